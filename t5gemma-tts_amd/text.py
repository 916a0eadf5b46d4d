"""Text front end of the generate() path: what the reference does to
the target / reference text before ``inference_tts`` sees token ids.

* ``normalize_text_with_lang`` -- inference_tts_utils.py:89-115 (Japanese-only
  normalisation: replacement map, full-width alphanumerics and digits to half-width,
  half-width katakana to full-width, ellipsis collapse; the language is resolved once
  and reused for the prefix transcript);
* ``detect_language`` -- duration_estimator.py:88-117, 185-187 (langdetect when it is
  importable, else the kana / CJK character heuristic, else English);
* ``estimate_duration`` -- duration_estimator.py:207-252 (phonemes x seconds-per-phoneme
  + punctuation pauses, clamped to [0.5, 120] s; with a reference clip the pace is
  derived from it and clamped per language);
* ``load_text_tokenizer`` -- the ``AutoTokenizer.from_pretrained(tokenizer_name)`` call of
  inference_commandline_hf.py:112-113, restricted to local directories (no network).

The reference's optional g2p back ends (g2p_en + nltk, pyopenjtalk, pypinyin) and
langdetect are used here exactly when they are importable, and fall back the way the
reference falls back (character counts / heuristic) when they are not; in this build
image none of them is installed, so the fallback path is the one pinned by the golden
fixtures (tests/golden/golden_text.json, produced by the reference's own functions).
This is host-side string work: nothing here touches the GPU.
"""
from __future__ import annotations

import os
import re
import wave
from typing import Optional, Tuple

# ---------------------------------------------------------------- normalisation
_REPLACE = [
    (r"\t", ""),
    (r"\[n\]", ""),
    (r" ", ""),
    (r"　", ""),
    (r"[;▼♀♂《》≪≫①②③④⑤⑥]", ""),
    (r"[\u02d7\u2010-\u2015\u2043\u2212\u23af\u23e4\u2500\u2501\u2e3a\u2e3b]", ""),
    (r"[\uff5e\u301C]", "ー"),
    (r"？", "?"),
    (r"！", "!"),
    (r"[●◯〇]", "○"),
    (r"♥", "♡"),
]
_ALNUM_FW = {0xFF21 + i: 0x41 + i for i in range(26)}
_ALNUM_FW.update({0xFF41 + i: 0x61 + i for i in range(26)})
_DIGITS_FW = {0xFF10 + i: 0x30 + i for i in range(10)}
_KATA_HW = "ｦｧｨｩｪｫｬｭｮｯｰｱｲｳｴｵｶｷｸｹｺｻｼｽｾｿﾀﾁﾂﾃﾄﾅﾆﾇﾈﾉﾊﾋﾌﾍﾎﾏﾐﾑﾒﾓﾔﾕﾖﾗﾘﾙﾚﾛﾜﾝ"
_KATA_FW = "ヲァィゥェォャュョッーアイウエオカキクケコサシスセソタチツテトナニヌネノハヒフヘホマミムメモヤユヨラリルレロワン"
_KATA = str.maketrans(_KATA_HW, _KATA_FW)


def normalize_japanese(text: str) -> str:
    """inference_tts_utils.py:89-100 (same rule order)."""
    for pat, rep in _REPLACE:
        text = re.sub(pat, rep, text)
    text = text.translate(_ALNUM_FW).translate(_DIGITS_FW).translate(_KATA)
    return re.sub(r"…{3,}", "……", text)


def normalize_text_with_lang(text: str, lang: Optional[str]) -> Tuple[str, Optional[str]]:
    """inference_tts_utils.py:103-115: normalise iff the (given or detected) language is
    Japanese; returns (text, resolved language) so callers do not detect twice."""
    resolved = lang.lower() if isinstance(lang, str) else None
    if not text:
        return text, resolved
    if resolved is None:
        resolved = detect_language(text)
    if resolved and resolved.startswith("ja"):
        return normalize_japanese(text), resolved
    return text, resolved


# ---------------------------------------------------------------- language detection
def _langdetect():
    try:
        from langdetect import DetectorFactory, LangDetectException, detect
        DetectorFactory.seed = 0
        return detect, LangDetectException
    except ImportError:
        return None, Exception


def detect_language(text: str) -> str:
    """duration_estimator.py:88-117: coarse en / ja / zh / other."""
    text = text.strip()
    if not text:
        return "other"
    detect, err = _langdetect()
    if detect is not None:
        try:
            lang = detect(text)
            if lang.startswith("ja"):
                return "ja"
            if lang.startswith("zh") or lang in {"yue"}:
                return "zh"
            if lang.startswith("en"):
                return "en"
        except err:
            pass
    if re.search(r"[\u3040-\u30ff]", text):
        return "ja"
    if re.search(r"[\u4e00-\u9fff]", text):
        return "zh"
    return "en"


def canonical_lang(lang: Optional[str]) -> Optional[str]:
    """duration_estimator.py:190-200."""
    if not lang:
        return None
    lang = lang.lower()
    if lang.startswith("ja"):
        return "ja"
    if lang.startswith("zh") or lang in {"yue"}:
        return "zh"
    if lang.startswith("en"):
        return "en"
    return lang


# ---------------------------------------------------------------- duration estimate
SPP_DEFAULT = {"en": 0.085, "ja": 0.10, "zh": 0.27, "other": 0.11}
SPP_MINMAX = {"en": (0.06, 0.12), "ja": (0.07, 0.15), "zh": (0.18, 0.36), "other": (0.07, 0.18)}
MIN_DURATION_SEC, MAX_DURATION_SEC = 0.5, 120.0
_g2p_en = None


def _count_en(text: str) -> int:
    global _g2p_en
    try:
        from g2p_en import G2p
    except ImportError:
        return len(text)
    if _g2p_en is None:
        _g2p_en = G2p()
    return len([p for p in _g2p_en(text) if p and p not in {" ", "<pad>", "<s>", "</s>", "<unk>"}])


def _count_ja(text: str) -> int:
    try:
        import pyopenjtalk
    except ImportError:
        return len(text)
    return len([p for p in pyopenjtalk.g2p(text).split(" ") if p and p not in {"pau", "sil"}])


def _count_zh(text: str) -> int:
    try:
        from pypinyin import Style, lazy_pinyin
    except ImportError:
        return len(text)
    syl = lazy_pinyin(text, style=Style.NORMAL, neutral_tone_with_five=True)
    return len([s for s in syl if s and re.search(r"[a-zA-Z]", s)])


def phoneme_count(text: str, lang: str) -> int:
    """duration_estimator.py:147-155."""
    if lang == "en":
        return _count_en(text)
    if lang == "ja":
        return _count_ja(text)
    if lang == "zh":
        return _count_zh(text)
    return max(len(text), 1)


def punctuation_bonus_sec(text: str) -> float:
    """duration_estimator.py:158-182."""
    t = text.strip()
    major = len(re.findall(r"[.!?。！？]", t))
    minor = len(re.findall(r"[、，,;；:]", t))
    if t and t[-1] in ".!?。！？":
        major = max(0, major - 1)
    ellipsis = len(re.findall(r"(…|\.\.\.)", t))
    dash = len(re.findall(r"(—|--)", t))
    return min(10.0, major * 0.40 + minor * 0.20 + ellipsis * 1.0 + dash * 0.12)


def audio_duration_sec(path: str) -> Optional[float]:
    """Length of an audio file in seconds (the reference reads torchaudio.info's
    num_frames / sample_rate): WAV through the standard library, other formats through
    soundfile when it is importable; None when unreadable."""
    try:
        with wave.open(path, "rb") as w:
            return w.getnframes() / float(w.getframerate())
    except (wave.Error, EOFError, OSError):
        pass
    try:
        import soundfile as sf
        info = sf.info(path)
        return info.frames / float(info.samplerate)
    except Exception:
        return None


def estimate_duration(target_text: str, reference_speech: Optional[str] = None,
                      reference_transcript: Optional[str] = None, target_lang: Optional[str] = None,
                      reference_lang: Optional[str] = None) -> float:
    """duration_estimator.py:207-252: target seconds from phoneme-aware pacing."""
    target_text = target_text or ""
    ref_has_audio = bool(reference_speech) and os.path.isfile(reference_speech)
    tgt_lang = canonical_lang(target_lang) or (detect_language(target_text) if target_text else "en")
    tgt_ph = max(phoneme_count(target_text, tgt_lang), 1)
    spp = SPP_DEFAULT.get(tgt_lang, SPP_DEFAULT["other"])
    if ref_has_audio:
        dur = audio_duration_sec(reference_speech)
        if dur and dur > 0:
            ref_text = reference_transcript or target_text
            ref_lang = canonical_lang(reference_lang) or detect_language(ref_text)
            ref_ph = max(phoneme_count(ref_text, ref_lang), 1)
            lo, hi = SPP_MINMAX.get(ref_lang, SPP_MINMAX["other"])
            spp = max(lo, min(hi, dur / ref_ph))
    bonus = punctuation_bonus_sec(target_text) * (0.3 if ref_has_audio else 1.0)
    return max(MIN_DURATION_SEC, min(tgt_ph * spp + bonus, MAX_DURATION_SEC))


# ---------------------------------------------------------------- tokenizer
def load_text_tokenizer(name_or_dir: str):
    """``AutoTokenizer.from_pretrained`` on a local directory (the Gemma SentencePiece
    tokenizer the checkpoint names, inference_commandline_hf.py:112-113). Hub names are
    refused: there is no network in this deployment."""
    if not name_or_dir or not os.path.isdir(name_or_dir):
        raise FileNotFoundError(f"text tokenizer directory not found: {name_or_dir!r} (hub downloads are not "
                                "available; pass a local directory holding tokenizer.json / tokenizer.model)")
    from transformers import AutoTokenizer
    return AutoTokenizer.from_pretrained(name_or_dir)
