"""Golden fixtures for the host plumbing around generate(), produced by the REFERENCE's own
functions in this container (never on the GPU box):

* ``inference_tts_utils.inference_one_sample`` (:141-379) driven with a recording fake
  model / audio tokenizer / text tokenizer: what it hands ``model.inference_tts``
  (x, x_lens, y, tgt_y_lens, keyword arguments), what it passes to the codec decoder,
  and what it returns -- over reference audio with and without a sample cut, repeat
  prompts ("max" and an int), Japanese normalisation, x_sep / eos / bos insertion,
  silence tokens given as a string, parallel_pattern;
* ``data/tokenizer.tokenize_audio`` (:125-143) inside it, with a stand-in ``torchaudio``
  (load honours frame_offset / num_frames, Resample yields ceil(n * new / old) samples)
  and a fake encoder emitting n16k // 320 + 1 codes ([tf] Xcodec2 feature extractor
  padding);
* ``normalize_text_with_lang`` (:103-115) and ``duration_estimator.estimate_duration``
  (:207-252) on English / Japanese / Chinese / mixed strings, with and without a
  reference clip (a real 16-bit WAV written here; torchaudio.info reads its header).

Modules that are not installed here and that these functions import at top level are
replaced by a minimal stand-in (``torchaudio``); langdetect / g2p_en /
pyopenjtalk / pypinyin are absent, so the reference's own fallback branches are what
the fixtures pin. No reference source is copied: it is imported read-only.
Output: tests/golden/golden_pipeline.json, tests/golden/golden_text.json.
"""
from __future__ import annotations

import json
import math
import os
import sys
import tempfile
import types
import wave

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

AUDIO = {}   # path -> (n_samples, sample_rate, channels)


def _stub_modules():
    ta = types.ModuleType("torchaudio")

    def load(path, frame_offset=0, num_frames=-1):
        n, sr, ch = AUDIO[path]
        start = frame_offset or 0
        end = n if num_frames in (None, -1) else min(n, start + num_frames)
        t = torch.arange(start, end, dtype=torch.float32)
        wav = torch.stack([torch.sin(t * (0.01 + 0.003 * c)) for c in range(ch)])
        return wav, sr

    class Resample:
        def __init__(self, orig, new):
            self.orig, self.new = orig, new

        def __call__(self, wav):
            n = wav.shape[-1]
            m = math.ceil(n * self.new / self.orig)
            return torch.nn.functional.interpolate(wav[None], size=m, mode="linear")[0]

    class _Info:
        def __init__(self, n, sr):
            self.num_frames, self.sample_rate = n, sr

    def info(path):
        with wave.open(path, "rb") as w:
            return _Info(w.getnframes(), w.getframerate())

    ta.load = load
    ta.info = info
    ta.transforms = types.SimpleNamespace(Resample=Resample)
    sys.modules["torchaudio"] = ta


class FakeCodec:
    """Stands in for the reference's AudioTokenizer: encode emits n // 320 + 1 codes for n
    16 kHz samples; decode records the frames and returns zeros [B, 1, T * 882]."""
    encode_sample_rate = 16000
    sample_rate = 44100
    device = torch.device("cpu")

    def __init__(self):
        self.encoded, self.decoded = [], []

    def encode(self, wav):
        n = int(wav.shape[-1])
        self.encoded.append(n)
        T = n // 320 + 1
        return (torch.arange(T, dtype=torch.long) * 7919 % 65536).view(1, 1, T)

    def decode(self, frames):
        self.decoded.append(frames.tolist())
        return torch.zeros(frames.shape[0], 1, frames.shape[-1] * 882)


class FakeText:
    """Deterministic text tokenizer: one id per character (records every text)."""

    def __init__(self):
        self.texts = []

    def encode(self, text, add_special_tokens=True):
        assert add_special_tokens is False
        self.texts.append(text)
        return [10 + (ord(ch) * 31) % 250000 for ch in text]


class FakeModel:
    """Records the inference_tts call; 'generates' a fixed continuation with a y_sep and
    an EOS in it so the output stripping is exercised."""

    def __init__(self, gen):
        self.calls, self.gen = [], gen

    def inference_tts(self, x, x_lens, y, tgt_y_lens=None, **kw):
        self.calls.append({"x": x.tolist(), "x_lens": x_lens.tolist(), "y": y.tolist(),
                           "tgt_y_lens": tgt_y_lens.tolist(), "kw": {k: (list(v) if isinstance(v, (list, tuple))
                                                                         else v) for k, v in kw.items()}})
        g = torch.tensor(self.gen, dtype=torch.long).view(1, 1, -1)
        return torch.cat([y.transpose(2, 1), g], dim=2), g


class Args:
    def __init__(self, **kw):
        self.n_codebooks = 1
        self.empty_token, self.eog, self.eos, self.y_sep_token, self.x_sep_token = 65536, 65537, 65539, 65540, 255999
        self.audio_max_length = 40.0
        for k, v in kw.items():
            setattr(self, k, v)


def write_wav(path, n, sr):
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes((np.sin(np.arange(n) * 0.01) * 8000).astype("<i2").tobytes())


def pipeline_cases(td):
    a16 = os.path.join(td, "ref16k.wav")
    a44 = os.path.join(td, "ref44k.wav")
    AUDIO[a16] = (16000 * 3 + 77, 16000, 1)
    AUDIO[a44] = (44100 * 2 + 5, 44100, 2)
    base = dict(top_k=30, top_p=0.9, min_p=0.0, temperature=0.8, stop_repetition=3, codec_sr=50,
                codec_audio_sr=44100, silence_tokens=[], sample_batch_size=1)
    eos, sep = 65539, 65540
    return [
        dict(name="ja_ref_cut", audio=a44, text="こんにちは！　今日は、いい天気ですね～ＡＢＣ１２３", lang=None,
             prefix="ﾃｽﾄです…………", prompt_end_frame=int(1.5 * 44100), dur=2.0, repeat=0, args={},
             dc=dict(base), gen=[5, 6, sep, 7, eos]),
        dict(name="en_noref_eos_bos", audio=None, text="Hello there, world.", lang="en", prefix=None,
             prompt_end_frame=0, dur=3.5, repeat=0, args={"add_eos_to_text": 1, "add_bos_to_text": 2},
             dc=dict(base, silence_tokens="[1, 2, 3]", top_k=5), gen=[9, 9, 9, eos]),
        dict(name="en_ref_full_repeat2", audio=a16, text="A short test.", lang=None, prefix="The reference said this.",
             prompt_end_frame=0, dur=1.2, repeat=2, args={}, dc=dict(base, min_p=0.05), gen=[1, 2, 3, eos]),
        dict(name="repeat_max_parallel", audio=a16, text="More words here", lang="EN", prefix="ref words",
             prompt_end_frame=int(0.5 * 16000), dur=4.0, repeat="max", args={"parallel_pattern": 1,
                                                                           "audio_max_length": 6.0},
             dc=dict(base), gen=[4, eos]),
        dict(name="zh_text_ref_cut", audio=a16, text="你好，世界。", lang=None, prefix="参考文本",
             prompt_end_frame=int(0.33 * 16000), dur=1.0, repeat=0, args={}, dc=dict(base, temperature=1.0),
             gen=[3, 3, sep, eos]),
    ]


def gen_pipeline(IU):
    out = []
    with tempfile.TemporaryDirectory() as td:
        for c in pipeline_cases(td):
            model, codec, tt = FakeModel(c["gen"]), FakeCodec(), FakeText()
            res = IU.inference_one_sample(model, Args(**c["args"]), tt, codec, c["audio"], c["text"], c["lang"], "cpu",
                                          c["dc"], c["prompt_end_frame"], c["dur"], prefix_transcript=c["prefix"],
                                          quiet=True, repeat_prompt=c["repeat"], return_frames=True)
            cs, gs, cf, gf = res
            full_codes = None
            if c["audio"] is not None:
                n, sr, _ = AUDIO[c["audio"]]
                n16 = math.ceil(n * 16000 / sr)
                full_codes = (torch.arange(n16 // 320 + 1) * 7919 % 65536).tolist()
            rec = {k: v for k, v in c.items() if k not in ("audio",)}
            rec.update(audio=None if c["audio"] is None else {"n": AUDIO[c["audio"]][0], "sr": AUDIO[c["audio"]][1],
                                                              "channels": AUDIO[c["audio"]][2]},
                       full_codes=full_codes, encoded_samples=codec.encoded, texts=tt.texts, call=model.calls[0],
                       decoded=codec.decoded, concat_frames=cf.tolist(), gen_frames=gf.tolist(),
                       concat_shape=list(cs.shape), gen_shape=list(gs.shape))
            out.append(rec)
            print(f"[pipeline] {c['name']}: x {len(rec['call']['x'][0])} y {len(rec['call']['y'][0])} "
                  f"tgt {rec['call']['tgt_y_lens']}")
    return out


def gen_text(IU, DE):
    texts = ["Hello there, world.", "What? No... really -- yes!", "こんにちは！　今日は、いい天気ですね～",
             "ﾃｽﾄ１２３です…………", "你好，世界。我们走吧", "", "  spaced  ", "Mixed 日本語 text", "ＡＢＣ；ｄｅｆ"]
    norm = []
    for t in texts:
        for lang in (None, "ja", "EN", "zh-cn"):
            o, l = IU.normalize_text_with_lang(t, lang)
            norm.append({"text": t, "lang": lang, "out": o, "resolved": l})
    dur = []
    with tempfile.TemporaryDirectory() as td:
        wav = os.path.join(td, "ref.wav")
        write_wav(wav, 16000 * 4 + 123, 16000)
        for t in texts:
            for tl in (None, "ja", "en"):
                dur.append({"text": t, "target_lang": tl, "ref": None,
                            "seconds": DE.estimate_duration(t, target_lang=tl)})
            for rt, rl in (("the reference transcript here", None), ("参照の文章です", "ja"), (None, None)):
                dur.append({"text": t, "target_lang": None, "ref": {"n": 16000 * 4 + 123, "sr": 16000},
                            "reference_transcript": rt, "reference_lang": rl,
                            "seconds": DE.estimate_duration(t, reference_speech=wav, reference_transcript=rt,
                                                            reference_lang=rl)})
    det = [{"text": t, "lang": DE.detect_language(t)} for t in texts]
    return {"normalize": norm, "estimate_duration": dur, "detect_language": det}


if __name__ == "__main__":
    _stub_modules()
    sys.path.insert(0, REF)
    import duration_estimator as DE  # noqa: E402
    import inference_tts_utils as IU  # noqa: E402
    with open(os.path.join(HERE, "golden_pipeline.json"), "w") as f:
        json.dump({"torch": torch.__version__, "cases": gen_pipeline(IU)}, f, ensure_ascii=False, indent=0)
    with open(os.path.join(HERE, "golden_text.json"), "w") as f:
        json.dump(gen_text(IU, DE), f, ensure_ascii=False, indent=0)
    print("ok")
