"""Command-line / Python entry with the reference CLI's surface:
``run_inference`` keeps ``inference_commandline_hf.py:72-242``'s arguments, defaults,
errors and outputs (``generated.wav`` + the max_abs / rms line, optional
``generated_frames.npy`` / ``concat_frames.npy``), running the MI355X engine and codec.

    python -m t5gemma_tts_amd.cli --model_dir ./t5gemma_voice_hf --codec_dir ./xcodec2_hf \\
        --tokenizer_dir ./gemma_tokenizer --target_text "..." --target_duration 3

Differences, all explicit:
* no network: the checkpoint (``model_dir``), the codec (``codec_dir``: a transformers
  ``Xcodec2Model`` directory, config.json + safetensors) and the Gemma tokenizer
  (``tokenizer_dir``; default: the checkpoint's ``text_tokenizer_name`` /
  ``t5gemma_model_name`` when that is a local directory) are local directories;
* ``synthetic="2b2b" | "tiny"`` runs seeded random weights of that architecture (and of the
  codec, ``codec`` "44k" | "16k" | "tiny") with a byte-level stand-in tokenizer -- for
  smoke runs and benchmarks only, the output is not speech;
* Whisper auto-transcription of ``reference_speech`` without ``reference_text``
  (:144-150) runs ``whisper_asr.load_model(whisper_model).transcribe(...)`` on the GPU;
  ``whisper_model`` names a local openai checkpoint (``~/.cache/whisper/<name>.pt``, the
  path whisper.load_model reads) or a transformers Whisper directory -- nothing is
  downloaded; ``asr_model`` may pass a loaded recognizer;
* ``fire`` is not installed: ``main`` parses the same flag names with argparse.
"""
from __future__ import annotations

import argparse
import os
import random
from typing import Optional

import numpy as np
import torch


def seed_everything(seed: int = 1) -> None:
    """inference_commandline_hf.py:62-69 (CUDA seeding is the ROCm device here)."""
    os.environ["PYTHONHASHSEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)


class ByteTokenizer:
    """Stand-in text tokenizer for synthetic-weight runs: UTF-8 bytes -> ids 3..258
    (below the x_sep id of every config). Not the Gemma tokenizer."""

    def encode(self, text, add_special_tokens=False):
        return [3 + b for b in str(text).encode("utf-8")]


def _none(v) -> bool:
    return v is None or str(v).strip().lower() in {"", "none", "null"}


# The reference CLI's extremes: a prompt cut at cut_off_sec = 100 s (inference_commandline_hf.py:91,
# 181) and a target clamped at 120 s by the duration estimator (duration_estimator.py:79, 251).
# The engine and codec are sized for them once; every call's work is sized by its own request
# (the decode attention grids follow the call's key bound, engine.py key_bound).
MAX_PROMPT_SECONDS = 100.0


def load_codec(codec_dir: Optional[str] = None, codec: str = "44k", device="cuda:0", max_batch: int = 4,
               max_frames: Optional[int] = None, seed: int = 22, max_encode_seconds: float = MAX_PROMPT_SECONDS):
    """XCodec2 decoder: from a local transformers ``Xcodec2Model`` directory, or seeded
    synthetic weights of the named size. ``max_frames`` (default: the engine's key capacity,
    prompt + target codes) bounds one decode; ``max_encode_seconds`` one prompt encode."""
    from .engine import MAX_AUDIO
    max_frames = MAX_AUDIO if max_frames is None else max_frames
    from .codec import AudioTokenizer, CodecConfig, codec_16k, codec_44k, codec_tiny, synthetic_codec_weights
    from .codec_enc import EncoderConfig, encoder_16k, encoder_tiny, synthetic_encoder_weights
    if codec_dir:
        import json

        from .weights import load_hf_checkpoint
        with open(os.path.join(codec_dir, "config.json")) as f:
            d = json.load(f)
        cfg = CodecConfig.from_hf_dict(d)
        sd = {k: v.float() for k, v in load_hf_checkpoint(codec_dir).items()}
        ecfg = EncoderConfig.from_hf_dict(d)
        esd = sd if "fc_encoder.weight" in sd else None     # a decoder-only export has no encoder
    else:
        cfg = {"44k": codec_44k, "16k": codec_16k, "tiny": codec_tiny}[codec]()
        sd = synthetic_codec_weights(cfg, seed)
        ecfg = encoder_tiny() if codec == "tiny" else encoder_16k()
        esd = synthetic_encoder_weights(ecfg, seed + 1)
    return AudioTokenizer(device=device, cfg=cfg, state_dict=sd, encoder_cfg=ecfg, encoder_state_dict=esd,
                          max_batch=max_batch, max_frames=max_frames, max_encode_seconds=max_encode_seconds)


def load_model(model_dir: Optional[str] = None, synthetic: Optional[str] = None, device="cuda:0",
               max_text: int = 512, max_audio: Optional[int] = None, seed: int = 7):
    """The voice model, sized for the reference CLI's longest request by default (max_audio =
    engine.MAX_AUDIO keys: a 100 s prompt + the 120 s duration cap; 1.3 GB of KV cache at
    batch 1) -- a shorter request runs on its own key bound, not the capacity."""
    from .engine import MAX_AUDIO, T5GemmaVoiceForConditionalGeneration
    kw = dict(device=device, max_batch=1, max_text=max_text, max_audio=MAX_AUDIO if max_audio is None else max_audio)
    if synthetic:
        from .config import named_config
        from .weights import synthetic_weights
        cfg = named_config(synthetic)
        return T5GemmaVoiceForConditionalGeneration(cfg, synthetic_weights(cfg, seed), **kw)
    if not model_dir or not os.path.isdir(model_dir):
        raise FileNotFoundError(f"model_dir {model_dir!r} is not a local HF export directory")
    return T5GemmaVoiceForConditionalGeneration.from_pretrained(model_dir, **kw)


def run_inference(reference_speech=None, target_text="こんにちは、私はAIです。これは音声合成のテストです。",
                  model_dir="./t5gemma_voice_hf", reference_text=None, target_duration=None, codec_audio_sr=16000,
                  codec_sr=50, top_k=30, top_p=0.9, min_p=0, temperature=0.8, silence_tokens=None, multi_trial=None,
                  repeat_prompt=0, stop_repetition=3, sample_batch_size=1, seed=1, output_dir="./generated_tts",
                  cut_off_sec=100, dump_tokens=False, lang=None, codec_dir=None, tokenizer_dir=None, synthetic=None,
                  codec="44k", device="cuda:0", whisper_model="large-v3-turbo", model=None, audio_tokenizer=None,
                  text_tokenizer=None, asr_model=None, parity=True):
    """inference_commandline_hf.py:72-242. ``model`` / ``audio_tokenizer`` /
    ``text_tokenizer`` / ``asr_model`` may be passed pre-built (then nothing is loaded).
    ``parity`` (default True, ``--parity False`` on the command line): reproduce the
    reference's tokens bit for bit (exact-order kernels, reference RNG stream, one host sync
    per step); False runs the fast graph-replayed path with on-device noise.
    Returns the path of the written wav."""
    from .audio import audio_info, write_wav
    from .pipeline import inference_one_sample, parse_silence_tokens
    from .text import estimate_duration, load_text_tokenizer, normalize_text_with_lang

    seed_everything(seed)
    if model is None:
        model = load_model(model_dir, synthetic, device)
    cfg = model.config
    if text_tokenizer is None:
        if synthetic and _none(tokenizer_dir):
            text_tokenizer = ByteTokenizer()
        else:
            name = tokenizer_dir or getattr(cfg, "text_tokenizer_name", None) or getattr(cfg, "t5gemma_model_name", None)
            text_tokenizer = load_text_tokenizer(name)
    if audio_tokenizer is None:
        audio_tokenizer = load_codec(codec_dir, codec, device)
    codec_sr = getattr(cfg, "encodec_sr", codec_sr)
    codec_audio_sr = audio_tokenizer.sample_rate            # :121-124
    silence_tokens = parse_silence_tokens(silence_tokens or [])
    multi_trial = multi_trial or []

    no_reference_audio = _none(reference_speech)
    has_reference_text = not _none(reference_text)
    if no_reference_audio and has_reference_text:              # :138-142
        raise ValueError("reference_text was provided but reference_speech is missing. "
                         "Please supply a reference_speech or omit reference_text.")
    if no_reference_audio:
        prefix_transcript = ""
    elif not has_reference_text:                               # :144-150
        if asr_model is None:
            from .whisper_asr import load_model as load_whisper
            asr_model = load_whisper(whisper_model, device=device)
        result = asr_model.transcribe(reference_speech)
        prefix_transcript = result["text"]
        print(f"[Info] Whisper transcribed text: {prefix_transcript}")
    else:
        prefix_transcript = reference_text

    lang = None if _none(lang) else str(lang)
    target_text, lang_code = normalize_text_with_lang(target_text, lang)
    if prefix_transcript:
        prefix_transcript, _ = normalize_text_with_lang(prefix_transcript, lang_code)
    if target_duration is None:
        target_generation_length = estimate_duration(
            target_text=target_text, reference_speech=None if no_reference_audio else reference_speech,
            reference_transcript=None if no_reference_audio else prefix_transcript, target_lang=lang_code,
            reference_lang=lang_code)
        print(f"[Info] target_duration not provided, estimated as {target_generation_length:.2f} seconds.")
    else:
        target_generation_length = float(target_duration)
    prompt_end_frame = 0
    prompt_sr = 16000
    if not no_reference_audio:
        if os.path.isfile(str(reference_speech)):
            _, prompt_sr = audio_info(reference_speech)
        prompt_end_frame = int(float(cut_off_sec) * prompt_sr)   # :172-183 (samples of the file)

    decode_config = {"top_k": top_k, "top_p": top_p, "min_p": min_p, "temperature": temperature,
                     "stop_repetition": stop_repetition, "codec_audio_sr": codec_audio_sr, "codec_sr": codec_sr,
                     "silence_tokens": silence_tokens, "sample_batch_size": sample_batch_size}
    res = inference_one_sample(model=model, model_args=cfg, text_tokenizer=text_tokenizer,
                               audio_tokenizer=audio_tokenizer,
                               audio_fn=None if no_reference_audio else reference_speech, target_text=target_text,
                               lang=lang_code, device=device, decode_config=decode_config,
                               prompt_end_frame=prompt_end_frame, target_generation_length=target_generation_length,
                               prefix_transcript=prefix_transcript, multi_trial=multi_trial,
                               repeat_prompt=repeat_prompt, return_frames=dump_tokens, prompt_sample_rate=prompt_sr,
                               parity=parity)
    if dump_tokens:
        concat_audio, gen_audio, concat_frames, gen_frames = res
    else:
        concat_audio, gen_audio = res
    gen_audio = gen_audio[0].cpu()
    os.makedirs(output_dir, exist_ok=True)
    out_path = os.path.join(output_dir, "generated.wav")
    write_wav(out_path, gen_audio.squeeze(), codec_audio_sr)
    max_abs = torch.max(gen_audio.abs()).item()
    rms = torch.sqrt((gen_audio ** 2).mean()).item()
    print(f"[Info] Generated audio stats -> max_abs: {max_abs:.6f}, rms: {rms:.6f}")
    if dump_tokens:
        np.save(os.path.join(output_dir, "generated_frames.npy"), gen_frames.squeeze(0).cpu().numpy())
        np.save(os.path.join(output_dir, "concat_frames.npy"), concat_frames.squeeze(0).cpu().numpy())
        print(f"[Info] Saved token arrays to {output_dir}")
    print(f"[Success] Generated audio saved to {out_path}")
    return out_path


def _arg(v: str):
    """fire-like literal parsing of a flag value (numbers, None, booleans, lists)."""
    import ast
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        low = v.strip().lower()
        return {"true": True, "false": False, "none": None}.get(low, v)


_SIGNATURE_OF = run_inference   # the flags (main() calls whatever run_inference is bound to)
_STR_ARGS = {"reference_speech", "target_text", "model_dir", "reference_text", "output_dir", "lang", "codec_dir",
             "tokenizer_dir", "synthetic", "codec", "device", "whisper_model"}


def main(argv=None) -> None:
    import inspect
    sig = inspect.signature(_SIGNATURE_OF)
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    for name, p in sig.parameters.items():
        if name in ("model", "audio_tokenizer", "text_tokenizer", "asr_model"):
            continue
        ap.add_argument(f"--{name}", type=str if name in _STR_ARGS else _arg, default=p.default)
    args = ap.parse_args(argv)
    run_inference(**vars(args))


if __name__ == "__main__":
    main()
