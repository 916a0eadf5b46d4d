"""Whisper recognizer on the GPU (whs_* C ABI) against transformers'
WhisperForConditionalGeneration goldens (tests/golden/make_golden_whisper.py) at test
dims and at large-v3-turbo dims (128 mels, 32 x 1280 encoder, 4 x 1280 decoder):

* log-mel vs the oracle's torch.stft restatement of openai's log_mel_spectrogram
  (fp32 DFT GEMM vs FFT: <= 2e-3 on the (x + 4) / 4 scale);
* encoder output of the first window and teacher-forced decoder logits (prefill, then one
  token at a time through the self-attention cache) within 2e-3 x their RMS, argmax equal;
* detect_language's choice, and the tokens of transcribe(audio, temperature=0) -- the
  host control flow over the GPU logits -- equal to the oracle's.
Parity against the openai-whisper package itself is unpinned (absent)."""
import json
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, GOLDEN)


def _load(name):
    with open(os.path.join(GOLDEN, f"golden_whisper_{name}.json")) as f:
        meta = json.load(f)
    return meta, dict(np.load(os.path.join(GOLDEN, f"golden_whisper_{name}.npz")))


def _setup(name, tmp_path):
    from t5gemma_tts_amd import whisper_asr as w
    from make_golden_codec_enc import test_wave
    from whisper_oracle import write_synthetic_tiktoken
    meta, z = _load(name)
    dims = w.WhisperDims(**meta["model_dims"])
    p = str(tmp_path / "v.tiktoken")
    write_synthetic_tiktoken(p, 50257, meta["tok_seed"])
    tok = w.WhisperTokenizer.from_tiktoken(p, dims.num_languages)
    m = w.WhisperModel(dims, w.synthetic_weights(dims, meta["weight_seed"]), device="cuda:0", max_seconds=30.0,
                       tokenizer=tok)
    audio = test_wave(int(meta["audio_seconds"] * 16000), meta["audio_seed"])
    return w, meta, z, m, tok, audio


@pytest.mark.parametrize("name", ["tiny", "turbo"])
def test_whisper_model_vs_transformers_golden(name, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from whisper_oracle import ref_log_mel
    w, meta, z, m, tok, audio = _setup(name, tmp_path)
    mel = m.log_mel(audio, out=True).cpu()
    ref = ref_log_mel(audio, m.dims.n_mels).T
    merr = (mel - ref).abs().max().item()
    assert m.mel_frames == meta["content_frames"] + 3000
    feat = m.encode(0, meta["content_frames"], out=True).cpu()[::25]
    ref_feat = torch.from_numpy(z["feat_rows"])
    ferr = ((feat - ref_feat).abs().max() / ref_feat.pow(2).mean().sqrt()).item()
    toks = meta["teacher_tokens"]
    rows = [m.logits(toks[:3], 0).cpu().clone()]
    for i in range(3, len(toks)):
        rows.append(m.logits(toks[i:i + 1], i).cpu().clone())
    lg = torch.cat(rows, 0)
    sub = torch.from_numpy(z["sub"]).long()
    ref_lg = torch.from_numpy(z["logits_sub"])
    lerr = ((lg[:, sub] - ref_lg).abs().max() / ref_lg.pow(2).mean().sqrt()).item()
    print(f"{name}: mel max err {merr:.2e}, encoder err/rms {ferr:.2e}, logits err/rms {lerr:.2e}")
    assert merr <= 2e-3, merr
    assert ferr <= 2e-3, ferr
    assert lerr <= 2e-3, lerr
    assert lg.argmax(-1).tolist() == meta["logit_argmax"]


@pytest.mark.parametrize("name", ["tiny", "turbo"])
def test_whisper_transcribe_vs_oracle(name, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    w, meta, z, m, tok, audio = _setup(name, tmp_path)
    m.log_mel(audio)
    lang, probs = m.detect_language(tok.with_language("en"))
    assert lang == meta["language"]
    for code, p in meta["language_top5"]:
        assert abs(probs[code] - p) < 1e-3 * max(p, 1e-3) + 1e-5, (code, probs[code], p)
    r = m.transcribe(audio, temperature=0.0)
    got = [s["tokens"] for s in r["segments"]]
    want = [s["tokens"] for s in meta["segments"]]
    print(f"{name}: language {r['language']}, {len(got)} segments, tokens equal: {got == want}")
    assert r["language"] == meta["transcribe_language"]
    assert got == want
    for s, g in zip(r["segments"], meta["segments"]):
        assert abs(s["start"] - g["start"]) < 1e-9 and abs(s["end"] - g["end"]) < 1e-9


def test_transcribe_wav_file_and_capacity(tmp_path):
    """A reference WAV at 44.1 kHz is resampled to 16 kHz as openai's ffmpeg loader does;
    audio longer than the recognizer's capacity is refused."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from t5gemma_tts_amd.audio import resample, write_wav
    w, meta, z, m, tok, audio = _setup("tiny", tmp_path)
    path = str(tmp_path / "ref.wav")
    write_wav(path, resample(audio[None], 16000, 44100)[0], 44100)
    r = m.transcribe(path, temperature=0.0, language="en")
    assert r["language"] == "en" and isinstance(r["text"], str)
    with pytest.raises(ValueError):
        m.log_mel(torch.zeros(31 * 16000))
