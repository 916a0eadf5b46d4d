"""The host plumbing around generate() against fixtures captured from the REFERENCE's own
functions (tests/golden/make_golden_pipeline.py, run in the build container):

* pipeline.inference_one_sample vs inference_tts_utils.inference_one_sample (:141-379):
  the exact (x, x_lens, y, tgt_y_lens, kwargs) handed to inference_tts, the frames
  handed to the codec decoder, and the returned frames / shapes -- for reference audio
  cut by a sample count (44.1 kHz stereo and 16 kHz files), no reference, repeat_prompt
  2 and "max", Japanese normalisation, eos / bos / x_sep insertion, string silence
  tokens, parallel_pattern;
* text.normalize_text_with_lang / detect_language / estimate_duration vs the reference's
  (inference_tts_utils.py:103-115, duration_estimator.py:88-252), g2p back ends absent
  on both sides (their fallbacks are what is pinned).
The reference's prompt went through data/tokenizer.tokenize_audio with a stand-in
encoder of n16k // 320 + 1 codes; here the same codes are passed as ids and cut by
pipeline.prompt_frames_for_samples."""
import json
import os
import tempfile
import wave

import numpy as np
import pytest
import torch

from conftest import GOLDEN

import t5gemma_tts_amd  # noqa: F401
from t5gemma_tts_amd.pipeline import inference_one_sample
from t5gemma_tts_amd import text as T


def _load(name):
    with open(os.path.join(GOLDEN, name), encoding="utf-8") as f:
        return json.load(f)


class FakeText:
    def encode(self, text, add_special_tokens=True):
        assert add_special_tokens is False
        return [10 + (ord(ch) * 31) % 250000 for ch in text]


class FakeModel:
    def __init__(self, gen):
        self.calls, self.gen = [], gen

    def inference_tts(self, x, x_lens, y, tgt_y_lens=None, **kw):
        self.calls.append({"x": x.tolist(), "x_lens": x_lens.tolist(), "y": y.tolist(),
                           "tgt_y_lens": tgt_y_lens.tolist(), "kw": kw})
        g = torch.tensor(self.gen, dtype=torch.long).view(1, 1, -1)
        return torch.cat([y.transpose(2, 1), g], dim=2), g


class FakeCodec:
    def __init__(self):
        self.decoded = []

    def decode(self, frames):
        self.decoded.append(frames.tolist())
        return torch.zeros(frames.shape[0], 1, frames.shape[-1] * 882)


class Args:
    def __init__(self, **kw):
        self.n_codebooks = 1
        self.empty_token, self.eog, self.eos, self.y_sep_token, self.x_sep_token = 65536, 65537, 65539, 65540, 255999
        self.audio_max_length = 40.0
        for k, v in kw.items():
            setattr(self, k, v)


@pytest.mark.parametrize("case", [c["name"] for c in _load("golden_pipeline.json")["cases"]])
def test_inference_one_sample_matches_reference(case):
    c = next(c for c in _load("golden_pipeline.json")["cases"] if c["name"] == case)
    model, codec = FakeModel(c["gen"]), FakeCodec()
    audio = None if c["audio"] is None else c["full_codes"]
    sr = 16000 if c["audio"] is None else c["audio"]["sr"]
    cs, gs, cf, gf = inference_one_sample(model, Args(**c["args"]), FakeText(), codec, audio, c["text"], c["lang"],
                                          "cpu", c["dc"], c["prompt_end_frame"], c["dur"],
                                          prefix_transcript=c["prefix"], quiet=True, repeat_prompt=c["repeat"],
                                          return_frames=True, prompt_sample_rate=sr)
    got, want = model.calls[0], c["call"]
    assert got["x"] == want["x"] and got["x_lens"] == want["x_lens"]
    assert got["y"] == want["y"]
    assert got["tgt_y_lens"] == want["tgt_y_lens"]
    for k, v in want["kw"].items():
        gv = got["kw"][k]
        assert (list(gv) if isinstance(gv, (list, tuple)) else gv) == v, k
    assert codec.decoded == c["decoded"]
    assert cf.tolist() == c["concat_frames"] and gf.tolist() == c["gen_frames"]
    assert list(cs.shape) == c["concat_shape"] and list(gs.shape) == c["gen_shape"]


def test_normalize_and_detect_match_reference():
    g = _load("golden_text.json")
    for r in g["normalize"]:
        assert list(T.normalize_text_with_lang(r["text"], r["lang"])) == [r["out"], r["resolved"]], r
    for r in g["detect_language"]:
        assert T.detect_language(r["text"]) == r["lang"], r


def test_estimate_duration_matches_reference():
    g = _load("golden_text.json")
    with tempfile.TemporaryDirectory() as td:
        for r in g["estimate_duration"]:
            ref = None
            if r["ref"] is not None:
                ref = os.path.join(td, "ref.wav")
                if not os.path.exists(ref):
                    with wave.open(ref, "wb") as w:
                        w.setnchannels(1)
                        w.setsampwidth(2)
                        w.setframerate(r["ref"]["sr"])
                        w.writeframes(np.zeros(r["ref"]["n"], dtype="<i2").tobytes())
            got = T.estimate_duration(r["text"], reference_speech=ref,
                                      reference_transcript=r.get("reference_transcript"),
                                      target_lang=r["target_lang"], reference_lang=r.get("reference_lang"))
            assert got == r["seconds"], r


def test_audio_resample_and_wav_roundtrip():
    from t5gemma_tts_amd.audio import load_audio, resample, write_wav
    x = torch.sin(torch.arange(44100 * 2 + 5, dtype=torch.float32) * 0.05)[None] * 0.5
    y = resample(x, 44100, 16000)
    assert y.shape[-1] == -(-(44100 * 2 + 5) * 16000 // 44100)
    # a band-limited tone keeps its amplitude through the sinc resampler (away from edges)
    assert abs(y[0, 2000:-2000].abs().max().item() - 0.5) < 0.01
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "a.wav")
        write_wav(p, x[0], 44100)
        w, sr = load_audio(p, frame_offset=10, num_frames=1000)
        assert sr == 44100 and w.shape == (1, 1000)
        assert (w[0] - x[0, 10:1010]).abs().max().item() < 1.0 / 32767 + 1e-6
