"""Host plumbing of inference_one_sample on CPU: token assembly,
prompt framing, target length, _strip_sep_and_eos, and the call sequence against
stand-in model / codec objects. Expected values follow inference_tts_utils.py:140-378
line by line (the reference module itself is not importable here: it imports
torchaudio/whisper at top level)."""
import torch
import pytest

import t5gemma_tts_amd  # noqa: F401
from t5gemma_tts_amd.config import config_tiny
from t5gemma_tts_amd.pipeline import (build_prompt, build_text_tokens, inference_one_sample, strip_sep_and_eos,
                                      target_length)


class FakeTok:
    def encode(self, text, add_special_tokens=True):
        assert add_special_tokens is False
        return [len(w) + 10 for w in text.split()]


def test_text_tokens_order():
    assert build_text_tokens([5, 6], [1, 2], x_sep_token=99) == [1, 2, 99, 5, 6]
    assert build_text_tokens([5, 6], [1, 2], x_sep_token=None) == [1, 2, 5, 6]
    assert build_text_tokens([5], None, x_sep_token=99, add_eos_token=7, add_bos_token=3) == [3, 5, 7]
    assert build_text_tokens("  ab c ", "xyz", FakeTok(), 99) == [13, 99, 12, 11]
    with pytest.raises(ValueError):
        build_text_tokens("text")


def test_prompt_framing():
    oa = build_prompt([4, 5, 6], y_sep_token=68, codec_sr=50, target_generation_length=1.0)
    assert oa.shape == (1, 4, 1) and oa[0, :, 0].tolist() == [4, 5, 6, 68]
    assert build_prompt(None, 68, 50, 1.0).shape == (1, 0, 1)          # no reference -> no y_sep
    assert build_prompt(torch.tensor([[4], [5]]), 68, 50, 1.0)[0, :, 0].tolist() == [4, 5, 68]   # [T, 1]
    rep = build_prompt([4, 5], 68, 50, 1.0, repeat_prompt=2)
    assert rep[0, :, 0].tolist() == [4, 5, 4, 5, 4, 5, 68]
    mx = build_prompt([4, 5], 68, 50, 0.5, repeat_prompt="max", audio_max_length=1.0)
    # grows while 2k + 25 + 2 < 50
    assert mx.shape[1] == 24 + 1
    with pytest.raises(ValueError):
        build_prompt(torch.zeros(2, 2, 3, dtype=torch.long), 68, 50, 1.0)


def test_target_length():
    assert target_length(151, 50, 10.0) == 651
    assert target_length(0, 50, 3.0) == 150
    assert target_length(10, 50, 1.01) == 60
    assert target_length(10, 50, 1.0, parallel_pattern=1) == 62


def test_strip_sep_and_eos():
    f = torch.tensor([[[1, 2, 68, 3, 67]]])
    assert strip_sep_and_eos(f, 68, 67).tolist() == [[[1, 2, 3]]]
    g = torch.tensor([[[1, 2, 3]]])
    assert strip_sep_and_eos(g, 68, 67) is g
    # the reference compares kept counts across CODEBOOKS only (keep[..., :1]): with one
    # codebook, batch rows that keep different counts reach .view() and raise
    r = torch.tensor([[[1, 68, 2, 3]], [[4, 5, 6, 67]]])
    assert strip_sep_and_eos(r, 68, 67).tolist() == [[[1, 2, 3]], [[4, 5, 6]]]
    with pytest.raises(RuntimeError):
        strip_sep_and_eos(torch.tensor([[[1, 68, 67, 3]], [[4, 5, 6, 67]]]), 68, 67)
    # codebooks with different kept counts: cut to the minimum (ragged branch)
    k2 = torch.tensor([[[1, 68, 2, 3], [4, 5, 6, 67]]])
    assert strip_sep_and_eos(k2, 68, 67).tolist() == [[[1, 2, 3], [4, 5, 6]]]
    k3 = torch.tensor([[[1, 68, 67, 3], [4, 5, 6, 67]]])
    assert strip_sep_and_eos(k3, 68, 67).tolist() == [[[1, 3], [4, 5]]]
    assert strip_sep_and_eos(torch.tensor([[[68, 67]]]), 68, 67).shape == (1, 1, 0)


class FakeModel:
    def __init__(self, cfg):
        self.cfg, self.calls = cfg, []

    def inference_tts(self, x, x_lens, y, tgt_y_lens, **kw):
        self.calls.append((x, x_lens, y, tgt_y_lens, kw))
        gen = torch.tensor([[[7, 8, 9, self.cfg.eos]]])
        return torch.cat([y.transpose(1, 2), gen], 2), gen


class FakeCodec:
    def __init__(self):
        self.calls = []

    def decode(self, frames):
        self.calls.append(frames.clone())
        return torch.zeros(frames.shape[0], 1, frames.shape[-1] * 320)


def test_inference_one_sample_call_sequence():
    cfg = config_tiny()
    model, codec = FakeModel(cfg), FakeCodec()
    dc = {"top_k": 30, "top_p": 0.9, "min_p": 0.0, "temperature": 0.8, "stop_repetition": 3, "codec_sr": 50,
          "silence_tokens": "[1, 2]", "sample_batch_size": 1}
    cs, gs, cf, gf = inference_one_sample(model, cfg, None, codec, [3, 4, 5, 6], [20, 21], None, "cpu", dc,
                                          prompt_end_frame=800, target_generation_length=2.0, prefix_transcript=[9],
                                          quiet=True, return_frames=True)
    x, xl, y, tgt, kw = model.calls[0]
    assert x.tolist() == [[9, cfg.x_sep_token, 20, 21]] and xl.tolist() == [4]
    # prompt_end_frame counts audio SAMPLES (inference_commandline_hf.py:181): 800 samples at
    # 16 kHz encode to 800 // 320 + 1 = 3 codes
    assert y[0, :, 0].tolist() == [3, 4, 5, cfg.y_sep_token]
    assert tgt.tolist() == [4 + 100]
    assert kw["prompt_frames"] == 4 and kw["silence_tokens"] == [1, 2] and kw["top_k"] == 30
    assert cf.tolist() == [[[3, 4, 5, 7, 8, 9]]] and gf.tolist() == [[[7, 8, 9]]]
    assert len(codec.calls) == 2 and cs.shape == (1, 1, 6 * 320) and gs.shape == (1, 1, 3 * 320)
    # no reference audio: only the generated frames are decoded
    model2, codec2 = FakeModel(cfg), FakeCodec()
    cs2, gs2 = inference_one_sample(model2, cfg, None, codec2, None, [20], None, "cpu", dc, 0, 1.0, quiet=True)
    assert len(codec2.calls) == 1 and cs2 is gs2
    assert model2.calls[0][2].shape == (1, 0, 1) and model2.calls[0][3].tolist() == [50]
    with pytest.raises(AssertionError):
        inference_one_sample(model2, cfg, None, codec2, None, [20], None, "cpu", dict(dc, sample_batch_size=2), 0,
                             1.0, quiet=True)


def test_prompt_end_frame_is_a_sample_count():
    """0.05 s of a 44.1 kHz file (2205 samples) -> 800 samples at 16 kHz -> 3 codes; the
    reference's default cut_off_sec = 100 keeps every code of a short prompt."""
    from t5gemma_tts_amd.pipeline import prompt_frames_for_samples
    assert prompt_frames_for_samples(2205, 44100) == 3
    assert prompt_frames_for_samples(800, 16000) == 3
    assert prompt_frames_for_samples(639, 16000) == 2
    assert prompt_frames_for_samples(0, 16000) == 1
    cfg = config_tiny()
    model, codec = FakeModel(cfg), FakeCodec()
    dc = {"top_k": 30, "top_p": 0.9, "temperature": 0.8, "codec_sr": 50}
    inference_one_sample(model, cfg, None, codec, list(range(10)), [20], None, "cpu", dc,
                         prompt_end_frame=2205, target_generation_length=1.0, quiet=True, prompt_sample_rate=44100)
    assert model.calls[0][2][0, :, 0].tolist() == [0, 1, 2, cfg.y_sep_token]
    model, codec = FakeModel(cfg), FakeCodec()
    inference_one_sample(model, cfg, None, codec, list(range(10)), [20], None, "cpu", dc,
                         prompt_end_frame=int(100 * 44100), target_generation_length=1.0, quiet=True,
                         prompt_sample_rate=44100)
    assert model.calls[0][2][0, :, 0].tolist() == list(range(10)) + [cfg.y_sep_token]
