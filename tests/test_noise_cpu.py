"""Parity-mode noise (t5gemma_tts_amd/noise.py, csrc/noise.hip): the restatement of torch's
CPU exponential_ stream (SURVEY a14' 6) against torch itself, on the CPU.

The reference's torch.multinomial(p, 1) (hf_export/modeling_t5gemma_voice.py:133-138)
draws V exponential variates per call from torch's global MT19937 generator. The device
kernel computes raw MT19937 outputs; here numpy's MT19937, started from the words
noise.mt_words extracts from a torch generator, plays the device's role."""
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import noise as N  # noqa: E402

V = 65541


def _numpy_stream(words, n):
    bg = np.random.MT19937(0)
    bg.state = {"bit_generator": "MT19937", "state": {"key": words[:624].astype(np.uint32), "pos": int(words[624])}}
    return bg.random_raw(n).astype(np.uint32), bg


@pytest.mark.parametrize("seed", [1, 1234, 2**40 + 7])
def test_restated_draws_equal_torch(seed):
    """q of 3 consecutive multinomial calls (bf16, V draws each) from the raw MT19937 pairs
    equals torch's exponential_ bit for bit; the generator ends where torch's does."""
    g = torch.Generator().manual_seed(seed)
    w = N.mt_words(g)
    raw, bg = _numpy_stream(w, 3 * 2 * V)
    q = N.host_q(raw.reshape(3, V, 2))
    for s in range(3):
        ref = torch.empty(V, dtype=torch.bfloat16).exponential_(1, generator=g).float().numpy()
        assert np.array_equal(q[s], ref), f"step {s}: {(q[s] != ref).sum()} draws differ"
    st = bg.state["state"]
    w2 = N.mt_words(g)
    assert np.array_equal(w2[:624], st["key"].astype(np.uint32)) and int(w2[624]) == int(st["pos"])


def test_generator_mid_stream():
    """A generator that already drew (the reference's global generator after
    seed_everything and model loading) continues from its saved position."""
    g = torch.Generator().manual_seed(99)
    torch.empty(1001, dtype=torch.float64).exponential_(1, generator=g)   # odd position within a state
    w = N.mt_words(g)
    raw, _ = _numpy_stream(w, 2 * V)
    q = N.host_q(raw.reshape(V, 2))
    ref = torch.empty(V, dtype=torch.bfloat16).exponential_(1, generator=g).float().numpy()
    assert np.array_equal(q, ref)


def test_set_generator_roundtrip():
    g = torch.Generator().manual_seed(5)
    torch.empty(3 * V, dtype=torch.bfloat16).exponential_(1, generator=g)
    w = N.mt_words(g)
    g2 = torch.Generator().manual_seed(12345)
    N.set_generator(g2, w)
    a = torch.empty(V, dtype=torch.bfloat16).exponential_(1, generator=g)
    b = torch.empty(V, dtype=torch.bfloat16).exponential_(1, generator=g2)
    assert torch.equal(a, b)
    with pytest.raises(ValueError):
        w_bad = w.copy()
        w_bad[624] = 0
        N.set_generator(g2, w_bad)
