"""The device sampler's sparse emulation of torch.sort's tie order (csrc/sort_emu.h, host
build t5g_sort_emu) against libstdc++ std::sort run in full (oracle/sort_order.cpp, the
order torch 2.10's CPU sort leaves equal keys in; SURVEY a14' 5).

Arrays of n entries, -inf except S survivors (the top-k filter's output,
hf_export/modeling_t5gemma_voice.py:101-105), sorted descending as top_k_top_p_filtering
does (:107-108): the emulation must give every survivor the slot std::sort gives it."""
import ctypes as C
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


@pytest.fixture(scope="module")
def libs():
    import importlib.util
    spec = importlib.util.spec_from_file_location("_b", os.path.join(REPO, "t5gemma-tts_amd", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    ol = C.CDLL(mod.build_oracle())
    ol.oracle_sort_desc.argtypes = [C.c_void_p, C.c_int64, C.c_void_p]
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd import _lib
    return ol, _lib.lib()


def _check(libs, n, idx, vals):
    ol, L = libs
    idx = np.asarray(idx, np.int64)
    vals = np.asarray(vals, np.float32)
    full = np.full(n, -np.inf, np.float32)
    full[idx] = vals
    perm = np.empty(n, np.int64)
    ol.oracle_sort_desc(full.ctypes.data, n, perm.ctypes.data)
    o = np.argsort(idx)
    pos = idx[o].astype(np.int32).copy()
    val = vals[o].copy()
    tag = idx[o].astype(np.int32).copy()
    rc = L.t5g_sort_emu(n, len(pos), pos.ctypes.data, val.ctypes.data, tag.ctypes.data)
    assert rc == 0, rc
    S = len(idx)
    want = perm[:S]
    assert np.array_equal(tag.astype(np.int64), want), (tag[:20], want[:20])
    assert np.array_equal(pos, np.arange(S, dtype=np.int32))


@pytest.mark.parametrize("n", [17, 40, 100, 1000, 4099, 65541])
def test_sort_emu_random_ties(libs, n):
    rng = np.random.default_rng(n)
    for it in range(60):
        S = int(rng.integers(1, min(n, 256) + 1))
        idx = rng.choice(n, size=S, replace=False)
        nv = int(rng.integers(1, 6))
        vals = rng.choice(np.linspace(-3, 3, nv), size=S).astype(np.float32)
        _check(libs, n, idx, vals)


def test_sort_emu_clusters(libs):
    """Survivors packed together (leading / trailing / mid runs): survivor pivots."""
    n = 65541
    rng = np.random.default_rng(3)
    for start in (0, 5, 100, 32767, 65541 - 300, 65541 - 64):
        for S in (16, 30, 64, 200):
            if start + S > n:
                continue
            idx = np.arange(start, start + S)
            vals = rng.choice(np.array([1.0, 1.0, 2.0, 0.5], np.float32), size=S)
            _check(libs, n, idx, vals)


def test_sort_emu_topk_logits(libs):
    """Realistic rows: bf16 logits / T, top-k 30 survivors (ties kept)."""
    V = 65541
    g = torch.Generator().manual_seed(11)
    for it in range(40):
        x = (torch.randn(V, generator=g) * (0.5 + it % 4)).to(torch.bfloat16)
        x = (x.float() / 0.8).to(torch.bfloat16).float()
        thr = torch.topk(x, 30).values[-1]
        keep = torch.nonzero(x >= thr).view(-1).numpy()
        _check(libs, V, keep, x.numpy()[keep])
