"""The sampler's one-wave replay of torch.sort's tie order (csrc/sort_emu.h se_sort_wave,
the device path for <= 63 finite survivors) == the single-thread replay (se_sort, itself
pinned against libstdc++ std::sort in tests/test_sort_emu_cpu.py): same final slot of
every survivor, same fail code, on random tie-heavy rows, packed clusters and top-k 30
logit rows of the real vocabulary. Bitwise (slots are integers)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _cases():
    rng = np.random.default_rng(21)
    out = []
    for n in (17, 40, 100, 1000, 4099, 65541):
        for _ in range(25):
            S = int(rng.integers(1, min(n, 63) + 1))
            idx = np.sort(rng.choice(n, size=S, replace=False))
            vals = rng.choice(np.linspace(-3, 3, int(rng.integers(1, 6))), size=S).astype(np.float32)
            out.append((n, idx, vals))
    for start in (0, 5, 100, 32767, 65541 - 64):
        for S in (16, 30, 63):
            idx = np.arange(start, start + S)
            out.append((65541, idx, rng.choice(np.array([1.0, 1.0, 2.0, 0.5], np.float32), size=S)))
    g = torch.Generator().manual_seed(12)
    for it in range(30):
        x = (torch.randn(65541, generator=g) * (0.5 + it % 4)).to(torch.bfloat16)
        x = (x.float() / 0.8).to(torch.bfloat16).float()
        keep = torch.nonzero(x >= torch.topk(x, 30).values[-1]).view(-1).numpy()
        if len(keep) <= 63:
            out.append((65541, keep, x.numpy()[keep]))
    return out


def test_sort_emu_wave_equals_single_thread():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    n_fail_match = 0
    for n, idx, vals in _cases():
        pos = idx.astype(np.int32).copy()
        val = vals.astype(np.float32).copy()
        tag = np.arange(len(idx), dtype=np.int32)
        rc_h = L.t5g_sort_emu(n, len(pos), pos.ctypes.data, val.ctypes.data, tag.ctypes.data)
        dp = torch.from_numpy(idx.astype(np.int32)).cuda()
        dv = torch.from_numpy(vals.astype(np.float32)).cuda()
        dt = torch.arange(len(idx), dtype=torch.int32, device="cuda")
        fail = torch.full((1,), -7, dtype=torch.int32, device="cuda")
        assert L.t5g_sort_emu_wave(n, len(idx), C.c_void_p(dp.data_ptr()), C.c_void_p(dv.data_ptr()),
                                   C.c_void_p(dt.data_ptr()), C.c_void_p(fail.data_ptr()), st) == 0
        torch.cuda.synchronize()
        rc_d = int(fail.item())
        assert rc_d == rc_h, (n, len(idx), rc_d, rc_h)
        if rc_h == 0:
            assert np.array_equal(dp.cpu().numpy(), pos), (n, len(idx))
            assert np.array_equal(dt.cpu().numpy(), tag), (n, len(idx))
            assert np.array_equal(dv.cpu().numpy(), val)
        else:
            n_fail_match += 1
    assert n_fail_match < len(_cases()) // 4
