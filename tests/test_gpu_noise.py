"""Device MT19937 noise (csrc/noise.hip via t5g_mt_stream / t5g_mt_exponential) against
numpy's MT19937 and torch's own CPU exponential_ -- the draws of the reference's
torch.multinomial (hf_export/modeling_t5gemma_voice.py:133-138, SURVEY a14' 6)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

pytestmark = pytest.mark.gpu
V = 65541


def _np_stream(words, n):
    bg = np.random.MT19937(0)
    bg.state = {"bit_generator": "MT19937", "state": {"key": words[:624].astype(np.uint32), "pos": int(words[624])}}
    return bg.random_raw(n).astype(np.uint32), bg


def _gens():
    g0 = torch.Generator().manual_seed(3)
    g1 = torch.Generator().manual_seed(2**33 + 17)
    torch.empty(777, dtype=torch.float64).exponential_(1, generator=g1)   # mid-state position
    g2 = torch.Generator().manual_seed(8)
    torch.empty(312, dtype=torch.float64).exponential_(1, generator=g2)   # a state boundary (pos 624)
    return [g0, g1, g2]


def test_mt_stream_raw_and_snapshots():
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd import noise as N
    L = _lib.lib()
    gens = _gens()
    words = np.stack([N.mt_words(g) for g in gens])
    steps, V2 = 3, 2 * V
    n_out, stride = steps * V2, steps * V2 + 1000
    init = torch.from_numpy(words.view(np.int32)).cuda()
    out = torch.zeros(len(gens), stride, dtype=torch.int32, device="cuda")
    snap = torch.zeros(len(gens), steps + 1, 625, dtype=torch.int32, device="cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(L.t5g_mt_stream(C.c_void_p(init.data_ptr()), len(gens), n_out, stride, C.c_void_p(out.data_ptr()),
                               V2, steps + 1, C.c_void_p(snap.data_ptr()), st), "mt_stream")
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    sn = snap.cpu().numpy().view(np.uint32)
    for b, w in enumerate(words):
        ref, _ = _np_stream(w, n_out)
        assert np.array_equal(got[b, :n_out], ref), f"row {b}: {(got[b, :n_out] != ref).sum()} outputs differ"
        assert not got[b, n_out:].any(), "wrote past n_out"
        for s in range(steps + 1):
            _, bg = _np_stream(w, s * V2)
            stt = bg.state["state"]
            # the same generator: either identical words + position, or the position-624
            # form of the state numpy has already twisted
            r1, _ = _np_stream(sn[b, s], 4096)
            r2 = bg.random_raw(4096).astype(np.uint32)
            assert np.array_equal(r1, r2), f"row {b} snapshot {s} continues differently"
            assert 1 <= int(sn[b, s, 624]) <= 624 or (s == 0 and int(sn[b, s, 624]) == int(w[624]))
            del stt


def test_mt_exponential_equals_torch():
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd import noise as N
    L = _lib.lib()
    gens = _gens()
    ref_gens = [torch.Generator() for _ in gens]
    for g, r in zip(gens, ref_gens):
        r.set_state(g.get_state())
    dn = N.DeviceNoise(V, "cuda")
    steps = 4
    dn.generate(gens, steps, steps + 2, snapshots=True)
    dn.wait()
    for b, r in enumerate(ref_gens):
        for s in range(steps):
            want = torch.empty(V, dtype=torch.bfloat16).exponential_(1, generator=r)
            got = dn.q_row(b, s)
            assert torch.equal(got, want), f"row {b} step {s}: {(got != want).sum().item()} draws differ"
    # advancing by 2 and 4 steps leaves the torch generators where torch leaves them
    dn.advance_generators(gens, [2, 4, 0])
    chk = [torch.Generator() for _ in gens]
    for g, st_ in zip(chk, _gens()):
        g.set_state(st_.get_state())
    for g, n in zip(chk, [2, 4, 0]):
        for _ in range(n):
            torch.empty(V, dtype=torch.bfloat16).exponential_(1, generator=g)
    for g, c in zip(gens, chk):
        a = torch.empty(1000, dtype=torch.float64).exponential_(1, generator=g)
        b = torch.empty(1000, dtype=torch.float64).exponential_(1, generator=c)
        assert torch.equal(a, b)
    del L
