"""CPU-side checks of libt5gtts.so: it loads, exports every symbol include/t5gtts.h
declares, and its host-only parity sampler (std::sort tie order) reproduces the
reference's sampler golden cases. No GPU compute is invoked."""
import ctypes as C
import json
import os
import re

import pytest
import torch

from conftest import GOLDEN, REPO


def _header_symbols():
    src = open(os.path.join(REPO, "include", "t5gtts.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(t5g_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_struct_layouts_match_header():
    from t5gemma_tts_amd import _lib
    assert C.sizeof(_lib.SamplerRow) == 48
    assert C.sizeof(_lib.SamplerState) == 48
    assert C.sizeof(_lib.LayerWeights) == 13 * 8
    assert C.sizeof(_lib.AttnDecodeArgs) == 4 * 4 + 3 * 8 + 8 + 8 + 4 * 4 + 2 * 8
    assert C.sizeof(_lib.GemvArgs) == 152


def test_packed_bytes():
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    assert L.t5g_packed_bytes(4096, 2304) == 4096 * 2304 * 2
    assert L.t5g_packed_bytes(65541, 2304) == 4100 * 16 * 2304 * 2  # row groups padded to x4
    assert L.t5g_packed_bytes(16, 33) < 0


def test_host_sampler_matches_reference_golden():
    """t5g_host_sample (exact std::sort tie order) on every reference sampler case."""
    from tests.golden.make_golden import make_sampler_logits
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.engine import reference_noise
    L = _lib.lib()
    meta = json.load(open(os.path.join(GOLDEN, "golden_sampler.json")))
    for c in meta["cases"]:
        V = c["V"]
        logits = make_sampler_logits(c["logit_seed"], V, c["scale"], c["quant"]).contiguous()
        noise = reference_noise(c["noise_seed"], 1, V)[0].contiguous()
        row = _lib.SamplerRow(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"],
                              temperature=c["temperature"])
        st = _lib.SamplerState(cur_num_gen=100, current_length=200, prompt_offset=1, target_total=-1,
                               est_total=1000, prev_token=-1, first_input_len=5)
        out = _lib.SamplerState()
        tok = C.c_int32()
        tk = (C.c_int32 * 1)()
        rc = L.t5g_host_sample(C.c_void_p(logits.data_ptr()), V, C.byref(row), tk, tk, C.byref(st),
                               C.c_void_p(noise.data_ptr()), 65539, 10, 250.0, 0, 2000.0, 4096, 4096,
                               C.byref(out), C.byref(tok))
        assert rc == 0
        assert tok.value == c["token"], c
        assert out.cur_num_gen == 101 and out.prev_token == c["token"]


@pytest.mark.parametrize("layout,M,K,splits,epi,nw", [
    (1, 33, 2304, 1, 3, 12),    # register-X: at most 32 rows
    (1, 8, 2304, 2, 3, 12),     # split K only into fp32 slabs
    (1, 8, 2048, 1, 4, 8),      # unsplit slices must be 72 k-steps
    (1, 8, 9216, 8, 4, 8),      # 36-k-step slices: nw must divide 36
    (1, 8, 9216, 3, 4, 12),     # 96-k-step slices: not instantiated
    (1, 8, 2304, 5, 4, 4),      # 72 k-steps do not split in 5
    (0, 17, 2304, 1, 3, 8),     # LDS-staged X: at most 16 rows
    (2, 8, 2304, 1, 3, 8),      # no third layout
    (1, 8, 2304, 1, 3, 16),     # register-X wave counts: 4 / 6 / 8 / 9 / 12 only
    (1, 8, 2304, 1, 3, 5),
])
def test_gemv_rejects_unsupported_shapes(layout, M, K, splits, epi, nw):
    """t5g_gemv validates on the host and returns an error code before any launch for the
    shapes its kernels are not built for (csrc/gemv.hip gemv_rx / gemv_dec)."""
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    a = _lib.GemvArgs()
    a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, K, 2304, epi, 0, nw, 8
    a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = 16, K, 16, 2304, splits, layout, 0
    a.W = 16   # never dereferenced: every case is rejected before a launch
    assert L.t5g_gemv(C.byref(a), None) < 0


def test_status_codes_map_to_python_errors():
    """The C ABI's statuses raise what the reference's code paths would (ValueError for bad
    arguments / capacity) and a FusedHandoffError for a fused decode launch whose hand-off
    gave up (engine.generate reruns such a call on the per-op launches)."""
    import pytest as _pt
    from t5gemma_tts_amd import _lib
    _lib.check(0, "ok")
    with _pt.raises(ValueError):
        _lib.check(-1, "x")
    with _pt.raises(ValueError):
        _lib.check(-5, "x")
    with _pt.raises(_lib.FusedHandoffError):
        _lib.check(-6, "x")
    with _pt.raises(_lib.T5GError):
        _lib.check(-2, "x")
    assert issubclass(_lib.FusedHandoffError, _lib.T5GError)
