"""CPU checks for the XCodec2 decoder row: the oracle restatement
against the transformers Xcodec2Model goldens, the host-side weight layouts the HIP
kernels consume, and the xc2_* C ABI exports. No GPU compute is invoked."""
import ctypes as C
import json
import math
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO

CASES = ["tiny", "full16k", "hop882"]


def load_case(name):
    from t5gemma_tts_amd.codec import CodecConfig
    m = json.load(open(os.path.join(GOLDEN, f"golden_codec_{name}.json")))
    wav = np.load(os.path.join(GOLDEN, f"golden_codec_{name}.npz"))["wav"]
    cfg = CodecConfig(**{k: (tuple(v) if isinstance(v, list) else v) for k, v in m["config"].items()})
    return m, cfg, wav


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_transformers_golden(name):
    from oracle import xc2_oracle as xo
    from t5gemma_tts_amd.codec import synthetic_codec_weights
    m, cfg, wav = load_case(name)
    sd = synthetic_codec_weights(cfg, m["weight_seed"])
    out = xo.decode(sd, torch.tensor(m["codes"]), cfg).numpy()
    assert out.shape == wav.shape
    err = out.astype(np.float64) - wav
    assert np.abs(err).max() <= 1e-6, np.abs(err).max()
    assert math.sqrt((err ** 2).mean()) <= 1e-7


def test_oracle_ragged_lens_decode_rows_independently():
    from oracle import xc2_oracle as xo
    from t5gemma_tts_amd.codec import synthetic_codec_weights
    m, cfg, wav = load_case("tiny")
    sd = synthetic_codec_weights(cfg, m["weight_seed"])
    codes = torch.tensor(m["codes"])
    out = xo.decode(sd, codes, cfg, lens=[codes.shape[1], 20])
    ref1 = xo.decode(sd, codes[1:, :20], cfg)
    assert torch.equal(out[1, :, :20 * cfg.hop_length], ref1[0])
    assert torch.all(out[1, :, 20 * cfg.hop_length:] == 0)


def test_fsq_special_ids_wrap():
    """Special audio ids 65536..65538 can reach the codec (SURVEY a16 edge case): the
    digit formula maps id -> id mod 4^8."""
    from oracle.xc2_oracle import fsq_codes
    ids = torch.tensor([0, 1, 65535, 65536, 65537, 65538])
    c = fsq_codes(ids, (4,) * 8)
    assert torch.equal(c[3], c[0]) and torch.equal(c[4], c[1]) and torch.equal(c[5], fsq_codes(torch.tensor([2]),
                                                                                          (4,) * 8)[0])
    assert torch.equal(c[0], torch.full((8,), -1.0))
    assert torch.equal(c[2], torch.full((8,), 0.5))


def test_irfft_basis_matches_torch():
    from t5gemma_tts_amd.codec import irfft_basis
    n_fft = 1280
    spec_ld = (n_fft + 2 + 31) // 32 * 32
    win = torch.hann_window(n_fft)
    B = irfft_basis(n_fft, spec_ld, win).double()
    g = torch.Generator().manual_seed(0)
    X = torch.randn(3, n_fft // 2 + 1, dtype=torch.complex128, generator=g)
    ref = torch.fft.irfft(X, n_fft, dim=1) * win.double()
    v = torch.zeros(3, spec_ld, dtype=torch.float64)
    v[:, 0:2 * (n_fft // 2 + 1):2] = X.real
    v[:, 1:2 * (n_fft // 2 + 1):2] = X.imag
    got = v @ B.T
    assert torch.allclose(got, ref, atol=1e-6, rtol=0), (got - ref).abs().max()


def _header_symbols():
    src = open(os.path.join(REPO, "include", "xc2.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(xc2_[a-z_0-9]+)\s*\(", src)))


def test_xc2_exports_and_struct_sizes():
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd import codec
    L = _lib.lib()
    syms = _header_symbols()
    assert set(syms) == set(codec.XC2_SIGNATURES), set(syms) ^ set(codec.XC2_SIGNATURES)
    for s in syms:
        assert hasattr(L, s), s
    assert C.sizeof(codec.XC2Config) == 18 * 4
    assert C.sizeof(codec.XC2ResBlock) == 8 * 8
    assert C.sizeof(codec.XC2Layer) == 6 * 8
    assert C.sizeof(codec.XC2Weights) == (6 + 4 * 8 + 32 * 6 + 8) * 8


def test_xc2_create_rejects_bad_config():
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd import codec
    L = _lib.lib()
    fn = L.xc2_create
    fn.restype, fn.argtypes = codec.XC2_SIGNATURES["xc2_create"]
    kc = codec.XC2Config(hidden=1000, head_dim=64, n_heads=16)   # hidden != heads * 64
    h = C.c_void_p()
    assert fn(C.byref(kc), C.byref(codec.XC2Weights()), C.byref(h)) == -1
