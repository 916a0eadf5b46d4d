"""oracle/sdpa_emu.py (the GPU attention kernels' reference) against torch's own CPU SDPA
on bf16 inputs, bit for bit: the numerics the reference's attention has in the build
container (AVX-512 aten kernels; the goldens were produced there). Other CPU builds of
aten take different code (AVX2 / default) and are skipped."""
import pytest
import torch
import torch.nn.functional as F

from oracle import sdpa_emu

BF16 = torch.bfloat16
pytestmark = pytest.mark.skipif(torch.backends.cpu.get_cpu_capability() != "AVX512",
                                reason="aten AVX-512 kernels are what the goldens were made with")


def _cmp(q, k, v, scale, causal, gqa):
    kw = {"enable_gqa": True} if gqa else {}
    ref = F.scaled_dot_product_attention(q[None], k[None], v[None], scale=scale, is_causal=causal, **kw)[0]
    got = sdpa_emu.attention(q, k, v, scale, is_causal=causal)
    return (got.view(torch.int16) == ref.view(torch.int16)).float().mean().item(), \
        (got.float() - ref.float()).abs().max().item()


@pytest.mark.parametrize("L", [1, 17, 40, 64, 152, 527, 903])
def test_decode_row_matches_torch_sdpa(L):
    g = torch.Generator().manual_seed(L)
    q = torch.randn(8, 1, 256, generator=g).to(BF16)
    k = torch.randn(4, L, 256, generator=g).to(BF16)
    v = torch.randn(4, L, 256, generator=g).to(BF16)
    eq, err = _cmp(q, k, v, 256 ** -0.5, False, True)
    assert eq >= 0.999, (eq, err)


@pytest.mark.parametrize("T,causal", [(30, True), (152, True), (200, True), (60, False), (20, False)])
def test_prefill_and_encoder_match_torch_sdpa(T, causal):
    g = torch.Generator().manual_seed(T)
    H, D = (2, 64) if T <= 30 else (8, 256)
    q = torch.randn(H, T, D, generator=g).to(BF16)
    k = torch.randn(H // 2, T, D, generator=g).to(BF16)
    v = torch.randn(H // 2, T, D, generator=g).to(BF16)
    eq, err = _cmp(q, k, v, D ** -0.5, causal, True)
    assert eq >= 0.999, (eq, err)


def test_fexp_matches_aten_vector_exp():
    """The fast exp alone: p of every key of a one-hot attention row (exact scores)."""
    g = torch.Generator().manual_seed(0)
    ok = tot = 0
    for trial in range(20):
        Tk = 256 - 9 * (trial % 7)
        q = torch.zeros(1, 1, 256, dtype=BF16)
        q[0, 0, 0] = 1.0
        k = (torch.randn(1, Tk, 256, generator=g) * 16).to(BF16)
        v = torch.zeros(1, Tk, 256, dtype=BF16)
        v[0, torch.arange(Tk), torch.arange(Tk)] = 1.0
        ref = F.scaled_dot_product_attention(q[None], k[None], v[None], scale=1 / 16)[0]
        got = sdpa_emu.attention(q, k, v, 1 / 16)
        ok += int((got.view(torch.int16) == ref.view(torch.int16)).sum())
        tot += got.numel()
    assert ok == tot


def test_expf_restatement_equals_host_libm():
    """oracle.sdpa_emu.expf (oracle/glibc_expf.c) == this host's glibc expf -- the
    std::exp(float) of aten's flash attention on the reference host -- on 2^22 floats of the
    softmax's range (-104, 0] plus the edge inputs; and it is not the correctly rounded exp
    there (the round-4 model): the test also finds inputs where the two differ. The exhaustive
    2^32 check is tools/cpu_order/check_glibc_expf.c (profiles/r05_s2_glibc_expf_exhaustive.log)."""
    import ctypes

    import numpy as np

    from oracle import sdpa_emu as E
    libm = ctypes.CDLL("libm.so.6")
    libm.expf.restype, libm.expf.argtypes = ctypes.c_float, [ctypes.c_float]
    rng = np.random.default_rng(7)
    x = np.concatenate([-rng.random(1 << 22, dtype=np.float32) * 104.0,
                        np.array([0.0, -0.0, -87.3365478515625, -88.0, -103.2789, -103.9721, -104.0, -np.inf,
                                  -1e-30, -0.45788383], np.float32)]).astype(np.float32)
    got = E.expf(torch.from_numpy(x)).numpy()
    idx = np.concatenate([np.arange(20000), np.arange(x.size - 10, x.size)])
    ref = np.array([libm.expf(float(v)) for v in x[idx]], np.float32)
    assert np.array_equal(got[idx].view(np.int32), ref.view(np.int32))
    cr = np.exp(x.astype(np.float64)).astype(np.float32)
    assert (cr != got).sum() > 0   # glibc expf is not correctly rounded on this range
