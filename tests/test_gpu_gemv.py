"""GPU numerics of the fused decode GEMV (csrc/gemv.hip via t5g_gemv) against a
plain PyTorch fp32 reference of the same ops: the RMSNorm(1+w)/residual prologue
([tf] T5GemmaRMSNorm :61-78, PMDecoderLayer :285-323) and the Linear epilogues."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu

BF16 = torch.bfloat16
EPS = 1e-6


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rms(x, w):
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + EPS)
    return ((xf * r) * (1.0 + w.float())).to(BF16)


def _epilogue(acc, epi, bias):
    M, N = acc.shape
    if epi == 4:
        return acc
    if epi == 0:
        return acc.to(BF16).float()
    if epi == 1:
        return (acc + bias.float()).to(BF16).float()
    if epi == 2:
        return torch.nn.functional.gelu((acc + bias.float()).to(BF16).float()).to(BF16).float()
    a3 = acc.view(M, N // 16, 2, 8)   # 8 gate rows, then the same 8 features' up rows
    gate, up = a3[:, :, 0].reshape(M, -1), a3[:, :, 1].reshape(M, -1)
    act = torch.nn.functional.gelu(gate.to(BF16).float(), approximate="tanh").to(BF16).float()
    return (act * up.to(BF16).float()).to(BF16).float()


def _check_resid(got, h, v, post_w):
    """h' = bf16(h + bf16(RMSNorm(v))): a one-ulp flip of the normed term (fp32 sum order)
    moves h' by up to one ulp of that term, so the bound is relative to |h| + |a|."""
    a = _rms(v, post_w).float()
    ref = (h.float() + a).to(BF16).float()
    diff = (got.float() - ref).abs()
    tol = 2 ** -7 * (h.float().abs() + a.abs() + ref.abs()) * 1.01 + 1e-6
    assert (diff <= tol).all(), diff.max()
    assert (diff == 0).float().mean() >= 0.99


def _close_bf16(got, ref, frac=0.99):
    """<= 1 bf16 ulp everywhere (fp32 sum order may flip a rounding), mostly exact."""
    diff = (got.float() - ref.float()).abs()
    ulp = ref.float().abs().clamp(min=1e-30) * 2 ** -7
    assert (diff <= ulp * 1.01 + 1e-6).all(), diff.max()
    assert (diff == 0).float().mean() >= frac


CASES = [  # pro, epi, M, N, K, nw
    (1, 4, 8, 4096, 2304, 8),     # self q|k|v with the post_ff/pre_self prologue
    (1, 4, 8, 2048, 2304, 8),     # cross q
    (1, 3, 8, 18432, 2304, 4),    # gate/up GeGLU
    (1, 3, 16, 18432, 2304, 8),
    (1, 2, 8, 2304, 2304, 8),     # head1 (final norm prologue, bias + GELU erf)
    (1, 0, 1, 2304, 2304, 4),
    (1, 4, 3, 192, 64, 4),        # tiny widths: most lanes idle
    (1, 4, 5, 300, 3584, 8),      # wider hidden (8 chunks per lane)
    (2, 4, 8, 4096, 2304, 8),     # layer-0 embedding prologue
    (0, 0, 8, 2304, 2048, 8),     # o / cross-o (rows staged through LDS)
    (0, 1, 16, 6000, 2304, 8),
    (3, 0, 8, 2304, 9216, 8),     # down, X straight from L2
    (3, 0, 16, 2304, 9216, 16),
    (3, 4, 1, 200, 96, 4),
]


@pytest.mark.parametrize("pro,epi,M,N,K,nw,splits", [c + (1,) for c in CASES] + [
    (0, 4, 8, 4096, 2304, 4, 2), (0, 4, 8, 2304, 9216, 4, 8), (3, 4, 8, 2304, 9216, 8, 16), (0, 4, 3, 200, 96, 4, 3),
    (0, 3, 8, 18432, 2304, 4, 1)])
def test_gemv_fused_vs_fp32(pro, epi, M, N, K, nw, splits):
    _need_gpu()
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(pro * 1000 + M * 7 + N + K)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16)
    bias = (torch.randn(N, generator=g) * 0.02).to(BF16)
    X = torch.randn(M, K, generator=g).to(BF16)
    v = (torch.randn(M, K, generator=g) * 3).to(BF16)
    h = torch.randn(M, K, generator=g).to(BF16)
    post_w = (torch.randn(K, generator=g) * 0.1).to(BF16)
    pre_w = (torch.randn(K, generator=g) * 0.1).to(BF16)
    vocab = 50
    table = (torch.randn(vocab, K, generator=g) * 0.05).to(BF16)
    ids = torch.randint(0, vocab, (M,), generator=g, dtype=torch.int32)
    scale = float(torch.tensor(K ** 0.5).to(BF16))

    Wd = W.to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device=dev)
    assert L.t5g_pack_weight(C.c_void_p(Wd.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0
    n_out = N // 2 if epi == 3 else N
    Y = torch.zeros(splits, M, n_out, dtype=torch.float32 if epi == 4 else BF16, device=dev)
    h_out = torch.zeros(M, K, dtype=BF16, device=dev)
    x_out = torch.zeros(M, K, dtype=BF16, device=dev)
    keep = [t.to(dev) for t in (bias, X, v, h, post_w, pre_w, table, ids)]
    bd, Xd, vd, hd, pd, qd, td, idd = keep
    a = _lib.GemvArgs()
    a.M, a.K, a.N, a.epi, a.pro, a.nw, a.splits = M, K, N, epi, pro, nw, splits
    a.W, a.bias, a.Y, a.ldy, a.ldx = Wp.data_ptr(), bd.data_ptr(), Y.data_ptr(), n_out, K
    a.X, a.v, a.h_in, a.ids, a.table = Xd.data_ptr(), vd.data_ptr(), hd.data_ptr(), idd.data_ptr(), td.data_ptr()
    a.scale, a.eps, a.post_w, a.pre_w = scale, EPS, pd.data_ptr(), qd.data_ptr()
    a.h_out, a.x_out = h_out.data_ptr(), x_out.data_ptr()
    assert L.t5g_gemv(C.byref(a), st) == 0
    torch.cuda.synchronize()

    if pro == 1:
        _check_resid(h_out.cpu(), h, v, post_w)
    elif pro == 2:
        _close_bf16(h_out.cpu(), (table[ids.long()].float() * scale).to(BF16))
    if pro in (1, 2):
        _close_bf16(x_out.cpu(), _rms(h_out.cpu(), pre_w))   # second norm on the kernel's own h'
        xin = x_out.cpu()
    else:
        xin = X
    acc = xin.float() @ W.float().t()
    ref = _epilogue(acc, epi, bias)
    got = Y.float().sum(0).cpu()
    if epi == 4:
        assert torch.allclose(got, ref, rtol=1e-5, atol=1e-4 * ref.abs().max().item())
    elif epi == 3:
        assert (got - ref).abs().max() <= 2 ** -6 * ref.abs().max()
    else:
        _close_bf16(got, ref, frac=0.97)


def test_gemv_batch_invariant():
    """Row m of an M-row launch equals the same row run alone (bitwise)."""
    _need_gpu()
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = "cuda"
    M, N, K = 8, 4096, 2304
    g = torch.Generator(device="cpu").manual_seed(5)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16).to(dev)
    v = (torch.randn(M, K, generator=g) * 3).to(BF16).to(dev)
    h = torch.randn(M, K, generator=g).to(BF16).to(dev)
    pw = (torch.randn(K, generator=g) * 0.1).to(BF16).to(dev)
    qw = (torch.randn(K, generator=g) * 0.1).to(BF16).to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device=dev)
    assert L.t5g_pack_weight(C.c_void_p(W.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0

    def run(rows):
        Y = torch.zeros(len(rows), N, dtype=torch.float32, device=dev)
        vv, hh = v[rows].contiguous(), h[rows].contiguous()
        a = _lib.GemvArgs()
        a.M, a.K, a.N, a.epi, a.pro, a.nw = len(rows), K, N, 4, 1, 8
        a.W, a.Y, a.ldy = Wp.data_ptr(), Y.data_ptr(), N
        a.v, a.h_in, a.eps, a.post_w, a.pre_w = vv.data_ptr(), hh.data_ptr(), EPS, pw.data_ptr(), qw.data_ptr()
        assert L.t5g_gemv(C.byref(a), st) == 0
        torch.cuda.synchronize()
        return Y.cpu()

    full = run(list(range(M)))
    for m in (0, 3, 7):
        assert torch.equal(run([m])[0], full[m])


RM_CASES = [  # pro, epi, M, N, K  (row-major VALU GEMV, layout 1; M <= 8)
    (1, 4, 8, 4096, 2304),    # q|k|v, 16 rows per block
    (2, 4, 8, 4096, 2304),    # layer-0 embedding prologue
    (1, 4, 8, 2048, 2304),    # cross q, 8 rows per block
    (1, 3, 8, 18432, 2304),   # gate/up (gate rows then up rows), 36 features per block
    (1, 2, 8, 2304, 2304),    # head1, 9 rows per block
    (3, 0, 8, 2304, 2048),    # o / cross o, X from L2
    (3, 0, 8, 2304, 9216),    # down, K split over 8 waves
    (0, 0, 5, 2304, 2048),
    (1, 4, 3, 192, 64),       # tiny widths, ragged blocks
    (1, 3, 2, 256, 64),
    (3, 0, 1, 64, 128),
    (1, 0, 7, 300, 2304),
]


@pytest.mark.parametrize("pro,epi,M,N,K", RM_CASES)
def test_gemv_rowmajor_vs_fp32(pro, epi, M, N, K):
    _need_gpu()
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(77 + pro * 1000 + M * 7 + N + K)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16)
    bias = (torch.randn(N, generator=g) * 0.02).to(BF16)
    X = torch.randn(M, K, generator=g).to(BF16)
    v = (torch.randn(M, K, generator=g) * 3).to(BF16)
    h = torch.randn(M, K, generator=g).to(BF16)
    post_w = (torch.randn(K, generator=g) * 0.1).to(BF16)
    pre_w = (torch.randn(K, generator=g) * 0.1).to(BF16)
    table = (torch.randn(50, K, generator=g) * 0.05).to(BF16)
    ids = torch.randint(0, 50, (M,), generator=g, dtype=torch.int32)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    n_out = N // 2 if epi == 3 else N
    Y = torch.zeros(M, n_out, dtype=torch.float32 if epi == 4 else BF16, device=dev)
    h_out = torch.zeros(M, K, dtype=BF16, device=dev)
    x_out = torch.zeros(M, K, dtype=BF16, device=dev)
    keep = [t.to(dev) for t in (W, bias, X, v, h, post_w, pre_w, table, ids)]
    Wd, bd, Xd, vd, hd, pd, qd, td, idd = keep
    a = _lib.GemvArgs()
    a.M, a.K, a.N, a.epi, a.pro, a.nw, a.layout = M, K, N, epi, pro, 4, 1
    a.W, a.bias, a.Y, a.ldy, a.ldx = Wd.data_ptr(), bd.data_ptr(), Y.data_ptr(), n_out, K
    a.X, a.v, a.h_in, a.ids, a.table = Xd.data_ptr(), vd.data_ptr(), hd.data_ptr(), idd.data_ptr(), td.data_ptr()
    a.scale, a.eps, a.post_w, a.pre_w = 48.0, EPS, pd.data_ptr(), qd.data_ptr()
    a.h_out, a.x_out = h_out.data_ptr(), x_out.data_ptr()
    assert L.t5g_gemv(C.byref(a), st) == 0
    torch.cuda.synchronize()
    if pro == 1:
        _check_resid(h_out.cpu(), h, v, post_w)
    elif pro == 2:
        _close_bf16(h_out.cpu(), (table[ids.long()].float() * 48.0).to(BF16))
    if pro in (1, 2):
        _close_bf16(x_out.cpu(), _rms(h_out.cpu(), pre_w))
        xin = x_out.cpu()
    else:
        xin = X
    acc = xin.float() @ W.float().t()
    got = Y.float().cpu()
    if epi == 3:
        F = N // 2
        act = torch.nn.functional.gelu(acc[:, :F].to(BF16).float(), approximate="tanh").to(BF16).float()
        ref = (act * acc[:, F:].to(BF16).float()).to(BF16).float()
        assert (got - ref).abs().max() <= 2 ** -6 * ref.abs().max()
    elif epi == 4:
        assert torch.allclose(got, acc, rtol=1e-5, atol=1e-4 * acc.abs().max().item())
    else:
        _close_bf16(got, _epilogue(acc, epi, bias), frac=0.97)


def test_gemv_rowmajor_batch_invariant():
    """VALU GEMV: row m of an 8-row launch equals the same row run alone (bitwise)."""
    _need_gpu()
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = "cuda"
    M, N, K = 8, 2304, 9216
    g = torch.Generator(device="cpu").manual_seed(9)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16).to(dev)
    X = torch.randn(M, K, generator=g).to(BF16).to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run(rows):
        Y = torch.zeros(len(rows), N, dtype=BF16, device=dev)
        xx = X[rows].contiguous()
        a = _lib.GemvArgs()
        a.M, a.K, a.N, a.epi, a.pro, a.nw, a.layout = len(rows), K, N, 0, 3, 4, 1
        a.W, a.Y, a.ldy, a.X, a.ldx = W.data_ptr(), Y.data_ptr(), N, xx.data_ptr(), K
        assert L.t5g_gemv(C.byref(a), st) == 0
        torch.cuda.synchronize()
        return Y.cpu()

    full = run(list(range(M)))
    for m in (0, 5):
        assert torch.equal(run([m])[0], full[m])
