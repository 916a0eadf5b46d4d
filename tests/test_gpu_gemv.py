"""GPU numerics of the decode GEMV (csrc/gemv.hip via t5g_gemv; the decode step's gate/up
launch) against a plain PyTorch fp32 reference of the same ops ([tf] T5GemmaMLP :81-97
GeGLU epilogue, Linear / bias / split-K epilogues)."""
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


def _close_bf16(got, ref, frac=0.99):
    """<= 1 bf16 ulp everywhere (fp32 sum order may flip a rounding), mostly exact."""
    diff = (got.float() - ref.float()).abs()
    ulp = ref.float().abs().clamp(min=1e-30) * 2 ** -7
    assert (diff <= ulp * 1.01 + 1e-6).all(), diff.max()
    assert (diff == 0).float().mean() >= frac


CASES = [  # epi, M, N, K, nw, splits
    (3, 8, 18432, 2304, 8, 1),    # decode gate/up GeGLU at 2b-2b (the product launch)
    (3, 8, 18432, 2304, 4, 1),
    (3, 16, 18432, 2304, 8, 1),
    (0, 8, 2304, 2048, 8, 1),     # o-shaped
    (1, 16, 6000, 2304, 8, 1),
    (0, 1, 2304, 2304, 4, 1),
    (4, 3, 192, 64, 4, 1),        # tiny widths: most lanes idle
    (4, 8, 4096, 2304, 4, 2),     # split-K fp32 slabs
    (4, 8, 2304, 9216, 4, 8),
    (4, 3, 200, 96, 4, 3),
]


def _run(epi, M, N, K, nw, splits, seed, max_grid=0, X=None, W=None, layout=0):
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(seed)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16) if W is None else W
    bias = (torch.randn(N, generator=g) * 0.02).to(BF16)
    X = torch.randn(M, K, generator=g).to(BF16) if X is None else X
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Wd = W.to(dev)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device=dev)
    assert L.t5g_pack_weight(C.c_void_p(Wd.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0
    n_out = N // 2 if epi == 3 else N
    Y = torch.zeros(splits, M, n_out, dtype=torch.float32 if epi == 4 else BF16, device=dev)
    bd, Xd = bias.to(dev), X.to(dev)
    a = _lib.GemvArgs()
    a.M, a.K, a.N, a.epi, a.pro, a.nw, a.splits, a.max_grid = M, K, N, epi, 0, nw, splits, max_grid
    a.layout = layout
    a.W, a.bias, a.Y, a.ldy, a.ldx, a.X = Wp.data_ptr(), bd.data_ptr(), Y.data_ptr(), n_out, K, Xd.data_ptr()
    assert L.t5g_gemv(C.byref(a), st) == 0
    torch.cuda.synchronize()
    return Y.float().sum(0).cpu(), X, W, bias


@pytest.mark.parametrize("epi,M,N,K,nw,splits", CASES)
def test_gemv_vs_fp32(epi, M, N, K, nw, splits):
    _need_gpu()
    got, X, W, bias = _run(epi, M, N, K, nw, splits, seed=M * 7 + N + K + splits)
    ref = _epilogue(X.float() @ W.float().t(), epi, bias)
    if epi == 4:
        assert torch.allclose(got, ref, rtol=1e-5, atol=1e-4 * ref.abs().max().item())
    elif epi == 3:
        assert (got - ref).abs().max() <= 2 ** -6 * ref.abs().max()
    else:
        _close_bf16(got, ref, frac=0.97)


def test_gemv_stream_tail_regression():
    """Round-1 LDS race (fixed in e2f4e11): the padded tail of a block's fragment stream
    (steps past its nu units; the loop rounds to 2*UN) stored partial sums past red[]
    into the staged X rows other waves were still reading. Deterministic guard: grid caps
    that leave blocks with nu = 4 / 5 / 11 / 12 units (not multiples of 2*UN) on the
    gate/up shape, each launch compared with the fp32 reference and the uncapped launch."""
    _need_gpu()
    M, N, K = 8, 18432, 2304
    full, X, W, bias = _run(3, M, N, K, 8, 1, seed=11)
    ref = _epilogue(X.float() @ W.float().t(), 3, bias)
    for cap in (251, 233, 97):   # 1152 units over the capped grid
        got, *_ = _run(3, M, N, K, 8, 1, seed=11, max_grid=cap, X=X, W=W)
        assert torch.equal(got, full), cap
        assert (got - ref).abs().max() <= 2 ** -6 * ref.abs().max()


def test_gemv_batch_invariant():
    """Row m of an M-row launch equals the same row run alone (bitwise)."""
    _need_gpu()
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = "cuda"
    M, N, K = 8, 4096, 2304
    g = torch.Generator(device="cpu").manual_seed(5)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16).to(dev)
    X = torch.randn(M, K, generator=g).to(BF16).to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device=dev)
    assert L.t5g_pack_weight(C.c_void_p(W.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0

    def run(rows):
        Y = torch.zeros(len(rows), N, dtype=torch.float32, device=dev)
        xx = X[rows].contiguous()
        a = _lib.GemvArgs()
        a.M, a.K, a.N, a.epi, a.pro, a.nw = len(rows), K, N, 4, 0, 8
        a.W, a.Y, a.ldy, a.X, a.ldx = Wp.data_ptr(), Y.data_ptr(), N, xx.data_ptr(), K
        assert L.t5g_gemv(C.byref(a), st) == 0
        torch.cuda.synchronize()
        return Y.cpu()

    full = run(list(range(M)))
    for m in (0, 3, 7):
        assert torch.equal(run([m])[0], full[m])



@pytest.mark.parametrize("epi,M", [(3, 8), (3, 1), (3, 16), (0, 8), (3, 32), (3, 24), (1, 17)])
def test_gemv_register_x_variant(epi, M):
    """layout 1 (register-resident X, 1..32 rows, K = 2304): vs the fp32 reference, and
    bitwise equal to the LDS-staged kernel on every 16-row slice of the batch."""
    _need_gpu()
    N, K = (18432, 2304) if epi == 3 else (6000, 2304)
    g = torch.Generator(device="cpu").manual_seed(M + epi)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16)
    X = torch.randn(M, K, generator=g).to(BF16)
    got, _, _, bias = _run(epi, M, N, K, 8, 1, seed=3, X=X, W=W, layout=1)
    ref = _epilogue(X.float() @ W.float().t(), epi, bias)
    if epi == 3:
        assert (got - ref).abs().max() <= 2 ** -6 * ref.abs().max()
    else:
        _close_bf16(got, ref, frac=0.97)
    parts = [_run(epi, min(16, M - r0), N, K, 8, 1, seed=3, X=X[r0:r0 + 16].contiguous(), W=W, layout=0)[0]
             for r0 in range(0, M, 16)]
    assert torch.equal(got, torch.cat(parts)), "register-X rows differ from the LDS-staged kernel"


@pytest.mark.parametrize("nw,M,epi", [(12, 8, 3), (12, 1, 3), (12, 16, 3), (9, 8, 3), (6, 5, 3), (4, 8, 3),
                                      (4, 32, 1), (4, 21, 1), (8, 16, 1)])
def test_gemv_register_x_wave_counts(nw, M, epi):
    """layout 1 at other wave counts (the decode gate/up runs 12 waves at K = 2304; the
    65 541-row head 8 waves up to 16 rows, 4 waves -- the partial-sum buffer's LDS limit --
    up to 32): vs the fp32 reference, and batch-invariant (every row bitwise equal to the
    same row alone)."""
    _need_gpu()
    N, K = (18432, 2304) if epi == 3 else (65541, 2304)
    g = torch.Generator(device="cpu").manual_seed(nw * 31 + M)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16)
    X = torch.randn(M, K, generator=g).to(BF16)
    got, _, _, bias = _run(epi, M, N, K, nw, 1, seed=5, X=X, W=W, layout=1)
    ref = _epilogue(X.float() @ W.float().t(), epi, bias)
    if epi == 3:
        assert (got - ref).abs().max() <= 2 ** -6 * ref.abs().max()
    else:
        _close_bf16(got, ref, frac=0.97)
    for m in sorted({0, M // 2, M - 1}):
        one = _run(epi, 1, N, K, nw, 1, seed=5, X=X[m:m + 1].contiguous(), W=W, layout=1)[0]
        assert torch.equal(one[0], got[m]), f"row {m} depends on the batch at nw={nw}"


@pytest.mark.parametrize("nw,M", [(12, 8), (12, 32), (12, 19), (4, 8), (9, 1)])
def test_gemv_register_x_split_k(nw, M):
    """layout 1 over 8 k-slices of K = 9216 (the decode down projection: fp32 slabs, 32
    blocks per slice each streaming several units): slab sum vs the fp32 reference, and
    batch-invariant."""
    _need_gpu()
    N, K, S = 2304, 9216, 8
    g = torch.Generator(device="cpu").manual_seed(nw * 7 + M)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16)
    X = torch.randn(M, K, generator=g).to(BF16)
    got = _run(4, M, N, K, nw, S, seed=5, X=X, W=W, layout=1)[0]
    ref = X.float() @ W.float().t()
    assert (got - ref).abs().max() <= 1e-5 * ref.abs().max()
    for m in sorted({0, M // 2, M - 1}):
        one = _run(4, 1, N, K, nw, S, seed=5, X=X[m:m + 1].contiguous(), W=W, layout=1)[0]
        assert torch.equal(one[0], got[m]), f"row {m} depends on the batch at nw={nw}"


@pytest.mark.parametrize("M", [8, 3, 16])
def test_resid_norm_vs_fp32(M):
    """The decode step's residual + RMSNorm kernel (t5g_resid_norm; norm.hip): against a
    PyTorch fp32 restatement of [tf] T5GemmaRMSNorm :61-78 wired as the residual add of
    PMDecoderLayer :285-323 -- within the bf16 roundings of the two norms."""
    _need_gpu()
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = "cuda"
    K = 2304
    g = torch.Generator(device="cpu").manual_seed(77 + M)
    delta = (torch.randn(M, K, generator=g) * 3.0).to(BF16)
    h = torch.randn(M, K, generator=g).to(BF16)
    post_w = (torch.randn(K, generator=g) * 0.1).to(BF16)
    pre_w = (torch.randn(K, generator=g) * 0.1).to(BF16)
    dd, hd, pd, qd = delta.to(dev), h.to(dev), post_w.to(dev), pre_w.to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    h1 = torch.empty_like(hd)
    xn = torch.empty_like(hd)
    assert L.t5g_resid_norm(M, K, C.c_void_p(dd.data_ptr()), C.c_void_p(hd.data_ptr()), C.c_void_p(pd.data_ptr()),
                            C.c_void_p(qd.data_ptr()), C.c_float(EPS), C.c_void_p(h1.data_ptr()),
                            C.c_void_p(xn.data_ptr()), st) == 0
    torch.cuda.synchronize()
    hr = (h.float() + _rms(delta, post_w).float()).to(BF16)
    xr = _rms(hr, pre_w)
    for got, ref in ((h1.cpu(), hr), (xn.cpu(), xr)):
        diff = (got.float() - ref.float()).abs()
        ulp = ref.float().abs().clamp(min=2.0 ** -20) * 2 ** -7
        assert (diff <= 2 * ulp).all(), diff.max()
        assert (diff == 0).float().mean() > 0.95


@pytest.mark.parametrize("epi,K,splits,nw,M,caps", [(3, 2304, 1, 12, 8, (200, 100)),
                                                    (4, 9216, 8, 12, 32, (96 * 8, 40 * 8)),
                                                    (4, 2048, 4, 8, 8, (96 * 4, 40 * 4)),
                                                    (1, 2304, 1, 4, 24, (241, 230))])
def test_gemv_register_x_grid_invariant(epi, K, splits, nw, M, caps):
    """The register-X GEMV's results do not depend on how many blocks share the units (a
    unit's sums are one block's fixed wave order): bitwise equal at the default grid (one
    block per CU per slice) and at capped grids, e.g. a partitioned GPU with fewer CUs."""
    _need_gpu()
    N = 18432 if epi == 3 else (65541 if epi == 1 else 2304)
    g = torch.Generator(device="cpu").manual_seed(K + splits + M)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16)
    X = torch.randn(M, K, generator=g).to(BF16)
    base = _run(epi, M, N, K, nw, splits, seed=9, X=X, W=W, layout=1)[0]
    for cap in caps:   # units per block stay within the partial-sum buffer's LDS
        got = _run(epi, M, N, K, nw, splits, seed=9, X=X, W=W, layout=1, max_grid=cap)[0]
        assert torch.equal(got, base), f"max_grid {cap}"
