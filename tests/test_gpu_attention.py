"""Decode attention through the C ABI (t5g_attention_decode: the split-K decode kernel +
combine the engine runs every step) against an fp64 softmax-attention reference of the
same bf16 q / K / V, at the C3 lengths: self attention over L in {1, 63, 64, 65, 152,
527, 903} keys (1 to 15 key chunks per (row, kv head), ragged rows in one launch) and
cross attention over T_x = 60 encoder keys. Reference semantics:
[tf] T5GemmaSelfAttention :264-304 / PMCrossAttention :167-253 through torch's CPU
SDPA, whose bf16 path rounds exp(s - max) to bf16 before P.V."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _reference(q, K, V, lens, scale, causal, pround):
    """fp64 attention per row over its first lens[b] keys (query = last key). pround:
    exp values rounded to bf16 before P.V (CPU SDPA bf16 numerics); else exact."""
    B, Hq, D = q.shape
    Hkv = K.shape[1]
    G = Hq // Hkv
    out = torch.zeros(B, Hq, D, dtype=torch.float64)
    for b in range(B):
        L = int(lens[b])
        for h in range(Hq):
            k = K[b, h // G, :L].double()
            v = V[b, h // G, :L].double()
            s = (k @ q[b, h].double()).float() * scale
            p = torch.exp((s - s.max()).double())
            l = p.sum()
            if pround:
                p = p.float().to(BF16).double()
            out[b, h] = (p @ v) / l
    return out


def _run(L, B, lens, Hq=8, Hkv=4, D=256, causal=1, seed=0):
    from t5gemma_tts_amd import _lib
    lib = _lib.lib()
    g = torch.Generator().manual_seed(seed)
    cap = L
    q = torch.randn(B, Hq, D, generator=g).to(BF16)
    K = torch.randn(B, Hkv, cap, D, generator=g).to(BF16)
    V = torch.randn(B, Hkv, cap, D, generator=g).to(BF16)
    dev = "cuda"
    qd, Kd, Vd = q.to(dev), K.to(dev), V.to(dev)
    lens_d = torch.tensor(lens, dtype=torch.int32, device=dev)
    out = torch.zeros(B, Hq * D, dtype=BF16, device=dev)
    nb = lib.t5g_attention_decode_work_bytes(B, Hq, Hkv, D, cap)
    assert nb > 0
    work = torch.empty(nb // 4, dtype=torch.float32, device=dev)
    a = _lib.AttnDecodeArgs(B=B, n_heads=Hq, n_kv_heads=Hkv, head_dim=D, q=qd.data_ptr(), k_cache=Kd.data_ptr(),
                            v_cache=Vd.data_ptr(), cap=cap, kv_len=lens_d.data_ptr(), causal=causal, window=0,
                            scale=D ** -0.5, out=out.data_ptr(), work=work.data_ptr())
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.t5g_attention_decode(C.byref(a), st), "attention_decode")
    torch.cuda.synchronize()
    got = out.cpu().view(B, Hq, D).double()
    return got, q, K, V


@pytest.mark.parametrize("L", [1, 63, 64, 65, 152, 527, 903])
def test_self_attention_decode_vs_fp64(L):
    """8 rows x 8 q heads / 4 kv heads x 256 (2b-2b), ragged lengths up to L."""
    _need_gpu()
    B = 8
    lens = [L, max(1, L - 1), max(1, L // 2), max(1, L - 64), 1, max(1, L - 3), max(1, (3 * L) // 4), L]
    got, q, K, V = _run(L, B, lens, seed=L)
    exact = _reference(q, K, V, lens, 256 ** -0.5, True, pround=False)
    emu = _reference(q, K, V, lens, 256 ** -0.5, True, pround=True)
    # bf16 output: half an ulp of the result + fp32 accumulation; the P-rounding of the
    # reference numerics moves a value by at most 2^-9 relative per term, i.e. <= 2^-9 of
    # sum_j p_j |v_j| / l  (bounded by max |v| <= ~5 for these draws)
    vmax = V.abs().max().item()
    tol = 2.0 ** -8 * got.abs() + 2.0 ** -8 * vmax + 1e-6
    assert ((got - exact).abs() <= tol).all(), (got - exact).abs().max()
    err_emu = (got - emu).abs()
    ulp = torch.exp2(torch.floor(torch.log2(emu.abs().clamp(min=2.0 ** -60))) - 7)
    assert (err_emu <= 2 * ulp + 1e-6 * vmax).float().mean() > 0.999, err_emu.max()
    # rows of <= 64 keys are one chunk (no merge): bit-identical to the P-rounded reference
    # whenever it lands off a bf16 rounding boundary; the merged rows agree within 1 ulp
    same = (got == emu.float().to(BF16).double()).float().mean().item()
    print(f"L={L}: bit-equal to the P-rounded fp64 reference {same:.4f}, max |err| vs exact "
          f"{(got - exact).abs().max().item():.3g}")
    assert same > 0.9


def test_cross_attention_decode_tx60():
    """PMCrossAttention shape: T_x = 60 encoder keys (non-causal), 8 rows, ragged text."""
    _need_gpu()
    B, T = 8, 60
    lens = [60, 59, 33, 1, 60, 17, 48, 60]
    got, q, K, V = _run(T, B, lens, causal=0, seed=60)
    emu = _reference(q, K, V, lens, 256 ** -0.5, False, pround=True)
    same = (got == emu.float().to(BF16).double()).float().mean().item()
    assert same > 0.97, same
    assert (got - emu).abs().max().item() <= 2.0 ** -7 * max(1.0, emu.abs().max().item())
