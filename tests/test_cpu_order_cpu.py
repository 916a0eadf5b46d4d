"""CPU tests of the reference-host accumulation-order restatement (oracle/cpu_order.py) and
of the exact-mode elementwise functions (csrc/exact_math.h, data/gelu_erf_bf16.bin).

* Against torch itself: only meaningful on the reference host (the build container the
  golden vectors were made on: torch 2.10 CPU with oneDNN AMX); skipped elsewhere.
* Against the reference's golden vectors: machine-independent (numpy arithmetic)."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN, REPO

BF16 = torch.bfloat16


def _reference_host():
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return False
    return "amx_bf16" in flags and torch.__version__.startswith("2.10")


ref_host = pytest.mark.skipif(not _reference_host(), reason="torch comparison needs the reference host (AMX, torch 2.10)")


def _hdr(shape, g):
    v = torch.randn(shape, generator=g) * torch.exp2(torch.randint(-10, 11, shape, generator=g).float())
    big = torch.rand(shape, generator=g) < 4.0 / shape[-1]
    return torch.where(big, torch.randn(shape, generator=g) * 2.0 ** 14, v).to(BF16)


@ref_host
@pytest.mark.parametrize("n", [2304, 128, 64, 9216, 100, 8])
def test_sum_last_matches_torch(n):
    from oracle import cpu_order
    torch.set_num_threads(8)
    g = torch.Generator().manual_seed(n)
    x = torch.randn(16, n, generator=g) * torch.exp2(torch.randint(-12, 13, (16, n), generator=g).float())
    assert np.array_equal(cpu_order.sum_last(x.numpy()), x.sum(-1).numpy())
    assert np.array_equal((cpu_order.sum_last((x * x).numpy()) / np.float32(n)).astype(np.float32),
                          x.pow(2).mean(-1).numpy())


@ref_host
@pytest.mark.parametrize("M,N,K", [(1, 2048, 2304), (1, 2304, 9216), (60, 2304, 9216), (152, 2304, 9216),
                                   (60, 1024, 2304), (7, 128, 256), (1, 2304, 2048)])
def test_linear_order_matches_torch(M, N, K):
    """The E/O chunk model with the measured K split == torch's F.linear, on a sample of
    output columns of order-revealing data."""
    from oracle import cpu_order
    torch.set_num_threads(8)
    g = torch.Generator().manual_seed(M + N + K)
    x = _hdr((M, K), g)
    cols = torch.randperm(N, generator=g)[:64]
    w = torch.zeros(N, K, dtype=BF16)
    w[cols] = _hdr((64, K), g)
    ref = F.linear(x, w)[:, cols]
    kb = cpu_order.ksplit(N, K, M)
    got = torch.from_numpy(cpu_order.linear_f32(x.float().numpy(), w[cols].float().numpy(), kb)).to(BF16)
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))


@ref_host
@pytest.mark.parametrize("Tq,Tk,causal", [(1, 903, False), (1, 60, False), (60, 60, False), (152, 152, True),
                                          (152, 60, False), (33, 33, True), (300, 300, True)])
def test_sdpa_order_matches_torch(Tq, Tk, causal):
    from oracle import cpu_order
    torch.set_num_threads(8)
    g = torch.Generator().manual_seed(Tq * 7 + Tk)
    q = torch.randn(1, 8, Tq, 256, generator=g).to(BF16)
    k = torch.randn(1, 4, Tk, 256, generator=g).to(BF16)
    v = torch.randn(1, 4, Tk, 256, generator=g).to(BF16)
    ref = F.scaled_dot_product_attention(q, k, v, scale=1 / 16, is_causal=causal and Tq > 1, enable_gqa=True)[0]
    got = cpu_order.sdpa(q[0], k[0].repeat_interleave(2, 0), v[0].repeat_interleave(2, 0), 1 / 16,
                         is_causal=causal, Hq=8)
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize("name", ["golden_tiny", "golden_tiny_window"])
def test_cpu_order_oracle_reproduces_reference_goldens(name):
    """With every Linear / RMSNorm / SDPA restated (no oneDNN, no aten reductions), the
    oracle reproduces the reference's runs bit for bit: tokens and every logit row."""
    import oracle.t5g_oracle as O
    from oracle import cpu_order
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.weights import synthetic_weights
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    arrs = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    cpu_order.install(O)
    try:
        orc = O.T5GemmaTTSOracle(cfg, sd)
        for ci, c in enumerate(meta["cases"]):
            p = O.SamplerParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                                stop_repetition=c["stop_repetition"], silence_tokens=tuple(c["silence_tokens"]))
            out = orc.generate(c["x"], c["y"], c["tgt"], p, seed=c["seed"], record_logits=True)
            assert out["gen"].view(-1).tolist() == c["gen"], ci
            assert np.array_equal(out["logits"].contiguous().view(torch.int16).numpy(), arrs[f"logits_{ci}"]), ci
    finally:
        cpu_order.uninstall(O)


# ------------------------------------------------------------------- exact_math.h
_SHIM = r"""
#define T5G_HD
#include "exact_math.h"
extern "C" void eval_all(unsigned short* tanh_out, unsigned short* erf_out) {
    for (int i = 0; i < 65536; ++i) {
        unsigned int u = (unsigned int)i << 16; float x; __builtin_memcpy(&x, &u, 4);
        float a = t5g_exact::gelu_tanh(x), b = t5g_exact::gelu_erf(x);
        unsigned int ua, ub; __builtin_memcpy(&ua, &a, 4); __builtin_memcpy(&ub, &b, 4);
        // RNE to bf16 (NaN kept NaN)
        tanh_out[i] = (ua & 0x7fffffff) > 0x7f800000 ? (unsigned short)((ua >> 16) | 0x40)
                                                     : (unsigned short)((ua + 0x7fff + ((ua >> 16) & 1)) >> 16);
        erf_out[i] = (ub & 0x7fffffff) > 0x7f800000 ? (unsigned short)((ub >> 16) | 0x40)
                                                    : (unsigned short)((ub + 0x7fff + ((ub >> 16) & 1)) >> 16);
    }
}
"""


@pytest.fixture(scope="module")
def exact_math_lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("exact_math")
    src = d / "shim.cpp"
    src.write_text(_SHIM)
    so = d / "shim.so"
    inc = os.path.join(REPO, "t5gemma-tts_amd", "csrc")
    r = subprocess.run(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-I", inc, str(src), "-o", str(so)],
                       capture_output=True, text=True)
    if r.returncode:
        pytest.skip(f"g++ unavailable: {r.stderr[-300:]}")
    lib = C.CDLL(str(so))
    t = np.zeros(65536, np.uint16)
    e = np.zeros(65536, np.uint16)
    lib.eval_all(t.ctypes.data_as(C.c_void_p), e.ctypes.data_as(C.c_void_p))
    return t, e


def _finite_mask():
    x = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(BF16).float()
    return torch.isfinite(x).numpy()


def test_gelu_tanh_matches_torch_every_bf16(exact_math_lib):
    """gelu_tanh of exact_math.h == torch's CPU gelu(approximate='tanh') on every finite bf16."""
    tanh_out, _ = exact_math_lib
    x = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(BF16)
    ref = F.gelu(x, approximate="tanh").view(torch.int16).numpy().astype(np.uint16)
    ok = _finite_mask()
    assert np.array_equal(tanh_out[ok], ref[ok]), int((tanh_out[ok] != ref[ok]).sum())


def test_gelu_erf_table_and_exact_form(exact_math_lib):
    """The shipped GELU(erf) table is torch's CPU nn.GELU() of the reference host; the
    exact-erf fallback differs from it only on the 24 documented inputs in [-5.4, -3.1]."""
    _, erf_out = exact_math_lib
    tab = np.fromfile(os.path.join(REPO, "t5gemma-tts_amd", "data", "gelu_erf_bf16.bin"), dtype="<u2")
    assert tab.shape == (65536,)
    ok = _finite_mask()
    diff = np.nonzero(ok & (erf_out != tab))[0]
    xs = torch.from_numpy(diff.astype(np.int32)).to(torch.int16).view(BF16).float()
    assert len(diff) == 24 and bool(((xs >= -5.4) & (xs <= -3.1)).all()), xs.tolist()
    if _reference_host():
        x = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(BF16)
        assert np.array_equal(F.gelu(x).view(torch.int16).numpy().astype(np.uint16)[ok], tab[ok])


# ------------------------------------------------------------------- RoPE cos / sin
_ROPE_SHIM = r"""
#define T5G_HD
#include "exact_math.h"
extern "C" void rope_eval(const float* ang, long n, const unsigned* exc, int ne, unsigned short* c,
                          unsigned short* s) {
    for (long i = 0; i < n; ++i) {
        const float a = t5g_exact::rope_trig(ang[i], 0, exc, ne), b = t5g_exact::rope_trig(ang[i], 1, exc, ne);
        unsigned ua, ub;
        __builtin_memcpy(&ua, &a, 4);
        __builtin_memcpy(&ub, &b, 4);
        c[i] = (unsigned short)(ua >> 16);
        s[i] = (unsigned short)(ub >> 16);
    }
}
"""


@pytest.fixture(scope="module")
def rope_lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("rope_trig")
    src = d / "shim.cpp"
    src.write_text(_ROPE_SHIM)
    so = d / "shim.so"
    inc = os.path.join(REPO, "t5gemma-tts_amd", "csrc")
    r = subprocess.run(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-I", inc, str(src), "-o", str(so)],
                       capture_output=True, text=True)
    if r.returncode:
        pytest.skip(f"g++ unavailable: {r.stderr[-300:]}")
    return C.CDLL(str(so))


def _rope_eval(lib, ang, exc):
    ang = np.ascontiguousarray(ang, np.float32)
    c = np.zeros(ang.size, np.uint16)
    s = np.zeros(ang.size, np.uint16)
    e = np.ascontiguousarray(exc, "<u4") if exc is not None else None
    lib.rope_eval(ang.ctypes.data_as(C.c_void_p), C.c_long(ang.size),
                  e.ctypes.data_as(C.c_void_p) if e is not None else None, 0 if e is None else len(e),
                  c.ctypes.data_as(C.c_void_p), s.ctypes.data_as(C.c_void_p))
    return c, s


def test_rope_trig_matches_reference_host(rope_lib):
    """RoPE cos / sin of exact_math.h (correctly rounded + data/rope_trig_exc.bin) == the
    reference host's torch (MKL VML) cos / sin after the bf16 cast, on the angles of the
    601-code prompt golden, of random position sets of the enumerated family and of every
    table entry; without the table they differ exactly on the table's angles."""
    if not _reference_host():
        pytest.skip("MKL's cos / sin are compared on the reference host only")
    from t5gemma_tts_amd import _lib
    exc = _lib.rope_exc_table()
    assert exc.ndim == 2 and exc.shape[1] == 2 and np.all(np.diff(exc[:, 0].astype(np.int64)) > 0)
    inv = (1.0 / (10000.0 ** (torch.arange(0, 256, 2, dtype=torch.float) / 256))).numpy()
    rng = np.random.default_rng(5)
    pos = [np.array([0.0, 2000.0], np.float32)]
    # lengths across the table's whole coverage (ROPE_EXC_MAX_LEN: 12 288)
    for e in [603, 2, 3, 4096, 9503, _lib.ROPE_EXC_MAX_LEN] + rng.integers(2, _lib.ROPE_EXC_MAX_LEN + 1, size=40).tolist():
        t = torch.arange(e, dtype=torch.float32)
        pos.append(((t / (e - 1)) * 2000.0).numpy())
        pos.append(np.minimum(np.arange(e, dtype=np.float64) / float(e - 1) * 2000.0, 2000.0).astype(np.float32))
    pos = np.unique(np.concatenate(pos))
    ang = np.unique(np.concatenate([(np.float32(f) * pos).astype(np.float32) for f in inv] +
                                   [exc[:, 0].copy().view(np.float32)]))
    c, s = _rope_eval(rope_lib, ang, exc)
    at = torch.from_numpy(ang)
    rc = torch.cos(at).to(BF16).view(torch.int16).numpy().astype(np.uint16)
    rs = torch.sin(at).to(BF16).view(torch.int16).numpy().astype(np.uint16)
    assert np.array_equal(c, rc), int((c != rc).sum())
    assert np.array_equal(s, rs), int((s != rs).sum())
    c0, s0 = _rope_eval(rope_lib, ang, None)
    differ = set(ang[(c0 != rc) | (s0 != rs)].view(np.uint32).tolist())
    assert differ <= set(exc[:, 0].tolist()) and len(differ) > 0


def test_eager_softmax_restatement_bitwise():
    """oracle.cpu_order.softmax_lastdim == nn.functional.softmax(bf16, -1, dtype=float32) on
    this host, bit for bit, at lengths 1 ... 903 (the eager attention's softmax, [tf]
    modeling_t5gemma.py:226)."""
    import torch
    from oracle import cpu_order
    g = torch.Generator().manual_seed(3)
    for L in (1, 5, 16, 17, 60, 64, 152, 527, 903):
        x = (torch.randn(32, L, generator=g) * 3).to(torch.bfloat16)
        ref = torch.softmax(x, dim=-1, dtype=torch.float32)
        got = cpu_order.softmax_lastdim(x)
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), L


def test_eager_pv_one_row_regimes_bitwise():
    """oracle.cpu_order.matmul_m1_pv == torch.matmul(p [1,1,1,K], v [1,1,K,256]) in bf16 on
    this host for K in each measured regime, on absorption inputs (+-2^24 pairs whose
    survivors reveal the summation order)."""
    import numpy as np
    import torch
    from oracle import cpu_order
    rng = np.random.default_rng(5)
    for K in (4, 7, 13, 16, 17, 33, 60, 63, 64, 100):
        p = rng.integers(1, 4, size=K).astype(np.float32)
        v = rng.integers(0, 4, size=(K, 256)).astype(np.float32)
        for n in range(256):
            i, j = rng.choice(K, 2, replace=False)
            v[i, n], v[j, n] = 2.0 ** 24, -2.0 ** 24
            p[i] = p[j] = 1.0
        pt, vt = torch.from_numpy(p).to(torch.bfloat16), torch.from_numpy(v).to(torch.bfloat16)
        ref = torch.matmul(pt.view(1, 1, 1, K), vt.view(1, 1, K, 256)).view(256)
        got = torch.from_numpy(cpu_order.matmul_m1_pv(pt.float().numpy(), vt.float().numpy())).to(torch.bfloat16)
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), K


def test_eager_attention_restatement_reproduces_reference_full_depth():
    """The reference default attn_implementation 'eager' (softcap 50) on the full 2b-2b model:
    with only the attention restated (oracle.cpu_order.eager_attention: the measured oneDNN
    matmul selection, the Sleef-exp softmax; Linears / norms stay torch's, the reference's
    own ops on this host), the oracle reproduces golden_2b2b_eager -- a C3 voice-clone row,
    a prompt-less short text and a 6-query prefill -- tokens and every logit row (sha)."""
    import hashlib
    import oracle.t5g_oracle as O
    from oracle import cpu_order
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.weights import state_dict_digest, synthetic_weights
    meta = json.load(open(os.path.join(GOLDEN, "golden_2b2b_eager.json")))
    torch.set_num_threads(meta["threads"])
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    assert state_dict_digest(sd) == meta["weight_sha256"]
    cpu_order.install_eager_attention(O)
    try:
        orc = O.T5GemmaTTSOracle(cfg, sd)
        for ci, c in enumerate(meta["cases"]):
            p = O.SamplerParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                                stop_repetition=c["stop_repetition"], silence_tokens=tuple(c["silence_tokens"]))
            out = orc.generate(c["x"], c["y"], c["tgt"], p, seed=c["seed"], record_logits=True)
            assert out["gen"].view(-1).tolist() == c["gen"], ci
            bits = out["logits"].contiguous().view(torch.int16).numpy()
            shas = [hashlib.sha256(r.astype(np.int16).tobytes()).hexdigest()[:16] for r in bits]
            assert shas == c["logit_sha"], ci
    finally:
        cpu_order.uninstall(O)
