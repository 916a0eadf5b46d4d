"""GPU parity of the exact-order kernels (csrc/exact.hip, parity mode): bit-for-bit
against the reference's own runs (golden vectors made by importing the reference in the
build container) and against the machine-independent restatement of the reference
host's accumulation orders (oracle/cpu_order.py). Run on an MI355X (``pytest -m gpu``).

Tolerance: none. Every comparison here is bitwise (bf16 bits, token ids)."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    npz = os.path.join(GOLDEN, name + ".npz")
    return meta, (dict(np.load(npz)) if os.path.exists(npz) else {})


def _st():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _pack(L, W):
    N, K = W.shape
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device="cuda")
    assert L.t5g_pack_weight(C.c_void_p(W.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), _st()) == 0
    return Wp


def _hdr(shape, g):
    """bf16 values over a wide exponent range plus rare huge entries: sums whose bits
    depend on the association order (a plain randn rarely exposes a wrong order)."""
    v = torch.randn(shape, generator=g) * torch.exp2(torch.randint(-10, 11, shape, generator=g).float())
    big = torch.rand(shape, generator=g) < 4.0 / shape[-1]
    return torch.where(big, torch.randn(shape, generator=g) * 2.0 ** 14, v).to(BF16)


# ------------------------------------------------------------------------- Linear
@pytest.mark.parametrize("M,N,K,kb,epi", [
    (1, 2048, 2304, 0, 0), (8, 4096, 2304, 0, 4), (3, 2304, 9216, 4608, 0), (60, 2304, 9216, 3072, 4),
    (152, 2304, 9216, 2304, 0), (8, 2304, 2048, 0, 0), (5, 2304, 2304, 0, 1), (4, 2304, 2304, 0, 2),
    (8, 18432, 2304, 0, 3), (2, 65541, 2304, 0, 1), (17, 300, 128, 0, 0), (9, 256, 128, 0, 3),
    # split-K launches (<= 8 rows, < 256 row tiles): K parts, bias, GEGLU, a ragged last tile
    (8, 2304, 9216, 2304, 3), (7, 1024, 9216, 3072, 1), (1, 1028, 2304, 0, 1), (6, 2304, 9216, 4608, 4),
    # f32-MFMA shapes: 17-32 decode rows (two row tiles), prefill tiles of 4 x 16 rows
    (32, 2304, 9216, 4608, 0), (24, 18432, 2304, 0, 3), (100, 4096, 2304, 768, 0), (160, 2304, 2304, 0, 4),
    # a 602-token prefill (601-code voice prompt): the K splits of the measured table at M = 602
    (602, 2048, 2304, 1152, 0), (602, 2304, 2048, 1024, 0), (602, 4608, 2304, 768, 3), (602, 2304, 9216, 1536, 0),
])
@pytest.mark.parametrize("fn", ["t5g_exact_linear", "t5g_xmm_linear"])
def test_exact_linear_bitwise_vs_cpu_order(M, N, K, kb, epi, fn):
    """t5g_exact_linear (VALU chains) and t5g_xmm_linear (the engine's f32-MFMA chains) ==
    oracle.cpu_order.linear (the reference host's F.linear order)."""
    _need_gpu()
    from oracle import cpu_order
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    g = torch.Generator().manual_seed(M * 131 + N + kb)
    X = _hdr((M, K), g)
    W = _hdr((N, K), g)
    bias = (torch.randn(N, generator=g)).to(BF16)
    Wp = _pack(L, W.cuda())
    Xd, bd = X.cuda(), bias.cuda()
    lut = torch.frombuffer(bytearray(_lib.gelu_erf_table()), dtype=torch.int16).cuda()
    n_out = N // 2 if epi == 3 else N
    Y = torch.zeros(M, n_out, dtype=torch.float32 if epi == 4 else BF16, device="cuda")
    rc = getattr(L, fn)(C.c_void_p(Xd.data_ptr()), K, M, C.c_void_p(Wp.data_ptr()), N, K, kb // 32,
                            C.c_void_p(bd.data_ptr()), C.c_void_p(lut.data_ptr()), C.c_void_p(Y.data_ptr()), n_out,
                            epi, _st())
    assert rc == 0
    torch.cuda.synchronize()
    y32 = cpu_order.linear_f32(X.float().numpy(), W.float().numpy(), kb or None)
    if epi == 4:
        assert np.array_equal(Y.cpu().numpy().view(np.int32), y32.view(np.int32))
        return
    if epi in (1, 2):
        y32 = (y32 + bias.float().numpy()[None]).astype(np.float32)
    ref = torch.from_numpy(y32).to(BF16)
    if epi == 2:
        tab = np.frombuffer(bytes(_lib.gelu_erf_table()), dtype=np.uint16)
        ref = torch.from_numpy(tab[ref.view(torch.int16).numpy().astype(np.uint16)].astype(np.int16)).view(BF16)
    if epi == 3:   # interleaved 8-row gate / up groups
        r3 = ref.float().view(M, N // 16, 2, 8)
        gate, up = r3[:, :, 0].reshape(M, -1).to(BF16), r3[:, :, 1].reshape(M, -1).to(BF16)
        ref = (torch.nn.functional.gelu(gate, approximate="tanh") * up)
    got = Y.cpu()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), \
        int((got.view(torch.int16) != ref.view(torch.int16)).sum())


@pytest.mark.parametrize("M,N,K,kb", [
    (1, 2304, 9216, 4608), (8, 2304, 9216, 4608), (13, 2304, 9216, 4608), (32, 2304, 9216, 3072),
    (5, 1028, 2304, 1152), (3, 300, 256, 96),
])
def test_xmm_decode_parts_bitwise(M, N, K, kb):
    """The decode part mode (one workgroup per (group, K part), the engine's down projection
    at M = 1): each part's fp32 fold, added in order from 0 as the consumer norm does, ==
    the reference order's unrounded sum (oracle.cpu_order.linear_f32 with the same split)."""
    _need_gpu()
    from oracle import cpu_order
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    g = torch.Generator().manual_seed(M * 71 + N + kb)
    X = _hdr((M, K), g)
    W = _hdr((N, K), g)
    Wp = _pack(L, W.cuda())
    Xd = X.cuda()
    parts = -(-K // kb)
    Y = torch.full((parts, M, N), float("nan"), dtype=torch.float32, device="cuda")
    rc = L.t5g_xmm_linear(C.c_void_p(Xd.data_ptr()), K, M, C.c_void_p(Wp.data_ptr()), N, K, kb // 32, None, None,
                          C.c_void_p(Y.data_ptr()), N, 0x2000 | 4, _st())
    assert rc == 0
    torch.cuda.synchronize()
    p = Y.cpu().numpy()
    tot = np.zeros((M, N), np.float32)
    for i in range(parts):
        tot = (tot + p[i]).astype(np.float32)
    y32 = cpu_order.linear_f32(X.float().numpy(), W.float().numpy(), kb)
    assert np.array_equal(tot.view(np.int32), y32.view(np.int32)), int((tot.view(np.int32) != y32.view(np.int32)).sum())


# ------------------------------------------------------------------------- SDPA
@pytest.mark.parametrize("Tk,window,G", [(1, 0, 2), (60, 0, 2), (64, 0, 2), (65, 0, 2), (152, 0, 2), (513, 0, 2),
                                         (903, 0, 2), (40, 8, 2), (600, 0, 1), (200, 0, 1), (518, 0, 2),
                                         (4102, 0, 2), (4103, 0, 2), (4103, 4096, 2), (6150, 4096, 2)])
def test_decode_attention_launches_bitwise_vs_cpu_order(Tk, window, G):
    """The engine's decode attention launches (csrc/xattn.hip: the scores launch, four threads
    per key keeping the gemv's lane accumulators, and the P.V launch) == oracle.cpu_order.sdpa
    for one query per row at its last key: 3 rows of different lengths, 4 kv heads."""
    _need_gpu()
    from oracle import cpu_order
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    Hkv, D = 4, 256
    Hq = Hkv * G
    lens = [Tk, max(1, Tk - 7), max(1, Tk // 2)]
    B, cap = len(lens), max(Tk, 64)
    g = torch.Generator().manual_seed(Tk * 31 + window + G)
    q = torch.randn(B, Hq, D, generator=g).to(BF16)
    kc = torch.randn(B, Hkv, cap, D, generator=g).to(BF16)
    vc = torch.randn(B, Hkv, cap, D, generator=g).to(BF16)
    if Tk > 512:   # the last, partial 512-key block of row 0 holds its maximum (a rescale)
        tail = Tk - Tk % 512
        kc[0, :, tail:Tk] = (kc[0, :, tail:Tk].float() + 2.0 * q[0].view(Hkv, G, D)[:, :1].float()).to(BF16)
    i32 = dict(dtype=torch.int32, device="cuda")
    kv_len = torch.tensor(lens, **i32)
    o = torch.zeros(B, Hq * D, dtype=BF16, device="cuda")
    qd, kd, vd = q.reshape(B, Hq * D).cuda(), kc.cuda(), vc.cuda()   # held: the call reads them
    rc = L.t5g_exact_attention(C.c_void_p(qd.data_ptr()), B, None, None, None, C.c_void_p(kd.data_ptr()),
                               C.c_void_p(vd.data_ptr()), cap, C.c_void_p(kv_len.data_ptr()), Hq, Hkv, D, 1,
                               window, 1.0 / 16, 8, C.c_void_p(o.data_ptr()), _st())
    assert rc == 0
    torch.cuda.synchronize()
    got = o.cpu().view(B, Hq, D)
    for b, n in enumerate(lens):
        lo = n - window if (window and n >= window) else 0
        kk = kc[b, :, lo:n].repeat_interleave(G, 0)
        vv = vc[b, :, lo:n].repeat_interleave(G, 0)
        ref = cpu_order.sdpa(q[b][:, None], kk, vv, 1.0 / 16, is_causal=True, Hq=Hq)[:, 0]
        assert torch.equal(got[b].view(torch.int16), ref.view(torch.int16)), (b, n)


@pytest.mark.parametrize("Tq,Tk,causal,window", [
    (1, 1, 1, 0), (1, 60, 0, 0), (1, 152, 1, 0), (1, 903, 1, 0), (1, 600, 1, 0),   # decode (gemv)
    (60, 60, 0, 0), (33, 33, 0, 0), (152, 152, 1, 0), (152, 60, 0, 0), (200, 200, 1, 0),   # prefill / encoder
    (17, 17, 1, 8), (1, 40, 1, 8), (20, 20, 0, 8),                                       # sliding window
    (602, 602, 1, 0), (602, 60, 0, 0), (1, 603, 1, 0),                                    # 601-code prompt
])
def test_exact_attention_bitwise_vs_cpu_order(Tq, Tk, causal, window):
    """t5g_exact_attention == oracle.cpu_order.sdpa (aten CPU flash attention + the GEMM it
    selects) for decode, prefill, cross and encoder shapes, 8 q heads over 4 kv heads."""
    _need_gpu()
    from oracle import cpu_order
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    Hq, Hkv, D, cap = 8, 4, 256, max(Tk, 64)
    g = torch.Generator().manual_seed(Tq * 1000 + Tk + window)
    q = torch.randn(Tq, Hq, D, generator=g).to(BF16)
    k = torch.randn(Hkv, Tk, D, generator=g).to(BF16)
    v = torch.randn(Hkv, Tk, D, generator=g).to(BF16)
    kc = torch.zeros(1, Hkv, cap, D, dtype=BF16)
    vc = torch.zeros(1, Hkv, cap, D, dtype=BF16)
    kc[0, :, :Tk], vc[0, :, :Tk] = k, v
    qd, kd, vd = q.reshape(Tq, Hq * D).cuda(), kc.cuda(), vc.cuda()
    i32 = dict(dtype=torch.int32, device="cuda")
    q_row = torch.zeros(Tq, **i32)
    q_pos = torch.arange(Tq, **i32)
    q_len = torch.tensor([Tq], **i32)
    kv_len = torch.tensor([Tk], **i32)
    out = torch.zeros(Tq, Hq * D, dtype=BF16, device="cuda")
    rc = L.t5g_exact_attention(C.c_void_p(qd.data_ptr()), Tq, C.c_void_p(q_row.data_ptr()),
                               C.c_void_p(q_pos.data_ptr()), C.c_void_p(q_len.data_ptr()), C.c_void_p(kd.data_ptr()),
                               C.c_void_p(vd.data_ptr()), cap, C.c_void_p(kv_len.data_ptr()), Hq, Hkv, D, causal,
                               window, 1.0 / 16, 8, C.c_void_p(out.data_ptr()), _st())
    assert rc == 0
    torch.cuda.synchronize()
    # the reference call: decode sliding-window layers see the last `window` keys (all
    # visible, explicit mask); long-enough sliding layers an explicit band mask
    kk, vv = k.repeat_interleave(Hq // Hkv, 0), v.repeat_interleave(Hq // Hkv, 0)
    mask = None
    if window and Tk >= window:
        if Tq == 1 and causal:
            kk, vv = kk[:, Tk - window:], vv[:, Tk - window:]
            mask = torch.ones(1, window, dtype=torch.bool)
        else:
            qi = torch.arange(Tq)[:, None] + (Tk - Tq)
            ki = torch.arange(Tk)[None, :]
            mask = ((ki <= qi) & (ki > qi - window)) if causal else ((qi - ki).abs() <= window)
    ref = cpu_order.sdpa(q.transpose(0, 1), kk, vv, 1.0 / 16, is_causal=bool(causal), mask=mask, Hq=Hq)
    ref = ref.transpose(0, 1).reshape(Tq, Hq * D)
    got = out.cpu()
    bad = int((got.view(torch.int16) != ref.view(torch.int16)).sum())
    assert bad == 0, f"{bad} of {got.numel()} outputs differ"


# ------------------------------------------------------------------------- engine
def _engine(cfg, sd, **kw):
    from t5gemma_tts_amd.engine import T5GemmaTTSEngine
    return T5GemmaTTSEngine(cfg, sd, device="cuda:0", **kw)


def _params(c):
    from t5gemma_tts_amd.engine import SamplingParams
    return SamplingParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                          stop_repetition=c["stop_repetition"], silence_tokens=tuple(c["silence_tokens"]))


def _sha(row_bits):
    return hashlib.sha256(row_bits.astype(np.int16).tobytes()).hexdigest()[:16]


def _run_golden(name, max_audio=256, max_text=64, max_gen=200, cases=None, batch=1):
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    if not os.path.exists(os.path.join(GOLDEN, name + ".json")):
        pytest.skip("fixture missing")
    meta, arrs = _load(name)
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    eng = _engine(cfg, sd, max_batch=max(batch, 1), max_text=max_text, max_audio=max_audio, max_gen=max_gen)
    todo = list(range(len(meta["cases"]))) if cases is None else cases
    report = []
    for i0 in range(0, len(todo), batch):
        idx = todo[i0:i0 + batch]
        cs = [meta["cases"][i] for i in idx]
        utts = [Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"]) for c in cs]
        out = eng.generate(utts, [_params(c) for c in cs], seeds=[c["seed"] for c in cs], parity=True,
                           record_logits=True)
        for b, (ci, c) in enumerate(zip(idx, cs)):
            g = out["gen"][b].tolist()
            n = len(c["gen"])
            rows = [lg[b].cpu().view(torch.int16).numpy() for lg in out["logits"][:n]]
            if f"logits_{ci}" in arrs:
                exp = arrs[f"logits_{ci}"]
                eq = [bool(np.array_equal(r, e)) for r, e in zip(rows, exp)]
            else:
                eq = [_sha(r) == s for r, s in zip(rows, c["logit_sha"])]
            first_bad = next((t for t, ok in enumerate(eq) if not ok), None)
            report.append({"case": ci, "tokens_equal": g == c["gen"], "steps": n, "logit_rows_equal": sum(eq),
                           "first_unequal_row": first_bad})
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"exact_{name}.json"), "w") as f:
        json.dump(report, f, indent=1)
    print(name, json.dumps(report))
    return report


@pytest.mark.parametrize("name", ["golden_tiny", "golden_tiny_window"])
def test_exact_engine_tiny_goldens_bitwise(name):
    """Parity mode reproduces the reference's own runs: every case's tokens and every
    step's full logit row bit for bit (free-running, no teacher forcing)."""
    _need_gpu()
    rep = _run_golden(name)
    assert all(r["tokens_equal"] for r in rep), rep
    assert all(r["logit_rows_equal"] == r["steps"] for r in rep), rep


def test_exact_engine_tiny_batched_bitwise():
    """Rows of a parity-mode batch are the reference's single-utterance runs, bitwise."""
    _need_gpu()
    rep = _run_golden("golden_tiny", batch=4)
    assert all(r["tokens_equal"] and r["logit_rows_equal"] == r["steps"] for r in rep), rep


def test_exact_engine_mid_golden_bitwise():
    """2b-2b widths (d 2304, 8/4 heads of 256, FFN 9216, V 65541), 2+2 layers."""
    _need_gpu()
    rep = _run_golden("golden_mid", max_audio=256, max_text=64, max_gen=64)
    assert all(r["tokens_equal"] and r["logit_rows_equal"] == r["steps"] for r in rep), rep


def test_exact_engine_full_golden_bitwise():
    """Full depth (26+26 layers) at the C3 shapes (T_x 60, T_p 151), 16 steps per case:
    tokens and every step's logit-row sha equal the reference's."""
    _need_gpu()
    rep = _run_golden("golden_full", max_audio=200, max_text=64, max_gen=32, batch=2)
    assert all(r["tokens_equal"] and r["logit_rows_equal"] == r["steps"] for r in rep), rep


def test_exact_engine_long_golden():
    """The C3 bench workload's first two rows to the full 751-token budget (L up to 903):
    the reference's tokens, and every step's logit-row sha."""
    _need_gpu()
    rep = _run_golden("golden_long", max_audio=1024, max_text=64, max_gen=760, batch=2)
    assert all(r["tokens_equal"] and r["logit_rows_equal"] == r["steps"] for r in rep), rep


def test_sdpa_expf_device_equals_glibc_restatement():
    """csrc/common.h sdpa_expf (the exact attention kernels' std::exp(float)) == the reference
    host's glibc expf (oracle/glibc_expf.c, equal to libm on all 2^32 inputs) on 2^24 floats
    of (-104, 0] plus every input where glibc differs from the correctly rounded exp in a
    dense scan of (-1, 0]."""
    _need_gpu()
    from oracle import sdpa_emu as E
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    g = np.random.default_rng(11)
    x = np.concatenate([-g.random(1 << 24, dtype=np.float32) * 104.0,
                        -np.arange(0, 1 << 23, dtype=np.float32) / np.float32(1 << 23),
                        np.array([0.0, -87.3365478515625, -88.0, -103.2789, -103.9721, -104.0, -np.inf], np.float32)])
    x = x.astype(np.float32)
    ref = E.expf(torch.from_numpy(x)).numpy()
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty_like(xd)
    assert L.t5g_sdpa_expf(C.c_void_p(xd.data_ptr()), C.c_void_p(yd.data_ptr()), x.size, _st()) == 0
    torch.cuda.synchronize()
    got = yd.cpu().numpy()
    bad = int((got.view(np.int32) != ref.view(np.int32)).sum())
    assert bad == 0, bad
