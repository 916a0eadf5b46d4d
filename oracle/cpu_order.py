"""Machine-independent restatement of the reference host's CPU accumulation orders --
TEST INFRASTRUCTURE ONLY (the checker of the exact-order GPU kernels, csrc/exact.hip).

The reference runs inference_tts on CPU in bf16 (inference_commandline_hf.py:102-106).
Its bits depend on the order in which torch 2.10's CPU kernels accumulate fp32 sums.
These orders were measured in the build container -- the machine the golden vectors were
made on -- with absorption probes (tools/cpu_order/*: a partial sum of 2^25 swallows
small terms, so the surviving terms reveal the association tree), then confirmed bit for
bit on random data against torch itself and, with ``install``, on the reference's own
generate() runs (tests/test_cpu_order_cpu.py). numpy float32 arithmetic (each add rounded)
restates them; products of two bf16 values are exact in fp32.

* ``linear``: F.linear -> oneDNN AMX matmul: per output, per 32-element chunk of K an
  even-k chain and an odd-k chain, chunk = E + O, chunk sums folded in order; K cut into
  parts of ``kb`` elements folded in order (kb depends on M, N, K and the thread count:
  tools/cpu_order/ksplit_2b2b_*.jsonl); bias added last.
* ``sum_last``: aten SumKernel.cpp cascade_sum, AVX2 kernel (8-float vectors, 4
  interleaved vector accumulators, a 4-level cascade of 16 rows, lanes summed in order) --
  the mean inside T5Gemma's RMSNorm ([tf] modeling_t5gemma.py:61-78).
* ``sdpa``: aten cpu_flash_attention for bf16 with the GEMM it selects: oneDNN gemv for a
  one-row q block without packing, else the E/O chunk GEMM (q.k over 32-element chunks of
  the head dim; P.V over 32-key chunks + tail, or, when aten packs, chunks of the largest
  even divisor <= 32 of the even-padded block length); later kv blocks accumulate onto the
  rescaled output. Softmax pieces from ``oracle.sdpa_emu``.
* eager attention pieces (the reference default attn_implementation, [tf]
  modeling_t5gemma.py:199-230; the full restatement is not done yet):
  ``softmax_lastdim`` = nn.functional.softmax(x_bf16, -1, dtype=float32) on this host
  (aten's AVX-512 float path: Sleef expf_u10 on every element, reduce_all with one 16-lane
  accumulator and a zero-filled partial tail, halves tree, x * (1 / sum)); ``matmul_m1_pv``
  = torch.matmul of one bf16 probability row with a bf16 V, per its three measured regimes
  (K <= 16: 4 interleaved accumulators, remainder into the first, folded in order;
  17 <= K < 64: one VDPBF16PS pair chain, odd product first; K >= 64: the E/O 32-element
  chunks with no K split).
"""
from __future__ import annotations

import json
import math
import os
from typing import Optional

import numpy as np
import torch

from . import sdpa_emu as E

BF16 = torch.bfloat16
f32 = np.float32
_HERE = os.path.dirname(os.path.abspath(__file__))
_KSPLIT_DIR = os.path.join(os.path.dirname(_HERE), "tools", "cpu_order")


# ------------------------------------------------------------------------- Linear
def eo_chunk_matmul(A: np.ndarray, B: np.ndarray, chunk: int = 32, C: Optional[np.ndarray] = None) -> np.ndarray:
    """A [M, K], B [K, N] fp32 holding bf16 values -> fp32 [M, N]: per chunk of ``chunk``
    k, even and odd product chains, chunk = E + O, folded into the total (which starts at
    C if given)."""
    M, K = A.shape
    N = B.shape[1]
    tot = None if C is None else C.astype(f32).copy()
    for c in range(0, K, chunk):
        n = min(chunk, K - c)
        e = (A[:, c, None] * B[None, c]).astype(f32)
        o = (A[:, c + 1, None] * B[None, c + 1]).astype(f32) if n > 1 else np.zeros((M, N), f32)
        for t in range(2, n):
            p = (A[:, c + t, None] * B[None, c + t]).astype(f32)
            if t % 2 == 0:
                e = (e + p).astype(f32)
            else:
                o = (o + p).astype(f32)
        s = (e + o).astype(f32)
        tot = s if tot is None else (tot + s).astype(f32)
    return tot


def linear_f32(x: np.ndarray, w: np.ndarray, kb: Optional[int] = None) -> np.ndarray:
    """x [M, K], w [N, K] (fp32 of bf16) -> unrounded fp32 [M, N] in the reference order."""
    K = x.shape[1]
    kb = kb or K
    wt = np.ascontiguousarray(w.T)
    tot = None
    for p0 in range(0, K, kb):
        part = eo_chunk_matmul(x[:, p0:p0 + kb], wt[p0:p0 + kb])
        tot = part if tot is None else (tot + part).astype(f32)
    return tot


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, kb: Optional[int] = None,
           threads: int = 8) -> torch.Tensor:
    """F.linear(x, w, bias) for bf16 tensors as the reference host computes it."""
    sh = x.shape
    x2 = x.reshape(-1, sh[-1]).float().numpy()
    if kb is None:
        kb = ksplit(w.shape[0], w.shape[1], x2.shape[0], threads)
    y = linear_f32(x2, w.float().numpy(), kb)
    if bias is not None:
        y = (y + bias.float().numpy()[None]).astype(f32)
    return torch.from_numpy(y).to(BF16).reshape(*sh[:-1], w.shape[0])


_KSPLIT = None


def ksplit(N: int, K: int, M: int, threads: int = 8) -> int:
    """Part length of the reference host's K split for a Linear (N, K) over M rows."""
    global _KSPLIT
    if threads != 8:
        raise ValueError("only the 8-thread K-split table was measured")
    if _KSPLIT is None:
        _KSPLIT = {}
        for fn in sorted(os.listdir(_KSPLIT_DIR)):
            if fn.startswith("ksplit_2b2b_") and fn.endswith(".jsonl"):
                for line in open(os.path.join(_KSPLIT_DIR, fn)):
                    if line.startswith("{"):
                        r = json.loads(line)
                        _KSPLIT[(r["N"], r["K"], r["M"])] = r["Kb"][0]
    return _KSPLIT.get((N, K, M), K)


# ------------------------------------------------------------------------- sums
def sum_last(x: np.ndarray) -> np.ndarray:
    """torch CPU float sum over a contiguous last dim (x [R, n] fp32) -> [R]."""
    x = np.asarray(x, f32)
    R, n = x.shape
    vec, ilp = 8, 4
    vec_size = n // vec
    size_ilp = vec_size // ilp
    V = x[:, :vec_size * vec].reshape(R, vec_size, vec)
    level_power = max(4, (0 if size_ilp <= 1 else int(math.ceil(math.log2(size_ilp)))) // 4)
    level_step = 1 << level_power
    level_mask = level_step - 1
    acc = np.zeros((4, ilp, R, vec), f32)
    i = 0
    while i + level_step <= size_ilp:
        for _ in range(level_step):
            for k in range(ilp):
                acc[0, k] = (acc[0, k] + V[:, i * ilp + k]).astype(f32)
            i += 1
        for j in range(1, 4):
            acc[j] = (acc[j] + acc[j - 1]).astype(f32)
            acc[j - 1] = 0
            if i & (level_mask << (j * level_power)):
                break
    while i < size_ilp:
        for k in range(ilp):
            acc[0, k] = (acc[0, k] + V[:, i * ilp + k]).astype(f32)
        i += 1
    for j in range(1, 4):
        acc[0] = (acc[0] + acc[j]).astype(f32)
    p0 = acc[0, 0].copy()
    for t in range(size_ilp * ilp, vec_size):
        p0 = (p0 + V[:, t]).astype(f32)
    for k in range(1, ilp):
        p0 = (p0 + acc[0, k]).astype(f32)
    fin = np.zeros(R, f32)
    for t in range(vec_size * vec, n):
        fin = (fin + x[:, t]).astype(f32)
    for lane in range(vec):
        fin = (fin + p0[:, lane]).astype(f32)
    return fin


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """T5GemmaRMSNorm ([tf] :61-78) with the reference host's mean order."""
    xf = x.float()
    sh = xf.shape
    s = sum_last((xf * xf).reshape(-1, sh[-1]).numpy())
    ms = torch.from_numpy((s / f32(sh[-1])).astype(f32)).reshape(*sh[:-1], 1)
    out = xf * torch.rsqrt(ms + eps)
    return (out * (1.0 + w.float())).type_as(x)


# ------------------------------------------------------------------------- SDPA
def _gemv_qk(q: np.ndarray, k: np.ndarray) -> np.ndarray:
    """q [D], k [L, D] -> [L]: oneDNN gemv (VDPBF16PS lanes + hadd tree)."""
    L, D = k.shape
    P = (q[None, :] * k).astype(f32)
    acc = np.zeros((L, 16), f32)
    for c in range(0, D, 32):
        blk = P[:, c:c + 32].reshape(L, 16, 2)
        acc = (acc + blk[..., 1]).astype(f32)
        acc = (acc + blk[..., 0]).astype(f32)
    v8 = (acc[:, :8] + acc[:, 8:]).astype(f32)
    v4 = (v8[:, 0::2] + v8[:, 1::2]).astype(f32)
    v2 = (v4[:, 0::2] + v4[:, 1::2]).astype(f32)
    return (v2[:, 0] + v2[:, 1]).astype(f32)


def _gemv_pv(p: np.ndarray, v: np.ndarray, init: Optional[np.ndarray]) -> np.ndarray:
    """p [L], v [L, D] -> [D]: groups of 8 keys, pair chains odd first, added to init."""
    L, D = v.shape
    acc = np.zeros(D, f32) if init is None else init.astype(f32).copy()
    for g0 in range(0, L, 8):
        tmp = np.zeros(D, f32)
        for j in range(g0, min(L, g0 + 8), 2):
            if j + 1 < L:
                tmp = (tmp + p[j + 1] * v[j + 1]).astype(f32)
            tmp = (tmp + p[j] * v[j]).astype(f32)
        acc = (acc + tmp).astype(f32)
    return acc


def need_pack(Tq: int, Tk: int, Hq: int, D: int = 256, threads: int = 8, causal: bool = False) -> bool:
    if not (Tk >= 64 and Tq >= 64):
        return False
    qs = E.qsplit(Tq)
    q_slice = (Tq + qs - 1) // qs
    qs_per_thread = (Hq * q_slice + threads - 1) // threads
    return qs_per_thread * qs * (Tq if causal else Tk) * D / (Hq * Tk * D) >= 4


def even_div_chunk(K: int) -> int:
    Ke = K + (K & 1)
    for c in range(32, 2, -2):
        if Ke % c == 0:
            return c
    return 2


def sdpa(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float, is_causal: bool = False,
         mask: Optional[torch.Tensor] = None, Hq: Optional[int] = None, threads: int = 8,
         row_from: int = 0, row_to: Optional[int] = None) -> torch.Tensor:
    """F.scaled_dot_product_attention on CPU bf16 as the reference host computes it.
    q [H, Tq, D], k / v [H, Tk, D] (GQA already expanded), mask bool [Tq, Tk] (True =
    attend) or None. Returns bf16 [H, Tq, D]. ``row_from`` / ``row_to``: only the q blocks
    holding rows in [row_from, row_to) are computed (aten's q blocks are independent; the
    other rows are left 0)."""
    H, Tq, D = q.shape
    Tk = k.shape[1]
    causal = bool(is_causal and mask is None and Tq > 1)
    pk = need_pack(Tq, Tk, Hq or H, D, threads, causal)
    out = torch.zeros(H, Tq, D, dtype=BF16)
    qsz = E.qsplit(Tq)
    scale_t = torch.tensor(scale, dtype=torch.float32)
    for h in range(H):
        qh, kh, vh = q[h].float().numpy(), k[h].float().numpy(), v[h].float().numpy()
        for r0 in range(0, Tq, qsz):
            r1 = min(r0 + qsz, Tq)
            if r1 <= row_from or (row_to is not None and r0 >= row_to):
                continue
            M = r1 - r0
            nk = min(Tk - Tq + r1, Tk) if causal else Tk
            gemv = M == 1 and not pk
            m = np.full(M, -np.inf, f32)
            l = np.zeros(M, f32)
            dst = None
            for bs in range(0, nk, 512):
                blen = min(512, Tk - bs)
                if gemv:
                    S = _gemv_qk(qh[r0], kh[bs:bs + blen])[None]
                else:
                    S = eo_chunk_matmul(qh[r0:r1], np.ascontiguousarray(kh[bs:bs + blen].T), 32)
                S = torch.from_numpy(S) * scale_t
                if causal:
                    pos = torch.arange(r0, r1)[:, None] + (Tk - Tq)
                    S = S.masked_fill(torch.arange(bs, bs + blen)[None, :] > pos, float("-inf"))
                if mask is not None:
                    S = S.masked_fill(~mask[r0:r1, bs:bs + blen], float("-inf"))
                mt = torch.from_numpy(m)
                mn = torch.maximum(mt, S.max(-1).values)
                p = E.block_p(S - mn[:, None], blen)
                ts = E.block_sum(p)
                et = torch.where(torch.isinf(mt), torch.zeros_like(mt), E.expf(mt - mn))
                l = E._fma(et, torch.from_numpy(l), ts).numpy()
                pb = p.to(BF16).float().numpy()
                init = None if dst is None else (dst * et.numpy()[:, None]).astype(f32)
                if gemv:
                    dst = _gemv_pv(pb[0], vh[bs:bs + blen], None if init is None else init[0])[None]
                else:
                    ch = even_div_chunk(blen) if pk else 32
                    dst = eo_chunk_matmul(pb, vh[bs:bs + blen], ch, C=init)
                m = mn.numpy()
            out[h, r0:r1] = (torch.from_numpy(dst) * torch.from_numpy((f32(1.0) / l).astype(f32))[:, None]).to(BF16)
    return out


# ------------------------------------------------------------------------- oracle hook
def install(oracle_module, threads: int = 8) -> None:
    """Route oracle.t5g_oracle's Linear / RMSNorm / SDPA through these restatements (the
    oracle then no longer depends on the CPU it runs on). Undo with ``uninstall``."""
    O = oracle_module
    if getattr(O, "_cpu_order_saved", None) is None:
        O._cpu_order_saved = (O.T5GemmaTTSOracle._lin, O.rms_norm, O.attention)

    def _lin(self, x, name, bias=None):
        return linear(x, self.w[name], self.w[bias] if bias else None, threads=threads)

    def _attention(q, k, v, *, scale, softcap, n_rep, mask, is_causal, impl):
        if impl != "sdpa":
            raise NotImplementedError("cpu_order restates the sdpa path only")
        B, H, Tq, D = q.shape
        k = k.repeat_interleave(n_rep, 1) if n_rep > 1 else k
        v = v.repeat_interleave(n_rep, 1) if n_rep > 1 else v
        mk = None if mask is None else mask.view(mask.shape[-2], mask.shape[-1])
        o = sdpa(q[0], k[0], v[0], scale, is_causal=is_causal, mask=mk, Hq=H, threads=threads)[None]
        return o.transpose(1, 2).reshape(B, Tq, H * D)

    O.T5GemmaTTSOracle._lin = _lin
    O.rms_norm = rms_norm
    O.attention = _attention


def uninstall(oracle_module) -> None:
    O = oracle_module
    saved = getattr(O, "_cpu_order_saved", None)
    if saved is not None:
        O.T5GemmaTTSOracle._lin, O.rms_norm, O.attention = saved
        O._cpu_order_saved = None


# ------------------------------------------------------------------------- eager pieces
_R_LN2 = f32(1.442695040888963407359924681001892137426645954152985934135449406931)
_L2U, _L2L = f32(0.693145751953125), f32(1.428606765330187045e-06)
_EXPC = [f32(x) for x in (0.000198527617612853646278381, 0.00139304355252534151077271, 0.00833336077630519866943359,
                          0.0416664853692054748535156, 0.166666671633720397949219, 0.5)]


def _fma32(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """fp32 fused multiply-add: the double product of two fp32 values is exact."""
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def sleef_expf(d: np.ndarray) -> np.ndarray:
    """Sleef_expf16_u10 (sleefsimdsp.c xexpf; aten Vectorized<float>::exp,
    ATen/cpu/vec/vec512/vec512_float.h:307) for arguments <= 0 (softmax's x - max)."""
    d0 = np.asarray(d, f32)
    d = np.maximum(d0, f32(-110.0))   # below -104 the result is 0 (selected at the end)
    q = np.rint((d * _R_LN2).astype(f32)).astype(np.int32)
    qf = q.astype(f32)
    s = _fma32(qf, np.full_like(d, -_L2U), d)
    s = _fma32(qf, np.full_like(d, -_L2L), s)
    u = np.full_like(d, _EXPC[0])
    for c in _EXPC[1:]:
        u = _fma32(u, s, np.full_like(d, c))
    u = (f32(1.0) + _fma32((s * s).astype(f32), u, s)).astype(f32)
    e1 = q >> 1
    u = (u * np.exp2(e1).astype(f32)).astype(f32)
    u = (u * np.exp2(q - e1).astype(f32)).astype(f32)
    return np.where(d0 < -104, f32(0), u).astype(f32)


def _reduce_all16(x: np.ndarray) -> np.ndarray:
    """aten vec::reduce_all<float>(+) over the last dim of x [R, n], 16-lane vectors."""
    R, n = x.shape
    if n < 16:
        acc = x[:, 0].copy()
        for i in range(1, n):
            acc = (acc + x[:, i]).astype(f32)
        return acc
    acc = x[:, :16].copy()
    d = 16
    while d < n - (n % 16):
        acc = (acc + x[:, d:d + 16]).astype(f32)
        d += 16
    if n - d > 0:
        acc[:, :n - d] = (acc[:, :n - d] + x[:, d:]).astype(f32)
    w = 16
    while w > 1:
        w //= 2
        acc = (acc[:, :w] + acc[:, w:2 * w]).astype(f32)
    return acc[:, 0]


def softmax_lastdim(x: torch.Tensor) -> torch.Tensor:
    """nn.functional.softmax(x, dim=-1, dtype=torch.float32) for a bf16 x, as the reference
    host computes it (tests/test_cpu_order_cpu.py pins it bitwise)."""
    sh = x.shape
    xf = x.float().reshape(-1, sh[-1]).numpy()
    e = sleef_expf((xf - xf.max(-1, keepdims=True)).astype(f32))
    inv = (f32(1.0) / _reduce_all16(e)).astype(f32)
    return torch.from_numpy((e * inv[:, None]).astype(f32)).reshape(sh)


def matmul_m1_pv(p: np.ndarray, v: np.ndarray) -> np.ndarray:
    """torch.matmul of one bf16 row p [K] with a bf16 v [K, N] (fp32 values) -> unrounded
    fp32 [N], in the reference host's order for that K (three measured regimes)."""
    K, N = v.shape
    P = (p[:, None] * v).astype(f32)
    if K >= 64:
        return eo_chunk_matmul(p[None, :].astype(f32), v.astype(f32))[0]
    if K >= 17:
        acc = np.zeros(N, f32)
        for k in range(0, K, 2):
            if k + 1 < K:
                acc = (acc + P[k + 1]).astype(f32)
            acc = (acc + P[k]).astype(f32)
        return acc
    a = np.zeros((4, N), f32)
    main = K - K % 4
    for k in range(main):
        a[k % 4] = (a[k % 4] + P[k]).astype(f32)
    for k in range(main, K):
        a[0] = (a[0] + P[k]).astype(f32)
    return (((a[0] + a[1]).astype(f32) + a[2]).astype(f32) + a[3]).astype(f32)


def _eo32_b(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """eo_chunk_matmul batched over heads: A [H, M, K], B [H, K, N] -> [H, M, N]."""
    H, M, K = A.shape
    N = B.shape[2]
    tot = None
    for c in range(0, K, 32):
        n = min(32, K - c)
        e = (A[:, :, c, None] * B[:, None, c, :]).astype(f32)
        o = (A[:, :, c + 1, None] * B[:, None, c + 1, :]).astype(f32) if n > 1 else np.zeros((H, M, N), f32)
        for t in range(2, n):
            pr = (A[:, :, c + t, None] * B[:, None, c + t, :]).astype(f32)
            if t % 2 == 0:
                e = (e + pr).astype(f32)
            else:
                o = (o + pr).astype(f32)
        sm = (e + o).astype(f32)
        tot = sm if tot is None else (tot + sm).astype(f32)
    return tot


def _pair_b(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """one VDPBF16PS pair chain per output (odd product first), batched: [H,M,K] x [H,K,N]."""
    H, M, K = A.shape
    acc = np.zeros((H, M, B.shape[2]), f32)
    for k in range(0, K, 2):
        if k + 1 < K:
            acc = (acc + (A[:, :, k + 1, None] * B[:, None, k + 1, :]).astype(f32)).astype(f32)
        acc = (acc + (A[:, :, k, None] * B[:, None, k, :]).astype(f32)).astype(f32)
    return acc


def _u4_b(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """4 interleaved accumulators (remainder into the first), folded in order; batched."""
    H, M, K = A.shape
    a = np.zeros((4, H, M, B.shape[2]), f32)
    main = K - K % 4
    for k in range(K):
        u = k % 4 if k < main else 0
        a[u] = (a[u] + (A[:, :, k, None] * B[:, None, k, :]).astype(f32)).astype(f32)
    return (((a[0] + a[1]).astype(f32) + a[2]).astype(f32) + a[3]).astype(f32)


def eager_matmul(A: np.ndarray, B: np.ndarray, op: str) -> np.ndarray:
    """torch.matmul of the eager attention's bf16 [1, 8, M, K] x [1, 8, K, N] on the reference
    host (the 2b-2b call: batch 1, 8 query heads, head_dim 256), with the accumulation model
    oneDNN selects for that shape (tools/cpu_order/probe_eager_table.py ->
    eager_table_2b2b.jsonl): q.k^T ('qk') 4 accumulators when M * N == 2 else the E/O
    32-element chunks; P.V ('pv') the pair chain when M * K < 64 and (M == 1 or K even), else
    the E/O chunks. No K split at any probed size."""
    H, M, K = A.shape
    N = B.shape[2]
    if op == "qk":
        return _u4_b(A, B) if M * N == 2 else _eo32_b(A, B)
    if M * K < 64 and (M == 1 or K % 2 == 0):
        return _pair_b(A, B)
    return _eo32_b(A, B)


def _bf(x: np.ndarray) -> np.ndarray:
    return torch.from_numpy(np.ascontiguousarray(x, dtype=f32)).to(BF16).float().numpy()


def eager_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float, softcap: float,
                    mask: Optional[torch.Tensor]) -> torch.Tensor:
    """[tf] eager_attention_forward (:199-230) for one call of the reference (q [H, Tq, D],
    k / v [H, Tk, D] bf16 with the GQA heads already repeated; mask bool [Tq, Tk], True =
    attend, or None): q.k^T, x scale, / softcap -> tanh -> x softcap, + finfo.min where
    masked, fp32 softmax -> bf16, P.V -- every bf16 tensor op an fp32 operation rounded
    once (checked over all bf16 inputs for / 50, x 50 and tanh), the matmuls and the softmax
    in the orders above. Returns [H, Tq, D] bf16."""
    qf, kf, vf = q.float().numpy(), k.float().numpy(), v.float().numpy()
    w = _bf(eager_matmul(qf, np.ascontiguousarray(kf.transpose(0, 2, 1)), "qk"))
    w = _bf(w * f32(scale))
    if softcap:
        w = _bf(w / f32(softcap))
        w = torch.tanh(torch.from_numpy(w).to(torch.float64)).to(BF16).float().numpy()
        w = _bf(w * f32(softcap))
    if mask is not None:
        add = np.where(mask.numpy(), f32(0), f32(torch.finfo(BF16).min)).astype(f32)
        w = _bf(w + add[None])
    p = softmax_lastdim(torch.from_numpy(w).to(BF16)).to(BF16).float().numpy()
    o = eager_matmul(p, vf, "pv")
    return torch.from_numpy(o).to(BF16)


def install_eager_attention(oracle_module) -> None:
    """Route only the oracle's eager attention through ``eager_attention`` (its Linears and
    norms stay torch's -- the reference's own ops on this host); ``uninstall`` undoes it."""
    O = oracle_module
    if getattr(O, "_cpu_order_saved", None) is None:
        O._cpu_order_saved = (O.T5GemmaTTSOracle._lin, O.rms_norm, O.attention)
    base = O._cpu_order_saved[2]

    def _attention(q, k, v, *, scale, softcap, n_rep, mask, is_causal, impl):
        if impl != "eager":
            return base(q, k, v, scale=scale, softcap=softcap, n_rep=n_rep, mask=mask, is_causal=is_causal, impl=impl)
        B, H, Tq, D = q.shape
        Tk = k.shape[2]
        k = k.repeat_interleave(n_rep, 1) if n_rep > 1 else k
        v = v.repeat_interleave(n_rep, 1) if n_rep > 1 else v
        if mask is None and is_causal and Tq > 1:
            mask = (torch.arange(Tq)[:, None] + (Tk - Tq) >= torch.arange(Tk)[None, :])
        mk = None if mask is None else mask.reshape(mask.shape[-2], mask.shape[-1])
        outs = [eager_attention(q[b], k[b], v[b], scale, softcap, mk) for b in range(B)]
        o = torch.stack(outs)
        return o.transpose(1, 2).reshape(B, Tq, H * D)

    O.attention = _attention
