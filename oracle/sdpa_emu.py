"""Machine-independent restatement of torch's CPU SDPA for bf16 inputs -- TEST
INFRASTRUCTURE ONLY (imported by tests/ as the reference of the GPU attention kernels).

The reference calls ``F.scaled_dot_product_attention`` on CPU bf16 tensors
([tf] integrations/sdpa_attention.py:79-162 from modeling_t5gemma.py's attention), which
dispatches to aten's ``cpu_flash_attention`` (AVX-512 build in the container the goldens
were made in). Its numerics, read off the shipped kernel and confirmed bit-for-bit
against torch 2.10 here (tests/test_sdpa_emu_cpu.py):

* s = fp32(q . k) * scale; per query row, kv blocks of 512 keys with a running max m;
* a causal row t only sees its q-block's key range: keys [0, min(t - t % qs + qs, Tk))
  with qs = 32 / 64 / 256 for Tq < 192 / < 768 / >= 768 (keys > t masked to -inf);
* p = exp(s - m): the first (blen & ~15) keys of each block through at::vec's fast exp
  (``fexp`` below: x*log2e, floor, a cubic correction, exponent bits built by one
  fma + truncation), the tail through std::exp(float) -- the host's glibc expf (``expf``
  below, restated in oracle/glibc_expf.c; not correctly rounded: round 4 used the
  correctly rounded value, which differed at one element of a 4 101-token prefill);
* tmp_sum = 16 lane accumulators (key % 16, in order), xor-8/4/2/1 tree, then the tail in
  order; l = fma(expf(m_old - m), l_old, tmp_sum); dst = dst * expf(m_old - m) + bf16(p) . V;
* out = bf16(dst * (1 / l)).

The q.k and P.V products are accumulated in fp64 and rounded once here; aten's fp32 GEMM
order differs in the last fp32 bit, which moves ~1e-4 of the bf16 outputs by one ulp.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import torch

BF16 = torch.bfloat16
F32, F64 = torch.float32, torch.float64
_C = [torch.tensor(v, dtype=F32).double() for v in
      (-0.07920423895120621, -0.2243383675813675, 0.3035426139831543, 0.00010703434963943437)]
_LOG2E = torch.tensor([0x3fb8aa3b], dtype=torch.int32).view(F32)[0]


_EXPF = None


def _expf_lib():
    global _EXPF
    if _EXPF is None:
        here = os.path.dirname(os.path.abspath(__file__))
        src, lib = os.path.join(here, "glibc_expf.c"), os.path.join(here, "lib", "liboracle_expf.so")
        if not os.path.exists(lib) or os.path.getmtime(lib) < os.path.getmtime(src):
            os.makedirs(os.path.dirname(lib), exist_ok=True)
            subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", lib, src], check=True)
        L = ctypes.CDLL(lib)
        L.oracle_glibc_expf_v.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
        _EXPF = L
    return _EXPF


def expf(x) -> torch.Tensor:
    """std::exp on fp32 values as the reference host computes it (glibc 2.35 expf,
    oracle/glibc_expf.c); fp32 tensor in, fp32 tensor out."""
    a = np.ascontiguousarray(torch.as_tensor(x, dtype=F32).numpy(), dtype=np.float32)
    out = np.empty_like(a)
    _expf_lib().oracle_glibc_expf_v(a.ctypes.data, out.ctypes.data, a.size)
    return torch.from_numpy(out)


def _fma(a, b, c):
    """fp32 fused multiply-add (the product is exact in fp64, one final rounding)."""
    return (a.double() * (b.double() if torch.is_tensor(b) else b) + (c.double() if torch.is_tensor(c) else c)).float()


def fexp(x: torch.Tensor) -> torch.Tensor:
    """aten's vectorised fast exp (bf16 flash-attention softmax), fp32 in / out."""
    x = x.to(F32)
    t = x * _LOG2E
    n = torch.floor(t)
    f = t - n
    p = _fma(f, _C[0], _C[1])
    p = _fma(f, p, _C[2])
    q = _fma(p, f, _C[3])
    y = _fma(t - q, 8388608.0, 1065353216.0)
    bits = torch.trunc(y.double()).to(torch.int64).clamp(0, 0x7f800000).to(torch.int32)
    out = bits.view(F32)
    return torch.where(x < -87.3365478515625, torch.zeros_like(out), out)


def block_p(d: torch.Tensor, blen: int) -> torch.Tensor:
    """p of one kv block: d = s - m [..., blen] (masked keys -inf)."""
    n16 = blen & ~15
    head = fexp(d[..., :n16])
    tail = expf(d[..., n16:].contiguous())
    return torch.cat([head, tail], dim=-1)


def block_sum(p: torch.Tensor) -> torch.Tensor:
    """aten's tmp_sum over the last axis (fp32)."""
    blen = p.shape[-1]
    n16 = blen & ~15
    acc = torch.zeros(p.shape[:-1] + (16,), dtype=F32)
    for i in range(0, n16, 16):
        acc = acc + p[..., i:i + 16]
    idx = torch.arange(16)
    for sh in (8, 4, 2, 1):
        acc = acc + acc[..., idx ^ sh]
    s = acc[..., 0]
    for i in range(n16, blen):
        s = s + p[..., i]
    return s


def qsplit(Tq: int) -> int:
    return 256 if Tq >= 768 else (64 if Tq >= 192 else 32)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float, is_causal: bool = False,
              kv_block: int = 512) -> torch.Tensor:
    """q [H, Tq, D], k / v [H or Hkv, Tk, D] bf16 (GQA by head repeat) -> bf16 [H, Tq, D].
    Causal: query i sits at key position Tk - Tq + i (Tq == Tk for prefill)."""
    H, Tq, D = q.shape
    if k.shape[0] != H:
        rep = H // k.shape[0]
        k = k.repeat_interleave(rep, 0)
        v = v.repeat_interleave(rep, 0)
    Tk = k.shape[1]
    S = (q.double() @ k.double().transpose(1, 2)).float() * torch.tensor(scale, dtype=F32)
    out = torch.empty(H, Tq, D, dtype=BF16)
    qs = qsplit(Tq)
    groups = [(0, Tq, Tk)] if not is_causal else \
        [(q0, min(q0 + qs, Tq), min(Tk - Tq + q0 + qs, Tk)) for q0 in range(0, Tq, qs)]
    for r0, r1, nk in groups:
        s = S[:, r0:r1, :nk].clone()
        if is_causal:
            pos = torch.arange(r0, r1)[:, None] + (Tk - Tq)
            s = s.masked_fill(torch.arange(nk)[None, :] > pos, float("-inf"))
        m = torch.full((H, r1 - r0), float("-inf"), dtype=F32)
        l = torch.zeros(H, r1 - r0, dtype=F32)
        dst = torch.zeros(H, r1 - r0, D, dtype=F32)
        for bs in range(0, nk, kv_block):
            blen = min(kv_block, nk - bs)
            sb = s[..., bs:bs + blen]
            mn = torch.maximum(m, sb.max(dim=-1).values)
            p = block_p(sb - mn[..., None], blen)
            ts = block_sum(p)
            et = torch.where(torch.isinf(m), torch.zeros_like(m), expf(m - mn))
            l = _fma(et, l, ts)
            pv = (p.to(BF16).double() @ v[:, bs:bs + blen].double()).float()
            dst = dst * et[..., None] + pv
            m = mn
        out[:, r0:r1] = (dst * (1.0 / l)[..., None]).to(BF16)
    return out
