"""CPU-only probe: which fp32 accumulation order of q.k and P.V reproduces torch 2.10's
CPU bf16 SDPA (aten cpu_flash_attention) bit for bit? Candidates on top of
oracle/sdpa_emu.py (softmax parts already exact):
  S  : fp64-rounded-once | E/O chains per 32-element chunk, chunk sums folded in order
  PV : fp64 | chunk model then dst * et + pv | chunk model accumulating onto dst * et
Run: python tools/cpu_order/sdpa_order_probe.py
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import sdpa_emu as E  # noqa: E402

BF16, F32 = torch.bfloat16, torch.float32


def chunk_dot(a, b, init=None):
    """a [..., K], b [..., K] fp32 exact products; E/O chains per 32-chunk, folded."""
    P = (a.double() * b.double()).float()
    K = P.shape[-1]
    tot = init.clone() if init is not None else None
    for c in range(0, K, 32):
        blk = P[..., c:c + 32]
        n = blk.shape[-1]
        e = blk[..., 0].clone()
        o = blk[..., 1].clone() if n > 1 else torch.zeros_like(e)
        for m in range(1, (n + 1) // 2):
            e = e + blk[..., 2 * m]
            if 2 * m + 1 < n:
                o = o + blk[..., 2 * m + 1]
        s = e + o
        tot = s if tot is None else tot + s
    return tot


def attention(q, k, v, scale, s_mode, pv_mode):
    H, Tq, D = q.shape
    rep = H // k.shape[0]
    k = k.repeat_interleave(rep, 0)
    v = v.repeat_interleave(rep, 0)
    Tk = k.shape[1]
    if s_mode == "f64":
        S = (q.double() @ k.double().transpose(1, 2)).float()
    else:
        S = chunk_dot(q[:, :, None, :].float(), k[:, None, :, :].float())
    S = S * torch.tensor(scale, dtype=F32)
    m = torch.full((H, Tq), float("-inf"))
    l = torch.zeros(H, Tq)
    dst = torch.zeros(H, Tq, D)
    for bs in range(0, Tk, 512):
        blen = min(512, Tk - bs)
        sb = S[..., bs:bs + blen]
        mn = torch.maximum(m, sb.max(-1).values)
        p = E.block_p(sb - mn[..., None], blen)
        ts = E.block_sum(p)
        et = torch.where(torch.isinf(m), torch.zeros_like(m), torch.exp((m - mn).double()).float())
        l = E._fma(et, l, ts)
        pb = p.to(BF16).float()
        vb = v[:, bs:bs + blen].float()
        if pv_mode == "f64":
            pv = (pb.double() @ vb.double()).float()
            dst = dst * et[..., None] + pv
        else:
            a = pb[:, :, None, :]                       # [H, Tq, 1, blen]
            b = vb.transpose(1, 2)[:, None, :, :]       # [H, 1, D, blen]
            if pv_mode == "chunk_add":
                dst = dst * et[..., None] + chunk_dot(a, b)
            else:                                       # chunk sums onto the rescaled dst
                dst = chunk_dot(a, b, init=dst * et[..., None] if bs > 0 else None)
        m = mn
    return (dst * (1.0 / l)[..., None]).to(BF16)


def main():
    torch.set_num_threads(8)
    for L in (17, 64, 152, 527, 903):
        g = torch.Generator().manual_seed(L)
        q = torch.randn(8, 1, 256, generator=g).to(BF16)
        k = torch.randn(4, L, 256, generator=g).to(BF16)
        v = torch.randn(4, L, 256, generator=g).to(BF16)
        ref = F.scaled_dot_product_attention(q[None], k[None], v[None], scale=256 ** -0.5, enable_gqa=True)[0]
        res = {}
        for s_mode in ("f64", "chunk"):
            for pv_mode in ("f64", "chunk_add", "chunk_onto"):
                got = attention(q, k, v, 256 ** -0.5, s_mode, pv_mode)
                res[f"{s_mode}/{pv_mode}"] = round((got.view(torch.int16) == ref.view(torch.int16)).float().mean().item(), 5)
        print(L, res, flush=True)


if __name__ == "__main__":
    main()
