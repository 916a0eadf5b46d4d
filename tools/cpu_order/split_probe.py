"""CPU-only probe (build container): for each Linear shape of the voice model and a set
of row counts M, which K-split reproduces torch's CPU bf16 F.linear bit for bit?

Model (gemm_order_model.py): per output, per 32-element chunk of K an even-k and an
odd-k fp32 chain, chunk sum E + O, chunk sums folded in order; K cut into parts of Kb
folded in order; bias added last. This probe searches Kb per (M, N, K) on random
high-dynamic-range data, over a sample of output columns.

Run: python tools/cpu_order/split_probe.py [--threads 8] [--shapes 2b2b|tiny|mid]
Prints one JSON line per (N, K, M): {"N", "K", "M", "Kb": [matching candidates]}.
"""
import argparse
import json

import numpy as np
import torch

f32 = np.float32


def chunk_model(x, w, Kb=None):
    """x [M, K] fp32 (bf16 values), w [N, K] -> fp32 [M, N] per the E/O chunk model."""
    M, K = x.shape
    N = w.shape[0]
    Kb = Kb or K
    tot = None
    for p0 in range(0, K, Kb):
        part = None
        for c in range(p0, min(K, p0 + Kb), 32):
            n = min(32, K - c)
            E = x[:, c, None] * w[None, :, c]
            O = x[:, c + 1, None] * w[None, :, c + 1] if n > 1 else np.zeros((M, N), f32)
            for m in range(1, (n + 1) // 2):
                E = (E + x[:, c + 2 * m, None] * w[None, :, c + 2 * m]).astype(f32)
                if c + 2 * m + 1 < c + n:
                    O = (O + x[:, c + 2 * m + 1, None] * w[None, :, c + 2 * m + 1]).astype(f32)
            s = (E + O).astype(f32)
            part = s if part is None else (part + s).astype(f32)
        tot = part if tot is None else (tot + part).astype(f32)
    return tot


def hdr(shape, g):
    """bf16 values with a wide exponent range (order-revealing sums)."""
    v = torch.randn(shape, generator=g) * torch.exp2(torch.randint(-14, 15, shape, generator=g).float())
    # a few huge entries per row: partial sums that absorb small terms reveal the tree
    big = torch.rand(shape, generator=g) < 8.0 / shape[-1]
    v = torch.where(big, torch.sign(torch.randn(shape, generator=g)) * 2.0 ** 24, v)
    return v.to(torch.bfloat16)


def absorb_rows(N, K, g, rows, n_small=12):
    """Rows of +2^25 / -2^25 at random k plus small integers elsewhere (x = ones): the
    output counts the small terms a partial sum of magnitude 2^25 did not absorb, which
    differs between association trees (K splits) far more often than random data does."""
    w = torch.zeros(N, K)
    for r in rows.tolist():
        idx = torch.randperm(K, generator=g)[:2 + n_small]
        w[r, idx[0]] = 2.0 ** 25
        w[r, idx[1]] = -2.0 ** 25
        w[r, idx[2:]] = torch.randint(1, 4, (n_small,), generator=g).float()
    return w.to(torch.bfloat16)


def probe(M, N, K, cands, ncols=256, seed=0):
    g = torch.Generator().manual_seed(seed + 7 * M + N + K)
    x = torch.ones(M, K, dtype=torch.bfloat16)
    cols = torch.randperm(N, generator=g)[:ncols].sort().values
    w = absorb_rows(N, K, g, cols)
    ref = torch.nn.functional.linear(x, w)
    xr = x[:1].float().numpy()   # x = ones: every row of the product is the same
    wr = w[cols].float().numpy()
    refc = ref[:, cols].float().numpy()
    hits = []
    for kb in cands:
        emu = torch.from_numpy(chunk_model(xr, wr, kb)).to(torch.bfloat16).float().numpy()
        if np.array_equal(np.broadcast_to(emu, refc.shape), refc):
            hits.append(kb)
    return hits


SHAPES = {
    # (N, K): q, k/v, o, gate/up, down, head1, head2 of T5Gemma-2b-2b
    "2b2b": [(2048, 2304), (1024, 2304), (2304, 2048), (9216, 2304), (2304, 9216), (2304, 2304), (65541, 2304)],
    "tiny": [(128, 128), (64, 128), (128, 128), (256, 128), (128, 256), (69, 128)],
    # the decoder / encoder layer shapes only: the calls made with one utterance's prompt or
    # text (M > 512 for long reference clips); the head is called on one row
    "2b2b_layers": [(2048, 2304), (1024, 2304), (2304, 2048), (9216, 2304), (2304, 9216)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--shapes", default="2b2b")
    ap.add_argument("--ms", default="1,2,8,13,20,32,40,42,43,48,60,64,65,100,128,152,200,256,257,300,512",
                    help="comma list, or lo-hi for a range")
    ap.add_argument("--only", default="", help="N,K of one shape of the set (resume a run)")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    shapes = SHAPES[args.shapes]
    if args.only:
        shapes = [tuple(int(v) for v in args.only.split(","))]
    for N, K in shapes:
        cands = sorted({K} | {K // d for d in (2, 3, 4, 6, 8, 9, 12, 16) if K % d == 0 and (K // d) % 32 == 0}, reverse=True)
        if "-" in args.ms:
            lo, hi = (int(v) for v in args.ms.split("-"))
            ms = list(range(lo, hi + 1))
        else:
            ms = [int(v) for v in args.ms.split(",")]
        for M in ms:
            hits = probe(M, N, K, cands)
            print(json.dumps({"N": N, "K": K, "M": M, "threads": args.threads, "Kb": hits}), flush=True)


if __name__ == "__main__":
    main()
