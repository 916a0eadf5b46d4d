"""Kernel-selection table of the reference host's bf16 torch.matmul for the eager attention
shapes of the 2b-2b model (batch 1, 8 query heads after repeat_kv, head_dim 256): for
q.k^T [1,8,M,256] x [1,8,256,N] and P.V [1,8,M,K] x [1,8,K,256], which accumulation model
reproduces every output bit on absorption inputs: 'eo32' (E/O 32-element chunks, no K
split), 'pair' (one VDPBF16PS pair chain, odd product first), 'u4' (4 interleaved
accumulators, remainder into the first, folded in order). Writes JSON lines to
tools/cpu_order/eager_table_2b2b.jsonl. Run here only (the reference host)."""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import cpu_order as co  # noqa: E402

torch.set_num_threads(8)
f32 = np.float32
BF = torch.bfloat16
BIG = 2.0 ** 24


def _add(a, b):
    return (a + b).astype(f32)


def m_u4(A, B):
    M, K = A.shape
    N = B.shape[1]
    out = np.zeros((M, N), f32)
    main = K - K % 4
    for m in range(M):
        P = (A[m][:, None] * B).astype(f32)
        a = [np.zeros(N, f32) for _ in range(4)]
        for k in range(main):
            a[k % 4] = _add(a[k % 4], P[k])
        for k in range(main, K):
            a[0] = _add(a[0], P[k])
        out[m] = _add(_add(_add(a[0], a[1]), a[2]), a[3])
    return out


def m_pair(A, B):
    M, K = A.shape
    N = B.shape[1]
    out = np.zeros((M, N), f32)
    for m in range(M):
        P = (A[m][:, None] * B).astype(f32)
        acc = np.zeros(N, f32)
        for k in range(0, K, 2):
            if k + 1 < K:
                acc = _add(acc, P[k + 1])
            acc = _add(acc, P[k])
        out[m] = acc
    return out


def m_eo(A, B):
    return co.eo_chunk_matmul(A, B, chunk=32)


MODELS = (("eo32", m_eo), ("pair", m_pair), ("u4", m_u4))


def probe(M, K, N, H=8, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.integers(1, 4, size=(1, H, M, K)).astype(f32)
    b = rng.integers(0, 4, size=(1, H, K, N)).astype(f32)
    if K >= 2:
        for h in range(H):
            for n in range(N):
                i, j = rng.choice(K, 2, replace=False)
                b[0, h, i, n], b[0, h, j, n] = BIG, -BIG
                a[0, h, :, i] = a[0, h, :, j] = 1.0
    at, bt = torch.from_numpy(a).to(BF), torch.from_numpy(b).to(BF)
    ref = torch.matmul(at, bt).contiguous().view(torch.int16).numpy()
    hits = []
    for name, fn in MODELS:
        got = np.stack([fn(at[0, h].float().numpy(), bt[0, h].float().numpy()) for h in range(H)])
        g = torch.from_numpy(got).to(BF).view(1, H, M, N).contiguous().view(torch.int16).numpy()
        if (g == ref).all():
            hits.append(name)
    return hits


def main():
    out = os.path.join(HERE, "eager_table_2b2b.jsonl")
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    with open(out, "a") as f:
        if which in ("qk", "all"):
            for M in range(2, 17):
                for N in range(1, 65):
                    r = probe(M, 256, N)
                    f.write(json.dumps({"op": "qk", "M": M, "K": 256, "N": N, "models": r}) + "\n")
                    f.flush()
        if which in ("pv", "all"):
            for M in range(2, 17):
                for K in range(1, 65):
                    r = probe(M, K, 256)
                    f.write(json.dumps({"op": "pv", "M": M, "K": K, "N": 256, "models": r}) + "\n")
                    f.flush()


if __name__ == "__main__":
    main()
