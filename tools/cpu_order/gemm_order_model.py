"""CPU-only probe (build container): the accumulation order of torch 2.10's CPU bf16
F.linear (oneDNN, AMX build), as restated in DESIGN.md §5 "reference GEMM order".

Probe rows hold +2^25 / -2^25 / small values at chosen k so that the bf16 result reveals
which small products were absorbed by a partial sum of magnitude 2^25, i.e. the
association tree. Model that reproduces every probe (and random high-dynamic-range data)
bit for bit: per output, for each 32-element chunk of K, an even-k chain and an odd-k
chain (sequential fp32 adds of exact products), chunk sum = E + O, chunk sums folded
sequentially; bias added in fp32 at the end; K split into independent parts of Kb that
are folded sequentially -- Kb depends on M (8 threads, K = 9216: M <= 42 -> 4608,
43..64 -> 3072, 65..256 -> 2304). Run: python tools/cpu_order/gemm_order_model.py
"""
import torch, numpy as np, sys
torch.set_num_threads(8)
f32 = np.float32
BIG = 2.0**25
def chunk_model(P, bias=None):
    """P: [N, K] fp32 products (x = 1), returns fp32 totals per the E/O 32-chunk model."""
    N, K = P.shape
    tot = np.zeros(N, f32)
    for c in range(0, K, 32):
        blk = P[:, c:c+32]
        E = blk[:, 0].copy(); O = blk[:, 1].copy()
        for m in range(1, 16):
            E = (E + blk[:, 2*m]).astype(f32); O = (O + blk[:, 2*m+1]).astype(f32)
        tot = (tot + (E + O).astype(f32)).astype(f32)
    if bias is not None: tot = (tot + bias).astype(f32)
    return tot
def check(M, N, K, with_bias, seed=0):
    rng = np.random.default_rng(seed)
    W = np.zeros((N, K), f32)
    for r in range(N):
        i, j = rng.choice(K, 2, replace=False)
        W[r, i] = BIG; W[r, j] = -BIG
        for s in rng.choice(K, 3, replace=False):
            if W[r, s] == 0: W[r, s] = rng.choice([1.0, 1.5, 3.0])
    b = None
    if with_bias:
        b = (rng.choice([0.0, 1.0, 2.5, BIG, -BIG], N)).astype(f32)
    Wt = torch.tensor(W).to(torch.bfloat16)
    bt = None if b is None else torch.tensor(b).to(torch.bfloat16)
    out = torch.nn.functional.linear(torch.ones(M, K, dtype=torch.bfloat16), Wt, bt).float().numpy()
    emu = torch.from_numpy(chunk_model(W, None if b is None else bt.float().numpy())).to(torch.bfloat16).float().numpy()
    ok = (out == emu[None, :]).mean()
    return ok
for (M, N, K, bias) in [(1, 4096, 2304, 0), (1, 2304, 2048, 0), (1, 18432, 2304, 0), (1, 2304, 9216, 0),
                        (1, 2304, 2304, 1), (1, 65541, 2304, 1), (152, 4096, 2304, 0), (152, 2304, 9216, 0),
                        (60, 1024, 2304, 0), (1, 256, 128, 0), (1, 128, 256, 0), (1, 69, 128, 1), (1, 128, 128, 1),
                        (20, 256, 128, 0), (13, 128, 256, 0)]:
    print(M, N, K, "bias" if bias else "", "chunk-model exact frac:", check(M, N, K, bias), flush=True)

print("--- K=9216 split hypotheses")
def split_model(P, Kb, comb="seq"):
    parts = [chunk_model(P[:, a:a+Kb]) for a in range(0, P.shape[1], Kb)]
    if comb == "seq":
        t = parts[0]
        for q in parts[1:]: t = (t + q).astype(f32)
        return t
    while len(parts) > 1:
        nxt = [(parts[i] + parts[i+1]).astype(f32) if i + 1 < len(parts) else parts[i] for i in range(0, len(parts), 2)]
        parts = nxt
    return parts[0]
def check2(M, N, K, Kb, comb, seed=0):
    rng = np.random.default_rng(seed)
    W = np.zeros((N, K), f32)
    for r in range(N):
        i, j = rng.choice(K, 2, replace=False)
        W[r, i] = BIG; W[r, j] = -BIG
        for s in rng.choice(K, 3, replace=False):
            if W[r, s] == 0: W[r, s] = rng.choice([1.0, 1.5, 3.0])
    out = torch.nn.functional.linear(torch.ones(M, K, dtype=torch.bfloat16), torch.tensor(W).to(torch.bfloat16)).float().numpy()
    emu = torch.from_numpy(split_model(W, Kb, comb)).to(torch.bfloat16).float().numpy()
    return (out == emu[None, :]).mean()
for Kb in (512, 768, 1024, 1152, 1536, 2048, 2304, 3072, 4096, 4608):
    for comb in ("seq", "tree"):
        print(Kb, comb, check2(1, 2304, 9216, Kb, comb), check2(152, 2304, 9216, Kb, comb), flush=True)
