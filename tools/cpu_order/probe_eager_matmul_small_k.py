"""Eager attention P.V at M = 1 with K < 64 keys (the decode cross attention over the text):
none of the chunked / sequential / gemv orders reproduce torch.matmul there (it does at
K >= 64). Candidates and match fractions per K; round-4 result in DESIGN.md section 3."""
import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from oracle import cpu_order as co
torch.set_num_threads(8)
rng = np.random.default_rng(3)
BF = torch.bfloat16
f32 = np.float32
def bits(t): return t.contiguous().view(torch.int16).numpy()
BIG = 2.0 ** 24
def seq(A, B):
    tot = np.zeros((A.shape[0], B.shape[1]), f32)
    for k in range(A.shape[1]):
        tot = (tot + A[:, k, None] * B[None, k]).astype(f32)
    return tot
def probe(M, K, N=256, H=2):
    a = rng.integers(1, 4, size=(1, H, M, K)).astype(f32)
    b = rng.integers(0, 4, size=(1, H, K, N)).astype(f32)
    for h in range(H):
        for n in range(N):
            if K >= 2:
                i, j = rng.choice(K, 2, replace=False)
                b[0, h, i, n], b[0, h, j, n] = BIG, -BIG
                a[0, h, :, i] = a[0, h, :, j] = 1.0
    at, bt = torch.from_numpy(a).to(BF), torch.from_numpy(b).to(BF)
    ref = bits(torch.matmul(at, bt))
    out = {}
    cands = {f"eo{c}": (lambda A, B, c=c: co.eo_chunk_matmul(A, B, chunk=c)) for c in (32, 16, 8, 4, 2)}
    cands["eoK"] = lambda A, B: co.eo_chunk_matmul(A, B, chunk=max(K, 1))
    cands["seq"] = seq
    cands["gemv"] = lambda A, B: co._gemv_pv(A[0], B, None)[None]
    for name, fn in cands.items():
        got = np.stack([fn(at[0, h].float().numpy(), bt[0, h].float().numpy()) for h in range(H)])
        got = bits(torch.from_numpy(got.astype(f32)).to(BF).view(1, H, M, N))
        out[name] = round(float((got == ref).mean()), 3)
    return out
for K in (2, 7, 8, 15, 16, 17, 31, 32, 33, 40, 48, 56, 60, 63, 64):
    r = probe(1, K)
    print(K, {k: v for k, v in r.items() if v > 0.99} or r, flush=True)
