"""Eager attention (attn_implementation="eager", the reference default) matmul orders on the
reference host: torch.matmul of bf16 [1,H,M,K] x [1,H,K,N] against the E/O chunk model of
oracle/cpu_order.py with candidate chunk sizes and K splits, on absorption inputs (+-2^24
pairs whose survivors reveal the order). Output: the (chunk, K-part) pairs that reproduce
every output bit. Round-4 result in DESIGN.md section 3 (eager)."""
import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from oracle import cpu_order as co
torch.set_num_threads(8)
rng = np.random.default_rng(2)
BF = torch.bfloat16
f32 = np.float32
def bits(t): return t.contiguous().view(torch.int16).numpy()
BIG = 2.0 ** 24

def eo_split(A, B, chunk, kb):
    K = A.shape[1]
    tot = None
    for p0 in range(0, K, kb):
        part = co.eo_chunk_matmul(A[:, p0:p0 + kb], B[p0:p0 + kb], chunk=chunk)
        tot = part if tot is None else (tot + part).astype(f32)
    return tot

def probe(M, K, N, H=2):
    a = rng.integers(1, 4, size=(1, H, M, K)).astype(f32)
    b = rng.integers(0, 4, size=(1, H, K, N)).astype(f32)
    for h in range(H):
        for n in range(N):
            i, j = rng.choice(K, 2, replace=False)
            b[0, h, i, n], b[0, h, j, n] = BIG, -BIG
            a[0, h, :, i] = a[0, h, :, j] = 1.0
    at, bt = torch.from_numpy(a).to(BF), torch.from_numpy(b).to(BF)
    ref = bits(torch.matmul(at, bt))
    res = []
    for chunk in (32, 30, 28, 20, 16, 12, 10, 8, 6, 4, 2):
        for kb in sorted({K, 32 * ((K + 31) // 64), 64, 128, 256, 512}):
            if kb <= 0 or kb > K:
                continue
            got = np.stack([eo_split(at[0, h].float().numpy(), bt[0, h].float().numpy(), chunk, kb) for h in range(H)])
            got = bits(torch.from_numpy(got.astype(f32)).to(BF).view(1, H, M, N))
            m = (got == ref).mean()
            if m > 0.999:
                res.append((chunk, kb))
    return res

for (M, K, N) in [(1, 60, 256), (1, 64, 256), (1, 65, 256), (1, 100, 256), (1, 200, 256), (1, 600, 256), (1, 903, 256),
                  (1, 1500, 256), (60, 60, 256), (152, 152, 256), (152, 60, 256), (60, 256, 60), (152, 256, 152)]:
    print((M, K, N), probe(M, K, N), flush=True)
