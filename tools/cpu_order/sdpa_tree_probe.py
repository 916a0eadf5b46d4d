"""CPU-only probe (build container): the association tree of the fp32 dot products inside
torch 2.10's CPU bf16 scaled_dot_product_attention (aten cpu_flash_attention), decode-shaped
as the reference calls it (q [1, 8, 1, 256], k / v [1, 4, L, 256], enable_gqa, scale 1/16).

q.k: two keys, k0 = ones, k1 = zeros, v0 = ones, v1 = zeros. A query holding +B at dim i,
-B at dim j and a small c at dim s scores s0 = c or 0 depending on whether c was added
before B and -B cancelled (B = 2^30, c = 16: c is absorbed by a partial sum of B). The
output p0 / (p0 + p1) tells which.
P.V: L keys all scoring 0 (q = 0), so p = 1 for every key and out = bf16(sum_t V[t] / L);
a V column holding +B at key i, -B at key j and c at key s reveals the key-sum tree.

Each candidate model predicts absorbed / not for every probe; the script prints which
candidates reproduce every probe. Run: python tools/cpu_order/sdpa_tree_probe.py
"""
import itertools

import numpy as np
import torch
import torch.nn.functional as F

BF16 = torch.bfloat16
B, C = 2.0 ** 30, 16.0


def sdpa(q, k, v):
    return F.scaled_dot_product_attention(q, k, v, scale=1.0 / 16, enable_gqa=True)


# ---------------------------------------------------------------- candidate trees
def seq(vals):
    acc = np.float32(0)
    for v in vals:
        acc = np.float32(acc + np.float32(v))
    return acc


def eo_chunks(vals, chunk=32):
    tot = None
    for c in range(0, len(vals), chunk):
        blk = vals[c:c + chunk]
        e = np.float32(blk[0])
        o = np.float32(blk[1]) if len(blk) > 1 else np.float32(0)
        for m in range(2, len(blk)):
            if m % 2 == 0:
                e = np.float32(e + np.float32(blk[m]))
            else:
                o = np.float32(o + np.float32(blk[m]))
        s = np.float32(e + o)
        tot = s if tot is None else np.float32(tot + s)
    return tot


def lanes(vals, W):
    """W-lane vector accumulation (lane = index % W, each lane sequential), then a
    sequential horizontal sum of the lanes."""
    acc = [np.float32(0)] * W
    for t, v in enumerate(vals):
        acc[t % W] = np.float32(acc[t % W] + np.float32(v))
    return seq(acc)


def lanes_tree(vals, W):
    acc = [np.float32(0)] * W
    for t, v in enumerate(vals):
        acc[t % W] = np.float32(acc[t % W] + np.float32(v))
    while len(acc) > 1:
        h = len(acc) // 2
        acc = [np.float32(acc[i] + acc[i + h]) for i in range(h)]
    return acc[0]


CANDS = {
    "seq": seq,
    "eo32": eo_chunks,
    "eo16": lambda v: eo_chunks(v, 16),
    "eo64": lambda v: eo_chunks(v, 64),
    "lanes8": lambda v: lanes(v, 8),
    "lanes16": lambda v: lanes(v, 16),
    "lanes16tree": lambda v: lanes_tree(v, 16),
    "lanes8tree": lambda v: lanes_tree(v, 8),
    "lanes32": lambda v: lanes(v, 32),
    "lanes64": lambda v: lanes(v, 64),
}


def probe_qk(n=400, seed=0):
    rng = np.random.default_rng(seed)
    D = 256
    trip = [tuple(rng.choice(D, 3, replace=False)) for _ in range(n)]
    obs = []
    for g0 in range(0, n, 8):
        group = trip[g0:g0 + 8]
        q = torch.zeros(1, 8, 1, D)
        for h, (i, j, s) in enumerate(group):
            q[0, h, 0, i], q[0, h, 0, j], q[0, h, 0, s] = B, -B, C
        k = torch.zeros(1, 4, 2, D)
        k[:, :, 0] = 1.0
        v = torch.zeros(1, 4, 2, D)
        v[:, :, 0] = 1.0
        o = sdpa(q.to(BF16), k.to(BF16), v.to(BF16)).float()[0, :len(group), 0, 0]
        obs += [bool(x > 0.6) for x in o.tolist()]   # kept c -> s0 = 1 -> 0.73
    return trip, obs


def probe_pv(L, n=400, seed=1):
    rng = np.random.default_rng(seed + L)
    D = 256
    trip = [tuple(rng.choice(L, 3, replace=False)) for _ in range(n)]
    obs = []
    for g0 in range(0, n, D):
        group = trip[g0:g0 + D]
        q = torch.zeros(1, 8, 1, D)
        k = torch.zeros(1, 4, L, D)
        v = torch.zeros(1, 4, L, D)
        for d, (i, j, s) in enumerate(group):
            v[0, 0, i, d], v[0, 0, j, d], v[0, 0, s, d] = B, -B, C
        o = sdpa(q.to(BF16), k.to(BF16), v.to(BF16)).float()[0, 0, 0, :len(group)] * L
        obs += [bool(x > C / 2) for x in o.tolist()]
    return trip, obs


def check(name, trip, obs, size):
    ok = []
    for cname, fn in CANDS.items():
        good = True
        for (i, j, s), kept in zip(trip, obs):
            vals = np.zeros(size, np.float32)
            vals[i], vals[j], vals[s] = B, -B, C
            pred = bool(fn(vals) > C / 2)
            if pred != kept:
                good = False
                break
        if good:
            ok.append(cname)
    print(f"{name}: kept {sum(obs)}/{len(obs)}; matching candidates: {ok}", flush=True)


def main():
    torch.set_num_threads(8)
    trip, obs = probe_qk()
    check("q.k (D=256)", trip, obs, 256)
    for L in (16, 64, 100, 300, 512, 700):
        trip, obs = probe_pv(L)
        check(f"P.V (L={L})", trip, obs, L)


if __name__ == "__main__":
    main()
