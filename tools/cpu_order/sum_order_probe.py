import torch, numpy as np
torch.set_num_threads(8)
BIG = 2.0**25
def ranges(xs):
    out=[]
    for x in xs:
        if out and x == out[-1][1]+1: out[-1][1]=x
        else: out.append([x,x])
    return ",".join(f"{a}-{b}" if a!=b else f"{a}" for a,b in out)
for K in (2304, 128):
    S = list(range(0, min(K, 300)))
    for i, j in [(0,1),(0,16),(0,32),(0,64),(0,128),(0,256),(1,17),(0,2)] if K > 200 else [(0,1),(0,16),(0,32),(0,64),(0,2)]:
        rows = []
        for s in S:
            r = np.zeros(K, np.float32); r[i] = BIG; r[j] = -BIG
            if s not in (i, j): r[s] = 1
            rows.append(r)
        X = torch.tensor(np.array(rows))
        g = X.sum(-1).numpy()     # same reduction as .mean (mean = sum / n)
        m = X.mean(-1).numpy() * K
        ab = [s for s, v in zip(S, g) if v == 0 and s not in (i, j)]
        print(K, (i, j), "absorbed:", ranges(ab), "| mean agrees with sum:", np.array_equal(g == 0, m == 0))
