import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import t5gemma_tts_amd
from t5gemma_tts_amd import _lib
L = _lib.lib()
BF16 = torch.bfloat16
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
for (M, N, K, pro) in [(1, 64, 128, 3), (2, 64, 128, 3), (1, 2304, 2048, 3), (1, 64, 128, 0), (1, 4096, 2304, 0)]:
    W = torch.zeros(N, K)
    for n in range(N):
        W[n, n % K] = 1.0
    X = torch.arange(M * K, dtype=torch.float32).view(M, K) % 97
    Wd, Xd = W.to(BF16).cuda(), X.to(BF16).cuda()
    Y = torch.zeros(M, N, dtype=torch.float32, device="cuda")
    a = _lib.GemvArgs()
    a.M, a.K, a.N, a.epi, a.pro, a.nw, a.layout = M, K, N, 4, pro, 4, 1
    a.W, a.Y, a.ldy, a.X, a.ldx = Wd.data_ptr(), Y.data_ptr(), N, Xd.data_ptr(), K
    rc = L.t5g_gemv(C.byref(a), st)
    torch.cuda.synchronize()
    ref = X.to(BF16).float() @ W.t()
    y = Y.cpu()
    bad = (y - ref).abs() > 1e-3
    print(M, N, K, pro, "rc", rc, "bad", int(bad.sum()), "of", bad.numel())
    if bad.any():
        idx = bad.nonzero()[:8]
        for m, n in idx.tolist():
            print("   m", m, "n", n, "got", y[m, n].item(), "want", ref[m, n].item())
