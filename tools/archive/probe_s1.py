"""Probe for the fused-norm decode plan: o / cross-o projections (2304 x 2048) as one
K pass with bf16 output (split 1) vs the 4 fp32 k-slices the step runs, and cross-q
(2048 x 2304) on the register-resident-X GEMV with bf16 output vs the tiled GEMM at 4
k-slices; M = 8, weights rotated over >= 600 MB so every launch streams from HBM."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    M = 8
    for name, N, K in (("o", 2304, 2048), ("cross_q", 2048, 2304)):
        nbytes = N * K * 2
        n_w = max(2, -(-600_000_000 // nbytes))
        Ws = []
        for i in range(n_w):
            raw = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            dst = torch.empty(int(L.t5g_packed_bytes(N, K)) // 2, dtype=torch.bfloat16, device=dev)
            _lib.check(L.t5g_pack_weight(C.c_void_p(raw.data_ptr()), N, K, K, C.c_void_p(dst.data_ptr()), st), "pack")
            Ws.append(dst)
            del raw
        arr = (C.c_void_p * len(Ws))(*[w.data_ptr() for w in Ws])
        X = torch.randn(M, K, device=dev).to(torch.bfloat16)
        Y = torch.empty(8, M, N, dtype=torch.float32, device=dev)
        row = {"op": name, "M": M}
        for s, epi in ((4, 4), (2, 4), (1, 0)):
            us = C.c_float()
            _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(Ws), N, K, s,
                                       C.c_void_p(Y.data_ptr()), N, epi, 200, st, C.byref(us)), "gemm")
            row[f"gemm_s{s}_us"] = round(us.value, 2)
        if K == 2304:
            a = _lib.GemvArgs()
            a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, K, N, 0, 0, 8, 8
            a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), K, Y.data_ptr(), N, 1, 1, 0
            u2 = C.c_float()
            rc = L.t5g_time_gemv(C.byref(a), arr, len(Ws), 200, st, C.byref(u2))
            row["rx_s1_bf16_us"] = round(u2.value, 2) if rc == 0 else f"rc {rc}"
        print(json.dumps(row), flush=True)
        del Ws


if __name__ == "__main__":
    main()
