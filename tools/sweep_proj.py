"""Decode projection GEMMs at the 2b-2b shapes: the tiled decode GEMM (gemm_p16, split-K
fp32 slabs, what the step runs) vs the register-resident-X GEMV (layout 1) at the same and
other split factors, M = 8 and 32, rotating enough weight copies (>= 600 MB) that every
launch streams from HBM.  python tools/sweep_proj.py
"""
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
    shapes = [("qkv", 4096, 2304, 2, (1, 2, 4)), ("o", 2304, 2048, 4, (4, 3)), ("cross_q", 2048, 2304, 4, (4, 2, 1)),
              ("down", 2304, 9216, 8, (8, 4, 6))]
    for name, N, K, s_now, rx_splits in shapes:
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
        for M in (8, 32):
            X = torch.randn(M, K, device=dev).to(torch.bfloat16)
            Y = torch.empty(8, M, N, dtype=torch.float32, device=dev)
            us = C.c_float()
            _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(Ws), N, K, s_now,
                                       C.c_void_p(Y.data_ptr()), N, 4, 200, st, C.byref(us)), "gemm")
            row = {"op": name, "M": M, "gemm_p16_splits": s_now, "gemm_p16_us": round(us.value, 2)}
            for s in rx_splits:
                a = _lib.GemvArgs()
                a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, K, N, 4, 0, 8, 8
                a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), K, Y.data_ptr(), N, s, 1, 0
                u2 = C.c_float()
                rc = L.t5g_time_gemv(C.byref(a), arr, len(Ws), 200, st, C.byref(u2))
                row[f"rx_s{s}_us"] = round(u2.value, 2) if rc == 0 else f"rc {rc}"
            print(json.dumps(row), flush=True)
        del Ws


if __name__ == "__main__":
    main()
