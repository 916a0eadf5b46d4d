"""Probe: the 65 541-row head (2304 -> 65541 + bias) on the register-resident-X GEMV at
8 / 16 / 24 / 32 rows and the wave counts whose partial-sum buffer fits LDS, against the
tiled decode GEMM (HIP-event us per launch, weights rotated over >= 600 MB)."""
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
    N, K = 65541, 2304
    nbytes = N * K * 2
    n_w = max(2, -(-600_000_000 // nbytes))
    g = torch.Generator(device=dev).manual_seed(N)
    Ws = []
    for i in range(n_w):
        raw = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        dst = torch.empty(int(L.t5g_packed_bytes(N, K)) // 2, dtype=torch.bfloat16, device=dev)
        _lib.check(L.t5g_pack_weight(C.c_void_p(raw.data_ptr()), N, K, K, C.c_void_p(dst.data_ptr()), st), "pack")
        Ws.append(dst)
        del raw
    arr = (C.c_void_p * len(Ws))(*[w.data_ptr() for w in Ws])
    bias = (torch.randn(N, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    for M in (8, 16, 24, 32):
        X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        Y = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
        us = C.c_float()
        _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(Ws), N, K, 1,
                                   C.c_void_p(Y.data_ptr()), N, 0, 100, st, C.byref(us)), "gemm")
        row = {"op": "head2", "M": M, "gemm_us": round(us.value, 2)}
        for nw in (4, 6, 8, 9):
            a = _lib.GemvArgs()
            a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, K, N, 1, 0, nw, 8
            a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), K, Y.data_ptr(), N, 1, 1, 0
            a.bias = bias.data_ptr()
            a.W = Ws[0].data_ptr()
            u2 = C.c_float()
            rc = L.t5g_time_gemv(C.byref(a), arr, len(Ws), 100, st, C.byref(u2))
            row[f"rx_nw{nw}_us"] = round(u2.value, 2) if rc == 0 else f"rc {rc}"
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
