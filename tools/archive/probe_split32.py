"""Probe: k-slice count of the decode down projection (2304 x 9216) at 8 and 32 rows on
the tiled decode GEMM; weights rotated over >= 600 MB (HIP-event us per launch)."""
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
    N, K = 2304, 9216
    n_w = max(2, -(-600_000_000 // (N * K * 2)))
    Ws = []
    for i in range(n_w):
        raw = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        dst = torch.empty(int(L.t5g_packed_bytes(N, K)) // 2, dtype=torch.bfloat16, device=dev)
        _lib.check(L.t5g_pack_weight(C.c_void_p(raw.data_ptr()), N, K, K, C.c_void_p(dst.data_ptr()), st), "pack")
        Ws.append(dst)
    arr = (C.c_void_p * len(Ws))(*[w.data_ptr() for w in Ws])
    for M in (8, 32):
        X = torch.randn(M, K, device=dev).to(torch.bfloat16)
        Y = torch.zeros(24, M, N, dtype=torch.float32, device=dev)
        row = {"op": "down", "M": M}
        for s in (2, 3, 4, 6, 8, 12, 16, 24):
            us = C.c_float()
            _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(Ws), N, K, s,
                                       C.c_void_p(Y.data_ptr()), N, 4, 200, st, C.byref(us)), "gemm")
            row[f"s{s}"] = round(us.value, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
