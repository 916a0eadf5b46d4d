"""Probe: predict-head GEMMs (head1 2304 x 2304 + bias + GELU, head2 65541 x 2304 + bias)
on the tiled decode GEMM (what the step runs) vs the register-resident-X GEMV (layout 1),
M = 8 and 32; weights rotated over >= 600 MB; outputs compared between the two."""
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
    for name, N, K, epi in (("head1", 2304, 2304, 2), ("head2", 65541, 2304, 1)):
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
        for M in (8, 32):
            X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            Y = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            Y2 = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            us = C.c_float()
            # t5g_time_gemm passes no bias: time with the bias-free epilogue of the same shape
            _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(Ws), N, K, 1,
                                       C.c_void_p(Y.data_ptr()), N, 0, 200, st, C.byref(us)), "gemm")
            _lib.check(L.t5g_gemm(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(Ws[0].data_ptr()), N, K, 1,
                                  C.c_void_p(bias.data_ptr()), C.c_void_p(Y.data_ptr()), N, epi, st), "gemm1")
            a = _lib.GemvArgs()
            a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, K, N, epi, 0, 8, 8
            a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), K, Y2.data_ptr(), N, 1, 1, 0
            a.bias = bias.data_ptr()
            a.W = Ws[0].data_ptr()
            u2 = C.c_float()
            rc = L.t5g_time_gemv(C.byref(a), arr, len(Ws), 200, st, C.byref(u2))
            rc2 = L.t5g_gemv(C.byref(a), st)
            torch.cuda.synchronize()
            same = bool(torch.equal(Y, Y2)) if rc2 == 0 else None
            print(json.dumps({"op": name, "M": M, "gemm_us": round(us.value, 2),
                              "rx_us": round(u2.value, 2) if rc == 0 else f"rc {rc}",
                              "gemm_GBps": round(nbytes / us.value / 1e3, 1), "rx_equal_gemm": same}), flush=True)
        del Ws


if __name__ == "__main__":
    main()
