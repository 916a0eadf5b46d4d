"""Sweep the decode gate/up GEMV launch shape (waves per block, fragments in flight, block
cap) at the 2b-2b shape (M = 8, N = 2 x 9216, K = 2304, GeGLU), rotating over 8 packed
weight copies (680 MB >> the 256 MiB Infinity Cache) so every launch streams from HBM.

    python tools/sweep_gate_up.py
"""
import ctypes as C
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main32():
    """B = 32: the 17..32-row GEMV against the tiled decode GEMM (gemm_p16) it replaces."""
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = torch.device("cuda:0")
    M, d, f = 32, 2304, 9216
    N = 2 * f
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    g = torch.Generator(device="cpu").manual_seed(0)
    Ws = []
    for i in range(8):
        raw = (torch.randn(N, d, generator=g) * 0.02).to(torch.bfloat16).to(dev)
        dst = torch.empty(int(L.t5g_packed_bytes(N, d)) // 2, dtype=torch.bfloat16, device=dev)
        _lib.check(L.t5g_pack_weight(C.c_void_p(raw.data_ptr()), N, d, d, C.c_void_p(dst.data_ptr()), st), "pack")
        Ws.append(dst)
    X = torch.randn(M, d, device=dev).to(torch.bfloat16)
    Y = torch.empty(M, f, dtype=torch.bfloat16, device=dev)
    arr = (C.c_void_p * len(Ws))(*[w.data_ptr() for w in Ws])
    alg = N * d * 2 + M * d * 2 + M * f * 2
    for m in (1, 8, 16, 24, 32):
        res = {}
        for layout in (0, 1):
            if layout == 0 and m > 16:
                continue
            a = _lib.GemvArgs()
            a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = m, d, N, 3, 0, 8, 8
            a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), d, Y.data_ptr(), f, 1, layout, 0
            us = C.c_float()
            _lib.check(L.t5g_time_gemv(C.byref(a), arr, len(Ws), 240, st, C.byref(us)), "gemv")
            res[layout] = round(us.value, 2)
        us2 = C.c_float()
        _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), d, m, arr, len(Ws), N, d, 1, C.c_void_p(Y.data_ptr()), f,
                                   3, 240, st, C.byref(us2)), "gemm")
        print(json.dumps({"M": m, "gemv_lds_x_us": res.get(0), "gemv_reg_x_us": res[1],
                          "gemm_p16_us": round(us2.value, 2),
                          "reg_x_GBps": round(alg / (res[1] * 1e-6) / 1e9, 1)}), flush=True)


def main():
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = torch.device("cuda:0")
    M, d, f = 8, 2304, 9216
    N = 2 * f
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    g = torch.Generator(device="cpu").manual_seed(0)
    Ws = []
    for i in range(8):
        raw = (torch.randn(N, d, generator=g) * 0.02).to(torch.bfloat16).to(dev)
        dst = torch.empty(int(L.t5g_packed_bytes(N, d)) // 2, dtype=torch.bfloat16, device=dev)
        _lib.check(L.t5g_pack_weight(C.c_void_p(raw.data_ptr()), N, d, d, C.c_void_p(dst.data_ptr()), st), "pack")
        Ws.append(dst)
        del raw
    X = torch.randn(M, d, device=dev).to(torch.bfloat16)
    Y = torch.empty(M, f, dtype=torch.bfloat16, device=dev)
    arr = (C.c_void_p * len(Ws))(*[w.data_ptr() for w in Ws])
    alg = N * d * 2 + M * d * 2 + M * f * 2
    out = []
    for nw, un, grid in itertools.product((8, 4), (8, 16), (0, 192, 224, 288, 320, 384, 512)):
        a = _lib.GemvArgs()
        a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, d, N, 3, 0, nw, un
        a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), d, Y.data_ptr(), f, 1, 0, grid
        us = C.c_float()
        rc = L.t5g_time_gemv(C.byref(a), arr, len(Ws), 240, st, C.byref(us))
        row = {"nw": nw, "un": un, "max_grid": grid, "rc": rc,
               "us": round(us.value, 2) if rc == 0 else None,
               "GBps": round(alg / (us.value * 1e-6) / 1e9, 1) if rc == 0 else None}
        print(json.dumps(row), flush=True)
        out.append(row)


if __name__ == "__main__":
    main32() if "--m32" in sys.argv else main()
