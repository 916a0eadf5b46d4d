"""Probe: the decode down projection (2304 x 9216, fp32 slabs of 8 k-slices) on the
register-resident-X GEMV (32 blocks per slice, several units per block) vs the tiled
decode GEMM, at 8 and 32 rows; HIP-event us per launch over >= 600 MB of rotated weights,
and the slab sums' max |difference| between the two kernels relative to max |y|."""
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
    S = int(os.environ.get("PROBE_SPLITS", "8"))
    n_w = max(2, -(-600_000_000 // (N * K * 2)))
    g = torch.Generator(device=dev).manual_seed(7)
    Ws = []
    for i in range(n_w):
        raw = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        dst = torch.empty(int(L.t5g_packed_bytes(N, K)) // 2, dtype=torch.bfloat16, device=dev)
        _lib.check(L.t5g_pack_weight(C.c_void_p(raw.data_ptr()), N, K, K, C.c_void_p(dst.data_ptr()), st), "pack")
        Ws.append(dst)
        del raw
    arr = (C.c_void_p * len(Ws))(*[w.data_ptr() for w in Ws])
    for M in (8, 32):
        X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        Y = torch.zeros(S, M, N, dtype=torch.float32, device=dev)
        Y2 = torch.zeros(S, M, N, dtype=torch.float32, device=dev)
        us = C.c_float()
        _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(Ws), N, K, S,
                                   C.c_void_p(Y.data_ptr()), N, 4, 200, st, C.byref(us)), "gemm")
        _lib.check(L.t5g_gemm(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(Ws[0].data_ptr()), N, K, S, None,
                              C.c_void_p(Y.data_ptr()), N, 4, st), "gemm1")
        row = {"op": "down", "splits": S, "M": M, "gemm_us": round(us.value, 2)}
        for nw in ((4, 6, 9, 12) if S == 8 else (4, 6, 8, 9, 12)):
            for mg in (0, 512):
                a = _lib.GemvArgs()
                a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, K, N, 4, 0, nw, 8
                a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), K, Y2.data_ptr(), N, S, 1, mg
                a.W = Ws[0].data_ptr()
                u2 = C.c_float()
                rc = L.t5g_time_gemv(C.byref(a), arr, len(Ws), 200, st, C.byref(u2))
                rc2 = L.t5g_gemv(C.byref(a), st)
                torch.cuda.synchronize()
                key = f"rx_nw{nw}" + (f"_g{mg}" if mg else "")
                row[key + "_us"] = round(u2.value, 2) if rc == 0 else f"rc {rc}"
                if rc2 == 0:
                    ys, y2s = Y.sum(0), Y2.sum(0)
                    row[key + "_reldiff"] = float((ys - y2s).abs().max() / ys.abs().max())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
