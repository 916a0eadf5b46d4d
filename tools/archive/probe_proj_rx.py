"""Probe: the decode attention projections (qkv 2304->4096, o / cross-o 2048->2304,
cross-q 2304->2048; fp32 split-K slabs) on the register-resident-X GEMV with
cu_count / splits blocks per slice vs the tiled decode GEMM at the engine's split count,
at 8 and 32 rows (HIP-event us per launch, weights rotated over >= 600 MB)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("qkv", 4096, 2304, 2), ("o", 2304, 2048, 4), ("cross_q", 2048, 2304, 4)]
if os.environ.get("PROBE_ONLY"):
    SHAPES = [s for s in SHAPES if s[0] == os.environ["PROBE_ONLY"]]
NWS = {8: (4, 8), 16: (4, 8), 18: (6, 9), 32: (4, 8), 36: (4, 6, 9, 12)}


def main():
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for name, N, K, s_eng in SHAPES:
        n_w = max(2, -(-600_000_000 // (N * K * 2)))
        g = torch.Generator(device=dev).manual_seed(N + K)
        Ws = []
        for i in range(n_w):
            raw = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
            dst = torch.empty(int(L.t5g_packed_bytes(N, K)) // 2, dtype=torch.bfloat16, device=dev)
            _lib.check(L.t5g_pack_weight(C.c_void_p(raw.data_ptr()), N, K, K, C.c_void_p(dst.data_ptr()), st), "pack")
            Ws.append(dst)
            del raw
        arr = (C.c_void_p * len(Ws))(*[w.data_ptr() for w in Ws])
        for M in (8, 16, 32):
            X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            Y = torch.zeros(8, M, N, dtype=torch.float32, device=dev)
            us = C.c_float()
            _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(Ws), N, K, s_eng,
                                       C.c_void_p(Y.data_ptr()), N, 4, 200, st, C.byref(us)), "gemm")
            row = {"op": name, "M": M, f"gemm_s{s_eng}_us": round(us.value, 2)}
            for S in (2, 4, 8):
                per = K // 32 // S
                for nw in NWS.get(per, ()):
                    a = _lib.GemvArgs()
                    a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, K, N, 4, 0, nw, 8
                    a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), K, Y.data_ptr(), N, S, 1, 0
                    a.W = Ws[0].data_ptr()
                    u2 = C.c_float()
                    rc = L.t5g_time_gemv(C.byref(a), arr, len(Ws), 200, st, C.byref(u2))
                    row[f"rx_s{S}_nw{nw}_us"] = round(u2.value, 2) if rc == 0 else f"rc {rc}"
            print(json.dumps(row), flush=True)
        del Ws


if __name__ == "__main__":
    main()
