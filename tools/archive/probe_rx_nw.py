"""Probe: waves sharing each unit's K stream in the register-resident-X gate/up GEMV
(nw = 4 / 6 / 8 / 9 / 12: 72 k-steps split evenly) at M = 8 and 32, rotating 8 weight copies
(680 MB) so every launch streams from HBM; also a grid cap that balances 1152 units."""
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
    d, f = 2304, 9216
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
    arr = (C.c_void_p * len(Ws))(*[w.data_ptr() for w in Ws])
    for M in (8, 32):
        X = torch.randn(M, d, device=dev).to(torch.bfloat16)
        Y = torch.empty(M, f, dtype=torch.bfloat16, device=dev)
        alg = N * d * 2 + M * d * 2 + M * f * 2
        row = {"M": M}
        for nw in (8, 4, 6, 9, 12):
            for grid in (0, 192, 288):
                a = _lib.GemvArgs()
                a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, d, N, 3, 0, nw, 8
                a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), d, Y.data_ptr(), f, 1, 1, grid
                us = C.c_float()
                rc = L.t5g_time_gemv(C.byref(a), arr, len(Ws), 240, st, C.byref(us))
                row[f"nw{nw}_g{grid}"] = round(us.value, 2) if rc == 0 else f"rc {rc}"
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
