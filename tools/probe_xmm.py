"""Probe: hipEvent time of the parity Linears (csrc/xmm.hip) at the 2b-2b decode shapes,
weights rotated over 8 layers' worth (HBM-cold). Prints one JSON line per shape."""
import ctypes as C
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402

L = _lib.lib()
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
BF16 = torch.bfloat16
SHAPES = [("qkv", 4096, 2304, 0), ("o", 2304, 2048, 0), ("cross_q", 2048, 2304, 0), ("gate_up", 18432, 2304, 3),
          ("down", 2304, 9216, 0), ("head1", 2304, 2304, 2), ("head2", 65541, 2304, 1)]
Ms = [int(m) for m in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "8"])]
# optional 2nd argument "var": also time the decode kernel without its fold (var 1) and
# without its MFMA (var 2), epilogue bf16 (where each block's time goes)
VARS = [0, 1, 2] if len(sys.argv) > 2 and sys.argv[2] == "var" else [0]
for name, N, K, epi in SHAPES:
    nb = L.t5g_packed_bytes(N, K)
    n_w = max(2, min(8, int(2.0e9 // nb)))
    ws = []
    for i in range(n_w):
        w = torch.randn(nb // 2, device="cuda").to(BF16)   # any bits: timing only
        ws.append(w)
    arr = (C.c_void_p * n_w)(*[w.data_ptr() for w in ws])
    bias = torch.randn(N, device="cuda").to(BF16)
    for M in Ms:
        X16 = torch.randn(((M + 15) // 16) * 16 * K, device="cuda").to(BF16)
        n_out = N // 2 if epi == 3 else N
        Y = torch.empty(((M + 15) // 16) * 16 * max(n_out, N), device="cuda", dtype=BF16)
        for var in VARS:
            if var and M > 32:
                continue
            us = C.c_float()
            e = epi | (0x1000 if epi == 3 else 0)
            if var:
                e = 0 | (0x4000 if var == 1 else 0x8000)
            _lib.check(L.t5g_time_xmm(C.c_void_p(X16.data_ptr()), M, arr, n_w, N, K, e, C.c_void_p(bias.data_ptr()),
                                      C.c_void_p(Y.data_ptr()), n_out, 50, st, C.byref(us)), "time_xmm")
            gbs = nb / (us.value * 1e-6) / 1e9
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "var": var, "us": round(us.value, 2),
                              "weight_MB": round(nb / 1e6, 1), "GBps": round(gbs, 1)}), flush=True)
    del ws
