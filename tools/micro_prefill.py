"""Encoder / prefill GEMM shapes at the bench workload (B = 8: encoder 8 x 60 = 480 tokens,
decoder prefill 8 x 152 = 1216 tokens): old path (decode-style tiles, 64 tokens per block)
vs the register-tiled many-token kernel (T5G_GEMM_PREFILL). us per launch, TFLOP/s."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402

PREFILL = 0x100


def main():
    L = _lib.lib()
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for M in (480, 1216):
        for name, N, K, epi in [("qkv", 4096, 2304, 0), ("o", 2304, 2048, 0), ("gate_up", 18432, 2304, 3),
                                ("down", 2304, 9216, 0), ("cross_kv", 2048, 2304, 0)]:
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            p = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=torch.bfloat16, device=dev)
            _lib.check(L.t5g_pack_weight(C.c_void_p(w.data_ptr()), N, K, K, C.c_void_p(p.data_ptr()), st), "pack")
            X = torch.randn(M, K, device=dev).to(torch.bfloat16)
            Y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            arr = (C.c_void_p * 1)(p.data_ptr())
            res = []
            for flag in (0, PREFILL):
                us = C.c_float()
                _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, 1, N, K, 1, C.c_void_p(Y.data_ptr()),
                                           N // 2 if epi == 3 else N, epi | flag, 20, st, C.byref(us)), "time")
                res.append(us.value)
            fl = 2.0 * M * N * K
            print(f"M={M:5d} {name:9s} N={N:6d} K={K:5d}: old {res[0]:8.1f} us ({fl / res[0] / 1e6:6.1f} TF/s)  "
                  f"new {res[1]:8.1f} us ({fl / res[1] / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
