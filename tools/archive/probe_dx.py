"""Probe: decode GEMMs with the block's X slice staged in LDS and shared by RG row groups
(T5G_DX = RG, gemm_dx_kernel) vs the fragment-per-MFMA kernel (T5G_DX = 0), M = 8 / 32,
at the 2b-2b decode shapes and split factors; weights rotated over >= 600 MB. Prints the
HIP-event time per launch and a hash of the outputs (must match across modes: same
summation order)."""
import ctypes as C
import hashlib
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
    mode = os.environ.get("T5G_DX", "0")
    shapes = [("qkv", 4096, 2304, 2), ("o", 2304, 2048, 4), ("cross_q", 2048, 2304, 4), ("down", 2304, 9216, 8),
              ("head1", 2304, 2304, 1)]
    for name, N, K, s in shapes:
        nbytes = N * K * 2
        n_w = max(2, -(-600_000_000 // nbytes))
        g = torch.Generator(device=dev).manual_seed(N + K)
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
            epi = 4 if s > 1 else 0
            Y = torch.zeros(s, M, N, dtype=torch.float32, device=dev) if epi == 4 else \
                torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            us = C.c_float()
            _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(Ws), N, K, s,
                                       C.c_void_p(Y.data_ptr()), N, epi, 200, st, C.byref(us)), "gemm")
            Y.zero_()
            _lib.check(L.t5g_gemm(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(Ws[0].data_ptr()), N, K, s, None,
                                  C.c_void_p(Y.data_ptr()), N, epi, st), "gemm1")
            torch.cuda.synchronize()
            h = hashlib.sha1(Y.cpu().view(torch.int16 if epi == 0 else torch.int32).numpy().tobytes()).hexdigest()[:12]
            print(json.dumps({"mode": mode, "op": name, "M": M, "splits": s, "us": round(us.value, 2),
                              "GBps": round(nbytes / us.value / 1e3, 1), "hash": h}), flush=True)
        del Ws


if __name__ == "__main__":
    main()
