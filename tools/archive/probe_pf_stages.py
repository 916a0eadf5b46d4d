"""Probe: register ring depth of the many-token GEMM (gemm_pf_kernel<EPI, S>) at the bench's
encoder (480 tokens) and decoder-prefill (1 216 tokens) shapes. Run once per library built
with -DPF_STAGES=S (T5G_LIB=tools/bin/libt5gtts_pfS.so); prints HIP-event us per launch,
TFLOP/s and a hash of each output (ring depth must not change a bit)."""
import ctypes as C
import hashlib
import json
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
    out = {"lib": os.path.basename(_lib.LIB_PATH)}
    for M in (480, 1216):
        for name, N, K, epi in [("qkv", 4096, 2304, 0), ("o", 2304, 2048, 0), ("gate_up", 18432, 2304, 3),
                                ("down", 2304, 9216, 0)]:
            g = torch.Generator(device="cpu").manual_seed(N + K + M)
            w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16).to(dev)
            p = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=torch.bfloat16, device=dev)
            _lib.check(L.t5g_pack_weight(C.c_void_p(w.data_ptr()), N, K, K, C.c_void_p(p.data_ptr()), st), "pack")
            X = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
            ldy = N // 2 if epi == 3 else N
            Y = torch.zeros(M, ldy, dtype=torch.bfloat16, device=dev)
            _lib.check(L.t5g_gemm(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(p.data_ptr()), N, K, 1, None,
                                  C.c_void_p(Y.data_ptr()), ldy, epi | PREFILL, st), "gemm")
            torch.cuda.synchronize()
            h = hashlib.sha1(Y.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:12]
            arr = (C.c_void_p * 1)(p.data_ptr())
            us = C.c_float()
            _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, 1, N, K, 1, C.c_void_p(Y.data_ptr()),
                                       ldy, epi | PREFILL, 50, st, C.byref(us)), "time")
            out[f"{name}_{M}"] = {"us": round(us.value, 2), "tflops": round(2.0 * M * N * K / us.value / 1e6, 1),
                                  "hash": h}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
