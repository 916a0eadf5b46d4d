"""Probe: the LDS-staged many-token GEMM (gemm_pfl_kernel, buffer_load ... lds ring) against
the register-ring kernel (gemm_pf_kernel) at the bench's encoder (480 tokens), decoder
prefill (1 216 tokens) and a C5 prefill (4 864 tokens) shapes: HIP-event us per launch
(weights rotated over 8 copies so they stream from HBM at the big shapes), TFLOP/s, and
whether the two outputs are bitwise equal. GPU only."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402

PREFILL, PREFILL_REG = 0x100, 0x200


def main():
    L = _lib.lib()
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = []
    for M in (480, 1216, 4864):
        for name, N, K, epi in [("qkv", 4096, 2304, 0), ("o", 2304, 2048, 0), ("gate_up", 18432, 2304, 3),
                                ("down", 2304, 9216, 0)]:
            g = torch.Generator(device="cpu").manual_seed(N + K + M)
            ps = []
            for c in range(8):
                w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16).to(dev)
                p = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=torch.bfloat16, device=dev)
                _lib.check(L.t5g_pack_weight(C.c_void_p(w.data_ptr()), N, K, K, C.c_void_p(p.data_ptr()), st), "pack")
                ps.append(p)
            X = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
            ldy = N // 2 if epi == 3 else N
            row = {"shape": f"{name}_{M}", "M": M, "N": N, "K": K}
            outs = {}
            for tag, flag in (("lds", PREFILL), ("reg", PREFILL | PREFILL_REG)):
                Y = torch.zeros(M, ldy, dtype=torch.bfloat16, device=dev)
                _lib.check(L.t5g_gemm(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(ps[0].data_ptr()), N, K, 1, None,
                                      C.c_void_p(Y.data_ptr()), ldy, epi | flag, st), "gemm")
                torch.cuda.synchronize()
                outs[tag] = Y.clone()
                arr = (C.c_void_p * len(ps))(*[p.data_ptr() for p in ps])
                us = C.c_float()
                _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, len(ps), N, K, 1,
                                           C.c_void_p(Y.data_ptr()), ldy, epi | flag, 40, st, C.byref(us)), "time")
                row[f"{tag}_us"] = round(us.value, 2)
                row[f"{tag}_tflops"] = round(2.0 * M * N * K / us.value / 1e6, 1)
            row["bitwise_equal"] = bool(torch.equal(outs["lds"].view(torch.int16), outs["reg"].view(torch.int16)))
            res.append(row)
            print(json.dumps(row), flush=True)
            del ps


if __name__ == "__main__":
    main()
