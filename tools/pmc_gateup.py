"""Drive the decode-step gate/up GEMM (M = 8, 2304 -> 2 x 9216, GeGLU epilogue) over 26
layers' worth of packed weights (2.2 GB, beyond the 256 MiB Infinity Cache), exactly as
bench.py's roofline leg does, so rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE can count the
HBM bytes per launch. GPU only. Usage (two separate passes, see tools/gpu_pmc.sh):
  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 tools/pmc_gateup.py
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402


def main():
    L = _lib.lib()
    B, d, f, n_layers = 8, 2304, 9216, 26
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    packed = []
    for i in range(n_layers):
        w = (torch.randn(2 * f, d, device=dev) * 0.02).to(torch.bfloat16)
        dst = torch.empty(L.t5g_packed_bytes(2 * f, d) // 2, dtype=torch.bfloat16, device=dev)
        _lib.check(L.t5g_pack_weight(C.c_void_p(w.data_ptr()), 2 * f, d, d, C.c_void_p(dst.data_ptr()), st), "pack")
        packed.append(dst)
        del w
    torch.cuda.synchronize()
    X = torch.randn(B, d, device=dev).to(torch.bfloat16)
    Y = torch.empty(B, f, dtype=torch.bfloat16, device=dev)
    us = _lib.time_gate_up(X.data_ptr(), d, B, [p.data_ptr() for p in packed], 2 * f, d, Y.data_ptr(), 2 * n_layers, st)
    alg = 2 * f * d * 2 + B * d * 2 + B * f * 2
    print(f"gate_up avg {us:.2f} us/launch, algorithmic {alg} B -> {alg / us / 1e3:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
