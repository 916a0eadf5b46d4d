"""Write t5gemma-tts_amd/data/gelu_erf_bf16.bin: torch 2.10 CPU nn.GELU() (erf) on every
bf16 input, as the reference host computes it (bf16 tensor -> oneDNN eltwise_gelu_erf on
an AVX-512 host, aten gelu_out_cpu). 65,536 little-endian uint16 outputs indexed by the
input's bits. The exact-order head (csrc/exact.hip EPI_BIAS_GELU) looks its GELU up here:
oneDNN's erf approximation differs from the exact erf on 24 inputs in [-5.4, -3.1] after
the bf16 cast (tools/cpu_order notes). Run here only (build container).
"""
import os

import numpy as np
import torch

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                   "t5gemma-tts_amd", "data", "gelu_erf_bf16.bin")


def main():
    torch.set_num_threads(8)
    x = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    y = torch.nn.functional.gelu(x).view(torch.int16).numpy().astype("<u2")
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    y.tofile(OUT)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
