"""Write t5gemma-tts_amd/data/tanh_bf16.bin: torch 2.10 CPU tanh on every bf16 input, as the
reference host computes the eager attention's softcap tanh ([tf] modeling_t5gemma.py:220 on
a bf16 tensor). 65 536 little-endian uint16 outputs indexed by the input's bits; the
eager-attention kernels (csrc/eager.hip) look it up. Run here only (the reference host)."""
import os

import torch

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                   "t5gemma-tts_amd", "data", "tanh_bf16.bin")


def main():
    torch.set_num_threads(8)
    x = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    y = torch.tanh(x).view(torch.int16).numpy().astype("<u2")
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    y.tofile(OUT)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
