"""Drive the decode attention (t5g_attention_decode: scores, P.V and combine launches --
the kernels the engine runs every step) at the C3 shape: 8 rows x 8 q / 4 kv heads x 256,
ragged self-attention lengths around the C3 mean (L = 527), over 26 distinct KV caches
(26 x 16.8 MB = 436 MB > the 256 MiB Infinity Cache, as the 26 layers of a real step), so
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE can count the HBM bytes per call. GPU only.
Prints the algorithmic bytes per call (K and V rows of every key a row attends to,
q in, output out)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402

B, HQ, HKV, D, CAP, N_CACHES = 8, 8, 4, 256, 1024, 26
LENS = [527, 526, 520, 512, 530, 541, 515, 545]


def algorithmic_bytes():
    kv = sum(LENS) * HKV * D * 2 * 2
    return kv + B * HQ * D * 2 * 2


def main():
    flash = "--flash" in sys.argv   # the fast path's one-launch form (t5g_attention_decode_flash)
    L = _lib.lib()
    dev = torch.device("cuda:0")
    caches = [(torch.randn(B, HKV, CAP, D, device=dev).to(torch.bfloat16),
               torch.randn(B, HKV, CAP, D, device=dev).to(torch.bfloat16)) for _ in range(N_CACHES)]
    q = torch.randn(B, HQ, D, device=dev).to(torch.bfloat16)
    lens = torch.tensor(LENS, dtype=torch.int32, device=dev)
    out = torch.empty(B, HQ * D, dtype=torch.bfloat16, device=dev)
    work = torch.zeros(L.t5g_attention_decode_work_bytes(B, HQ, HKV, D, CAP) // 4, dtype=torch.float32, device=dev)
    fn = L.t5g_attention_decode_flash if flash else L.t5g_attention_decode
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(3):
        if it == 1:
            ev0.record()
        for K, V in caches:
            a = _lib.AttnDecodeArgs(B=B, n_heads=HQ, n_kv_heads=HKV, head_dim=D, q=q.data_ptr(), k_cache=K.data_ptr(),
                                    v_cache=V.data_ptr(), cap=CAP, kv_len=lens.data_ptr(), causal=1, window=0,
                                    scale=D ** -0.5, out=out.data_ptr(), work=work.data_ptr())
            _lib.check(fn(C.byref(a), st), "attention_decode")
    ev1.record()
    torch.cuda.synchronize()
    us = ev0.elapsed_time(ev1) * 1e3 / (2 * N_CACHES)
    alg = algorithmic_bytes()
    print(f"attention{' (flash, 1 launch)' if flash else ' (2 launches)'} avg {us:.2f} us/call, algorithmic {alg} B -> "
          f"{alg / us / 1e3:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
