"""The fast decode self attention at the C5 shape: t5g_attention_decode_flash over 32 rows x
8 q / 4 kv heads x 256, cache capacity 960 keys (15 chunks, as a C5 call's key bound), timed
with HIP events over 26 distinct KV caches (as the 26 layers of a step), at row lengths
across a C5 utterance. B / CAP from the environment. GPU only."""
import ctypes as C
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402

B, HQ, HKV, D, N_CACHES = int(os.environ.get("B", "32")), 8, 4, 256, 26
CAP = int(os.environ.get("CAP", "960"))


def main():
    L = _lib.lib()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    caches = [(torch.randn(B, HKV, CAP, D, device=dev).to(torch.bfloat16),
               torch.randn(B, HKV, CAP, D, device=dev).to(torch.bfloat16)) for _ in range(N_CACHES)]
    q = torch.randn(B, HQ, D, device=dev).to(torch.bfloat16)
    out = torch.empty(B, HQ * D, dtype=torch.bfloat16, device=dev)
    work = torch.zeros(L.t5g_attention_decode_work_bytes(B, HQ, HKV, D, CAP) // 4, dtype=torch.float32, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for base in (152, 340, 527, 715, 902):
        lens_l = [base - (i % 3) for i in range(B)]
        lens = torch.tensor(lens_l, dtype=torch.int32, device=dev)
        alg = sum(lens_l) * HKV * D * 2 * 2
        for name, fn in (("flash", L.t5g_attention_decode_flash),):
            for mode in ("cold",):
                seq = caches if mode == "cold" else [caches[0]] * N_CACHES
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for it in range(3):
                    if it == 1:
                        ev0.record()
                    for K, V in seq:
                        a = _lib.AttnDecodeArgs(B=B, n_heads=HQ, n_kv_heads=HKV, head_dim=D, q=q.data_ptr(),
                                                k_cache=K.data_ptr(), v_cache=V.data_ptr(), cap=CAP,
                                                kv_len=lens.data_ptr(), causal=1, window=0, scale=D ** -0.5,
                                                out=out.data_ptr(), work=work.data_ptr())
                        _lib.check(fn(C.byref(a), st), name)
                ev1.record()
                torch.cuda.synchronize()
                us = ev0.elapsed_time(ev1) * 1e3 / (2 * N_CACHES)
                h = hashlib.sha256(out.cpu().view(torch.int16).numpy().tobytes()).hexdigest()[:12]
                print(f"L~{base} {name:10s} {mode}: {us:6.2f} us/call, {alg / 1e6:.1f} MB -> {alg / us / 1e3:6.0f} GB/s"
                      f"  out {h}", flush=True)


if __name__ == "__main__":
    main()
