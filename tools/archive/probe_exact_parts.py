"""Probe: per-call time of the parity-mode kernels (t5g_exact_attention, t5g_exact_linear)
at the 2b-2b decode shapes, through the C-ABI, timed with HIP events on one stream.
Prints one JSON line per case. Run on the GPU box: python tools/probe_exact_parts.py"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import t5gemma_tts_amd  # noqa: F401,E402
from t5gemma_tts_amd import _lib  # noqa: E402

BF16 = torch.bfloat16


def _time(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def attn_case(L, B, Tk, cross=False):
    Hq, Hkv, D = 8, 4, 256
    cap = max(Tk, 64) if not cross else 64
    st = torch.cuda.current_stream().cuda_stream
    q = torch.randn(B, Hq * D, device="cuda").to(BF16)
    kc = torch.randn(B, Hkv, cap, D, device="cuda").to(BF16)
    vc = torch.randn(B, Hkv, cap, D, device="cuda").to(BF16)
    i32 = dict(dtype=torch.int32, device="cuda")
    q_row = torch.arange(B, **i32)
    kv_len = torch.full((B,), Tk, **i32)
    out = torch.zeros(B, Hq * D, dtype=BF16, device="cuda")

    def run():
        rc = L.t5g_exact_attention(C.c_void_p(q.data_ptr()), B, C.c_void_p(q_row.data_ptr()), None, None,
                                   C.c_void_p(kc.data_ptr()), C.c_void_p(vc.data_ptr()), cap,
                                   C.c_void_p(kv_len.data_ptr()), Hq, Hkv, D, 0 if cross else 1, 0, 1.0 / 16, 8,
                                   C.c_void_p(out.data_ptr()), C.c_void_p(st))
        assert rc == 0
    return _time(run)


def linear_case(L, M, N, K, epi=0):
    st = torch.cuda.current_stream().cuda_stream
    X = torch.randn(M, K, device="cuda").to(BF16)
    W = torch.randn(N, K, device="cuda").to(BF16)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device="cuda")
    assert L.t5g_pack_weight(C.c_void_p(W.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), C.c_void_p(st)) == 0
    del W
    n_out = N // 2 if epi == 3 else N
    Y = torch.zeros(M, n_out, dtype=BF16, device="cuda")

    def run():
        rc = L.t5g_exact_linear(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(Wp.data_ptr()), N, K, 0, None, None,
                                C.c_void_p(Y.data_ptr()), n_out, epi, C.c_void_p(st))
        assert rc == 0
    us = _time(run)
    return us, N * K * 2 / us / 1e6


def main():
    L = _lib.lib()
    for B in (1, 8):
        for Tk in (32, 128, 512, 513, 750, 1024):
            print(json.dumps({"kernel": "exact_attn", "B": B, "Tk": Tk, "us": round(attn_case(L, B, Tk), 2)}),
                  flush=True)
        print(json.dumps({"kernel": "exact_attn_cross", "B": B, "Tk": 32, "us": round(attn_case(L, B, 32, True), 2)}),
              flush=True)
    for M in (1, 8):
        for N, K, epi in ((4096, 2304, 0), (2304, 2048, 0), (2048, 2304, 0), (18432, 2304, 3), (2304, 9216, 0)):
            us, tbs = linear_case(L, M, N, K, epi)
            print(json.dumps({"kernel": "exact_linear", "M": M, "N": N, "K": K, "epi": epi, "us": round(us, 2),
                              "TB/s": round(tbs, 2)}), flush=True)


if __name__ == "__main__":
    main()
