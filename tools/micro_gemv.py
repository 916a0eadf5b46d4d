"""Per-launch timing of the decode-step GEMV shapes (csrc/gemv.hip) at batch 8, HBM-cold:
every launch rotates over 26 distinct packed weight sets (one per decoder layer, more
bytes than the 256 MiB Infinity Cache), as inside a decode step. Prints one line per
(shape, prologue, waves) with us/launch and weight GB/s. GPU only.

  python tools/micro_gemv.py [M]
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402

BF16 = torch.bfloat16
PRO = {"rows": 0, "norm": 1, "embed": 2, "direct": 3}


def main(M=8):
    L = _lib.lib()
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    d, f, q, nl = 2304, 9216, 2048, 26
    packs = {}

    def packed(N, K):
        if (N, K) not in packs:
            ws = []
            for _ in range(nl):
                w = (torch.randn(N, K, device=dev) * 0.02).to(BF16)
                p = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device=dev)
                _lib.check(L.t5g_pack_weight(C.c_void_p(w.data_ptr()), N, K, K, C.c_void_p(p.data_ptr()), st), "pack")
                ws.append(p)
                del w
            packs[(N, K)] = ws
        return packs[(N, K)]

    v = torch.randn(M, f, device=dev).to(BF16)
    h = torch.randn(M, f, device=dev).to(BF16)
    X = torch.randn(M, f, device=dev).to(BF16)
    nw_ = (torch.randn(2, f, device=dev) * 0.1).to(BF16)
    ids = torch.arange(M, dtype=torch.int32, device=dev)
    table = torch.randn(64, d, device=dev).to(BF16)
    bias = torch.zeros(65541, dtype=BF16, device=dev)
    Y = torch.empty(M * 65541, dtype=torch.float32, device=dev)
    hout = torch.empty(M, d, dtype=BF16, device=dev)
    # row-major VALU GEMV (layout 1): exact rows per CU, plain [N][K] weights
    rms = {}

    def rowmajor(N, K):
        if (N, K) not in rms:
            rms[(N, K)] = [(torch.randn(N, K, device=dev) * 0.02).to(BF16) for _ in range(nl)]
        return rms[(N, K)]
    for name, N, K, epi, pro in [("rm qkv", 4096, d, 4, "norm"), ("rm qkv-embed", 4096, d, 4, "embed"),
                                 ("rm o", d, q, 0, "direct"), ("rm o rows", d, q, 0, "rows"),
                                 ("rm cross_q", q, d, 4, "norm"), ("rm gate_up", 2 * f, d, 3, "norm"),
                                 ("rm down", d, f, 0, "direct"), ("rm head1", d, d, 2, "norm")]:
        wl = rowmajor(N, K)
        arr = (C.c_void_p * nl)(*[p.data_ptr() for p in wl])
        a = _lib.GemvArgs()
        a.layout = 1
        a.M, a.K, a.N, a.epi, a.pro, a.nw = M, K, N, epi, PRO[pro], 4
        a.Y, a.ldy, a.ldx, a.X, a.v, a.h_in = Y.data_ptr(), (N // 2 if epi == 3 else N), f, X.data_ptr(), \
            v.data_ptr(), h.data_ptr()
        a.ids, a.table, a.scale, a.eps = ids.data_ptr(), table.data_ptr(), 48.0, 1e-6
        a.post_w, a.pre_w, a.bias, a.h_out = nw_[0].data_ptr(), nw_[1].data_ptr(), bias.data_ptr(), hout.data_ptr()
        us = C.c_float()
        rc = L.t5g_time_gemv(C.byref(a), arr, nl, 4 * nl, st, C.byref(us))
        print(f"{name:14s} pro={pro:6s}: " + (f"rc={rc}" if rc else
              f"{us.value:7.2f} us  {N * K * 2 / us.value / 1e3:7.1f} GB/s"), flush=True)
    rms.clear()
    # split-K decomposition on the same kernel (fp32 slabs, like the unfused chain)
    for name, N, K, epi, pro, splits in [("qkv s2", 4096, d, 4, "rows", 2), ("qkv s4", 4096, d, 4, "rows", 4),
                                         ("o s4", d, q, 4, "rows", 4), ("o s2", d, q, 4, "rows", 2),
                                         ("gate_up rows", 2 * f, d, 3, "rows", 1),
                                         ("down s8", d, f, 4, "rows", 8), ("down s4", d, f, 4, "rows", 4),
                                         ("down s8 dir", d, f, 4, "direct", 8), ("down s16 dir", d, f, 4, "direct", 16)]:
        wl = packed(N, K)
        arr = (C.c_void_p * nl)(*[p.data_ptr() for p in wl])
        for nw, un in [(4, 8), (4, 16), (8, 8)]:
            a = _lib.GemvArgs()
            a.un, a.max_grid, a.splits = un, 0, splits
            a.M, a.K, a.N, a.epi, a.pro, a.nw = M, K, N, epi, PRO[pro], nw
            a.Y, a.ldy, a.ldx, a.X = Y.data_ptr(), (N // 2 if epi == 3 else N), f, X.data_ptr()
            us = C.c_float()
            rc = L.t5g_time_gemv(C.byref(a), arr, nl, 4 * nl, st, C.byref(us))
            if rc:
                print(f"{name:14s} nw={nw:2d} un={un:2d}: rc={rc}")
                continue
            print(f"{name:14s} nw={nw:2d} un={un:2d}: {us.value:7.2f} us  {N * K * 2 / us.value / 1e3:7.1f} GB/s",
                  flush=True)
    shapes = [  # name, N, K, epi, pro, nw list
        ("qkv", 4096, d, 4, "norm", [4, 8]), ("qkv-embed", 4096, d, 4, "embed", [8]),
        ("o", d, q, 0, "rows", [4, 8, 16]), ("o-direct", d, q, 0, "direct", [8, 16]),
        ("cross_q", q, d, 4, "norm", [4, 8]), ("gate_up", 2 * f, d, 3, "norm", [4, 8]),
("down", d, f, 0, "direct", [8, 16]),
        ("head1", d, d, 2, "norm", [4, 8]),
    ]
    for name, N, K, epi, pro, nws in shapes:
        wl = packed(N, K)
        arr = (C.c_void_p * nl)(*[p.data_ptr() for p in wl])
        for nw, un, mg in [(nw, un, mg) for nw in nws for un in (8, 16) for mg in (0, 100000)]:
            a = _lib.GemvArgs()
            a.un, a.max_grid = un, mg
            a.M, a.K, a.N, a.epi, a.pro, a.nw = M, K, N, epi, PRO[pro], nw
            a.Y, a.ldy, a.ldx, a.X, a.v, a.h_in = Y.data_ptr(), (N // 2 if epi == 3 else N), f, X.data_ptr(), \
                v.data_ptr(), h.data_ptr()
            a.ids, a.table, a.scale, a.eps = ids.data_ptr(), table.data_ptr(), 48.0, 1e-6
            a.post_w, a.pre_w, a.bias, a.h_out = nw_[0].data_ptr(), nw_[1].data_ptr(), bias.data_ptr(), \
                hout.data_ptr()
            us = C.c_float()
            rc = L.t5g_time_gemv(C.byref(a), arr, nl, 4 * nl, st, C.byref(us))
            if rc:
                print(f"{name:14s} pro={pro:6s} nw={nw:2d} un={un:2d} grid={'cu' if mg == 0 else 'all'}: rc={rc}")
                continue
            wbytes = N * K * 2
            print(f"{name:14s} pro={pro:6s} nw={nw:2d} un={un:2d} grid={'cu ' if mg == 0 else 'all'}: "
                  f"{us.value:7.2f} us  {wbytes / us.value / 1e3:7.1f} GB/s", flush=True)
    # the unfused chain for reference: split-K GEMM launches
    for name, N, K, epi, splits in [("old qkv s2", 4096, d, 4, 2), ("old o s4", d, q, 4, 4),
                                    ("old gate_up", 2 * f, d, 3, 1), ("old down s8", d, f, 4, 8)]:
        wl = packed(N, K)
        arr = (C.c_void_p * nl)(*[p.data_ptr() for p in wl])
        us = C.c_float()
        _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), f, M, arr, nl, N, K, splits, C.c_void_p(Y.data_ptr()),
                                   N // 2 if epi == 3 else N, epi, 4 * nl, st, C.byref(us)), "time_gemm")
        print(f"{name:14s}                : {us.value:7.2f} us  {N * K * 2 / us.value / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:]))
