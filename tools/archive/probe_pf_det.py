"""Probe: run-to-run determinism of the many-token GEMMs (LDS-staged gemm_pfl_kernel and the
register ring gemm_pf_kernel): each shape is launched 30 times on the same inputs, every
output compared bitwise with the first and with the other kernel's. GPU only."""
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
    for M in (480, 1216):
        for name, N, K, epi in [("qkv", 4096, 2304, 0), ("gate_up", 18432, 2304, 3), ("down", 2304, 9216, 0)]:
            g = torch.Generator(device="cpu").manual_seed(N + K + M)
            w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16).to(dev)
            p = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=torch.bfloat16, device=dev)
            _lib.check(L.t5g_pack_weight(C.c_void_p(w.data_ptr()), N, K, K, C.c_void_p(p.data_ptr()), st), "pack")
            X = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
            ldy = N // 2 if epi == 3 else N
            row = {"shape": f"{name}_{M}"}
            first = {}
            for tag, flag in (("lds", PREFILL), ("reg", PREFILL | PREFILL_REG)):
                diff_runs, diff_elems = 0, 0
                for it in range(30):
                    Y = torch.full((M, ldy), float("nan"), dtype=torch.bfloat16, device=dev)
                    _lib.check(L.t5g_gemm(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(p.data_ptr()), N, K, 1, None,
                                          C.c_void_p(Y.data_ptr()), ldy, epi | flag, st), "gemm")
                    torch.cuda.synchronize()
                    if it == 0:
                        first[tag] = Y.clone()
                        row[f"{tag}_nan"] = int(torch.isnan(Y.float()).sum())
                    else:
                        ne = int((Y.view(torch.int16) != first[tag].view(torch.int16)).sum())
                        diff_runs += ne > 0
                        diff_elems = max(diff_elems, ne)
                row[f"{tag}_runs_differing"] = diff_runs
                row[f"{tag}_max_elems_differing"] = diff_elems
            row["lds_vs_reg_elems_differing"] = int(
                (first["lds"].view(torch.int16) != first["reg"].view(torch.int16)).sum())
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
