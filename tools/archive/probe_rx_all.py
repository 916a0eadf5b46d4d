"""Probe: register-X GEMV with every unit's weight batch requested up front (un = -1) vs
one unit ahead, for the decode shapes it runs (gate/up, down slices, o projection) at 8
rows; HBM-cold (rotating over the 26 layers). Also bitwise equality of the outputs."""
import ctypes as C, json, os, sys
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import t5gemma_tts_amd  # noqa
from t5gemma_tts_amd import _lib
from t5gemma_tts_amd.config import config_2b2b
from t5gemma_tts_amd.engine import T5GemmaTTSEngine
from t5gemma_tts_amd.weights import synthetic_weights
cfg = config_2b2b()
dev = torch.device("cuda:0")
sd = synthetic_weights(cfg, seed=1234, device="cuda:0")
eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=8, max_text=64, max_audio=1024, max_gen=800)
L = _lib.lib()
st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
res = {}
shapes = {"gate_up": ("gate_up", 18432, 2304, 3, 1, 12), "down": ("down", 2304, 9216, 4, 8, 12),
          "o": ("o", 2304, 2048, 4, 4, 8), "cross_o": ("cross_o", 2304, 2048, 4, 4, 8)}
for M in (8, 1, 32):
    for name, (fld, N, K, epi, splits, nw) in shapes.items():
        X = torch.randn(M, K, device=dev).to(torch.bfloat16)
        outs = {}
        for un in (8, -1):
            a = _lib.GemvArgs()
            a.M, a.K, a.N, a.epi, a.pro, a.nw, a.un = M, K, N, epi, 0, nw, un
            ny = N // 2 if epi == 3 else N
            Y = torch.zeros(splits, M, ny, dtype=torch.float32 if epi == 4 else torch.bfloat16, device=dev)
            a.X, a.ldx, a.Y, a.ldy, a.splits, a.layout, a.max_grid = X.data_ptr(), K, Y.data_ptr(), ny, splits, 1, 0
            ws = [getattr(lw, fld) for lw in eng._dec]
            arr = (C.c_void_p * len(ws))(*ws)
            us = C.c_float()
            a.W = ws[0]
            _lib.check(L.t5g_gemv(C.byref(a), st), "gemv")
            torch.cuda.synchronize()
            outs[un] = Y.clone()
            _lib.check(L.t5g_time_gemv(C.byref(a), arr, len(ws), 208, st, C.byref(us)), "time")
            res[f"{name}_M{M}_un{un}"] = round(us.value, 2)
        res[f"{name}_M{M}_bitwise"] = bool(torch.equal(outs[8].view(torch.int32) if epi == 4 else outs[8].view(torch.int16),
                                                      outs[-1].view(torch.int32) if epi == 4 else outs[-1].view(torch.int16)))
print(json.dumps(res, indent=0))
json.dump(res, open(os.path.join(REPO, "gpurun_out", "r3_probe_rx_all.json"), "w"))
