"""Probe: decode GEMV time with weights warm in the Infinity Cache (same weights re-read)
vs cold (rotating over all 26 decoder layers), at 8 and 4 rows -- is a second chain's
re-read of a layer's weights (two half-batch chains in lockstep) cheaper than HBM?"""
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
d, f = 2304, 9216
st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
res = {}
for M in (8, 4):
    X = torch.randn(M, d, device=dev).to(torch.bfloat16)
    Y = torch.empty(M, f, dtype=torch.bfloat16, device=dev)
    ws = [lw.gate_up for lw in eng._dec]
    cold = _lib.time_gate_up(X.data_ptr(), d, M, ws, 2 * f, d, Y.data_ptr(), 208, st)
    warm1 = _lib.time_gate_up(X.data_ptr(), d, M, ws[:1], 2 * f, d, Y.data_ptr(), 200, st)
    warm2 = _lib.time_gate_up(X.data_ptr(), d, M, ws[:2], 2 * f, d, Y.data_ptr(), 200, st)   # 170 MB cycle
    warm3 = _lib.time_gate_up(X.data_ptr(), d, M, ws[:3], 2 * f, d, Y.data_ptr(), 201, st)   # 255 MB cycle
    res[M] = {"cold_26layers_us": round(cold, 2), "same_layer_us": round(warm1, 2), "2_layers_us": round(warm2, 2),
              "3_layers_us": round(warm3, 2)}
print(json.dumps(res))
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(REPO, "gpurun_out", "r3_probe_mall_reuse.json"), "w"))
