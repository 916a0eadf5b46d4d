"""How much of the token divergence comes from GEMM order vs RMSNorm order? Run the tiny
golden cases through the oracle with (a) GEMMs in fp64-then-bf16 (a different but valid
accumulation order), (b) RMSNorm sum of squares in fp64, (c) both; count token-exact cases."""
import json, os, sys
import numpy as np, torch
import torch.nn.functional as F
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import t5gemma_tts_amd  # noqa
import oracle.t5g_oracle as O
from t5gemma_tts_amd.config import named_config
from t5gemma_tts_amd.weights import synthetic_weights
torch.set_num_threads(8)
meta = json.load(open("/root/repo/tests/golden/golden_tiny.json"))
cfg = named_config(meta["config"], **meta["config_kw"]); sd = synthetic_weights(cfg, meta["weight_seed"])
orig_lin, orig_rms = O.T5GemmaTTSOracle._lin, O.rms_norm
def lin64(self, x, name, bias=None):
    w = self.w[name]; y = x.double() @ w.double().T
    if bias: y = y + self.w[bias].double()
    return y.to(torch.bfloat16) if not bias else (x.double() @ w.double().T).float().to(torch.bfloat16) + self.w[bias]
def rms64(x, w, eps):
    xf = x.float()
    ms = xf.double().pow(2).mean(-1, keepdim=True).float()
    out = xf * torch.rsqrt(ms + eps)
    return (out * (1.0 + w.float())).to(x.dtype)
def run(tag):
    orc = O.T5GemmaTTSOracle(cfg, sd)
    ex = 0
    for c in meta["cases"]:
        p = O.SamplerParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                            stop_repetition=c["stop_repetition"], silence_tokens=tuple(c["silence_tokens"]))
        r = orc.generate(c["x"], c["y"], c["tgt"], p, seed=c["seed"])
        ex += int(r["gen"].view(-1).tolist() == c["gen"])
    print(tag, "token-exact", ex, "/", len(meta["cases"]), flush=True)
run("reference-order")
O.rms_norm = rms64; run("rms fp64")
O.rms_norm = orig_rms; O.T5GemmaTTSOracle._lin = lin64; run("gemm fp64")
O.rms_norm = rms64; run("both fp64")
