"""Which reference op does the order restatement (oracle/cpu_order.py) get wrong on a golden
case? Runs the torch-CPU oracle (bitwise equal to the reference on this host) over a golden
case's encoder + prefill and, at every Linear / RMSNorm / SDPA call, recomputes the op with
the cpu_order restatement on the same inputs and reports differing elements. Debug tool
(CPU only, slow: numpy order emulation at prefill sizes).

usage: python tools/dbg/check_order_ops.py golden_longprompt [--skip-encoder] [--layers N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import t5gemma_tts_amd  # noqa: E402,F401
from oracle import cpu_order as CO  # noqa: E402
from oracle import t5g_oracle as O  # noqa: E402
from t5gemma_tts_amd.config import named_config  # noqa: E402
from t5gemma_tts_amd.weights import synthetic_weights  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("golden")
ap.add_argument("--skip-encoder", action="store_true")
ap.add_argument("--only", default="", help="comma list of op kinds to check: lin,rms,attn")
args = ap.parse_args()
kinds = set(args.only.split(",")) if args.only else {"lin", "rms", "attn"}

meta = json.load(open(os.path.join(REPO, "tests", "golden", args.golden + ".json")))
cfg = named_config(meta["config"], **meta["config_kw"])
sd = synthetic_weights(cfg, meta["weight_seed"])
orc = O.T5GemmaTTSOracle(cfg, sd)
case = meta["cases"][0]
phase = {"name": "encoder"}
n_bad = {"n": 0}


def report(tag, shape, y, y2, extra=""):
    a = y.contiguous().view(torch.int16)
    b = y2.contiguous().view(torch.int16)
    bad = int((a != b).sum())
    print(json.dumps({"phase": phase["name"], "op": tag, "shape": list(shape), "diff": bad, **({"x": extra} if extra else {})}),
          flush=True)
    if bad:
        n_bad["n"] += 1


orig_lin = O.T5GemmaTTSOracle._lin
orig_rms = O.rms_norm
orig_attn = O.attention


def lin(self, x, name, bias=None):
    y = orig_lin(self, x, name, bias)
    if "lin" in kinds and not (args.skip_encoder and phase["name"] == "encoder"):
        M = x.reshape(-1, x.shape[-1]).shape[0]
        w = self.w[name]
        kb = CO.ksplit(w.shape[0], w.shape[1], M)
        t = time.time()
        y2 = CO.linear(x, w, self.w[bias] if bias else None)
        report("lin " + name.replace("backbone.model.", ""), (M,) + tuple(w.shape), y, y2, f"kb={kb} {time.time() - t:.0f}s")
    return y


def rms(x, w, eps):
    y = orig_rms(x, w, eps)
    if "rms" in kinds and not (args.skip_encoder and phase["name"] == "encoder"):
        report("rms", x.shape, y, CO.rms_norm(x, w, eps))
    return y


def attn(q, k, v, *, scale, softcap, n_rep, mask, is_causal, impl):
    y = orig_attn(q, k, v, scale=scale, softcap=softcap, n_rep=n_rep, mask=mask, is_causal=is_causal, impl=impl)
    if "attn" in kinds and not (args.skip_encoder and phase["name"] == "encoder"):
        B, H, Tq, D = q.shape
        kk = k.repeat_interleave(n_rep, 1) if n_rep > 1 else k
        vv = v.repeat_interleave(n_rep, 1) if n_rep > 1 else v
        mk = None if mask is None else mask.view(mask.shape[-2], mask.shape[-1])
        o = CO.sdpa(q[0], kk[0], vv[0], scale, is_causal=is_causal, mask=mk, Hq=H)[None]
        y2 = o.transpose(1, 2).reshape(B, Tq, H * D)
        report("attn", (Tq, kk.shape[2]), y, y2, f"causal={is_causal} mask={mask is not None}")
    return y


O.T5GemmaTTSOracle._lin = lin
O.rms_norm = rms
O.attention = attn

orig_decode = O.T5GemmaTTSOracle.decode


def decode(self, *a, **kw):
    phase["name"] = "prefill" if phase["name"] == "encoder" else "decode"
    return orig_decode(self, *a, **kw)


O.T5GemmaTTSOracle.decode = decode
ctx = orc.prepare(case["x"], case["y"], case["tgt"])
phase["name"] = "head"
lg = orc.step_logits(ctx)
import hashlib  # noqa: E402
sha = hashlib.sha256(lg.view(torch.int16).numpy().tobytes()).hexdigest()[:16]
print(json.dumps({"step0_logit_sha": sha, "golden": case["logit_sha"][0], "ops_differing": n_bad["n"]}), flush=True)
