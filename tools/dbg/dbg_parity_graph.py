"""Diagnostic: parity-mode generate() with graph replay vs direct launches vs the CPU oracle
(teacher forced) on golden_tiny cases; prints the first step whose logits leave the oracle."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import t5gemma_tts_amd  # noqa: E402,F401
from test_gpu_parity import _engine, _load, _oparams, _params  # noqa: E402
from t5gemma_tts_amd.config import named_config  # noqa: E402
from t5gemma_tts_amd.engine import Utterance  # noqa: E402
from t5gemma_tts_amd.weights import synthetic_weights  # noqa: E402
from oracle.t5g_oracle import T5GemmaTTSOracle  # noqa: E402

meta, arrs = _load("golden_tiny")
cfg = named_config(meta["config"], **meta["config_kw"])
sd = synthetic_weights(cfg, meta["weight_seed"])
eng = _engine(cfg, sd, max_batch=8, max_text=64, max_audio=256, max_gen=200)
for ci, c in enumerate(meta["cases"][:4]):
    u = Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])
    outs = {}
    for g in (True, False):
        outs[g] = eng.generate([u], _params(c), seeds=[c["seed"]], parity=True, record_logits=True, use_graph=g)
    orc = T5GemmaTTSOracle(cfg, sd)
    ctx = orc.prepare(u.x, u.y, u.tgt_y_len)
    toks = outs[True]["gen"][0].tolist()
    print(f"case {ci}: tokens graph {toks[:8]} direct {outs[False]['gen'][0].tolist()[:8]} ref {c['gen'][:8]}")
    for t, tok in enumerate(toks):
        lo = orc.step_logits(ctx)
        lg = outs[True]["logits"][t][0].cpu()
        ld = outs[False]["logits"][t][0].cpu() if t < len(outs[False]["logits"]) else None
        e_g = (lg.float() - lo.float()).abs().max().item()
        e_d = (ld.float() - lo.float()).abs().max().item() if ld is not None else -1
        if e_g > 1e-3 or e_d > 1e-3 or t < 2:
            print(f"  step {t}: graph err {e_g:.4f} direct err {e_d:.4f} graph==direct "
                  f"{ld is not None and torch.equal(lg, ld)} tok {tok}")
        if e_g > 1e-3:
            break
        ctx["state"].cur_num_gen += 1
        ctx["state"].current_length += 1
        if tok == cfg.eog_inference:
            break
        orc.advance(ctx, tok)
