"""Localise golden_longprompt4k's 1-ulp decode steps on the CPU.

Runs the REFERENCE (tests/golden/make_golden.py's import) on the golden's case here, wraps
torch's scaled_dot_product_attention, and for the decoder self-attention calls of the first
decode steps records what aten receives (q / k shapes, mask shape + all-true, is_causal,
enable_gqa) and whether ``oracle.cpu_order.sdpa`` on the same inputs returns the same bits.
Run here only (imports /root/reference):
    python tools/cpu_order/diag_window_sdpa.py [--steps 4] > profiles/r05_diag_window_sdpa.jsonl
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="golden_longprompt4k")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--all", action="store_true", help="check every self-attention call, not only mismatches")
    ap.add_argument("--prefill-layers", type=int, default=0, help="also check the first N decoder prefill calls")
    ap.add_argument("--prefill-rows", type=int, default=16, help="... over their last rows (whole q blocks)")
    a = ap.parse_args()
    import make_golden as MG
    from oracle import cpu_order as CO
    from t5gemma_tts_amd.config import named_config

    meta = json.load(open(os.path.join(REPO, "tests", "golden", a.name + ".json")))
    torch.set_num_threads(meta["threads"])
    cfg = named_config(meta["config"], **meta["config_kw"])
    RT, _ = MG._import_reference()
    orig = F.scaled_dot_product_attention
    state = {"call": 0, "prefill": 0}
    ncalls_per_pass = 2 * cfg.backbone.num_decoder_layers   # self + cross per layer
    recs = []

    def wrapped(q, k, v, attn_mask=None, dropout_p=0.0, is_causal=False, scale=None, enable_gqa=False, **kw):
        o = orig(q, k, v, attn_mask=attn_mask, dropout_p=dropout_p, is_causal=is_causal, scale=scale,
                 enable_gqa=enable_gqa, **kw)
        Tq = q.shape[2]
        if Tq > 64 and Tq == k.shape[2] and state["prefill"] < a.prefill_layers:
            # decoder prefill self-attention (the first layers): the q blocks from row_from on
            li = state["prefill"]
            state["prefill"] += 1
            H = q.shape[1]
            kk, vv = k, v
            if enable_gqa and k.shape[1] != H:
                kk = k.repeat_interleave(H // k.shape[1], 1)
                vv = v.repeat_interleave(H // v.shape[1], 1)
            mk = None if attn_mask is None else attn_mask.reshape(attn_mask.shape[-2], attn_mask.shape[-1])
            r0 = max(0, Tq - a.prefill_rows)
            got = CO.sdpa(q[0], kk[0], vv[0], scale, is_causal=is_causal, mask=mk, Hq=H, row_from=r0)
            qs = CO.E.qsplit(Tq)
            rb = (r0 // qs) * qs
            diff = got[:, rb:].view(torch.int16) != o[0][:, rb:].view(torch.int16)
            bad_rows = torch.nonzero(diff.any(-1).any(0)).view(-1) + rb
            print(json.dumps({"prefill_layer": li, "Tq": Tq, "gqa": bool(enable_gqa), "is_causal": bool(is_causal),
                              "mask": None if attn_mask is None else [list(attn_mask.shape), str(attn_mask.dtype)],
                              "rows_checked": [rb, Tq], "ndiff": int(diff.sum()),
                              "bad_rows": bad_rows[:32].tolist()}), flush=True)
        if Tq == 1 and k.shape[2] > 64:   # decoder self-attention decode calls
            step = state["call"] // (cfg.backbone.num_decoder_layers)
            layer = state["call"] % cfg.backbone.num_decoder_layers
            state["call"] += 1
            if step < a.steps:
                H = q.shape[1]
                kk, vv = k, v
                if enable_gqa and k.shape[1] != H:
                    kk = k.repeat_interleave(H // k.shape[1], 1)
                    vv = v.repeat_interleave(H // v.shape[1], 1)
                mk = None
                if attn_mask is not None:
                    mk = attn_mask.reshape(attn_mask.shape[-2], attn_mask.shape[-1])
                    if mk.dtype != torch.bool:
                        mk = mk == 0
                got = CO.sdpa(q[0], kk[0], vv[0], scale, is_causal=is_causal, mask=mk, Hq=H)
                ref = o[0]
                diff = (got.view(torch.int16) != ref.view(torch.int16))
                rec = {"step": step, "layer": layer, "Tk": int(k.shape[2]), "k_heads": int(k.shape[1]),
                       "gqa": bool(enable_gqa), "is_causal": bool(is_causal),
                       "mask": None if attn_mask is None else {
                           "shape": list(attn_mask.shape), "dtype": str(attn_mask.dtype),
                           "all_true": bool((attn_mask if attn_mask.dtype == torch.bool else attn_mask == 0).all())},
                       "k_contig": bool(k.is_contiguous()), "k_stride": list(k.stride()),
                       "ndiff": int(diff.sum())}
                if rec["ndiff"] or a.all:
                    print(json.dumps(rec), flush=True)
                recs.append(rec)
        return o

    F.scaled_dot_product_attention = wrapped
    torch.nn.functional.scaled_dot_product_attention = wrapped
    c = meta["cases"][0]
    with tempfile.TemporaryDirectory(dir=os.environ.get("GOLDEN_TMP", "/tmp")) as td:
        m, _ = MG.build_reference_model(RT, cfg, meta["weight_seed"], td, lowmem=True)
        res, gen, logs, dt = MG.run_case(RT, m, cfg, c)
    print(json.dumps({"summary": True, "tokens_equal": gen == c["gen"], "calls": len(recs),
                      "mismatching_calls": [(r["step"], r["layer"]) for r in recs if r["ndiff"]]}), flush=True)


if __name__ == "__main__":
    main()
