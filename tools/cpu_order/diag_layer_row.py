"""Which op of one decoder layer differs between the reference and the restatement at one
prefill row? (golden_longprompt4k: the GPU's layer-25 K / V differ from the reference's at
position 2 765 only -- tools/dbg/dbg_window_kv.py -- so layer 24's ops at that row, or
layer 25's input norm / K / V projections, hold a rule the restatement misses.)

Runs the REFERENCE here (imports /root/reference through tests/golden/make_golden.py) with
forward hooks on the prefill call of decoder layer --layer and the input norm / k / v
projections of layer + 1, and checks ``oracle.cpu_order``'s Linear (the measured K split at
M = prefill length) and RMSNorm on the captured inputs of row --row against the captured
outputs; the self / cross attention of that row through ``cpu_order.sdpa``.
    python tools/cpu_order/diag_layer_row.py [--layer 24] [--row 2765]
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


def bits(t):
    return t.contiguous().view(torch.int16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="golden_longprompt4k")
    ap.add_argument("--layer", type=int, default=24)
    ap.add_argument("--row", type=int, default=2765)
    ap.add_argument("--save", default="", help="torch.save the layer's self-attention inputs / output here")
    a = ap.parse_args()
    import make_golden as MG
    from oracle import cpu_order as CO
    from t5gemma_tts_amd.config import named_config
    meta = json.load(open(os.path.join(REPO, "tests", "golden", a.name + ".json")))
    torch.set_num_threads(meta["threads"])
    cfg = named_config(meta["config"], **meta["config_kw"])
    c = meta["cases"][0]
    T = len(c["y"]) + 1
    R = a.row
    RT, _ = MG._import_reference()
    cap = {}
    orig_sdpa = F.scaled_dot_product_attention
    state = {"self": 0}

    def sdpa(q, k, v, attn_mask=None, dropout_p=0.0, is_causal=False, scale=None, enable_gqa=False, **kw):
        o = orig_sdpa(q, k, v, attn_mask=attn_mask, dropout_p=dropout_p, is_causal=is_causal, scale=scale,
                      enable_gqa=enable_gqa, **kw)
        if q.shape[2] == T:
            if k.shape[2] == T:
                li = state["self"]
                state["self"] += 1
                tag = "self"
            else:
                li = state.get("cross", 0)
                state["cross"] = li + 1
                tag = "cross"
            if li == a.layer:
                cap[tag + "_sdpa"] = (q, k, v, attn_mask, is_causal, scale, enable_gqa, o)
        return o

    F.scaled_dot_product_attention = sdpa
    torch.nn.functional.scaled_dot_product_attention = sdpa
    with tempfile.TemporaryDirectory(dir=os.environ.get("GOLDEN_TMP", "/tmp")) as td:
        m, _ = MG.build_reference_model(RT, cfg, meta["weight_seed"], td, lowmem=True)
        layers = None
        for name, mod in m.named_modules():
            if name.endswith("decoder.layers"):
                layers = mod
        assert layers is not None
        hooks = []

        def hook(tag):
            def f(mod, inp, out):
                x = inp[0]
                if x.dim() == 3 and x.shape[1] == T:
                    cap[tag] = (x[0, R].clone(), out[0, R].clone(), mod)
            return f

        for li in (a.layer, a.layer + 1):
            for name, mod in layers[li].named_modules():
                if isinstance(mod, torch.nn.Linear) or "norm" in type(mod).__name__.lower():
                    hooks.append(mod.register_forward_hook(hook(f"L{li}.{name}")))
        res, gen, logs, dt = MG.run_case(RT, m, cfg, c)
        for h in hooks:
            h.remove()
        out = []
        kb_of = {}
        for tag, val in sorted(cap.items()):
            if tag.endswith("_sdpa"):
                continue
            x, y, mod = val
            if isinstance(mod, torch.nn.Linear):
                N, K = mod.weight.shape
                kb = CO.ksplit(N, K, T)
                kb_of[tag] = kb
                got = CO.linear(x[None], mod.weight.detach(), None if mod.bias is None else mod.bias.detach(), kb=kb)[0]
            else:
                got = CO.rms_norm(x[None], mod.weight.detach(), float(mod.eps))[0]
            nd = int((bits(got) != bits(y)).sum())
            r = {"op": tag, "kind": type(mod).__name__, "ndiff": nd}
            if isinstance(mod, torch.nn.Linear):
                r["kb"] = kb_of[tag]
                if nd:
                    # which other split lengths reproduce the reference at this row?
                    K = mod.weight.shape[1]
                    r["kb_matching"] = [k for k in range(32, K + 1, 32) if K % k == 0 and int(
                        (bits(CO.linear(x[None], mod.weight.detach(), None, kb=k)[0]) != bits(y)).sum()) == 0]
            out.append(r)
            print(json.dumps(r), flush=True)
        if a.save and "self_sdpa" in cap:
            q, k, v, mask, is_causal, scale, gqa, o = cap["self_sdpa"]
            torch.save({"q": q, "k": k, "v": v, "mask": mask, "is_causal": is_causal, "scale": scale, "gqa": gqa,
                        "o": o}, a.save)
        for tag in ("self_sdpa", "cross_sdpa"):
            if tag not in cap:
                continue
            q, k, v, mask, is_causal, scale, gqa, o = cap[tag]
            H = q.shape[1]
            if k.shape[1] != H:
                k = k.repeat_interleave(H // k.shape[1], 1)
                v = v.repeat_interleave(H // v.shape[1], 1)
            mk = None if mask is None else mask.reshape(mask.shape[-2], mask.shape[-1])
            got = CO.sdpa(q[0], k[0], v[0], scale, is_causal=is_causal, mask=mk, Hq=H, row_from=R, row_to=R + 1)
            nd = int((bits(got[:, R]) != bits(o[0][:, R])).sum())
            r = {"op": f"L{a.layer}.{tag}", "Tk": int(k.shape[2]), "mask": mask is not None, "ndiff": nd}
            out.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
