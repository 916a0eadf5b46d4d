"""golden_longprompt4k: where do the GPU's caches first differ from the reference's?

``ref`` (here, imports /root/reference through tests/golden/make_golden.py): runs the
reference's inference_tts on the golden case, captures every decoder self-attention K / V
handed to the cache (DynamicCache.update: the 4 101-token prefill, then one position per
decode step) and writes per-(layer, K/V, kv head, position) hashes to
tools/dbg/kvref_<golden>.npy (diagnostic data, not committed).
``gpu`` (the box): runs the engine in parity mode on the same case, hashes its caches over
the same positions and prints, per layer, how many (head, position) rows differ in the
prefill part and in each decode step's appended row.
    python tools/dbg/dbg_window_kv.py ref|gpu [golden_longprompt4k]
"""
import ctypes as C
import json
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
mode = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "golden_longprompt4k"
meta = json.load(open(os.path.join(REPO, "tests", "golden", name + ".json")))
c = meta["cases"][0]
T = len(c["y"]) + 1
S = len(c["gen"]) - 1            # decode passes (no pass after the last token)
ref_path = os.path.join(REPO, "tools", "dbg", f"kvref_{name}.npy")


def hashes(kv):   # kv [hk, n, D] bf16 -> [hk, n] int64
    D = kv.shape[-1]
    v = kv.contiguous().view(torch.int16).to(torch.int64) & 0xFFFF
    w = torch.arange(1, D + 1, dtype=torch.int64, device=v.device) * 2654435761
    return (v * w).sum(-1)


if mode == "ref":
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import make_golden as MG
    from transformers import cache_utils
    from t5gemma_tts_amd.config import named_config
    torch.set_num_threads(meta["threads"])
    cfg = named_config(meta["config"], **meta["config_kw"])
    RT, _ = MG._import_reference()
    got = {}
    orig = cache_utils.DynamicCache.update

    def upd(self, key_states, value_states, layer_idx, *a, **k):
        if key_states.shape[-2] != len(c["x"]):   # self attention (cross K/V hold T_x rows)
            got.setdefault(layer_idx, []).append((hashes(key_states[0]), hashes(value_states[0])))
        return orig(self, key_states, value_states, layer_idx, *a, **k)

    cache_utils.DynamicCache.update = upd
    with tempfile.TemporaryDirectory(dir=os.environ.get("GOLDEN_TMP", "/tmp")) as td:
        m, _ = MG.build_reference_model(RT, cfg, meta["weight_seed"], td, lowmem=True)
        res, gen, logs, dt = MG.run_case(RT, m, cfg, c)
    assert gen == c["gen"], "reference run differs from the golden"
    nl = len(got)
    out = np.stack([np.stack([torch.cat([k for k, _ in got[l]], 1).numpy(), torch.cat([v for _, v in got[l]], 1).numpy()])
                    for l in range(nl)])
    np.save(ref_path, out)
    print("wrote", ref_path, out.shape)
else:
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    ref = np.load(ref_path)
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    bb = cfg.backbone
    nl, hk, D = bb.num_decoder_layers, bb.num_key_value_heads, bb.head_dim
    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=1, max_text=64, max_audio=T + S + 16,
                           max_gen=len(c["gen"]) + 8)
    p = SamplingParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                       stop_repetition=c["stop_repetition"])
    out = eng.generate([Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])], p, seeds=[c["seed"]], parity=True)
    print("tokens equal:", out["gen"][0].tolist() == c["gen"], flush=True)
    torch.cuda.synchronize()
    L = _lib.lib()
    hip = C.CDLL("libamdhip64.so")
    n = ref.shape[-1]
    rep = []
    for layer in range(nl):
        row = {"layer": layer, "sliding": bool(bb.layer_types("decoder")[layer] == "sliding_attention")}
        for which, key in enumerate(("k", "v")):
            hs, rs = C.c_int64(), C.c_int64()
            ptr = L.t5g_engine_cache_ptr(eng.h, layer, which, C.byref(hs), C.byref(rs))
            cap = hs.value // D
            buf = torch.empty(hk * cap * D, dtype=torch.bfloat16, device="cuda")
            torch.cuda.synchronize()
            assert hip.hipMemcpy(C.c_void_p(buf.data_ptr()), C.c_void_p(ptr), C.c_size_t(hk * cap * D * 2), 3) == 0
            g = hashes(buf.view(hk, cap, D)[:, :n]).cpu().numpy()
            bad = g != ref[layer, which]
            row[key + "_prefill_bad"] = int(bad[:, :T].sum())
            row[key + "_prefill_first"] = int(np.nonzero(bad[:, :T].any(0))[0][0]) if bad[:, :T].any() else None
            row[key + "_step_bad"] = [int(bad[:, T + s].sum()) for s in range(n - T)]
        rep.append(row)
        print(json.dumps(row), flush=True)
