"""Where does a golden case's prefill first differ? Hashes of every (decoder layer, self K / V,
kv head, position) of the prompt part of the cache -- on the GPU engine in parity mode
(``gpu``: writes gpurun_out/cache_hash_<golden>.npy) and in the torch-CPU oracle (``cpu``:
compares with that file and prints the first differing layer / head / position).

usage: python tools/dbg/dbg_cache_hash.py gpu|cpu golden_longprompt
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd.config import named_config  # noqa: E402
from t5gemma_tts_amd.weights import synthetic_weights  # noqa: E402

mode, name = sys.argv[1], sys.argv[2]
meta = json.load(open(os.path.join(REPO, "tests", "golden", name + ".json")))
cfg = named_config(meta["config"], **meta["config_kw"])
sd = synthetic_weights(cfg, meta["weight_seed"])
c = meta["cases"][0]
T = len(c["y"]) + 1            # the prefill: empty token + prompt
bb = cfg.backbone
nl, hk, D = bb.num_decoder_layers, bb.num_key_value_heads, bb.head_dim
out_path = os.path.join(REPO, "gpurun_out", f"cache_hash_{name}.npy")


def hashes(kv):   # kv [hk, T, D] bf16 -> [hk, T] int64
    v = kv.contiguous().view(torch.int16).to(torch.int64) & 0xFFFF
    w = torch.arange(1, D + 1, dtype=torch.int64, device=v.device) * 2654435761
    return (v * w).sum(-1)


if mode == "gpu":
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=1, max_text=64, max_audio=1024, max_gen=760)
    p = SamplingParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                       stop_repetition=c["stop_repetition"])
    eng.generate([Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])], p, seeds=[c["seed"]], parity=True)
    torch.cuda.synchronize()
    L = _lib.lib()
    hip = C.CDLL("libamdhip64.so")
    res = np.zeros((nl, 2, hk, T), np.int64)
    for layer in range(nl):
        for which in range(2):
            hs, rs = C.c_int64(), C.c_int64()
            ptr = L.t5g_engine_cache_ptr(eng.h, layer, which, C.byref(hs), C.byref(rs))
            cap = hs.value // D
            buf = torch.empty(hk * cap * D, dtype=torch.bfloat16, device="cuda")
            torch.cuda.synchronize()
            # device-to-device copy of the row-0 cache block (hipMemcpyDeviceToDevice = 3)
            assert hip.hipMemcpy(C.c_void_p(buf.data_ptr()), C.c_void_p(ptr), C.c_size_t(hk * cap * D * 2), 3) == 0
            kv = buf.view(hk, cap, D)[:, :T]
            res[layer, which] = hashes(kv).cpu().numpy()
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    np.save(out_path, res)
    print("wrote", out_path, res.shape)
else:
    ref_path = os.path.join(REPO, "gpurun_out", f"cache_hash_{name}_oracle.npy")
    if os.path.exists(ref_path):
        ref_all = np.load(ref_path)
    else:
        from oracle import t5g_oracle as O
        orc = O.T5GemmaTTSOracle(cfg, sd)
        cache = orc.prepare(c["x"], c["y"], c["tgt"])["cache"]
        ref_all = np.stack([np.stack([hashes(cache[key][layer][0]).numpy() for key in ("k", "v")])
                            for layer in range(nl)])
        np.save(ref_path, ref_all)
    if not os.path.exists(out_path):
        print("oracle hashes saved; no GPU file yet")
        sys.exit(0)
    got = np.load(out_path)
    first = None
    for layer in range(nl):
        for which, key in enumerate(("k", "v")):
            bad = np.nonzero(got[layer, which] != ref_all[layer, which])
            n = len(bad[0])
            print(f"layer {layer} {key}: {n} / {hk * T} (head, pos) rows differ" +
                  (f", first head {bad[0][0]} pos {bad[1][0]}" if n else ""), flush=True)
            if n and first is None:
                first = (layer, key)
    print("first differing:", first)
