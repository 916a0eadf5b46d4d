"""golden_longprompt4k (a 4 101-token prefill past the 4 096-key sliding window) in parity
mode: per step, whether the logits row's sha matches the reference's and the largest
difference over the reference's top-64 logits (bf16 ulps of the value).
    python tools/diag_window.py > gpurun_out/diag_window.json"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def main():
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    name = sys.argv[1] if len(sys.argv) > 1 else "golden_longprompt4k"
    meta = json.load(open(os.path.join(GOLDEN, name + ".json")))
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    c = meta["cases"][0]
    p = SamplingParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                       stop_repetition=c["stop_repetition"])
    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=1, max_text=64,
                           max_audio=len(c["y"]) + len(c["gen"]) + 16, max_gen=len(c["gen"]) + 8)
    out = eng.generate([Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])], p, seeds=[c["seed"]], parity=True,
                       record_logits=True)
    rows = []
    for s, lg in enumerate(out["logits"][:len(c["gen"])]):
        bits = lg[0].cpu().view(torch.int16).numpy()
        sha = hashlib.sha256(bits.tobytes()).hexdigest()[:16]
        idx, ref = z["top_idx_0"][s], z["top_vals_0"][s]
        got = bits[idx]
        rows.append({"step": s, "sha_equal": sha == c["logit_sha"][s], "top64_bits_differ": int((got != ref).sum()),
                     "max_bit_delta": int(np.abs(got.astype(np.int32) - ref.astype(np.int32)).max())})
    print(json.dumps({"name": name, "tokens_equal": out["gen"][0].tolist() == c["gen"], "steps": rows}))


if __name__ == "__main__":
    main()
