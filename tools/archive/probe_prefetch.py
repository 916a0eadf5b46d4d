"""ARCHIVED (round 6): needs the removed t5g_engine_set_prefetch plumbing.

The Infinity Cache prefetch (csrc/prefetch.hip, t5g_engine_set_prefetch) at C3 (8 rows):
the persistent layer launches timed with HIP events over the 26 layers (fast path
t5g_time_decode_layer, parity t5g_time_xlayer) and the whole fast decode step
(t5g_time_decode_step), prefetch off / plain loads / nt loads, plus the tokens of one
generate in each mode (must be equal: the prefetch only loads). GPU only."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402
from t5gemma_tts_amd.config import config_2b2b  # noqa: E402
from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance  # noqa: E402
from t5gemma_tts_amd.weights import synthetic_weights  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    cfg = config_2b2b()
    sd = synthetic_weights(cfg, seed=1234, device=str(dev))
    B = 8
    eng = T5GemmaTTSEngine(cfg, sd, device=str(dev), max_batch=B, max_text=128, max_audio=151 + 1 + 760, max_gen=760)
    g = torch.Generator().manual_seed(5)
    utts = [Utterance(x=torch.randint(3, 1000, (60,), generator=g).tolist(),
                      y=torch.randint(0, 65536, (150,), generator=g).tolist() + [cfg.y_sep_token], tgt_y_len=500)
            for _ in range(B)]
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3, eos_disabled=True)
    L = _lib.lib()
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    out, toks = {}, {}
    modes = [int(m) for m in os.environ.get("PF_MODES", "0,1,2").split(",")]
    for parity in (False, True):
        for m in modes:
            eng.set_prefetch(m)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = eng.generate(utts, p, seeds=list(range(B)), chunk=64, parity=parity)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            toks[(parity, m)] = [x.tolist() for x in r["gen"]]
            us, keys, step = C.c_float(), C.c_float(), C.c_float()
            name = ("parity" if parity else "fast") + f"_pf{m}"
            if parity:
                _lib.check(L.t5g_time_xlayer(eng.h, B, 208, st, C.byref(us)), "time_xlayer")
                out[name] = {"xlayer_us": round(us.value, 2)}
            else:
                _lib.check(L.t5g_time_decode_layer(eng.h, B, 208, st, C.byref(us), C.byref(keys)), "time_layer")
                _lib.check(L.t5g_time_decode_step(eng.h, 20, st, C.byref(step)), "time_step")
                out[name] = {"layer_us": round(us.value, 2), "step_us": round(step.value, 1)}
            out[name]["generate_s"] = round(wall, 3)
            out[name]["tok_per_s"] = round(sum(len(t) for t in toks[(parity, m)]) / wall, 1)
            out[name]["same_tokens_as_off"] = toks[(parity, m)] == toks[(parity, modes[0])]
            print(name, out[name], flush=True)
        eng.set_exact(False)
    eng.set_prefetch(0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
