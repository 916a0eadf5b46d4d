"""The parity layer launch's Infinity Cache warm-up (csrc/xlayer.hip, t5g_engine_set_xl_warm)
at C3 (8 rows): xlayer_kernel timed with HIP events over the 26 layers (t5g_time_xlayer) and
one parity generate, warm-up off / on; tokens must be equal (loads only). GPU only."""
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
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3)
    L = _lib.lib()
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    out, toks = {}, {}
    eng.generate(utts, p, seeds=list(range(B)), chunk=64, parity=True)   # exact images, graphs
    for rep in range(2):
        for on in (False, True):
            eng.set_xl_warm(on)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = eng.generate(utts, p, seeds=list(range(B)), chunk=64, parity=True)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            toks[on] = [x.tolist() for x in r["gen"]]
            us = C.c_float()
            _lib.check(L.t5g_time_xlayer(eng.h, B, 208, st, C.byref(us)), "time_xlayer")
            name = f"rep{rep}_warm{int(on)}"
            out[name] = {"xlayer_us": round(us.value, 2), "generate_s": round(wall, 3),
                         "tok_per_s": round(sum(len(t) for t in toks[on]) / wall, 1)}
            print(name, out[name], flush=True)
    out["same_tokens"] = toks[True] == toks[False]
    print(json.dumps(out))
    assert out["same_tokens"]


if __name__ == "__main__":
    main()
