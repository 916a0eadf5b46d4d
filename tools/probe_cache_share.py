"""Which bytes' Infinity Cache residency the persistent layer launches are sensitive to: the
fast path's fused_block_kernel (t5g_time_decode_layer) and the parity path's xlayer_kernel
(t5g_time_xlayer), timed over the 26 layers as in a decode step, and with
T5G_TIME_SHARE=chain (every launch reads layer 1's chain-stage weights -- o / cross q /
cross o / q|k|v -- and cross K / V, ~48 MB that then stay cached) or =gd (layer 1's gate/up
and down, 127 MB). Every launch keeps its own layer's hand-off counters. GPU only."""
import ctypes as C
import json
import os
import sys

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
    out = {}
    for parity in (False, True):
        eng.generate(utts, p, seeds=list(range(B)), chunk=64, parity=parity)
        for share in (None, "chain", "gd"):
            os.environ.pop("T5G_TIME_SHARE", None)
            if share:
                os.environ["T5G_TIME_SHARE"] = share
            us, keys = C.c_float(), C.c_float()
            if parity:
                _lib.check(L.t5g_time_xlayer(eng.h, B, 208, st, C.byref(us)), "time_xlayer")
            else:
                _lib.check(L.t5g_time_decode_layer(eng.h, B, 208, st, C.byref(us), C.byref(keys)), "time_layer")
            name = ("xlayer" if parity else "fused_block") + "_" + (share or "rotate")
            out[name] = round(us.value, 2)
            print(name, out[name], flush=True)
        eng.set_exact(False)
    os.environ.pop("T5G_TIME_SHARE", None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
