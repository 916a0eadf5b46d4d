"""Drive the fused decode launch (csrc/fused.hip; at M = 8 the fused_block_kernel) at C3 shape
(M = 8, T_x 60, 2b-2b widths) over
the 26 decoder layers' weights (3.3 GB, beyond the 256 MiB Infinity Cache), as bench.py's
roofline leg does, so rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE can count its HBM bytes per
launch (separate passes, tools/gpu_r3_pmc.sh). GPU only."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402


def main():
    self_stage = "--self" in sys.argv   # the launch with the self attention inside (stage S)
    from t5gemma_tts_amd.config import config_2b2b
    from t5gemma_tts_amd.engine import T5GemmaTTSEngine
    from t5gemma_tts_amd.weights import synthetic_weights
    L = _lib.lib()
    cfg = config_2b2b()
    B = 8
    sd = synthetic_weights(cfg, seed=1234, device="cuda:0")
    # --self: caches filled to the C3 bench rows' final length (903 keys: the length bench.py's
    # roofline leg times the launch at), the generate on the launches without S (another kernel
    # instantiation), so the PMC rows of fused_block_kernel<true> are the timed launches only
    n_gen = 751 if self_stage else 8
    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=B, max_text=64, max_audio=152 + n_gen + 16,
                           max_gen=n_gen + 16)
    if self_stage:
        eng.set_attn_in_block(False)
    del sd
    # one short C3-shaped generate (T_x 60) so the engine's rows, text lengths and cross K / V
    # are those of the bench workload
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    import numpy as np
    rng = np.random.default_rng(0)
    utts = [Utterance(x=rng.integers(3, 4000, size=60).tolist(),
                      y=rng.integers(0, 65536, size=150).tolist() + [cfg.y_sep_token], tgt_y_len=151 + n_gen)
            for _ in range(B)]
    eng.generate(utts, SamplingParams(top_k=30, top_p=0.9, temperature=0.8), seeds=list(range(B)))
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    us = C.c_float()
    if self_stage:
        eng.set_attn_in_block(True)
        keys = C.c_float()
        _lib.check(L.t5g_time_decode_layer(eng.h, B, 52, st, C.byref(us), C.byref(keys)), "time_decode_layer")
        alg = _lib.fused_block_bytes(B, 60, self_keys=keys.value)
        print(f"keys per kv head (rows summed, layer mean) {keys.value:.1f}", flush=True)
    else:
        _lib.check(L.t5g_time_decode_mlp(eng.h, B, 52, st, C.byref(us)), "time_decode_mlp")
        alg = _lib.fused_block_bytes(B, 60)
    print(f"fused_block avg {us.value:.2f} us/launch, algorithmic {alg} B -> {alg / us.value / 1e3:.1f} GB/s", flush=True)
    if len(sys.argv) > 2 and self_stage:
        import json
        json.dump({"algorithmic": alg, "keys": keys.value, "avg_us": us.value}, open(sys.argv[-1], "w"))


if __name__ == "__main__":
    main()
