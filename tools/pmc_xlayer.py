"""Drive parity mode's persistent layer launch (csrc/xlayer.hip) at the bench's C3 shape (8
rows, T_x 60, 2b-2b widths) over the 26 decoder layers' weights (4.5 GB, beyond the 256 MiB
Infinity Cache), as bench.py's parity roofline leg does, so rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE can count its HBM bytes per launch (separate passes, tools/gpu_r5_pmc.sh). GPU only."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402


def main():
    from t5gemma_tts_amd.config import config_2b2b
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    L = _lib.lib()
    cfg = config_2b2b()
    B = 8
    sd = synthetic_weights(cfg, seed=1234, device="cuda:0")
    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=B, max_text=128, max_audio=400, max_gen=64)
    del sd
    rng = np.random.default_rng(0)
    utts = [Utterance(x=rng.integers(3, 4000, size=60).tolist(),
                      y=rng.integers(0, 65536, size=151).tolist() + [cfg.y_sep_token], tgt_y_len=152 + 8)
            for _ in range(B)]
    eng.generate(utts, SamplingParams(top_k=30, top_p=0.9, temperature=0.8), seeds=list(range(B)), parity=True)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    us = C.c_float()
    _lib.check(L.t5g_time_xlayer(eng.h, B, 52, st, C.byref(us)), "time_xlayer")
    alg = _lib.xlayer_bytes(B, cfg.backbone, 60, cfg.backbone.num_decoder_layers)
    print(f"xlayer avg {us.value:.2f} us/launch, algorithmic {alg:.0f} B -> {alg / us.value / 1e3:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
