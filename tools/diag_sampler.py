"""Block timeline of the multi-block sampler (diagnostic library, T5G_LIB=.../libt5gtts_dbg.so):
per point, median time from the block's start; the merging (last) block's points 3-6."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402
from t5gemma_tts_amd.config import named_config  # noqa: E402
from t5gemma_tts_amd.engine import T5GemmaTTSEngine  # noqa: E402
from t5gemma_tts_amd.weights import synthetic_weights  # noqa: E402

B = 8
cfg = named_config("tiny")
cfg.audio_vocab_size = 65536
cfg.empty_token, cfg.eog, cfg.audio_pad_token, cfg.eos, cfg.y_sep_token = 65536, 65537, 65538, 65539, 65540
eng = T5GemmaTTSEngine(cfg, synthetic_weights(cfg, 3), max_batch=B, max_text=16, max_audio=4096, max_gen=4000)
L = eng.L
V = cfg.n_audio_tokens
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
lg = (torch.randn(B, V + 11, device="cuda") * 0.8).to(torch.bfloat16)
buf = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
L.t5g_dbg_set_sampler.argtypes = [C.c_void_p]
assert L.t5g_dbg_set_sampler(C.c_void_p(buf.data_ptr())) == 0
rows = (_lib.SamplerRow * B)(*[_lib.SamplerRow(top_k=30, top_p=0.9, temperature=0.8, eos_disabled=1, seed_lo=b + 1)
                              for b in range(B)])
sts = (_lib.SamplerState * B)(*[_lib.SamplerState(cur_num_gen=20, current_length=100, prompt_offset=1, target_total=-1,
                                                  est_total=4000, prev_token=-1, first_input_len=5) for _ in range(B)])
tk = (C.c_int32 * 1)()
_lib.check(L.t5g_sampler_setup(eng.h, B, rows, sts, tk, 0, tk, 0, None, 0, st), "setup")
for _ in range(5):
    L.t5g_sample_only(eng.h, B, C.c_void_p(lg.data_ptr()), V + 11, st)
torch.cuda.synchronize()
buf.zero_()
L.t5g_sample_only(eng.h, B, C.c_void_p(lg.data_ptr()), V + 11, st)
torch.cuda.synchronize()
t = buf.view(-1, 8).cpu().numpy()[:16 * B].astype(np.float64)
t0 = t[:, 0][t[:, 0] > 0].min()
for k in range(7):
    v = t[:, k]
    v = v[v > 0]
    if len(v):
        print(f"point {k}: n={len(v):3d} median {np.median(v - t0) / 100:7.2f} us  max {(v.max() - t0) / 100:7.2f} us")
