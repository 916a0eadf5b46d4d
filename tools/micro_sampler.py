"""Micro-benchmark of the on-device sampler kernel (t5g_sample_only) on 2b-2b-sized
logits (V = 65541), B rows, several parameter mixes. GPU only."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402
from t5gemma_tts_amd.config import named_config  # noqa: E402
from t5gemma_tts_amd.engine import T5GemmaTTSEngine  # noqa: E402
from t5gemma_tts_amd.weights import synthetic_weights  # noqa: E402


def main():
    B = int(os.environ.get("B", "8"))
    cfg = named_config("tiny")
    cfg.audio_vocab_size = 65536
    cfg.empty_token, cfg.eog, cfg.audio_pad_token, cfg.eos, cfg.y_sep_token = 65536, 65537, 65538, 65539, 65540
    eng = T5GemmaTTSEngine(cfg, synthetic_weights(cfg, 3), max_batch=B, max_text=16, max_audio=4096,
                           max_gen=4000)
    L = eng.L
    V = cfg.n_audio_tokens
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    lg = (torch.randn(B, V + 11, device="cuda") * 0.8).to(torch.bfloat16)
    for name, (k, p, t) in {"softmax-only": (0, 1.0, 1.0), "topk30": (30, 1.0, 1.0),
                            "topk30+topp0.9+T0.8": (30, 0.9, 0.8), "topp0.9 (no top-k)": (0, 0.9, 1.0)}.items():
        rows = (_lib.SamplerRow * B)(*[_lib.SamplerRow(top_k=k, top_p=p, temperature=t, eos_disabled=1,
                                                       seed_lo=b + 1) for b in range(B)])
        sts = (_lib.SamplerState * B)(*[_lib.SamplerState(cur_num_gen=20, current_length=100, prompt_offset=1,
                                                          target_total=-1, est_total=4000, prev_token=-1,
                                                          first_input_len=5) for _ in range(B)])
        tk = (C.c_int32 * 1)()
        _lib.check(L.t5g_sampler_setup(eng.h, B, rows, sts, tk, 0, tk, 0, None, 0, st), "setup")
        for _ in range(3):
            L.t5g_sample_only(eng.h, B, C.c_void_p(lg.data_ptr()), V + 11, st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            L.t5g_sample_only(eng.h, B, C.c_void_p(lg.data_ptr()), V + 11, st)
        e1.record()
        torch.cuda.synchronize()
        print(f"sampler B={B} {name:24s}: {e0.elapsed_time(e1) / n * 1000:8.1f} us/step", flush=True)


if __name__ == "__main__":
    main()
