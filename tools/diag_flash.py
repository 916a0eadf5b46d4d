"""Block timeline of the fast path's flash decode self attention (attn_decode_kernel FLASH,
diagnostic library T5G_DBG_TS): runs a C3-shaped generate() and prints, for the last
layer's self-attention launch of the last step, the median / max time from each chunk
workgroup's start to its points and the combining (last-arriving) workgroups' points.
Points: 1 q staged, 2 scores in LDS, 3 partial stored + drained, 4 ticket known,
6 (combiner) chunk weights known, 5 (combiner) output stored.
    python t5gemma-tts_amd/build.py --dbg && T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so \\
        python tools/diag_flash.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    assert "dbg" in os.environ.get("T5G_LIB", ""), "point T5G_LIB at libt5gtts_dbg.so"
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.config import config_2b2b
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    _lib.lib()
    raw = C.CDLL(os.environ["T5G_LIB"])
    dev = "cuda:0"
    buf = torch.zeros(4096 * 8 * 4, dtype=torch.int64, device=dev)
    fn = raw.t5g_dbg_set_attn
    fn.argtypes = [C.c_void_p]
    assert fn(C.c_void_p(buf.data_ptr())) == 0
    cfg = config_2b2b()
    sd = synthetic_weights(cfg, seed=1234, device=dev)
    eng = T5GemmaTTSEngine(cfg, sd, device=dev, max_batch=8, max_text=64, max_audio=1024, max_gen=760)
    rng = np.random.default_rng(0)
    for tgt in (151 + 400, 151 + 750):
        utts = []
        for b in range(8):
            x = rng.integers(3, cfg.backbone.text_vocab_size - 1, size=60).tolist()
            y = rng.integers(0, cfg.audio_vocab_size, size=150).tolist() + [cfg.y_sep_token]
            utts.append(Utterance(x=x, y=y, tgt_y_len=tgt))
        p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3, eos_disabled=True)
        buf.zero_()
        eng.generate(utts, p, seeds=list(range(8)), chunk=64)
        torch.cuda.synchronize()
        a = buf.view(-1, 8).cpu().numpy()
        rows = a[a[:, 2] > 0]   # chunk workgroups that computed scores
        t0 = rows[:, 0].astype(np.int64)
        base = t0.min()
        print(f"== L ~ {tgt + 1}: {len(rows)} chunk workgroups, starts spread {(t0.max() - base) * 10} ns")
        for k, name in ((1, "q staged"), (2, "scores in LDS"), (3, "partial stored+drained"), (4, "ticket known"),
                        (6, "combiner: weights"), (5, "combiner: output stored")):
            v = rows[:, k].astype(np.int64)
            ok = v > 0
            if not ok.any():
                continue
            d = (v[ok] - t0[ok]) * 10
            e = (v[ok] - base) * 10
            print(f"   {k} {name:24s}: from block start median {int(np.median(d))} ns (max {int(d.max())}); "
                  f"from first start median {int(np.median(e))} ns (max {int(e.max())}) [{int(ok.sum())}]")


if __name__ == "__main__":
    main()
