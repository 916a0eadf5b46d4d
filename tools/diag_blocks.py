"""Block timelines inside the decode step (diagnostic library, T5G_DBG_TS): runs a C3-shaped
generate() on lib/libt5gtts_dbg.so and prints, for the last launch of each instrumented
unit (norm: the final resid_norm of the last layer; attn: the last layer's cross attention;
gemm: head1; sampler: the last sampler_kernel), the spread of block start times and the
median time from block start to each numbered point (100 MHz device clock, 10 ns).
    python t5gemma-tts_amd/build.py --dbg && T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so \\
        python tools/diag_blocks.py"""
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
    L = _lib.lib()
    raw = C.CDLL(os.environ["T5G_LIB"])
    dev = "cuda:0"
    units = ["norm", "attn", "gemm", "sampler"]
    bufs = {}
    for u in units:
        b = torch.zeros(4096 * 8 * 4, dtype=torch.int64, device=dev)
        fn = getattr(raw, f"t5g_dbg_set_{u}")
        fn.argtypes = [C.c_void_p]
        assert fn(C.c_void_p(b.data_ptr())) == 0
        bufs[u] = b
    cfg = config_2b2b()
    sd = synthetic_weights(cfg, seed=1234, device=dev)
    eng = T5GemmaTTSEngine(cfg, sd, device=dev, max_batch=8, max_text=64, max_audio=1024, max_gen=600)
    rng = np.random.default_rng(0)
    utts = []
    for b in range(8):
        x = rng.integers(3, cfg.backbone.text_vocab_size - 1, size=60).tolist()
        y = rng.integers(0, cfg.audio_vocab_size, size=150).tolist() + [cfg.y_sep_token]
        utts.append(Utterance(x=x, y=y, tgt_y_len=151 + 400))
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3, eos_disabled=True)
    eng.generate(utts, p, seeds=list(range(8)), chunk=64)
    torch.cuda.synchronize()
    # the attn buffer holds the last layer's self-attention launches, each overwriting block
    # slots from 0: scores (480 blocks), then P.V/combine (slots 0-255); slots 256-479 keep
    # the scores launch. norm: the last per-op resid_norm; gemm: head1 (blocks 0-143)
    groups = [("norm", "norm (8 rows)", 0, 8), ("attn", "attn pvc", 0, 256),
              ("attn", "attn scores (blocks 256-479)", 256, 480), ("gemm", "gemm head1", 0, 144),
              ("sampler", "sampler_fast (last step with live rows)", 0, 128)]
    a = bufs["attn"].view(-1, 8).cpu().numpy()
    sc, pv = a[256:480], a[0:256]
    sc, pv = sc[sc[:, 0] > 0], pv[pv[:, 0] > 0]
    if len(sc) and len(pv):
        base = sc[:, 0].min()
        ends = np.maximum.reduce([sc[:, k] for k in range(1, 7)])
        print(f"== scores -> pvc (absolute, from the first scores block start): scores last end "
              f"{(ends.max() - base) * 10} ns, median end {int(np.median(ends - base)) * 10} ns; pvc first start "
              f"{(pv[:, 0].min() - base) * 10} ns, median start {int(np.median(pv[:, 0] - base)) * 10} ns, "
              f"median point 1 {int(np.median(pv[:, 1] - base)) * 10} ns, last point 1 {(pv[:, 1].max() - base) * 10} ns")
        print("   pvc points (one-pass rows): 2 = scores / chunk maxima in, 3 = p staged, 4 = P.V chains in LDS, "
              "1 = output stored")
    for u, name, lo, hi in groups:
        a = bufs[u].view(-1, 8).cpu().numpy()[lo:hi]
        rows = a[(a[:, 0] > 0)]
        u = name
        if len(rows) == 0:
            print(f"{u}: no records")
            continue
        t0 = rows[:, 0].astype(np.int64)
        base = t0.min()
        print(f"== {u}: {len(rows)} blocks, block starts spread {(t0.max() - base) * 10} ns")
        for k in range(1, 7):
            v = rows[:, k].astype(np.int64)
            ok = v > 0
            if ok.sum() == 0:
                continue
            d = (v[ok] - t0[ok]) * 10
            e = (v[ok] - base) * 10
            print(f"   point {k}: from block start median {int(np.median(d))} ns (max {int(d.max())}); "
                  f"from first block start median {int(np.median(e))} ns (max {int(e.max())}) [{int(ok.sum())} blocks]")


if __name__ == "__main__":
    main()
