"""Block timeline of the fused decode launch (csrc/fused.hip) inside a C3-shaped decode step,
on the diagnostic library (T5G_DBG_TS): for the last layer's launch, per numbered point the
time from the first block start (100 MHz device clock), over all workgroups and over the
norm workgroups. B <= 16 runs fused_block_kernel (points: 1 Q hand-off seen, 2 O hand-off
seen, 3 G hand-off seen, 4 gate/up published, 5 D hand-off seen, 6 leaving); B > 16
fused_mlp_kernel (1 norm published, 2 gate/up hand-off seen, 3 gate/up sums in LDS, 4 down
hand-off seen, 5 down sums in LDS, 6 leaving).
    python t5gemma-tts_amd/build.py --dbg && T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so \\
        python tools/diag_fused.py"""
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
    from t5gemma_tts_amd.config import config_2b2b
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    raw = C.CDLL(os.environ["T5G_LIB"])
    dev = "cuda:0"
    buf = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
    fn = raw.t5g_dbg_set_fused
    fn.argtypes = [C.c_void_p]
    assert fn(C.c_void_p(buf.data_ptr())) == 0
    cfg = config_2b2b()
    sd = synthetic_weights(cfg, seed=1234, device=dev)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    eng = T5GemmaTTSEngine(cfg, sd, device=dev, max_batch=B, max_text=64, max_audio=1024, max_gen=600)
    rng = np.random.default_rng(0)
    utts = []
    for b in range(B):
        x = rng.integers(3, cfg.backbone.text_vocab_size - 1, size=60).tolist()
        y = rng.integers(0, cfg.audio_vocab_size, size=150).tolist() + [cfg.y_sep_token]
        utts.append(Utterance(x=x, y=y, tgt_y_len=151 + 100))
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3, eos_disabled=True)
    eng.generate(utts, p, seeds=list(range(B)), chunk=64)
    torch.cuda.synchronize()
    a = buf.view(-1, 8).cpu().numpy()
    rows = a[a[:, 0] > 0]
    nb = len(rows)
    t0 = rows[:, 0].astype(np.int64)
    base = t0.min()
    print(f"fused launch B={B}: {nb} workgroups, block starts spread {(t0.max() - base) * 10} ns")
    if B <= 16:   # fused_block_kernel (cross-attention chain + MLP half)
        names = {1: "Q hand-off seen (N1)", 2: "O hand-off seen (attn)", 3: "G hand-off seen (N2)",
                 4: "gate/up published", 5: "D hand-off seen", 6: "leaving"}
    else:         # fused_mlp_kernel
        names = {1: "norm published", 2: "gate/up hand-off seen", 3: "gate/up sums in LDS", 4: "down hand-off seen",
                 5: "down sums in LDS", 6: "leaving"}
    norm = (rows[:, 1] > 0) if B > 16 else (np.arange(nb) >= nb - B)
    for k in range(1, 7):
        v = rows[:, k].astype(np.int64)
        ok = v > 0
        if ok.sum() == 0:
            continue
        e = (v[ok] - base) * 10
        pc = np.percentile(e, [0, 10, 50, 90, 100]).astype(int)
        print(f"  {k} {names[k]:24s} from first start: min {pc[0]} p10 {pc[1]} p50 {pc[2]} p90 {pc[3]} "
              f"max {pc[4]} ns [{int(ok.sum())}]")
        if (norm & ok).any() and (k > 1 or B <= 16):
            en = (v[norm & ok] - base) * 10
            print(f"      norm workgroups: p50 {int(np.median(en))} max {int(en.max())} ns")
    xcc = (rows[:, 7] >> 32) & 0xf
    for k in (3, 6):
        v = (rows[:, k].astype(np.int64) - base) * 10
        print(f"  point {k} by XCC median: " + " ".join(f"{int(np.median(v[xcc == x]))}" for x in range(8)
                                                       if (xcc == x).any()))


if __name__ == "__main__":
    main()
