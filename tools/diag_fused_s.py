"""Timeline of the fast path's persistent layer launch WITH the self attention (csrc/fused.hip
stage S) inside a C3-shaped decode step at ~527 keys, on the diagnostic library (T5G_DBG_TS):
for the last launch of the call, per point the time from the first workgroup start (100 MHz
device clock): 1 row geometry read, 2 q staged, 3 K in + scores, 4 P.V reduced, 5 partials
drained, 6 ticket seen, 7 att_self published (combiners / one-chunk rows), 8 S left, 9 O1
hand-off seen, 10 O1 published, 11 Q hand-off seen (N1 done), 12 N1 published (norm groups).
    python t5gemma-tts_amd/build.py --dbg && python tools/diag_fused_s.py [B] [n_gen]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["T5G_LIB"] = os.path.join(REPO, "t5gemma-tts_amd", "lib", "libt5gtts_dbg.so")
sys.path.insert(0, REPO)

NAMES = {17: "N3 seen (tail)", 18: "q|k|v published", 19: "q|k|v all seen", 20: "O1n hand-off seen",
         21: "O1n done", 14: "q rotated (wave 0)", 15: "first K row scored", 16: "scores done (wave 0)", 13: "second S run starts", 1: "row geometry", 2: "q staged", 3: "K in + scores", 4: "P.V reduced", 5: "partials drained",
         6: "ticket seen", 7: "att_self published", 8: "S left", 9: "O1 hand-off seen", 10: "O1 published",
         11: "Q hand-off seen", 12: "N1 published"}


def main():
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.config import config_2b2b
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n_gen = int(sys.argv[2]) if len(sys.argv) > 2 else 376
    dev = "cuda:0"
    cfg = config_2b2b()
    sd = synthetic_weights(cfg, seed=1234, device=dev)
    eng = T5GemmaTTSEngine(cfg, sd, device=dev, max_batch=B, max_text=64, max_audio=160 + n_gen + 64,
                           max_gen=n_gen + 16)
    mode = int(os.environ.get("FS_MODE", "2"))   # 1: stage S in front, 2: at the end (times of layer L-2's launch)
    eng.set_attn_in_block(mode)
    rng = np.random.default_rng(0)
    utts = [Utterance(x=rng.integers(3, 4000, size=60).tolist(),
                      y=rng.integers(0, 65536, size=150).tolist() + [cfg.y_sep_token], tgt_y_len=151 + n_gen)
            for _ in range(B)]
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    L = _lib.lib()
    L.t5g_dbg_set_fused_s.argtypes = [C.c_void_p]
    buf = torch.zeros(256 * 32, dtype=torch.int64, device=dev)
    assert L.t5g_dbg_set_fused_s(C.c_void_p(buf.data_ptr())) == 0
    L.t5g_dbg_set_fused_s_var.argtypes = [C.c_int]
    for rep, var in enumerate([int(v) for v in os.environ.get("FS_VARS", "0,0,1,2,3,4").split(",")]):
        # variants (timing only, results garbage): 1 no K / V loads, 2 one q|k|v slab address,
        # 3 every (row, kv head) on row 0 / kv head 0's cache
        assert L.t5g_dbg_set_fused_s_var(var) == 0
        buf.zero_()
        eng.generate(utts, p, seeds=list(range(B)))
        torch.cuda.synchronize()
        ts = buf.view(256, 32).cpu().numpy().astype(np.int64)
        live = ts[:, 0] > 0
        t0 = ts[live, 0].min()
        print(f"--- rep {rep} variant {var}: {int(live.sum())} workgroups, B={B}, keys ~{152 + n_gen}")
        for k in (17, 18, 19, 13, 1, 2, 14, 15, 16) + tuple(range(3, 13)) + (20, 21):
            v = ts[live, k]
            v = v[v > 0]
            if not len(v):
                continue
            d = (v - t0) * 0.01
            print(f"{k:2d} {NAMES[k]:20s} n={len(v):3d} min {d.min():7.2f} med {np.median(d):7.2f} max {d.max():7.2f} us")
        if os.environ.get("FS_SLOW"):
            # the workgroups that published att_self last: their own points 3-7 (and the ticket wait)
            wg = np.nonzero(live)[0]
            order = wg[np.argsort(ts[wg, 7])[::-1]][:int(os.environ["FS_SLOW"])]
            for w in order:
                pts = " ".join(f"{k}:{(ts[w, k] - t0) * 0.01:6.2f}" if ts[w, k] > 0 else f"{k}:   -  " for k in (19, 2, 3, 4, 5, 6, 7))
                print(f"   wg {w:3d} (xcd {w % 8}) {pts}")
    assert L.t5g_dbg_set_fused_s(C.c_void_p(0)) == 0
    assert L.t5g_dbg_set_fused_s_var(0) == 0


if __name__ == "__main__":
    main()
