"""Stage timeline of parity mode's persistent layer launch (csrc/xlayer.hip) at the bench's
C3 shape (2b-2b, 8 rows, 60 text keys): the T5G_DBG_TS library variant stores the 100 MHz
device clock at each stage boundary of every workgroup (XL_TS points); this prints, per
point, the earliest / median / latest workgroup relative to the launch's first start.

    python t5gemma-tts_amd/build.py --dbg      # on the CPU host, builds lib/libt5gtts_dbg.so
    python tools/xlayer_timeline.py            # on the GPU box
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("T5G_LIB", os.path.join(REPO, "t5gemma-tts_amd", "lib", "libt5gtts_dbg.so"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

POINTS = {20: "N1 delta in", 21: "N1 rms post", 22: "N1 resid", 23: "N1 rms pre", 24: "A q staged",
          25: "A scores", 26: "A softmax", 27: "A pv+store",0: "start", 1: "O1 end", 19: "N1 wait done", 2: "N1 end", 3: "Q wait done", 4: "Q end",
          5: "A wait done", 6: "A end", 7: "O wait done", 8: "O end", 9: "N2 wait done", 10: "N2 end",
          11: "G wait done", 12: "G end", 13: "D wait done", 14: "D end", 15: "N3 wait done", 16: "N3 end",
          17: "QKV wait done", 18: "QKV end"}


def main():
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.config import config_2b2b
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda:0")
    cfg = config_2b2b()
    sd = synthetic_weights(cfg, seed=1234, device=str(dev))
    eng = T5GemmaTTSEngine(cfg, sd, device=str(dev), max_batch=B, max_text=128, max_audio=400, max_gen=64)
    rng = np.random.default_rng(5)
    utts = []
    for _ in range(B):
        y = rng.integers(0, 65536, size=151).tolist() + [cfg.y_sep_token]
        utts.append(Utterance(x=rng.integers(3, 4000, size=60).tolist(), y=y, tgt_y_len=len(y) + 40))
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    eng.generate(utts, p, seeds=list(range(B)), parity=True)
    L = _lib.lib()
    L.t5g_dbg_set_xlayer.argtypes = [C.c_void_p]
    buf = torch.zeros(256 * 32, dtype=torch.int64, device=dev)
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    us = C.c_float()
    L.t5g_dbg_set_xlayer_var.argtypes = [C.c_int]
    for rep, var in enumerate([0, 0, 1, 2, 3]):
        assert L.t5g_dbg_set_xlayer_var(var) == 0
        buf.zero_()
        assert L.t5g_dbg_set_xlayer(C.c_void_p(buf.data_ptr())) == 0
        _lib.check(L.t5g_time_xlayer(eng.h, B, 1, stream, C.byref(us)), "time_xlayer")
        assert L.t5g_dbg_set_xlayer(C.c_void_p(0)) == 0
        torch.cuda.synchronize()
        assert L.t5g_dbg_set_xlayer_var(0) == 0
        ts = buf.view(256, 32).cpu().numpy().astype(np.int64)
        live = ts[:, 0] > 0
        t0 = ts[live, 0].min()
        print(f"--- rep {rep} variant {var} ({['product', 'no MFMA', 'no fold', 'no weight loads'][var]}): "
              f"{int(live.sum())} workgroups, avg launch {us.value:.2f} us (timed rotation)")
        for k in (0, 1, 19, 20, 21, 22, 23, 2, 3, 4, 5, 24, 25, 26, 27, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18):
            v = ts[live, k]
            v = v[v > 0]
            if not len(v):
                continue
            d = (v - t0) * 0.01   # 100 MHz ticks -> us
            if var and k not in (0, 1, 3, 4, 7, 8, 11, 12, 13, 14, 17, 18):
                continue
            print(f"{k:2d} {POINTS[k]:14s} n={len(v):3d} min {d.min():7.2f} med {np.median(d):7.2f} "
                  f"max {d.max():7.2f} us")


if __name__ == "__main__":
    main()
