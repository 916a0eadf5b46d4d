"""Time the XCodec2 encoder (xc2e_encode) at the real 16 kHz dims on a prompt of S seconds
(seeded weights, seeded speech-like audio). Prints one JSON line: ms per prompt, audio
seconds per wall second, and the dense fp32 FLOPs of the semantic and acoustic paths
with the rate they imply against the f32 MFMA peak.

    python tools/bench_codec_enc.py [--seconds 10] [--iters 5]
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def flops(cfg, n):
    """Dense multiply-add FLOPs (2 per MAC) of one encode of n samples."""
    from t5gemma_tts_amd.codec_enc import HOP
    T = n // HOP + 1
    F = 2 * T
    H, I = cfg.sem_hidden, cfg.sem_intermediate
    fb = 2 * F * 512 * 514 + 2 * F * 288 * 80
    layer = 2 * T * (2 * 2 * H * I + 3 * H * H + H * H + 2 * H * H + H * H) + 2 * T * T * H * 2 + 2 * T * H * 73
    sem = fb + 2 * T * 160 * H + cfg.sem_layers * layer + 4 * 2 * T * 3 * H * H
    Tl, c = T * HOP, cfg.ac_channels0
    ac = 2 * Tl * 7 * c
    for s in cfg.strides:
        ac += 3 * (2 * Tl * 7 * c * c + 2 * Tl * c * c)
        Tl //= s
        ac += 2 * Tl * 2 * s * c * 2 * c
        c *= 2
    ac += 2 * Tl * 3 * c * cfg.hidden
    head = 2 * T * cfg.fc_dim * cfg.fc_dim + 2 * T * cfg.fc_dim * len(cfg.levels)
    return sem, ac, head


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from t5gemma_tts_amd.codec_enc import XCodec2Encoder, encoder_16k, synthetic_encoder_weights
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
    from make_golden_codec_enc import test_wave
    cfg = encoder_16k()
    n = int(args.seconds * 16000)
    enc = XCodec2Encoder(cfg, synthetic_encoder_weights(cfg, 32), device="cuda:0", max_seconds=args.seconds + 1)
    wav = test_wave(n, 6).cuda()
    enc.encode(wav)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        enc.encode(wav)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters
    sem, ac, head = flops(cfg, n)
    tot = sem + ac + head
    print(json.dumps({"metric": "XCodec2 encode (prompt audio -> codes), 16 kHz dims", "seconds_audio": args.seconds,
                      "ms_per_prompt": round(dt * 1e3, 3), "audio_s_per_wall_s": round(args.seconds / dt, 2),
                      "gflop": {"semantic": round(sem / 1e9, 2), "acoustic": round(ac / 1e9, 2),
                                "fc_fsq": round(head / 1e9, 2)},
                      "tflops_achieved": round(tot / dt / 1e12, 2), "f32_mfma_peak_tflops": 157.3,
                      "workspace_gb": round(enc.workspace_bytes / 1e9, 3)}))


if __name__ == "__main__":
    main()
