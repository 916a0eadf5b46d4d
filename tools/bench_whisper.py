"""Time the Whisper recognizer at large-v3-turbo dims (seeded weights, seeded speech-like
audio): log-mel of S seconds, one 30 s encoder window, a decoder step with a full
self-attention cache, and a whole greedy window of 224 tokens (the openai sample_len cap
a random model runs into). Prints one JSON line with the encoder's dense FLOPs and the
rate against the f32 MFMA peak, and the decoder step's weight bytes and HBM rate.

    python tools/bench_whisper.py [--seconds 10] [--iters 5]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    from t5gemma_tts_amd import whisper_asr as w
    from make_golden_codec_enc import test_wave
    d = w.dims_large_v3_turbo()
    m = w.WhisperModel(d, w.synthetic_weights(d, 42), device="cuda:0", max_seconds=args.seconds + 1)
    audio = test_wave(int(args.seconds * 16000), 6).cuda()
    t_mel = timed(lambda: m.log_mel(audio), args.iters)
    content = m.mel_frames - 3000
    t_enc = timed(lambda: m.encode(0, min(content, 3000)), args.iters)
    C, T = d.n_audio_state, d.n_audio_ctx
    enc_flop = 2 * 3000 * 3 * d.n_mels * C + 2 * T * 3 * C * C + d.n_audio_layer * (
        2 * T * 4 * C * C + 2 * T * 8 * C * C + 4 * T * T * C) + d.n_text_layer * 2 * T * 2 * C * C
    toks = list(range(50258, 50261))
    m.logits(toks, 0)
    pos = 220

    def step():
        m.logits([50365], pos)
    t_step = timed(step, 50)
    Ct = d.n_text_state
    step_bytes = 4 * (d.n_text_layer * (4 * Ct * Ct + 2 * Ct * Ct + 8 * Ct * Ct) + d.n_vocab * Ct) + \
        4 * d.n_text_layer * 2 * (T + pos) * Ct

    def window():
        seq = list(toks)
        fed = 0
        for _ in range(224):
            lg = m.logits(seq[fed:], fed)
            fed = len(seq)
            seq.append(int(lg[-1].argmax()))
    t_win = timed(window, 1)
    print(json.dumps({"metric": "Whisper large-v3-turbo dims (fp32), batch 1", "seconds_audio": args.seconds,
                      "log_mel_ms": round(t_mel * 1e3, 3), "encode_window_ms": round(t_enc * 1e3, 3),
                      "encoder_gflop": round(enc_flop / 1e9, 1),
                      "encoder_tflops": round(enc_flop / t_enc / 1e12, 2), "f32_mfma_peak_tflops": 157.3,
                      "decode_step_ms": round(t_step * 1e3, 4), "decode_step_mb": round(step_bytes / 1e6, 1),
                      "decode_step_gbps": round(step_bytes / t_step / 1e9, 1),
                      "greedy_224_tokens_ms": round(t_win * 1e3, 1),
                      "workspace_gb": round(int(m.L.whs_workspace_bytes(m.h)) / 1e9, 3)}))


if __name__ == "__main__":
    main()
