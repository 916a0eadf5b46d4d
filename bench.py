"""Throughput benchmark: T5Gemma-TTS-2b-2b generate() on MI355X.

Default workload (BASELINE.json metric, configs[2], C3): bf16, batch 8 voice-cloning
utterances per GPU -- T_x = 60 text tokens (28 transcript + x_sep + 31 target),
T_p = 151 prompt frames (150 codes + y_sep), tgt_y_lens = T_p + 500 (10 s),
top-k 30 / top-p 0.9 / T 0.8, throughput mode (EOS never accepted before the
time budget) so every row emits exactly 751 tokens (incl. EOS).
A "step" = one full generate() (encoder + prefill + AR loop + on-device stop
rules) over the batch. Weights: seeded random at the exact 2b-2b shapes (no
checkpoint download); data: synthetic.

``--e2e`` (configs[4], C5): batch 32 per GPU, 10 s target, generate() plus the batched
XCodec2 decode of every row at 882 samples per token (Anime-XCodec2-44.1kHz-v2 rate)
inside the timed region; reports the real-time factor.

Multi-GPU: ``--gpus N`` launches N ranks itself (one process per GPU via
torch.distributed.run, before any GPU call) unless it already runs under a launcher
(WORLD_SIZE set, as the driver's torchrun). Rank 0 draws the global batch and broadcasts
it (RCCL), every rank generates its shard (weak scaling, no per-step collective), ids are
all-gathered. value = tokens of all ranks / max rank time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

T_X, T_P, DUR_FRAMES = 60, 151, 500
B_PER_GPU = 8
B_PER_GPU_E2E = 32
CPU_SAMPLE_TOKENS = 160


def make_batch(cfg, n: int, seed: int):
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n):
        x = rng.integers(3, cfg.backbone.text_vocab_size - 1, size=T_X)
        x[28] = cfg.x_sep_token
        y = rng.integers(0, cfg.audio_vocab_size, size=T_P - 1).tolist() + [cfg.y_sep_token]
        rows.append((x.tolist(), y, T_P + DUR_FRAMES))
    return rows


def cpu_baseline(cfg, sd_gpu, utt, n_tokens: int = CPU_SAMPLE_TOKENS):
    """Time the CPU oracle (the reference's algorithm restated in PyTorch CPU ops, pinned
    bitwise to the reference's golden vectors) over a complete, measured generate() of
    one utterance of the same workload: encoder + prefill + ``n_tokens`` AR steps, batch 1
    as the reference. Nothing is extrapolated; the rate is tokens / wall time like the
    reference's own [Speed] line (inference_tts_utils.py:289, 308-321)."""
    import torch
    from oracle.t5g_oracle import SamplerParams, T5GemmaTTSOracle
    threads = int(os.environ.get("OMP_NUM_THREADS", torch.get_num_threads()))
    torch.set_num_threads(threads)
    sd = {k: v.cpu() for k, v in sd_gpu.items()}
    orc = T5GemmaTTSOracle(cfg, sd)
    x, y, tgt = utt
    p = SamplerParams(top_k=30, top_p=0.9, temperature=0.8, eos_disabled=True)
    t0 = time.perf_counter()
    out = orc.generate(x, y, tgt, p, seed=1, max_steps=n_tokens)
    dt = time.perf_counter() - t0
    n = int(out["gen"].numel())
    return {"value": round(n / dt, 3), "unit": "audio tokens/s", "cores": threads, "kind": "port",
            "sample": f"1 utterance of this workload (T_x {T_X}, T_p {T_P}), complete generate(): encoder + "
                      f"prefill + {n} AR steps (self-attention keys {T_P + 1}..{T_P + n}) in {dt:.1f} s, "
                      f"batch 1 (reference semantics); the reference itself measured 7.04 tok/s on 8 cores "
                      f"(SURVEY 6)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--batch", type=int, default=0, help="utterances per GPU (default 8, --e2e 32)")
    ap.add_argument("--natural-eos", action="store_true",
                    help="accept EOS when sampled (SURVEY 8(d)'s second run) instead of throughput mode")
    ap.add_argument("--e2e", action="store_true", help="C5: generate + XCodec2 decode in the timed region")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, default) or gloo (CPU collectives; lets N ranks share one GPU "
                         "to rehearse the sharded path)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started before this process touches the GPU
        from t5gemma_tts_amd.distributed import launch_local_ranks
        sys.exit(launch_local_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus,
                                    require_gpus=args.dist_backend == "nccl"))

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(args.dist_backend)
        world = dist.get_world_size()
        rank = dist.get_rank()
    if args.dist_backend == "nccl" and torch.cuda.device_count() < world:
        raise SystemExit(f"{world} ranks but only {torch.cuda.device_count()} GPU(s)")
    dev = torch.device(f"cuda:{local % max(1, torch.cuda.device_count())}")
    comm_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    torch.cuda.set_device(dev)

    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd.config import config_2b2b, decode_weight_bytes
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights

    cfg = config_2b2b()
    B = args.batch or (B_PER_GPU_E2E if args.e2e else B_PER_GPU)
    torch.manual_seed(1234)
    sd = synthetic_weights(cfg, seed=1234, device=str(dev))
    n_tok_row = DUR_FRAMES + int(cfg.extra_budget) + 1
    eng = T5GemmaTTSEngine(cfg, sd, device=str(dev), max_batch=B, max_text=64,
                           max_audio=T_P + 1 + n_tok_row + 8, max_gen=n_tok_row + 4)
    codec = None
    if args.e2e:
        from t5gemma_tts_amd.codec import XCodec2Decoder, codec_44k, synthetic_codec_weights
        ccfg = codec_44k()
        codec = XCodec2Decoder(ccfg, synthetic_codec_weights(ccfg, 1), device=str(dev), max_batch=B,
                               max_frames=n_tok_row)

    # global batch drawn on rank 0; each step broadcasts it over RCCL, shards it (LPT over
    # the token budget, B per rank), generates, and all-gathers the ids (8(e))
    from t5gemma_tts_amd.distributed import run_sharded
    G = B * world
    rows = costs = None
    if rank == 0:
        rows = [[len(x), tgt] + x + y for x, y, tgt in make_batch(cfg, G, seed=20251226)]
        costs = [r[1] for r in rows]
    params = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3,
                            eos_disabled=not args.natural_eos)
    gen_tokens = [0]
    audio_frames = [0]

    def generate(shard, i):
        utts = [Utterance(x=r[2:2 + r[0]], y=r[2 + r[0]:], tgt_y_len=r[1]) for r in shard]
        out = eng.generate(utts, params, seeds=[1000 * i + rank * B + b for b in range(len(utts))], chunk=64)
        gen_tokens[0] += sum(len(g) for g in out["gen"])
        if codec is not None:
            # strip EOS (inference_tts_utils.py:323-354) and decode every row in one launch
            frames = [g[g != cfg.eog_inference] for g in out["gen"]]
            lens = [max(1, int(f.numel())) for f in frames]
            codes = torch.zeros(len(frames), max(lens), dtype=torch.long)
            for b, f in enumerate(frames):
                codes[b, :f.numel()] = f
            codec.decode(codes, lens=lens)
            audio_frames[0] += sum(lens)
        return [g.tolist() for g in out["gen"]]

    def step(i):
        if dist is None:
            return sum(len(g) for g in generate(rows, i))
        before = gen_tokens[0]
        run_sharded(rows, costs, lambda sh: generate(sh, i), comm_dev, max_per_rank=B, max_len=n_tok_row + 8)
        return gen_tokens[0] - before

    for i in range(args.warmup):
        step(i)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    audio_frames[0] = 0
    t0 = time.perf_counter()
    tokens = 0
    for i in range(args.steps):
        tokens += step(100 + i)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    tot = torch.tensor([float(tokens), dt, float(audio_frames[0])], dtype=torch.float64, device=comm_dev)
    if dist is not None:
        t_sum = tot[[0, 2]].clone()
        dist.all_reduce(t_sum, op=dist.ReduceOp.SUM)
        t_dt = tot[1:2].clone()
        dist.all_reduce(t_dt, op=dist.ReduceOp.MAX)
        tokens_all, frames_all, dt_max = float(t_sum[0].item()), float(t_sum[1].item()), float(t_dt.item())
    else:
        tokens_all, frames_all, dt_max = float(tokens), float(audio_frames[0]), dt
    value = tokens_all / dt_max

    # ---- roofline of the dominant kernel: decode GeGLU gate/up GEMV (largest weight stream)
    roof = None
    if rank == 0 and not args.e2e:
        import ctypes as C
        from t5gemma_tts_amd import _lib
        L = _lib.lib()
        d, f = cfg.backbone.hidden_size, cfg.backbone.intermediate_size
        # rotate over every decoder layer's gate/up weights (2.2 GB >> 256 MiB Infinity
        # Cache) so each launch streams its weights from HBM, as inside a decode step
        X = torch.randn(B, d, device=dev).to(torch.bfloat16)
        Y = torch.empty(B, f, dtype=torch.bfloat16, device=dev)
        st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        us_gu = _lib.time_gate_up(X.data_ptr(), d, B, [lw.gate_up for lw in eng._dec], 2 * f, d, Y.data_ptr(),
                                  208, st)
        alg_bytes = 2 * f * d * 2 + B * d * 2 + B * f * 2
        achieved = alg_bytes / (us_gu * 1e-6) / 1e9
        traffic = None
        pmc = os.path.join(REPO, "profiles", "r02_pmc_gate_up.json")
        if os.path.exists(pmc):
            traffic = json.load(open(pmc)).get("hbm_bytes_per_call")
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                "frac": round(achieved / 8000.0, 4), "traffic": traffic,
                "kernel": _lib.GATE_UP_KERNEL,
                "avg_us": round(us_gu, 2)}
        step_us = C.c_float()
        _lib.check(L.t5g_time_decode_step(eng.h, 20, st, C.byref(step_us)), "time_step")
        roof["decode_step_us"] = round(step_us.value, 1)
        roof["decode_step_GBps"] = round(decode_weight_bytes(cfg) / (step_us.value * 1e-6) / 1e9, 1)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.e2e:
        r0 = rows[0]
        cpu = cpu_baseline(cfg, sd, (r0[2:2 + r0[0]], r0[2 + r0[0]:], r0[1]))

    if rank == 0:
        ms = dt_max / args.steps * 1e3
        if args.e2e:
            hop = codec.cfg.hop_length
            audio_s = frames_all / 50.0
            line = {
                "metric": "end-to-end text->waveform RTF, T5Gemma-TTS-2b-2b + XCodec2 decode (882 samples/token)",
                "value": round(audio_s / dt_max, 3), "unit": "audio seconds per wall second", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "bf16 (voice model) + fp32 (codec)",
                "data": "synthetic (seeded random 2b-2b + codec weights, random text/prompt codes)",
                "config": {"workload": f"C5 end-to-end: 2b-2b bf16, {B} utterances/GPU, T_x 60, T_p 151, 10 s "
                                       f"target (751 tokens/utterance), generate + XCodec2 decode at {hop} "
                                       f"samples/token in the timed region",
                           "global_batch": B * world, "seq_len": T_P + 1 + n_tok_row,
                           "parallelism": f"dp{world} (utterance shards)"},
                "audio_tokens_per_s": round(value, 2), "wall_s_per_audio_s": round(dt_max / audio_s, 5),
                "samples_per_s": round(frames_all * hop / dt_max, 1),
            }
        else:
            line = {
                "metric": "XCodec2 audio tokens/sec (whole node) + RTF, T5Gemma-TTS-2b-2b bs=8",
                "value": round(value, 2), "unit": "audio tokens/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "bf16",
                "data": "synthetic (seeded random 2b-2b weights, random text/prompt codes)",
                "config": {"workload": f"C3 voice-clone: 2b-2b bf16, {B} utterances/GPU, T_x 60, T_p 151, "
                                       "10 s target (751 tokens/utterance), top-k 30/top-p 0.9/T 0.8"
                                       + (", EOS accepted when sampled" if args.natural_eos else ""),
                           "global_batch": B * world, "seq_len": T_P + 1 + n_tok_row,
                           "parallelism": f"dp{world} (utterance shards)"},
                "rtf_audio_s_per_wall_s": round(value / 50.0, 3),
                "roofline": roof, "cpu_baseline": cpu,
            }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
