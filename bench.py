"""Throughput benchmark: T5Gemma-TTS-2b-2b generate() on MI355X.

Workloads (BASELINE.json configs; ``--workload``, default c3 = the headline metric):
* c3 (configs[2], default): bf16, batch 8 voice-cloning utterances per GPU -- T_x = 60 text
  tokens (28 transcript + x_sep + 31 target), T_p = 151 prompt frames (150 codes + y_sep),
  tgt_y_lens = T_p + 500 (10 s), top-k 30 / top-p 0.9 / T 0.8, throughput mode (EOS never
  accepted before the time budget) so every row emits exactly 751 tokens.
* c2 (configs[1]): batch 1, T_x 32, no prompt, 10 s target (751 tokens).
* c4 (configs[3]): T_x 36 (a 128-character text), no prompt, 10 s, 8 utterances per GPU
  -- ``--gpus 8`` is the 64-utterance node batch.
* c5 (configs[4], also ``--e2e``): batch 32 per GPU, the c3 rows, generate() plus the
  batched XCodec2 decode of every row at 882 samples per token (Anime-XCodec2-44.1kHz-v2
  rate) inside the timed region; reports the real-time factor.
A "step" = one full generate() (encoder + prefill + AR loop + on-device stop rules) over
the batch. Weights: seeded random at the exact 2b-2b shapes (no checkpoint download);
data: synthetic.

``--parity``: time the drop-in default path instead (``inference_tts`` /
``inference_one_sample`` run ``parity=True``: exact-order kernels, the reference's CPU RNG
stream, one host sync per step, EOS accepted as in the reference), and print the
reference's own ``[Speed]`` line (inference_tts_utils.py:308-321) for it.

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

DUR_FRAMES = 500
# name -> (utterances per GPU, T_x, T_p incl. y_sep (0: no prompt), e2e, BASELINE configs index)
WORKLOADS = {
    "c2": (1, 32, 0, False, 1),
    "c3": (8, 60, 151, False, 2),
    "c4": (8, 36, 0, False, 3),
    "c5": (32, 60, 151, True, 4),
    # C3 with a 10 s voice prompt (500 codes + y_sep): rows end at ~1 253 keys, past the
    # decode attention stage's one-pass limits of round 5
    "c3p10": (8, 60, 501, False, 2),
}
T_X, T_P = 60, 151          # c3 (kept for tools that import them)
B_PER_GPU = 8
B_PER_GPU_E2E = 32


def make_batch(cfg, n: int, seed: int, T_x: int = T_X, T_p: int = T_P):
    """n synthetic utterances: text ids (x_sep after the 28-id transcript when there is a
    prompt), T_p - 1 prompt codes + y_sep (none when T_p = 0), tgt_y_lens = T_p + 500."""
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n):
        x = rng.integers(3, cfg.backbone.text_vocab_size - 1, size=T_x)
        if T_p:
            x[28] = cfg.x_sep_token
            y = rng.integers(0, cfg.audio_vocab_size, size=T_p - 1).tolist() + [cfg.y_sep_token]
        else:
            y = []
        rows.append((x.tolist(), y, T_p + DUR_FRAMES))
    return rows


def request_rows(cfg, G: int, T_x: int, T_p: int):
    """The step's global request batch (drawn on rank 0): [len(x), tgt, global index] + x + y.
    The global index seeds the request (request_seed), so a request samples the same
    tokens whatever rank / slot run_sharded gives it."""
    return [[len(x), tgt, gi] + x + y for gi, (x, y, tgt) in enumerate(make_batch(cfg, G, seed=20251226, T_x=T_x, T_p=T_p))]


def request_seed(step_i: int, gidx: int) -> int:
    """Sampling seed of global request gidx in step step_i (independent of the sharding)."""
    return 1000 * step_i + gidx


def cpu_model() -> str:
    """The host CPU (model name of /proc/cpuinfo, and the logical CPUs the process may use)."""
    name = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 0
    return f"{name} ({n} logical CPUs visible)"


def cpu_baseline(cfg, sd_gpu, utt, n_budget: int):
    """The CPU oracle (the reference's algorithm in PyTorch CPU ops, pinned bitwise to the
    reference's golden vectors) timed on ONE whole utterance of the workload, batch 1 as the
    reference runs it: encoder + prefill + every one of the row's ``n_budget`` AR steps
    (head, sampler with its noise draw, decoder step), EOS disabled so the row runs its full
    time budget like the GPU rows. rate = tokens / wall, the reference's [Speed] definition
    (inference_tts_utils.py:308-321). Threads: OMP_NUM_THREADS (16 on the GPU box: the
    box's CPU share per GPU, which the harness sets and asks jobs to keep)."""
    import torch
    from oracle.t5g_oracle import SamplerParams, T5GemmaTTSOracle
    threads = int(os.environ.get("OMP_NUM_THREADS", torch.get_num_threads()))
    torch.set_num_threads(threads)
    sd = {k: v.cpu() for k, v in sd_gpu.items()}
    orc = T5GemmaTTSOracle(cfg, sd)
    x, y, tgt = utt
    p = SamplerParams(top_k=30, top_p=0.9, temperature=0.8, eos_disabled=True)
    t0 = time.perf_counter()
    out = orc.generate(x, y, tgt, p, seed=1, max_steps=n_budget)
    wall = time.perf_counter() - t0
    n = int(out["gen"].numel())
    return {"value": round(n / wall, 3), "unit": "audio tokens/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"1 utterance of this workload (T_x {len(x)}, T_p {len(y)}), batch 1 (reference semantics), "
                      f"timed whole: encoder + prefill + {n} AR steps (L {len(y) + 1}..{len(y) + n}) in {wall:.1f} s "
                      f"on {threads} threads (the GPU box's per-GPU CPU share); the reference itself measured "
                      f"7.04 tok/s on 8 cores in the build container (SURVEY 6)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-steps", type=int, default=1,
                    help="timed generate() calls of the parity (drop-in default) path reported in the line's "
                         "`parity` object (0: skip)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3",
                    help="BASELINE config: c2 / c3 (default) / c4 / c5 (= --e2e)")
    ap.add_argument("--parity", action="store_true",
                    help="time the drop-in default path (parity=True: exact-order kernels, reference RNG, "
                         "one host sync per step, EOS accepted) and print the reference's [Speed] line")
    ap.add_argument("--batch", type=int, default=0, help="utterances per GPU (default: the workload's)")
    ap.add_argument("--natural-eos", action="store_true",
                    help="accept EOS when sampled (SURVEY 8(d)'s second run) instead of throughput mode")
    ap.add_argument("--e2e", action="store_true", help="C5: generate + XCodec2 decode in the timed region")
    ap.add_argument("--no-fused", action="store_true",
                    help="decode MLP half as three launches instead of the persistent fused launch (A/B)")
    ap.add_argument("--no-attn-flash", action="store_true",
                    help="fast path: decode self attention as the two-launch aten-order form (A/B)")
    ap.add_argument("--no-attn-in-block", action="store_true",
                    help="fast path: decode self attention as its own launch instead of inside the persistent "
                         "layer launch (A/B)")
    ap.add_argument("--attn-in-block", type=int, choices=(1, 2), default=None,
                    help="fast path: stage S in front of the layer's o-projection (1) or at the end of the "
                         "previous layer's launch (2, the engine default)")
    ap.add_argument("--attn", choices=("sdpa", "eager"), default="sdpa",
                    help="the checkpoint's attn_implementation: eager (the reference default, tanh softcap 50) "
                         "runs parity mode's eager.hip restatement")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, default) or gloo (CPU collectives; lets N ranks share one GPU "
                         "to rehearse the sharded path)")
    args = ap.parse_args()
    if args.e2e:
        args.workload = "c5"
    wl_b, wl_tx, wl_tp, wl_e2e, wl_cfg = WORKLOADS[args.workload]
    args.e2e = wl_e2e

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

    cfg = config_2b2b(attn_implementation=args.attn)
    B = args.batch or wl_b
    torch.manual_seed(1234)
    sd = synthetic_weights(cfg, seed=1234, device=str(dev))
    n_tok_row = DUR_FRAMES + int(cfg.extra_budget) + 1
    eng = T5GemmaTTSEngine(cfg, sd, device=str(dev), max_batch=B, max_text=128,   # the engine default
                           max_audio=wl_tp + 1 + n_tok_row + 8, max_gen=n_tok_row + 4)
    if args.no_fused:
        eng.set_fused(False)
    if args.no_attn_flash:
        eng.set_attn_flash(False)
    if args.no_attn_in_block:
        eng.set_attn_in_block(False)
    elif args.attn_in_block:
        eng.set_attn_in_block(args.attn_in_block)
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
        rows = request_rows(cfg, G, wl_tx, wl_tp)
        costs = [r[1] for r in rows]
    params = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3,
                            eos_disabled=not (args.natural_eos or args.parity))
    # the drop-in default path accepts EOS as the reference does
    params_parity = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3, eos_disabled=False)
    parity_stats = {"tokens": 0, "host_resolved": 0, "tie_cuts": 0}

    speed_lines = []
    gen_tokens = [0]
    audio_frames = [0]
    codec_s = [0.0]   # wall time inside XCodec2Decoder.decode (C5), the rest of a step is generate()

    def generate(shard, i, parity=None):
        parity = args.parity if parity is None else parity
        utts = [Utterance(x=r[3:3 + r[0]], y=r[3 + r[0]:], tgt_y_len=r[1]) for r in shard]
        t_call = time.perf_counter()
        out = eng.generate(utts, params_parity if parity else params, seeds=[request_seed(i, r[2]) for r in shard],
                           chunk=64, parity=parity)
        n_gen = sum(len(g) for g in out["gen"])
        gen_tokens[0] += n_gen
        if parity:
            parity_stats["tokens"] += n_gen
            parity_stats["host_resolved"] += out["ambiguous_fixed"]
            parity_stats["tie_cuts"] += sum(out["ambiguous"])
            # the reference's own report (inference_tts_utils.py:308-321)
            dt_call = time.perf_counter() - t_call
            speed_lines.append(f"[Speed] {n_gen / dt_call:.2f} tokens/s | RTF: {n_gen / 50.0 / dt_call:.2f}x | "
                               f"Generated {n_gen} tokens in {dt_call:.2f}s")
        if codec is not None:
            # strip EOS (inference_tts_utils.py:323-354) and decode every row in one launch
            frames = [g[g != cfg.eog_inference] for g in out["gen"]]
            lens = [max(1, int(f.numel())) for f in frames]
            codes = torch.zeros(len(frames), max(lens), dtype=torch.long)
            for b, f in enumerate(frames):
                codes[b, :f.numel()] = f
            torch.cuda.synchronize(dev)
            t_c = time.perf_counter()
            codec.decode(codes, lens=lens)
            torch.cuda.synchronize(dev)
            codec_s[0] += time.perf_counter() - t_c
            audio_frames[0] += sum(lens)
        return [g.tolist() for g in out["gen"]]

    def step(i):
        if dist is None:
            return sum(len(g) for g in generate(rows, i))
        before = gen_tokens[0]
        run_sharded(rows, costs, lambda sh: generate(sh, i), comm_dev, max_per_rank=B, max_len=n_tok_row + 8)
        return gen_tokens[0] - before

    s_before = eng.attn_in_block_launches()
    for i in range(args.warmup):
        step(i)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    audio_frames[0] = 0
    codec_s[0] = 0.0
    t0 = time.perf_counter()
    tokens = 0
    for i in range(args.steps):
        tokens += step(100 + i)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    s_launches = eng.attn_in_block_launches() - s_before
    s_mode = eng.attn_in_block_mode()
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

    # ---- the drop-in default path (parity mode: token-exact to the reference) on the same
    # workload, timed after the headline region: one untimed warm-up, PARITY_STEPS timed
    parity_line = None
    if world == 1 and not args.e2e and not args.parity and args.parity_steps > 0:
        saved = gen_tokens[0]
        generate(rows, 50, parity=True)   # warm-up: exact weight images, graphs
        torch.cuda.synchronize(dev)
        for k in parity_stats:
            parity_stats[k] = 0
        tp0 = time.perf_counter()
        for i in range(args.parity_steps):
            generate(rows, 200 + i, parity=True)
        torch.cuda.synchronize(dev)
        dtp = time.perf_counter() - tp0
        gen_tokens[0] = saved
        # roofline of the parity path's dominant kernel, timed with HIP events on the launching
        # stream, layers rotated (every launch streams its weights from HBM): the persistent
        # exact layer (xlayer.hip) where it serves the batch, else the six exact decode
        # Linears of one layer (xmm_dec_kernel)
        import ctypes as C
        from t5gemma_tts_amd import _lib
        stream_p = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        us_x = C.c_float()
        rc_xl = _lib.lib().t5g_time_xlayer(eng.h, B, 26 * 8, stream_p, C.byref(us_x))
        if rc_xl not in (0, _lib.T5G_EUNSUPPORTED):
            _lib.check(rc_xl, "time_xlayer")   # a real launch failure, not a shape the launch does not serve
        if rc_xl == 0:
            xbytes = _lib.xlayer_bytes(B, cfg.backbone, wl_tx, cfg.backbone.num_decoder_layers)
            pmc_x = os.path.join(REPO, "profiles", "r06_pmc_xlayer.json")
            kname = ("xlayer_kernel: one decoder layer after its self attention as one persistent launch (o, "
                     "norm, cross-q, PM cross attention, cross-o, norm, gate/up + GeGLU, down in the reference's "
                     "K parts, norm, next q|k|v; f32 MFMA in the reference host's fp32 orders)")
        else:
            _lib.check(_lib.lib().t5g_time_exact_linears(eng.h, B, 26 * 8, stream_p, C.byref(us_x)),
                       "time_exact_linears")
            xbytes = _lib.exact_linears_bytes(B, cfg.backbone)
            kname = ("xmm_dec_kernel: one layer's six exact decode Linears (q|k|v, o, cross-q, cross-o, "
                     "gate/up + GeGLU, down in the reference's K parts; f32 MFMA in the reference host's fp32 "
                     "orders)")
        traffic_x, tinfo_x = None, {"traffic_note": "PMC passes are at 8 rows"}
        if rc_xl != 0:
            tinfo_x = {"traffic_note": "no PMC pass of the per-op exact Linears"}
        elif B == 8:
            traffic_x, tinfo_x = _lib.pmc_traffic(pmc_x, "xlayer", "xlayer_kernel")
        ach_x = xbytes / (us_x.value * 1e-6) / 1e9
        parity_roof = {"bound": "hbm", "achieved": round(ach_x, 1), "peak": 8000.0, "unit": "GB/s",
                       "frac": round(ach_x / 8000.0, 4), "traffic": traffic_x, "kernel": kname,
                       "algorithmic_bytes": int(xbytes), "avg_us": round(us_x.value, 2), **tinfo_x}
        parity_line = {
            "value": round(parity_stats["tokens"] / dtp, 2), "unit": "audio tokens/s",
            "ms_per_step": round(dtp / args.parity_steps * 1e3, 2), "steps": args.parity_steps,
            "tokens": parity_stats["tokens"], "rtf_audio_s_per_wall_s": round(parity_stats["tokens"] / 50.0 / dtp, 3),
            "top_p_tie_cuts": parity_stats["tie_cuts"], "host_resolved_steps": parity_stats["host_resolved"],
            "mode": "parity (the drop-in default of inference_tts): exact-order kernels (logits bitwise the "
                    "reference CPU run's), the reference's MT19937 multinomial draws generated on the GPU, "
                    "torch.sort tie order on the GPU, EOS accepted; same workload and rows",
            "roofline": parity_roof,
        }

    # ---- roofline of the dominant kernel: the fused decode-MLP launch (norm + gate/up +
    # down, 127 MB of weights per layer), or the gate/up GEMV when the MLP runs unfused
    roof = None
    if rank == 0 and not args.e2e and not args.parity:
        import ctypes as C
        from t5gemma_tts_amd import _lib
        L = _lib.lib()
        eng.set_exact(False)   # the parity sub-run leaves the exact kernels selected
        d, f = cfg.backbone.hidden_size, cfg.backbone.intermediate_size
        st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        if not args.no_fused:
            us, keys = C.c_float(), C.c_float()
            # 208 launches rotated over the 26 layers' weights (3.3 GB >> 256 MiB Infinity
            # Cache): every launch streams from HBM, as inside a decode step; with the self
            # attention inside (stage S) when the step runs it so
            rc_s = _lib.T5G_EUNSUPPORTED if args.no_attn_in_block else \
                L.t5g_time_decode_layer(eng.h, B, 208, st, C.byref(us), C.byref(keys))
            if rc_s != 0:
                if rc_s != _lib.T5G_EUNSUPPORTED:
                    _lib.check(rc_s, "time_decode_layer")
                keys.value = 0.0
                _lib.check(L.t5g_time_decode_mlp(eng.h, B, 208, st, C.byref(us)), "time_decode_mlp")
            if B <= 16:   # the step runs the whole post-self-attention block in one launch
                us_k, kname = us.value, _lib.FUSED_BLOCK_KERNEL
                alg_bytes = _lib.fused_block_bytes(B, wl_tx, d, f, self_keys=keys.value)
                if keys.value > 0 and s_mode == 1:
                    kname = "fused_block_kernel<1> (the layer's self attention in front of its o-projection)"
                    pmc, pmc_op = os.path.join(REPO, "profiles", "r06_pmc_fused_block_s_front.json"), "fused_block_s"
                elif keys.value > 0:
                    kname = _lib.FUSED_BLOCK_S_KERNEL
                    pmc, pmc_op = os.path.join(REPO, "profiles", "r06_pmc_fused_block_s.json"), "fused_block_s"
                else:
                    pmc, pmc_op = os.path.join(REPO, "profiles", "r04_pmc_fused_block.json"), "fused_block"
            else:
                us_k, alg_bytes, kname = us.value, _lib.fused_mlp_bytes(B, d, f), _lib.FUSED_MLP_KERNEL
                pmc, pmc_op = os.path.join(REPO, "profiles", "r03_pmc_fused_mlp.json"), "fused_mlp"
        else:
            # rotate over every decoder layer's gate/up weights (2.2 GB >> 256 MiB Infinity
            # Cache) so each launch streams its weights from HBM, as inside a decode step
            X = torch.randn(B, d, device=dev).to(torch.bfloat16)
            Y = torch.empty(B, f, dtype=torch.bfloat16, device=dev)
            us_k = _lib.time_gate_up(X.data_ptr(), d, B, [lw.gate_up for lw in eng._dec], 2 * f, d, Y.data_ptr(),
                                     208, st)
            alg_bytes, kname = 2 * f * d * 2 + B * d * 2 + B * f * 2, _lib.GATE_UP_KERNEL
            pmc, pmc_op = os.path.join(REPO, "profiles", "r02_pmc_gate_up.json"), "gate_up"
        achieved = alg_bytes / (us_k * 1e-6) / 1e9
        traffic, tinfo = None, {"traffic_note": "PMC passes are at 8 rows"}
        if B == 8:
            # the PMC pass must be of the kernel this line prices, on the sources of this tree
            traffic, tinfo = _lib.pmc_traffic(pmc, pmc_op, kname)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                "frac": round(achieved / 8000.0, 4), "traffic": traffic, "kernel": kname,
                "algorithmic_bytes": int(alg_bytes), "avg_us": round(us_k, 2), **tinfo}
        step_us = C.c_float()
        _lib.check(L.t5g_time_decode_step(eng.h, 20, st, C.byref(step_us)), "time_step")
        roof["decode_step_us"] = round(step_us.value, 1)
        roof["decode_step_GBps"] = round(decode_weight_bytes(cfg) / (step_us.value * 1e-6) / 1e9, 1)

    # ---- C5: roofline of the codec's dominant kernel, gemm_f32_kernel (89 % of the decode's
    # device time, profiles/r06_c5_kernel_stats.csv), every GEMM launch of whole B x 751-frame
    # decodes between its own HIP events on the launching stream; 2 M N K flops against the
    # f32 MFMA peak (157.3 TFLOP/s: v_mfma_f32_32x32x2_f32 runs at the f32 vector rate)
    if rank == 0 and args.e2e:
        import ctypes as C
        Tc = n_tok_row
        g = torch.Generator(device="cpu").manual_seed(7)
        codes_c = torch.randint(0, codec.cfg.codebook_size, (B, Tc), generator=g, dtype=torch.int32).to(dev)
        wav_c = torch.empty(B, Tc * codec.cfg.hop_length, device=dev)
        st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        g_us, g_fl, g_n, d_us = C.c_float(), C.c_double(), C.c_int32(), C.c_float()
        rc = codec.L.xc2_time_gemms(codec.h, C.c_void_p(codes_c.data_ptr()), B, Tc, C.c_void_p(wav_c.data_ptr()), 5,
                                    st, C.byref(g_us), C.byref(g_fl), C.byref(g_n))
        if rc != 0:
            raise RuntimeError(f"xc2_time_gemms failed: {rc}")
        rc = codec.L.xc2_time_decode(codec.h, C.c_void_p(codes_c.data_ptr()), B, Tc, C.c_void_p(wav_c.data_ptr()), 5,
                                     st, C.byref(d_us))
        if rc != 0:
            raise RuntimeError(f"xc2_time_decode failed: {rc}")
        ach = g_fl.value / (g_us.value * 1e-6) / 1e12
        roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": 157.3, "unit": "TFLOP/s",
                "frac": round(ach / 157.3, 4), "traffic": None,
                "traffic_note": "compute-bound kernel: MFMA busy from the SQ_VALU_MFMA_BUSY_CYCLES pass "
                                "(profiles/r06_pmc_c5_codec.json: 0.72 of the SIMDs), HBM bytes not priced",
                "kernel": "gemm_f32_kernel (XCodec2 decoder GEMMs: fc, conv k7 / k3 as halo GEMMs, q|k|v, o, "
                          "fc1 + SiLU, fc2, head, iSTFT basis; 128 x 128 tiles, v_mfma_f32_32x32x2_f32)",
                "frames": f"{B} x {Tc}", "flops_per_decode": g_fl.value, "gemm_launches_per_decode": g_n.value,
                "gemm_us_per_decode": round(g_us.value, 1), "avg_us": round(g_us.value / max(1, g_n.value), 2),
                "decode_us": round(d_us.value, 1), "gemm_share_of_decode": round(g_us.value / d_us.value, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.e2e:
        r0 = rows[0]
        cpu = cpu_baseline(cfg, sd, (r0[2:2 + r0[0]], r0[2 + r0[0]:], r0[1]), n_tok_row)

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
                           "global_batch": B * world, "seq_len": wl_tp + 1 + n_tok_row,
                           "parallelism": f"dp{world} (utterance shards)"},
                "audio_tokens_per_s": round(value, 2), "wall_s_per_audio_s": round(dt_max / audio_s, 5),
                "samples_per_s": round(frames_all * hop / dt_max, 1),
                # rank 0's split of a step: generate() vs XCodec2Decoder.decode (synchronised
                # before and after the decode)
                "generate_ms_per_step": round((dt - codec_s[0]) / args.steps * 1e3, 2),
                "codec_decode_ms_per_step": round(codec_s[0] / args.steps * 1e3, 2),
                "codec_share": round(codec_s[0] / dt, 4),
                "roofline": roof,
            }
        else:
            prompt = f"T_p {wl_tp} (voice clone)" if wl_tp else "no prompt"
            desc = {"c2": "C2 single utterance", "c3": "C3 voice-clone", "c4": "C4 text-only",
                    "c3p10": "C3 voice-clone with a 10 s prompt"}[args.workload]
            mode = ("parity mode (drop-in default: exact-order kernels, reference RNG stream, host sync per "
                    "step, EOS accepted)" if args.parity else
                    "top-k 30/top-p 0.9/T 0.8" + (", EOS accepted when sampled" if args.natural_eos else ""))
            line = {
                "metric": "XCodec2 audio tokens/sec (whole node) + RTF, T5Gemma-TTS-2b-2b bs=8"
                          if args.workload == "c3" and not args.parity else
                          f"XCodec2 audio tokens/sec (whole node) + RTF, T5Gemma-TTS-2b-2b, BASELINE configs[{wl_cfg}]"
                          + (" parity mode" if args.parity else ""),
                "value": round(value, 2), "unit": "audio tokens/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "bf16",
                "data": "synthetic (seeded random 2b-2b weights, random text/prompt codes)",
                "config": {"workload": f"{desc}: 2b-2b bf16, {B} utterances/GPU, T_x {wl_tx}, {prompt}, "
                                       f"10 s target (751 tokens/utterance), {mode}"
                                       + (", eager attention (softcap 50)" if args.attn == "eager" else ""),
                           "global_batch": B * world, "seq_len": wl_tp + 1 + n_tok_row,
                           "parallelism": f"dp{world} (utterance shards)"},
                "rtf_audio_s_per_wall_s": round(value / 50.0, 3),
                "roofline": roof, "cpu_baseline": cpu,
                # persistent layer launches issued with the decode self attention inside (stage
                # S) during warm-up + timed steps -- graph-replayed steps count once, at capture;
                # 0: every layer's attention ran as its own launch
                "attn_in_block_launches": int(s_launches),
                "attn_in_block_mode": s_mode,   # 2 tail, 1 front (several passes past 3 slots / CU), 0 own launch
            }
            if not args.parity:
                # teacher-forced: the reference sampler on the reference CPU run's logits picks
                # the fast path's token (full-depth report of this tree's fast-path sources)
                from t5gemma_tts_amd import _lib
                line["fast_token_agreement"] = _lib.fast_token_agreement(
                    os.path.join(REPO, "profiles", "r06_parity_full.json"))
            if parity_line is not None:
                if cpu is not None:
                    parity_line["vs_cpu_baseline"] = round(parity_line["value"] / cpu["value"], 1)
                line["parity"] = parity_line
            if speed_lines:
                line["reference_speed_lines"] = speed_lines[-args.steps:]
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
