"""Utterance sharding over the GPUs of one node.

One process per GPU (torchrun), a full weight replica per GPU; the unit of work is the
utterance, so there is no per-step collective. The only exchanges are:
  1. rank 0 packs the request batch (token ids, lengths, sampler params, seeds) into one
     int64 tensor and broadcasts it (RCCL over xGMI on GPUs, gloo in the CPU tests);
  2. after generation, an all-gather of each rank's generated ids (padded int32 rows +
     lengths) so rank 0 can return results in request order.

Assignment is length-bucketed and balanced (longest-processing-time-first over the
per-utterance token budget), the inference-time analogue of the reference's
DistributedDynamicBatchSampler (steps/trainer_utils.py:210-660).
"""
from __future__ import annotations

import os
import subprocess
import sys
from typing import Callable, List, Sequence, Tuple

import torch
import torch.distributed as dist


def launch_local_ranks(script: str, argv: Sequence[str], n: int, require_gpus: bool = True,
                       master_port: int = 0) -> int:
    """Run ``script argv`` as ``n`` ranks of one node under torch.distributed.run (one
    process per GPU) and return the launcher's exit code. Called by a process that has
    not touched the GPU; the ranks are children (never an exec). ``require_gpus``: fail
    before launching when fewer than n GPUs are visible (``device_count`` does not
    initialise the GPU on this image)."""
    if n < 1:
        raise ValueError("n must be >= 1")
    if require_gpus:
        have = torch.cuda.device_count()
        if have < n:
            raise SystemExit(f"{os.path.basename(script)}: {n} ranks requested but only {have} GPU(s) visible")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this driver
    port = master_port or int(env.get("BENCH_MASTER_PORT", "29512"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), script] + list(argv)
    return subprocess.call(cmd, env=env)


def assign_shards(costs: Sequence[float], world: int, max_per_rank: int = 0) -> List[List[int]]:
    """LPT assignment: utterances sorted by cost (desc, index asc for ties) go to the
    least-loaded rank (lowest rank on ties). Deterministic; every rank computes the same
    answer. ``max_per_rank`` > 0 caps the batch per rank (engine max_batch)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = len(costs)
    if max_per_rank and n > world * max_per_rank:
        raise ValueError(f"{n} utterances exceed {world} ranks x max_batch {max_per_rank}")
    order = sorted(range(n), key=lambda i: (-float(costs[i]), i))
    load = [0.0] * world
    shards: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        cand = [r for r in range(world) if not max_per_rank or len(shards[r]) < max_per_rank]
        r = min(cand, key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += float(costs[i])
    return [sorted(s) for s in shards]


def pack_requests(rows: Sequence[Sequence[int]]) -> torch.Tensor:
    """Ragged int rows -> one int64 tensor [n, 1 + n_rows... ] = header(n, offsets) + data."""
    n = len(rows)
    lens = [len(r) for r in rows]
    flat = [v for r in rows for v in r]
    return torch.tensor([n] + lens + flat, dtype=torch.int64)


def unpack_requests(t: torch.Tensor) -> List[List[int]]:
    v = t.tolist()
    n = int(v[0])
    lens = v[1:1 + n]
    out, p = [], 1 + n
    for L in lens:
        out.append([int(x) for x in v[p:p + L]])
        p += L
    return out


def broadcast_rows(rows, device, src: int = 0) -> List[List[int]]:
    """Broadcast ragged int rows from ``src`` (two collectives: size, payload)."""
    rank = dist.get_rank()
    if rank == src:
        payload = pack_requests(rows).to(device)
        size = torch.tensor([payload.numel()], dtype=torch.int64, device=device)
    else:
        size = torch.zeros(1, dtype=torch.int64, device=device)
    dist.broadcast(size, src)
    if rank != src:
        payload = torch.empty(int(size.item()), dtype=torch.int64, device=device)
    dist.broadcast(payload, src)
    return unpack_requests(payload.cpu())


def gather_rows(local: Sequence[Sequence[int]], local_index: Sequence[int], n_total: int, device,
                max_len: int) -> List[List[int]]:
    """All-gather each rank's generated rows back into request order (every rank gets
    the full list). Rows are padded to ``max_len`` int32 + a length and an index column."""
    world = dist.get_world_size()
    cap_t = torch.tensor([len(local_index)], dtype=torch.int64, device=device)
    dist.all_reduce(cap_t, op=dist.ReduceOp.MAX)
    cap = max(1, int(cap_t.item()))
    buf = torch.full((cap, max_len + 2), -1, dtype=torch.int32, device=device)
    for j, (idx, row) in enumerate(zip(local_index, local)):
        if len(row) > max_len:
            raise ValueError("row longer than max_len")
        buf[j, 0], buf[j, 1] = int(idx), len(row)
        if row:
            buf[j, 2:2 + len(row)] = torch.tensor(list(row), dtype=torch.int32, device=device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out: List[List[int]] = [None] * n_total  # type: ignore
    for p in parts:
        for r in p.cpu().tolist():
            if r[0] >= 0:
                out[r[0]] = r[2:2 + r[1]]
    if any(o is None for o in out):
        raise RuntimeError("gather lost an utterance")
    return out


def run_sharded(rows: Sequence[Sequence[int]], costs: Sequence[float], generate: Callable[[List[List[int]]],
                List[List[int]]], device, max_per_rank: int, max_len: int) -> Tuple[List[List[int]], List[int]]:
    """Broadcast rank 0's request rows, run ``generate`` on this rank's shard, all-gather.
    Returns (results in request order, this rank's indices)."""
    rows = broadcast_rows(rows if dist.get_rank() == 0 else None, device)
    cost_rows = broadcast_rows([[int(c) for c in costs]] if dist.get_rank() == 0 else None, device)[0]
    shards = assign_shards(cost_rows, dist.get_world_size(), max_per_rank)
    mine = shards[dist.get_rank()]
    local = generate([rows[i] for i in mine]) if mine else []
    return gather_rows(local, mine, len(rows), device, max_len), mine
