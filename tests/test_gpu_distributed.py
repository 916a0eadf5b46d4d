"""The sharded engine path (distributed.run_sharded) on the real engine: two
ranks sharing one MI355X (gloo collectives, each rank its own engine and weight replica)
broadcast rank 0's requests, generate their LPT shards and all-gather the ids. The gathered
ids must equal one unsharded run of the same utterances and seeds, in the fast mode and in
parity mode (bitwise logits there)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _requests(cfg, n=6, seed=21):
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        tx = int(rng.integers(4, 20))
        x = rng.integers(3, cfg.backbone.text_vocab_size - 1, size=tx).tolist()
        tp = int(rng.integers(0, 10)) if i % 2 else 0
        y = rng.integers(0, cfg.audio_vocab_size, size=tp).tolist() + ([cfg.y_sep_token] if tp else [])
        tgt = len(y) + int(rng.integers(10, 40))
        rows.append([500 + i, len(x), tgt] + x + y)   # [seed, T_x, tgt_y_len, x..., y...]
    return rows


def _generate(eng, rows, parity):
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    utts = [Utterance(x=r[3:3 + r[1]], y=r[3 + r[1]:], tgt_y_len=r[2]) for r in rows]
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, stop_repetition=3)
    out = eng.generate(utts, p, seeds=[r[0] for r in rows], parity=parity)
    return [g.tolist() for g in out["gen"]]


def _engine():
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import T5GemmaTTSEngine
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    return cfg, T5GemmaTTSEngine(cfg, synthetic_weights(cfg, 7), device="cuda:0", max_batch=4, max_text=32,
                                 max_audio=128, max_gen=64)


def _worker(rank, world, port, parity, q, backend="gloo"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    import t5gemma_tts_amd  # noqa: F401
    from t5gemma_tts_amd.distributed import run_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        cfg, eng = _engine()
        rows = _requests(cfg, n=6 if world > 1 else 4) if rank == 0 else None
        costs = [r[2] for r in rows] if rank == 0 else None
        comm = torch.device("cuda:0") if backend == "nccl" else torch.device("cpu")
        out, mine = run_sharded(rows, costs, lambda shard: _generate(eng, shard, parity), comm,
                                max_per_rank=4, max_len=64)
        q.put((rank, out, mine))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("parity", [False, True])
def test_sharded_engine_equals_unsharded(parity):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, parity, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg, eng = _engine()
    rows = _requests(cfg)
    single = []
    for i in range(0, len(rows), 4):
        single += _generate(eng, rows[i:i + 4], parity)
    mines = []
    for rank, out, mine in res:
        assert out == single, (rank, parity)
        mines += mine
    assert sorted(mines) == list(range(len(rows)))
    assert all(len(r[2]) > 0 for r in res)   # both ranks generated a shard


@pytest.mark.timeout(300)
def test_run_sharded_rccl_world1():
    """bench.py's RCCL path (backend "nccl" = RCCL, collectives on cuda tensors) at world
    size 1: the broadcast / all-gather plumbing over the real communicator returns the
    unsharded ids."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), False, q, "nccl"))
    p.start()
    rank, out, mine = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    cfg, eng = _engine()
    rows = _requests(cfg, n=4)
    assert out == _generate(eng, rows, False)
    assert sorted(mine) == list(range(len(rows)))
