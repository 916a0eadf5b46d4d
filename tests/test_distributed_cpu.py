"""N>1 path on CPU: world_size-2 gloo runs of the utterance sharding --
broadcast of the request batch from rank 0, LPT shard assignment, per-rank generate,
all-gather back into request order. Same code as the RCCL path on GPUs."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import t5gemma_tts_amd  # noqa: F401
from t5gemma_tts_amd.distributed import assign_shards, pack_requests, run_sharded, unpack_requests


def test_assign_shards_balanced_and_deterministic():
    costs = [751, 300, 751, 120, 500, 500, 60, 900]
    s = assign_shards(costs, 2)
    assert sorted(i for sh in s for i in sh) == list(range(len(costs)))
    loads = [sum(costs[i] for i in sh) for sh in s]
    assert abs(loads[0] - loads[1]) <= max(costs)
    assert s == assign_shards(costs, 2)
    assert assign_shards(costs, 1) == [list(range(8))]
    capped = assign_shards([1] * 8, 4, max_per_rank=2)
    assert all(len(x) == 2 for x in capped)
    with pytest.raises(ValueError):
        assign_shards([1] * 9, 4, max_per_rank=2)
    # more ranks than utterances: empty shards allowed
    assert sum(len(x) for x in assign_shards([5, 4], 8)) == 2


def test_pack_roundtrip():
    rows = [[1, 2, 3], [], [7], list(range(100))]
    assert unpack_requests(pack_requests(rows)) == rows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = [[i] * (3 + i) for i in range(7)] if rank == 0 else None
        costs = [10 + (i * 37) % 11 for i in range(7)] if rank == 0 else None

        def generate(shard):   # stand-in for engine.generate: deterministic per utterance
            return [[v * 2 + rank * 0 for v in r] + [len(r)] for r in shard]

        out, mine = run_sharded(rows, costs, generate, torch.device("cpu"), max_per_rank=4, max_len=16)
        q.put((rank, out, mine))
    finally:
        dist.destroy_process_group()


def _seed_worker(rank, world, port, q):
    """bench.py's sharded step with the engine replaced by a recorder of the seeds and
    prompts each request is generated with."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from t5gemma_tts_amd.config import config_2b2b
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = config_2b2b()
        G = 4 * world
        rows = bench.request_rows(cfg, G, 40, 60) if rank == 0 else None
        costs = [r[1] for r in rows] if rank == 0 else None

        def generate(shard):
            return [[bench.request_seed(7, r[2]), r[2]] + r[3:3 + r[0]] for r in shard]

        out, _ = run_sharded(rows, costs, generate, torch.device("cpu"), max_per_rank=4, max_len=64)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_bench_seeds_independent_of_sharding(world):
    """A request samples with the same seed (and prompt) sharded over 2 or 8 ranks as in the
    unsharded batch: bench.py seeds by global request index."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from t5gemma_tts_amd.config import config_2b2b
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows = bench.request_rows(config_2b2b(), 4 * world, 40, 60)
    unsharded = [[bench.request_seed(7, r[2]), r[2]] + r[3:3 + r[0]] for r in rows]
    for _, out in res:
        assert out == unsharded
    assert len({o[0] for o in unsharded}) == len(unsharded)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_run_sharded_gloo(world):
    """7 utterances over `world` gloo ranks (8: the driver's node size, one rank with an
    empty shard): every rank ends with every utterance's output in request order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [[i * 2] * (3 + i) + [3 + i] for i in range(7)]
    mines = []
    for rank, out, mine in res:
        assert out == expect
        mines += mine
    assert sorted(mines) == list(range(7))


def test_launch_local_ranks_gloo(tmp_path):
    """bench.py --gpus N's launcher: N ranks under torch.distributed.run, each seeing
    WORLD_SIZE = N and its own rank through a gloo process group (the bench's N > 1 path
    reports n_gpus = dist.get_world_size())."""
    from t5gemma_tts_amd.distributed import launch_local_ranks
    script = tmp_path / "probe.py"
    script.write_text(
        "import os, sys, torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "t = __import__('torch').tensor([dist.get_rank() + 1])\n"
        "dist.all_reduce(t)\n"
        "open(os.path.join(sys.argv[1], f'rank{dist.get_rank()}'), 'w').write(f'{dist.get_world_size()} {int(t)}')\n"
        "dist.destroy_process_group()\n")
    rc = launch_local_ranks(str(script), [str(tmp_path)], 2, require_gpus=False, master_port=_free_port())
    assert rc == 0
    assert sorted(p.name for p in tmp_path.glob("rank*")) == ["rank0", "rank1"]
    assert all(p.read_text() == "2 3" for p in tmp_path.glob("rank*"))
    with pytest.raises(SystemExit):      # more ranks than GPUs: refused before launching
        launch_local_ranks(str(script), [str(tmp_path)], 4, require_gpus=True)
