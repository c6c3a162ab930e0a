"""The multi-GPU harness logic on CPU with gloo, world_size 2 (rvz/dist.py, bench.py's
aggregation): shards partition the global game space, seeds follow the global index, and the
whole-job rate is sum(units) / max(seconds)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_total, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-reversi_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from rvz import dist as rd
    assert rd.init("gloo")
    a, b = rd.shard_range(n_total, rank, world)
    seeds = rd.shard_seeds(42, n_total, rank, world)
    # each rank "plays" (b - a) plies in a rank-dependent time
    total, dt, rate = rd.aggregate_rate(b - a, 1.0 + rank)
    rd.barrier()
    q.put((rank, a, b, seeds.tolist(), total, dt, rate))
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [8192, 4097])
def test_two_rank_sharding_and_aggregation(n_total):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    covered = []
    for rank, a, b, seeds, total, dt, rate in res:
        covered += list(range(a, b))
        assert seeds == [42 + g for g in range(a, b)]
        assert total == n_total and dt == 2.0 and rate == n_total / 2.0
    assert covered == list(range(n_total))


def test_single_rank_is_identity():
    import rvz.dist as rd
    assert rd.shard_range(10, 0, 1) == (0, 10)
    assert rd.reduce_max(3.0) == 3.0 and rd.reduce_sum(3.0) == 3.0
    with pytest.raises(ValueError):
        rd.shard_range(10, 2, 2)
