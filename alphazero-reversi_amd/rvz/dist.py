"""Multi-GPU sharding of self-play: one process per GPU, games partitioned by rank.

Self-play shards embarrassingly: every game, tree and RNG stream is independent, so
rank r owns games [r*N/W, (r+1)*N/W) of the global game index space and runs its own engine on
its own device with no data-path collective. The only cross-rank traffic is the benchmark's
timing reduction (MAX over ranks) and the final sum of committed plies. The reference has no
counterpart (mcts.py:220-226,446-542 only chunks one batch over local replicas sequentially).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import time
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def env_rank_world() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from torchrun's environment (1 process when unset)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, stop) of the global game index space owned by `rank`."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard_seeds(seed_base: int, n_total: int, rank: int, world: int) -> torch.Tensor:
    """Per-game seeds of this rank's shard: global game g is always seeded seed_base + g."""
    a, b = shard_range(n_total, rank, world)
    return torch.arange(a, b, dtype=torch.int64) + seed_base


def init(backend: str = None, always: bool = False, device=None) -> bool:
    """Initialise the default process group when launched with several ranks (torchrun or
    spawn_ranks); with ``always`` also for a single rank (a one-member group, so a bench line's
    world size comes from the group itself). False when no group was created."""
    _, _, world = env_rank_world()
    if dist.is_initialized():
        return True
    if world <= 1 and not always:
        return False
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"   # nccl == RCCL on ROCm
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        if world > 1:
            raise RuntimeError("MASTER_PORT must be set for a multi-rank group")
        os.environ["MASTER_PORT"] = str(free_port())
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", str(world))
    dist.init_process_group(backend=backend,
                            device_id=device if backend == "nccl" and device is not None
                            else None)
    return True


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpu_count() -> Optional[int]:
    """GPUs this process may use, from the environment and sysfs only (no HIP call, so a launcher
    parent stays uninitialised): the entries of HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES when set, else the KFD topology nodes with a GPU (nonzero
    gfx_target_version). None when neither says."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = os.environ.get(var)
        if val is not None:
            return len([x for x in val.split(",") if x.strip() and x.strip() != "-1"])
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(root)
    except OSError:
        return None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(root, d, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "gfx_target_version" and int(v) != 0:
                        n += 1
                        break
        except (OSError, ValueError):
            continue
    return n


def spawn_ranks(n: int, cmd: List[str], poll_s: float = 0.2, kill_after_s: float = 10.0) -> int:
    """Run ``cmd`` as ``n`` rank processes on this node (one per GPU): each child gets RANK =
    LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = n and a shared 127.0.0.1 rendezvous, and
    inherits stdout/stderr. Children are separate processes started with Popen (never an exec of
    this one), so call this before anything touches the GPU. Returns 0 when every rank exits 0;
    otherwise the first failure's code (a signal maps to 1) after terminating the other ranks.
    If the launcher itself is interrupted (KeyboardInterrupt, or SIGTERM, which is turned into
    one here), every child still alive is terminated, then killed after ``kill_after_s``, so no
    rank keeps holding a GPU or the rendezvous port. This is what `bench.py --gpus N` runs when
    no launcher (torchrun) set WORLD_SIZE."""
    if n < 1:
        raise ValueError("need at least one rank")
    port = str(free_port())
    procs = []

    def on_term(signum, frame):
        raise KeyboardInterrupt(f"signal {signum}")

    installed, old = False, None
    try:
        old = signal.signal(signal.SIGTERM, on_term)
        installed = True                       # old may be None (a handler set outside Python)
    except ValueError:                         # not the main thread: no handler, finally still runs
        pass
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
            procs.append(subprocess.Popen(cmd, env=env))
        rc, alive = 0, list(procs)
        while alive:
            for p in list(alive):
                code = p.poll()
                if code is None:
                    continue
                alive.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    for q in alive:            # the exact children of this launcher, nothing else
                        q.terminate()
            if alive:
                time.sleep(poll_s)
        return rc
    finally:
        # a second SIGTERM during the cleanup must not raise out of it and strand live ranks
        # (ADVICE r04, r05): ignored from the first statement of the cleanup until every child is
        # gone, then the old handler is back (SIG_DFL if it was not a Python one)
        if installed:
            signal.signal(signal.SIGTERM, signal.SIG_IGN)
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.terminate()
        deadline = time.time() + kill_after_s
        for p in live:
            try:
                p.wait(max(0.0, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        if installed:
            signal.signal(signal.SIGTERM, old if old is not None else signal.SIG_DFL)


def _device_for_backend():
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def reduce_max(x: float) -> float:
    if not dist.is_initialized():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device_for_backend())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(x: float) -> float:
    if not dist.is_initialized():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device_for_backend())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def gather(obj) -> list:
    """Every rank's `obj` (picklable), in rank order, on every rank ([obj] without a group)."""
    if not dist.is_initialized():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def rank_report(local: dict, keys=("value", "seconds", "nn_rows_per_ply")) -> dict:
    """Per-rank fields of a multi-rank measurement and their spread: `local` is this rank's dict
    (its own rank, game range, plies, seconds, ...); returns {"per_rank": [dict per rank],
    "spread": {key: {min, max, argmin, argmax, max_over_min}}} on every rank, so a slow or
    unbalanced rank shows in the one JSON line instead of hiding in sum / max aggregates."""
    ranks = gather(dict(local))
    spread = {}
    for k in keys:
        vals = [(r.get(k), i) for i, r in enumerate(ranks) if isinstance(r.get(k), (int, float))]
        if not vals:
            continue
        lo, hi = min(vals), max(vals)
        spread[k] = {"min": lo[0], "max": hi[0], "argmin": lo[1], "argmax": hi[1],
                     "max_over_min": round(hi[0] / lo[0], 4) if lo[0] else None}
    return {"per_rank": ranks, "spread": spread}


def aggregate_rate(local_units: float, local_seconds: float) -> Tuple[float, float, float]:
    """Whole-job throughput: (sum of units over ranks, max seconds over ranks, units/s)."""
    total = reduce_sum(local_units)
    dt = reduce_max(local_seconds)
    return total, dt, total / dt if dt > 0 else float("nan")
