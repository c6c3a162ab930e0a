"""bench.py's multi-rank entry point on CPU (gloo): `bench.py --gpus N` with no launcher starts N
rank processes itself (rvz.dist.spawn_ranks), every rank checks the process group's world size
against --gpus, and rank 0 alone prints the one JSON line (VERDICT r02 'next' item 1; the
reference's only multi-device code, mcts.py:446-542, chunks batches over local replicas)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env.update(extra)
    return env


def _run(args, env=None, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=env or _env())


@pytest.mark.parametrize("n,games", [(2, 1024), (3, 100)])
def test_bench_gpus_n_starts_n_ranks(n, games):
    r = _run(["--gpus", str(n), "--dist-backend", "gloo", "--dry-run", "--games", str(games)])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]   # native logs go to stderr
    assert len(lines) == 1, r.stdout            # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["rccl_world"] == n and d["dist_backend"] == "gloo"
    assert d["global_games"] == n * games
    # contiguous shards of the global game space, one per rank, in rank order
    assert d["shards"] == [[k, k * games, (k + 1) * games] for k in range(n)]
    assert len(d["pids"]) == n                  # n distinct processes


def test_bench_world4_line_carries_per_rank_fields():
    """a line of N > 1 ranks must show each rank's own plies,
    seconds, rate, rows per ply and game range, and their spread (a slow rank would otherwise
    hide in sum-over-max). The dry run fills the same report (rvz.dist.rank_report) from a
    stand-in timed region."""
    n, games = 4, 96
    r = _run(["--gpus", str(n), "--dist-backend", "gloo", "--dry-run", "--games", str(games)])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    rep = d["ranks"]
    per = rep["per_rank"]
    assert [p["rank"] for p in per] == list(range(n))
    assert [p["games"] for p in per] == [[k * games, (k + 1) * games] for k in range(n)]
    assert len({p["pid"] for p in per}) == n
    for p in per:
        assert p["plies"] == games and p["seconds"] > 0
        assert abs(p["value"] - p["plies"] / p["seconds"]) <= 1e-3 * p["value"]
    for k in ("value", "seconds"):
        sp = rep["spread"][k]
        vals = [p[k] for p in per]
        assert sp["min"] == min(vals) and sp["max"] == max(vals)
        assert per[sp["argmin"]][k] == sp["min"] and per[sp["argmax"]][k] == sp["max"]
        assert sp["max_over_min"] >= 1.0


def test_bench_single_rank_forms_a_group_of_one():
    r = _run(["--dry-run", "--games", "64"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["rccl_world"] == 1 and d["shards"] == [[0, 0, 64]]


def test_bench_refuses_world_size_other_than_gpus():
    # a launcher (torchrun) set WORLD_SIZE: the rank must match --gpus or exit non-zero
    r = _run(["--gpus", "2", "--dry-run"], env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "WORLD_SIZE 1 != --gpus 2" in r.stderr


def test_spawn_ranks_propagates_a_failing_rank():
    sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
    from rvz.dist import spawn_ranks
    code = ("import os, sys, time\n"
            "r = int(os.environ['RANK'])\n"
            "assert os.environ['WORLD_SIZE'] == '3' and os.environ['LOCAL_RANK'] == str(r)\n"
            "sys.exit(3) if r == 1 else time.sleep(0 if r == 0 else 60)\n")
    assert spawn_ranks(3, [sys.executable, "-c", code]) == 3      # rank 2 is terminated
    ok = "import os; assert os.environ['MASTER_ADDR'] == '127.0.0.1'"
    assert spawn_ranks(2, [sys.executable, "-c", ok]) == 0


def test_launcher_parent_never_touches_hip(monkeypatch):
    """`bench.py --gpus N` (backend nccl) must start its ranks without any
    torch.cuda call in the parent (a device count may initialise HIP through hipGetDeviceCount,
    and a HIP-initialised parent must not fork the rank processes)."""
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
    import bench
    from rvz import dist as rdist

    def refuse(*a, **k):
        raise AssertionError("the launcher parent called into torch.cuda")

    for name in ("device_count", "is_available", "init", "_lazy_init", "current_device",
                 "set_device", "synchronize"):
        monkeypatch.setattr(torch.cuda, name, refuse)
    started = []
    monkeypatch.setattr(rdist, "spawn_ranks", lambda n, cmd: started.append((n, cmd)) or 0)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    args = bench.parse(["--gpus", "8", "--dist-backend", "nccl"])
    with pytest.raises(SystemExit) as ex:
        bench.launch(args)
    assert ex.value.code == 0 and started and started[0][0] == 8
    assert not torch.cuda.is_initialized()
    # more ranks than visible GPUs: refused from the environment alone, still without HIP
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    with pytest.raises(SystemExit) as ex:
        bench.launch(bench.parse(["--gpus", "4"]))
    assert ex.value.code == 2 and len(started) == 1
    assert not torch.cuda.is_initialized()


def test_visible_gpu_count_from_environment(monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
    from rvz.dist import visible_gpu_count
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3,5")
    assert visible_gpu_count() == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert visible_gpu_count() == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    n = visible_gpu_count()                      # sysfs (no GPU in this container: 0 or None)
    assert n is None or n >= 0


def test_spawn_ranks_terminates_children_when_the_launcher_is_killed(tmp_path):
    """a SIGTERM to the launcher must not leave rank processes holding GPUs or the
    rendezvous port."""
    import signal
    import time
    pkg = os.path.join(ROOT, "alphazero-reversi_amd")
    child = ("import os, time; open(os.path.join(%r, 'pid%%s' %% os.environ['RANK']), 'w')"
             ".write(str(os.getpid())); time.sleep(120)" % str(tmp_path))
    launcher = ("import sys; sys.path.insert(0, %r); from rvz.dist import spawn_ranks; "
                "sys.exit(spawn_ranks(2, [sys.executable, '-c', %r], kill_after_s=5))"
                % (pkg, child))
    p = subprocess.Popen([sys.executable, "-c", launcher], env=_env())
    pids = []
    t0 = time.time()
    while len(pids) < 2 and time.time() - t0 < 60:
        pids = [int(f.read_text()) for f in tmp_path.glob("pid*") if f.read_text()]
        time.sleep(0.1)
    assert len(pids) == 2, "ranks did not start"
    p.send_signal(signal.SIGTERM)
    p.wait(timeout=60)
    for pid in pids:
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)


@pytest.mark.parametrize("order", ["blocked", "interleaved"])
@pytest.mark.parametrize("n,L,world", [(4096, 60, 1), (16384, 32, 1), (32768, 60, 8), (1000, 60, 2),
                                       (512, 60, 4)])
def test_stagger_budgets_are_phase_neutral_per_rank(order, n, L, world):
    """bench.py's stagger: within EVERY rank's shard each ply of
    the game holds n / L games (floor or ceil), so every rank plays the same mix of phases
    (indexing the global game space gave rank r only plies [L r / W, L (r + 1) / W)); blocked
    keeps every fused-launch group of 6 consecutive games within two adjacent plies. The budgets
    come from the game's index in its shard (bench.stagger: seeds - seed - first_game)."""
    import torch
    import bench
    seed = 42
    for r in range(world):
        seeds = torch.arange(r * n, (r + 1) * n, dtype=torch.int64) + seed   # the rank's lane seeds
        bud = bench.stagger_budget(seeds - seed - r * n, L, n, order)
        counts = torch.bincount(bud.long(), minlength=L)
        assert counts.numel() == L and int(counts.min()) >= n // L and int(counts.max()) <= -(-n // L)
        assert int(bud.min()) == 0 and int(bud.max()) == L - 1
        if order == "blocked":
            groups = bud[: n // 6 * 6].view(-1, 6)
            assert int((groups.max(1).values - groups.min(1).values).max()) <= 1


def test_bench_world4_dry_run_ranks_cover_every_ply():
    """The world-4 dry run reports each rank's stagger: every rank's shard starts games at plies
    0..59 with 8 or 9 games per ply (512 games / 60 plies) — no rank holds one phase."""
    r = _run(["--gpus", "4", "--dist-backend", "gloo", "--dry-run", "--games", "512"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    for p in d["ranks"]["per_rank"]:
        assert p["stagger_plies"] == [0, 59], p
        assert p["stagger_games_per_ply"] == [8, 9], p


def test_stored_pmc_quoted_only_for_the_preset_shape():
    """bench.py quotes the committed PMC traffic and clock (profiles/pmc_traffic.json) only for
    the workload they were measured on: the preset's games, board, net and simulations. An
    override (--filters 256, --sims 400, --games ...) leaves roofline.traffic null."""
    import bench
    a = bench.parse(["--config", "c3"])
    b, src = bench.stored_traffic(a, "play", plies=20)
    assert b and "play_c3" in src
    assert bench.stored_pmc_clock(a) is not None
    for extra in (["--filters", "256"], ["--sims", "400"], ["--blocks", "5"], ["--games", "1024"]):
        o = bench.parse(["--config", "c3"] + extra)
        assert bench.stored_traffic(o, "play", plies=20) == (None, None), extra
        assert bench.stored_pmc_clock(o) is None, extra
