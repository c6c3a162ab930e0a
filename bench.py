#!/usr/bin/env python3
"""bench.py — self-play board-steps/sec @ 800 sims/move, 8x8 Reversi (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

A step is one self-play ply of every game on the GPU (one 800-simulation MCTS search + one move
per game: SelfPlay.generate_games' loop body, self_play.py:80-101). The N = 1 workload is
BASELINE.json configs[1]: 4,096 games, 800 sims, batch 64, 6-block/64-filter ResNet (random init,
torch.manual_seed(0)), fp32-class evaluator (the reference's precision). Games that end restart
at once from the next seed of their slot, so every step is a steady-state ply.

Multi-GPU: one process per GPU, each with its own 4,096 games (weak scaling), no collective in
the data path. `--gpus N` without a launcher starts the N rank processes itself
(rvz.dist.spawn_ranks, before anything touches the GPU); under torchrun the ranks come from its
environment. Either way every rank checks that the process group's world size equals --gpus.

Printed on rank 0: one JSON line with value = committed plies of all ranks / max-over-ranks wall
time, the roofline of the dominant kernel (the NN trunk: executed and algorithmic FLOPs per
launch / in-situ duration), the search kernels' HBM roofline, the CPU baseline (the oracle port +
the same net on the host cores, bounded sample) and, at N = 1, the largest single-GPU config
(C3) and the 6x6 config (C5) measured the same way.
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "alphazero-reversi_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA16_PEAK_TFLOPS = 2500.0      # dense 16-bit (f16/bf16) MFMA peak, same source


PRESETS = {   # BASELINE.json configs
    # lanes: independent game lanes per GPU (same games; measured best per config)
    # c1: the reference's own plumbing case (one game, 100 sims, the ModelConfig default 5x128
    # net; config.py:14-15) on one GPU, with the CPU port on the same single game beside it.
    # fused: the fused self-play launch (k_play, one workgroup plays the game: no per-batch
    # launches, and the cross-game table serves positions earlier searches evaluated) — C1
    # 11.3k vs 8.9k pull-style (round 6, profiles/r06s_c1_fused_vs_pull.txt); C2 (r03o: +4-5%
    # over 2 lanes), C3 and C5 since round 4 (with the table)
    "c1": dict(games=1, sims=100, blocks=5, filters=128, board=8, lanes=1, fused=True),
    "c2": dict(games=4096, sims=800, blocks=6, filters=64, board=8, lanes=2, fused=True,
               play_group=-6),
    "c3": dict(games=32768, sims=800, blocks=10, filters=128, board=8, lanes=1, fused=True,
               play_group=-16),
    # per GPU, x8; a step = one self-play + training iteration (main_c4)
    "c4": dict(games=32768, sims=800, blocks=10, filters=128, board=8, lanes=1, steps=1,
               warmup=0, fused=True, play_group=-16),
    "c5": dict(games=16384, sims=400, blocks=6, filters=64, board=6, lanes=2, fused=True,
               play_group=-24),
}
# measured beside the headline in the default N = 1 line (the largest single-GPU config and the
# 6x6 variant); each is a full workload of its preset over the same --steps
SUB_CONFIGS = ("c3", "c5")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(PRESETS), default="c2",
                    help="BASELINE.json workload preset; explicit flags override it")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without torchrun bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed plies; the default spans a whole 8x8 game (every stage, endgame "
                         "included): the steady-state mix of continuous self-play")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--games", type=int, default=None, help="games per GPU")
    ap.add_argument("--sims", type=int, default=None)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--blocks", type=int, default=None)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--board", type=int, default=None)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--instrument-plies", type=int, default=2)
    ap.add_argument("--evals", choices=("table", "lazy", "memo", "reference"), default="table",
                    help="which NN rows are evaluated (the games are bit-identical in all four, "
                         "tests/test_gpu_memo.py, tests/test_gpu_table.py): 'reference' = every "
                         "leaf of every batch, as the reference does (it rebuilds the tree every "
                         "move, mcts.py:334); 'memo' = a leaf the game's previous search already "
                         "evaluated takes that output (rvz_search_memo); 'lazy' = memo, and each "
                         "search's last batch is left unevaluated (rvz_search_skip: nothing reads "
                         "its output in that search) and evaluated by a later search only if one "
                         "reaches its position; 'table' = lazy, and (fused launch only) an opening "
                         "position any game evaluated before takes the stored output "
                         "(rvz_play_table)")
    ap.add_argument("--table-slots", type=int, default=1 << 20,
                    help="--evals table: slots of the cross-game NN-output table (power of two)")
    ap.add_argument("--table-discs", type=int, default=14,
                    help="--evals table: positions with at most this many discs use the table")
    ap.add_argument("--skip-last-eval", action="store_true",
                    help="leave each search's last batch unevaluated (also without the memo)")
    ap.add_argument("--no-memo", action="store_true",
                    help="no NN-output memo (with --evals lazy: the last batch is still skipped "
                         "only if --skip-last-eval)")
    ap.add_argument("--no-evals-ab", "--no-memo-ab", dest="no_evals_ab", action="store_true",
                    help="skip the measurements of the other --evals modes beside the headline")
    ap.add_argument("--torch-bookkeeping", action="store_true",
                    help="per-ply counting / autoreset as torch ops instead of rvz_env_autoreset")
    ap.add_argument("--no-compact", action="store_true",
                    help="evaluate all n_games leaf rows of every batch instead of only the U "
                         "live leaves (mcts.py:544-623 evaluates U; rows of games whose traversal "
                         "ended on a terminal are dead)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="independent game lanes per GPU, one stream each "
                         "(rvz.LaneRunner); the games are the same as with one lane")
    ap.add_argument("--plies-per-graph", type=int, default=0,
                    help="plies captured into each lane's HIP graph (one replay plays them all; "
                         "--steps must be a multiple; 0: --fused one launch for all --steps, "
                         "else 1)")
    ap.add_argument("--fused", dest="fused", action="store_true", default=None,
                    help="the fused self-play launch (rvz_play): each workgroup plays its own "
                         "games, search + h2 evaluator + act + autoreset in one persistent kernel "
                         "(the preset decides by default: C2 and C5 fused, C1/C3/C4 not)")
    ap.add_argument("--no-fused", dest="fused", action="store_false",
                    help="the pull-style per-batch launches (k_step / trunk / heads per lane)")
    ap.add_argument("--play-gate", default="default",
                    help="--fused at 10x128: the per-XCD pass gate (rvz_play_gate): 'default' "
                         "(0.8 of an XCD's running workgroups / 400 us / late join 200 us), 'off', "
                         "or 'fraction,us,late_us'")
    ap.add_argument("--play-group", type=int, default=None,
                    help="--fused: rvz_play games_per_workgroup (> 0 static ownership; <= 0 the "
                         "task queue with groups of -N games, 0 the default)")
    ap.add_argument("--joined-lanes", action="store_true",
                    help="one graph for all lanes with a fork / join per ply (default: one "
                         "graph per lane on its own stream, no per-ply join; +0.9%% at C2)")
    ap.add_argument("--stamps-dump", default=None,
                    help="save lane 0's trunk stamp ring of the timed region (int64 [launch, "
                         "workgroup, 2]; tools/xcd_balance.py) to this .npy path")
    ap.add_argument("--no-stamps", action="store_true",
                    help="no device stamps in the timed graph (roofline from the isolated "
                         "back-to-back launches)")
    ap.add_argument("--sub-configs", default=None,
                    help="comma-separated presets measured beside the headline (default at one "
                         "rank with --config c2: c3,c5; 'none' for none)")
    ap.add_argument("--no-stagger", action="store_true",
                    help="start the timed window with every game at the same ply (all games begin "
                         "together and stay in lockstep) instead of game g at ply g mod 60 of its "
                         "game (one budgeted rvz_play launch before the warm-up): without the "
                         "stagger a window shorter than a whole game measures one game phase")
    ap.add_argument("--stagger-order", choices=("blocked", "interleaved"), default="blocked",
                    help="which ply of its game the stagger puts global game g of N at (L = 60 "
                         "on 8x8): blocked floor(g * L / N) (the games of a ply are consecutive, "
                         "so a game group of the fused launch plays one ply of the game), "
                         "interleaved g mod L; both put N / L games at every ply")
    ap.add_argument("--serial-ranks", action="store_true",
                    help="N > 1 ranks sharing one card (gloo rehearsals): the ranks take turns "
                         "in the timed region, each with the card to itself, so the per-rank "
                         "report compares the shards and value (sum / max) predicts N cards")
    ap.add_argument("--cpu-seconds", type=float, default=30.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL) for real multi-GPU runs; gloo to rehearse several ranks "
                         "on one device")
    ap.add_argument("--dry-run", action="store_true",
                    help="start the ranks, form the process group and shard the games, print the "
                         "line without running self-play (launcher check; no GPU needed)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="stored rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE) whose HBM bytes "
                         "per launch are quoted as roofline.traffic, labelled with their source")
    ap.add_argument("--train-steps", type=int, default=100,
                    help="c4: DDP optimizer steps per iteration (batch --train-batch per rank)")
    ap.add_argument("--train-batch", type=int, default=64,
                    help="c4: per-rank training batch (TrainingConfig.batch_size = 64)")
    args = ap.parse_args(argv)
    apply_preset(args, args.config)
    args.force_skip = args.skip_last_eval
    if args.no_memo:
        args.evals = "reference"
    set_evals(args, args.evals)
    return args


def set_evals(args, mode):
    """--evals mode -> the engine switches (skip_last_eval stays on if asked for explicitly)."""
    args.evals = mode
    args.no_memo = mode == "reference"
    args.skip_last_eval = mode in ("lazy", "table") or getattr(args, "force_skip", False)
    args.table = mode == "table"


def apply_preset(args, name):
    for k, v in dict(dict(steps=60, warmup=3, play_group=0), **PRESETS[name]).items():
        if getattr(args, k, None) is None:
            setattr(args, k, v)


_LINE_FD = None     # the real stdout: only the JSON line goes there (see quiet_stdout)


def quiet_stdout():
    """Keep stdout for the one JSON line: native libraries print banners to fd 1 (RCCL's version
    block at communicator init, gloo's connection log), so fd 1 is pointed at stderr for the rest
    of the process and emit() writes the line to the saved descriptor."""
    global _LINE_FD
    if _LINE_FD is None:
        sys.stdout.flush()
        _LINE_FD = os.dup(1)
        os.dup2(2, 1)


def emit(obj):
    line = (json.dumps(obj) + "\n").encode()
    if _LINE_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_LINE_FD, line)


def fail(msg: str, code: int = 2):
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)
    sys.exit(code)


# ------------------------------------------------------------------------------ ranks
def launch(args):
    """`--gpus N` with no launcher around us: start N rank processes of this same command line
    (children, before any GPU call in this process) and exit with their combined status. Under
    torchrun (WORLD_SIZE set) or for N = 1 this is a no-op and the process is itself a rank."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return
    from rvz import dist as rdist
    # no torch.cuda call here: the parent never touches HIP before it starts the ranks (a device
    # count can fall back to hipGetDeviceCount, i.e. initialise HIP in the parent); each rank's
    # setup() refuses a LOCAL_RANK without a device
    if args.dist_backend == "nccl" and not args.dry_run:
        avail = rdist.visible_gpu_count()    # environment / sysfs only
        if avail is not None and args.gpus > avail:
            fail(f"--gpus {args.gpus} but only {avail} GPU(s) visible (backend nccl)")
    rc = rdist.spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:])
    sys.exit(rc)


def setup(args):
    """Join the process group (also at one rank) and pick this rank's device. Returns
    (rank, world, device, backend); device is None for --dry-run."""
    import torch.distributed as tdist

    from rvz import dist as rdist
    rank, local_rank, world = rdist.env_rank_world()
    if world != args.gpus:
        fail(f"WORLD_SIZE {world} != --gpus {args.gpus}")
    backend = args.dist_backend if not args.dry_run else "gloo"
    device = None
    if not args.dry_run:
        n_dev = torch.cuda.device_count()
        if n_dev < 1:
            fail("no HIP device")
        if backend == "nccl" and local_rank >= n_dev:
            fail(f"LOCAL_RANK {local_rank} has no device ({n_dev} visible, backend nccl)")
        device = torch.device("cuda", local_rank % n_dev)   # gloo rehearsals may share one GPU
        torch.cuda.set_device(device)
    rdist.init(backend, always=True, device=device)
    if tdist.get_world_size() != args.gpus:
        fail(f"process group world {tdist.get_world_size()} != --gpus {args.gpus}")
    return rank, tdist.get_world_size(), device, tdist.get_backend()


def dry_run(args, rank, world, backend):
    """The launcher check without a GPU: ranks, process group, shards, and the per-rank report
    of a real line (rvz.dist.rank_report) over a stand-in timed region (a short host loop per
    rank, one "ply" per game of the shard), so the fields of the first N > 1 record are tested
    on the CPU."""
    import torch.distributed as tdist

    from rvz import dist as rdist
    shards = [None] * world
    a, b = rdist.shard_range(args.games * world, rank, world)
    tdist.all_gather_object(shards, (rank, a, b, os.getpid()))
    rdist.barrier()
    t0 = time.perf_counter()
    acc = 0
    for g in range(a, b):                    # stand-in work, proportional to the shard
        acc += sum(range(200)) + g
    dt = max(time.perf_counter() - t0, 1e-9)
    rep = rdist.rank_report(rank_fields(rank, a, b, b - a, dt, None, "cpu (dry run)",
                                        **stagger_fields(args)))
    if rank == 0:
        emit({"metric": "dry-run (launcher check)", "n_gpus": world, "rccl_world": world,
              "dist_backend": backend, "games_per_gpu": args.games,
              "global_games": args.games * world,
              "shards": [[r, a, b] for r, a, b, _ in shards],
              "pids": sorted({p for *_, p in shards}), "ranks": rep})
    tdist.destroy_process_group()


def rank_fields(rank, first_game, end_game, plies, seconds, rows_per_ply, device, **extra):
    """One rank's part of a line: its global game range, committed plies, timed seconds, its own
    rate and NN rows per ply (rvz.dist.rank_report gathers them and their spread), plus extra
    fields (the stagger's ply range, table hits per ply)."""
    return dict({"rank": rank, "games": [first_game, end_game], "plies": int(plies),
                 "seconds": round(seconds, 9),
                 "value": round(plies / seconds, 2) if seconds > 0 else None,
                 "nn_rows_per_ply": rows_per_ply, "device": str(device), "pid": os.getpid()},
                **extra)


def stagger_fields(args):
    """A rank's stagger, for its report: the plies its shard's games start at (every rank covers
    0..L-1) and the fewest / most games at one ply."""
    if args.no_stagger:
        return {"stagger_plies": None}
    L = args.board * args.board - 4
    bud = stagger_budget(torch.arange(args.games, dtype=torch.int64), L, args.games,
                         args.stagger_order)
    cnt = torch.bincount(bud.long(), minlength=L)
    return {"stagger_plies": [int(bud.min()), int(bud.max())],
            "stagger_games_per_ply": [int(cnt.min()), int(cnt.max())]}


# ------------------------------------------------------------------------------ measurement
# every k_play dispatch this process makes (stagger, warm-up, timed, the --evals modes and the
# sub-configs), timed with HIP events without system fence on its stream: the line's
# k_play_dispatches, whose per-instantiation averages are what rocprofv3 --stats averages over
# the same command (its timed subset is roofline.avg_ms_per_launch)
DISPATCHES = []      # (kernel instantiation, label, ms)


def play_kernel(board, filters):
    """rvz_play's kernel instantiation for a geometry (csrc/rvz_engine.hip rvz_play)."""
    return {(8, 64): "k_play<64, 2, 2, 4, 8, 2>", (8, 128): "k_play<128, 1, 2, 4, 8, 2>",
            (8, 256): "k_play<256, 1, 4, 4, 8, 1>",
            (6, 64): "k_play<64, 3, 2, 4, 6, 2>", (6, 128): "k_play<128, 1, 2, 3, 6, 2>"}[
        (board, filters)]


class Dispatches:
    """HIP-event pairs around k_play dispatches on one stream, resolved after a synchronise."""

    def __init__(self, kernel, device, n=512):
        from rvz import _lib
        self.kernel, self.timer, self.stream = kernel, _lib.Timer(2 * n), _lib.stream_handle(device)
        self.marks = []

    def __call__(self, label, fn):
        a = self.timer.record(self.stream)
        fn()
        self.marks.append((label, a, self.timer.record(self.stream)))

    def flush(self):
        for label, a, b in self.marks:
            DISPATCHES.append((self.kernel, label, self.timer.elapsed(a, b)))
        self.marks = []


def dispatch_summary():
    out = {}
    for k, label, ms in DISPATCHES:
        d = out.setdefault(k, {"n": 0, "total_ms": 0.0, "by_label": {}})
        d["n"] += 1
        d["total_ms"] += ms
        b = d["by_label"].setdefault(label, [0, 0.0])
        b[0] += 1
        b[1] += ms
    for d in out.values():
        d["avg_ms"] = round(d.pop("total_ms") / d["n"], 4)
        d["by_label"] = {k: {"n": n, "avg_ms": round(t / n, 4)} for k, (n, t) in d["by_label"].items()}
    return out or None


def stagger_budget(idx: torch.Tensor, L: int, n: int, order: str) -> torch.Tensor:
    """The ply of its game each game of a rank's shard starts the run at (the stagger launch's
    per-game budgets), from the game's index in the shard: blocked floor(i * L / n), interleaved
    i mod L."""
    bud = idx * L // n if order == "blocked" else idx % L
    return bud.to(torch.int32).contiguous()


def stagger(args, runners, tag, device, first_game=0):
    """Phase-neutral start: every game begins at the start position together,
    and 99.9% of 8x8 games last exactly 60 plies, so without this the games stay in lockstep and a
    window of fewer than 60 plies samples one game phase. One rvz_play launch with per-game ply
    budgets puts game i of the rank's n = --games at ply floor(i * L / n) (--stagger-order
    blocked, the default) or i mod L (interleaved) of its first game (L = S*S - 4 = 60 on 8x8,
    the length of a full game): from then on every ply of the run holds a whole game's mix of
    phases, as continuous self-play does (self_play.py:80-101), with n / L games at every ply
    either way. The index is the game's place in THIS rank's shard (indexing
    the global game space gave rank r only plies [60 r / W, 60 (r + 1) / W), so rank 0 played
    openings and rank W - 1 endgames): every rank holds the same mix of phases, whatever W.
    Blocked keeps the games of one fused-launch group (consecutive games) at one ply, as
    self-play's lockstep start does (one box: +0.8% / +0.9% in 20- / 60-ply windows,
    profiles/r04o_ab_stagger_order_*). Runs on each lane's engine (the pull-style presets
    continue from the state k_play leaves:
    tests/test_gpu_play_oracle.py::test_stagger_then_pull_style_equals_fused). Returns the mean
    plies per game it played."""
    L = args.board * args.board - 4
    disp = Dispatches(play_kernel(args.board, args.filters), device, n=len(runners))
    tot, n = 0, 0
    for r in runners:
        # a lane's seeds are args.seed + its global game indices (seed_base + lane offset)
        bud = stagger_budget(r.seeds - args.seed - first_game, L, args.games, args.stagger_order)
        tot += int(bud.sum().item())
        n += bud.numel()
        disp(f"{tag}stagger", lambda r=r, bud=bud: r.eng.play(
            r.evaluator, L - 1, r.temperature, r.seeds, r.seed_stride, r._plies, r._done,
            reset=r.autoreset, skip_last_eval=r.skip_last_eval,
            games_per_workgroup=getattr(r, "play_group", 0) if r.fused else 0, budget=bud))
    torch.cuda.synchronize(device)
    disp.flush()
    for r in runners:
        r.eng.check()
    return tot / max(1, n)


def play_gate_setting(text):
    """--play-gate 'off' | 'fraction,us,late_us' -> rvz_play_gate's arguments."""
    if text == "off":
        return (0.0, 0.0, 0.0)
    vals = [float(v) for v in text.split(",")]
    if len(vals) != 3:
        raise SystemExit("--play-gate: 'default', 'off' or 'fraction,us,late_us'")
    return tuple(vals)


def make_net(args, device):
    import rvz
    torch.manual_seed(0)
    return rvz.AlphaZeroNetwork(args.board, args.blocks, args.filters).to(device).eval()


def instrumented(run, eng, ev, plies):
    """Eager plies, first with the engine's launch timing on (a HIP event pair, without system
    fence, around every k_step / k_act on the launch stream), then as many with the kernels'
    own algorithmic-byte counters on (per-game counter writes slow the search kernels, so they
    are never on while timing; both cover the same launches per ply). Each ply is enqueued
    behind a device-side sleep so the host runs ahead of the GPU and the intervals bracket only
    the kernels. The NN is timed separately (back-to-back calls)."""
    from rvz import _lib
    nn_calls = 0

    def one_ply():
        nonlocal nn_calls
        torch.cuda.synchronize(eng.device)
        torch.cuda._sleep(int(60e6))        # ~25-30 ms of device time: the host enqueues meanwhile
        eng.search_begin()
        while eng.search_step():
            logits, value = ev(eng.leaf_x)
            eng.search_submit(logits, value, True)
            nn_calls += 1
        eng.act(run.temperature, apply=True)
        run.restart_finished(eng.get_state()[2])

    eng.timing_enable(True)
    trunk_pairs, timer = [], _lib.Timer(2 * plies * eng.n_batches)
    ev.trunk_events = (timer, trunk_pairs)
    for _ in range(plies):
        one_ply()
    ev.trunk_events = None
    t = eng.timing_read()
    eng.timing_enable(False)
    eng.stats_enable(True)
    for _ in range(plies):
        one_ply()
    st, act, _ = eng.stats_read()
    eng.stats_enable(False)
    nn_calls //= 2
    # evaluator: 10 back-to-back calls on the same leaf tensor between two events
    stream = torch.cuda.current_stream(eng.device)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev(eng.leaf_x)
    a.record(stream)
    for _ in range(10):
        ev(eng.leaf_x)
    b.record(stream)
    torch.cuda.synchronize(eng.device)
    ms = {"step": t["step"][0], "act": t["act"][0], "nn": a.elapsed_time(b) / 10}
    n = {"step": t["step"][1], "act": t["act"][1], "nn": nn_calls}
    ms["nn_trunk"] = isolated_trunk_ms(ev, eng.leaf_x)
    if trunk_pairs:   # the trunk launches of the timed plies, in their k_step -> trunk -> heads order
        ms["nn_trunk_in_ply"] = sum(timer.elapsed(i, j) for i, j in trunk_pairs) / len(trunk_pairs)
    return ms, n, {"step": st, "act": act}


def isolated_trunk_ms(ev, x):
    """The trunk launch alone: HIP events over 10 back-to-back full-batch launches."""
    stream = torch.cuda.current_stream(x.device)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev.trunk_only(x)
    a.record(stream)
    for _ in range(10):
        ev.trunk_only(x)
    b.record(stream)
    torch.cuda.synchronize(x.device)
    return a.elapsed_time(b) / 10


def env_bench(device, board=8, n=1 << 23, reps=10):
    """SURVEY §8d env microbench: the batched rules kernels over n HBM-resident positions (random
    playouts of 0..40 plies, so every game stage is present), timed with HIP events on the launch
    stream. Algorithmic bytes per board in this layout (u64 black, u64 white, int32[4] status):
    legal = 8 + 8 + 4 (side) + 8 (mask out) = 28 B; apply (make_move: legality, flips, auto-pass,
    terminal, winner) = 8 + 8 + 16 + 4 (square) in, 8 + 8 + 16 + 4 (ok) out = 72 B."""
    import rvz
    g = torch.Generator(device=device)
    g.manual_seed(1)
    B0 = 0x0000000810000000 if board == 8 else 0x0000000408000000
    W0 = 0x0000001008000000 if board == 8 else 0x0000000810000000
    black = torch.full((n,), B0, dtype=torch.int64, device=device)
    white = torch.full((n,), W0, dtype=torch.int64, device=device)
    status = torch.zeros(n, 4, dtype=torch.int32, device=device)
    status[:, 0] = 1
    plies = torch.randint(0, 41, (n,), generator=g, device=device)

    def lowest_bit(x):                                              # index of the lowest set bit
        lsb = x & -x
        f = lsb.to(torch.float64).abs()                             # powers of two are exact
        return torch.where(lsb < 0, torch.full_like(x, 63), torch.log2(f).round().long())

    def random_legal(mask):
        """A legal square per board: the first legal square at or after a random start (cyclic;
        not uniform, enough to spread the positions); -1 (pass) without one."""
        s0 = torch.randint(0, board * board, (n,), generator=g, device=device)
        hi = mask & ~((torch.ones_like(mask) << s0) - 1)
        pick = lowest_bit(torch.where(hi != 0, hi, mask))
        return torch.where(mask != 0, pick, torch.full_like(pick, -1)).int()

    for k in range(40):
        sq = random_legal(rvz.board_legal(black, white, status, board))
        live = (plies > k) & (status[:, 1] == 0) & (sq >= 0)
        sq = torch.where(live, sq, torch.full_like(sq, -2))        # -2: no move this round
        rvz.board_apply(black, white, status, sq, board)
    sq = random_legal(rvz.board_legal(black, white, status, board))
    copies = [(black.clone(), white.clone(), status.clone()) for _ in range(reps)]
    torch.cuda.synchronize(device)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {}
    rvz.board_legal(black, white, status, board)
    a.record()
    for _ in range(reps):
        rvz.board_legal(black, white, status, board)
    b.record()
    torch.cuda.synchronize(device)
    t = a.elapsed_time(b) / reps * 1e-3
    out["legal"] = {"boards_per_s": round(n / t), "alg_bytes_per_board": 28,
                    "achieved_GBs": round(n * 28 / t / 1e9, 1),
                    "frac": round(n * 28 / t / 1e9 / HBM_PEAK_GBS, 4), "avg_us": round(t * 1e6, 1)}
    a.record()
    for cb, cw, cs in copies:
        rvz.board_apply(cb, cw, cs, sq, board)
    b.record()
    torch.cuda.synchronize(device)
    t = a.elapsed_time(b) / reps * 1e-3
    out["apply"] = {"plies_per_s": round(n / t), "alg_bytes_per_ply": 72,
                    "achieved_GBs": round(n * 72 / t / 1e9, 1),
                    "frac": round(n * 72 / t / 1e9 / HBM_PEAK_GBS, 4), "avg_us": round(t * 1e6, 1)}
    out["boards"] = n
    return out


def cpu_baseline(args, net):
    """The oracle port (oracle/, literal reference semantics) + the same net in fp32 on the host
    cores, from the start position, over a bounded sample of the C2 workload."""
    from oracle import oracle as O
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cores = max(1, min(cores, os.cpu_count() or 1))
    torch.set_num_threads(cores)
    cpu_net = make_net(args, "cpu")
    cpu_net.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
    G = min(384, args.games)                  # ~10 s of C2 work on the GPU box's 16 host threads
    games = [O.new_game(args.board) for _ in range(G)]
    mts = [O.MT(args.seed + g) for g in range(G)]
    srch = O.Search(G, args.sims, args.batch, 1.0, bs=args.board)
    npol = args.board ** 2 + 1
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds and not all(g.over for g in games):
        srch.begin(games)
        while (r := srch.step()) is not None:
            leaves, _ = r
            x = torch.from_numpy(O.leaf_planes(leaves, args.board))
            with torch.no_grad():
                logits, value = cpu_net(x)
            srch.submit(torch.softmax(logits, 1).numpy(), value.numpy())
        vis = srch.visits()
        for g in range(G):
            if games[g].over:
                continue
            nd = O.action_needs_draw(vis[g], 1.0)
            idx, _, _ = O.action(vis[g], 1.0, mts[g].random_sample() if nd else 0.0)
            O.make_move(games[g], -1 if idx == npol - 1 else idx, args.board)
            steps += 1
    dt = time.perf_counter() - t0
    # env + tree only: same searches with a zero-cost evaluator (uniform priors, value 0)
    stub = O.Search(G, args.sims, args.batch, 1.0, bs=args.board)
    roots = [O.new_game(args.board) for _ in range(G)]
    u = np.full((G, npol), 1.0 / npol, np.float32)
    z = np.zeros(G, np.float32)
    t1 = time.perf_counter()
    stub.begin(roots)
    while stub.step() is not None:
        stub.submit(u, z)
    dt_stub = time.perf_counter() - t1
    # the same on ONE core (OpenMP of the oracle library set to 1 thread), 48 searches
    import ctypes
    one = None
    try:
        gomp = ctypes.CDLL("libgomp.so.1")
        gomp.omp_set_num_threads(1)
        G1 = min(48, G)
        stub1 = O.Search(G1, args.sims, args.batch, 1.0, bs=args.board)
        t2 = time.perf_counter()
        stub1.begin([O.new_game(args.board) for _ in range(G1)])
        while stub1.step() is not None:
            stub1.submit(u[:G1], z[:G1])
        one = {"value": G1 / (time.perf_counter() - t2), "unit": "board-steps/s", "cores": 1,
               "sample": f"{G1} first-ply searches, zero-cost evaluator, 1 thread"}
        gomp.omp_set_num_threads(cores)
    except OSError:
        pass
    return {"value": steps / dt, "unit": "board-steps/s", "cores": cores, "kind": "port",
            "sample": f"{G} games from the start position, {steps} plies in {dt:.1f}s, "
                      f"{args.sims} sims, oracle/ C search + {args.blocks}x{args.filters} net "
                      f"fp32 on {cores} host threads; one NN row per game per batch (the "
                      f"reference evaluates {args.batch} identical rows, mcts.py:582-594)",
            "env_tree_only": {"value": G / dt_stub, "unit": "board-steps/s", "cores": cores,
                              "sample": f"{G} first-ply searches, zero-cost evaluator"},
            "env_tree_only_1core": one}


def preset_shape(args):
    """True when the run's board, net and simulations are its preset's (the stored PMC passes and
    clock were measured on the presets; an override such as --filters 256 makes them another
    workload's)."""
    p = PRESETS[args.config]
    return all(getattr(args, k) == p[k] for k in ("board", "blocks", "filters", "sims") if k in p)


def stored_traffic(args, kernel, plies=None):
    """HBM bytes per launch of `kernel` from the committed PMC passes (--pmc), quoted only for the
    configuration they were measured on, with their source named. k_play: key "play" (C2's
    launches) or "play_<config>" (tools/pmc_play_traffic.py: C3, C5), each with its games per
    GPU and plies per launch; a launch of another length gets the bytes scaled by its plies, and
    the label says so. The search kernels' entries were measured at C2 (4,096 games)."""
    if not os.path.exists(args.pmc):
        return None, None
    try:
        pmc = json.load(open(args.pmc))
    except Exception:
        return None, None
    key = f"play_{args.config}" if kernel == "play" and args.config != "c2" else kernel
    ent = pmc.get(key, {})
    games = ent.get("games", 4096)
    if ent.get("config", "c2") != args.config or games != args.games or not preset_shape(args):
        return None, None
    b = ent.get("hbm_bytes_per_launch")
    if b is None:
        return None, None
    src = (f"{os.path.relpath(args.pmc, ROOT)}[{key}] "
           f"({ent.get('source') or pmc.get('source', 'stored rocprofv3 PMC passes')}"
           "; not measured in this run)")
    pl = ent.get("plies_per_launch")
    if plies and pl and plies != pl:
        b = round(b * plies / pl)
        src += f"; scaled from {pl}-ply to {plies}-ply launches"
    return b, src


def stored_pmc_clock(args):
    """The k_play entry's PMC-pass clock and launch time (GRBM_GUI_ACTIVE / 8 / duration, the
    same stored passes as its traffic; tools/pmc_play_traffic.py), for the configuration it was
    measured on, else None."""
    try:
        pmc = json.load(open(args.pmc))
    except Exception:
        return None
    key = f"play_{args.config}" if args.config != "c2" else "play"
    ent = pmc.get(key, {})
    if (ent.get("config", "c2") != args.config or ent.get("games", 4096) != args.games or
            not preset_shape(args)):
        return None
    if "clock_GHz" not in ent:
        return None
    return {"clock_GHz": ent["clock_GHz"], "ms_per_launch": ent.get("ms_per_launch_clock_pass"),
            "plies_per_launch": ent.get("plies_per_launch"),
            "source": f"{os.path.relpath(args.pmc, ROOT)}[{key}] (not measured in this run)"}


def selfplay(args, device, rank, world, full=True):
    """One workload (args: a resolved preset) on this rank: warm-up, the ply graph(s) captured,
    `steps` timed replays, the dominant kernel's in-situ roofline. With `full`, also the eager
    instrumented plies (search kernels' durations and algorithmic bytes). Returns a dict with
    the measured pieces (rank-local except value / dt, which are whole-job)."""
    import rvz
    from rvz import _lib
    from rvz import dist as rdist
    from rvz.measure import trunk_spans

    net = make_net(args, device)

    def make_ev():
        return rvz.LeafEvaluator(net, device=device)

    def make_eng(n):
        e = rvz.Engine(n, args.sims, args.batch, 1.0, board_size=args.board, device=device,
                       compact_leaves=not args.no_compact, memo=not args.no_memo)
        if args.table and args.fused:      # the table serves rvz_play (the fused launch) only
            e.table(args.table_slots, args.table_discs)
        if args.fused and args.play_gate != "default":
            e.play_gate(*play_gate_setting(args.play_gate))
        return e

    first_game = rank * args.games          # global game index space: rank r owns a shard
    if args.fused:
        # one rvz_play launch per replay: every workgroup plays its own games (search + h2
        # evaluator + act + autoreset); lanes are not needed (no per-batch launch chain)
        args.lanes = 1
        lane0 = run = rvz.SelfPlayRunner(make_eng(args.games), make_ev(), temperature=1.0,
                                         fused_softmax=True, autoreset=True,
                                         seed_base=args.seed + first_game,
                                         seed_stride=args.games * world,
                                         skip_last_eval=args.skip_last_eval, fused=True)
        run.play_group = args.play_group
        engines = [run.eng]
    elif args.lanes > 1:
        run = rvz.LaneRunner(make_eng, make_ev, args.games, args.lanes, temperature=1.0,
                             fused_softmax=True, autoreset=True,
                             seed_base=args.seed + first_game, seed_stride=args.games * world,
                             skip_last_eval=args.skip_last_eval)
        lane0 = run.runners[0]
        engines = [r.eng for r in run.runners]
    else:
        lane0 = run = rvz.SelfPlayRunner(make_eng(args.games), make_ev(), temperature=1.0,
                                         fused_softmax=True, autoreset=True,
                                         seed_base=args.seed + first_game,
                                         seed_stride=args.games * world,
                                         skip_last_eval=args.skip_last_eval,
                                         fused_bookkeeping=not args.torch_bookkeeping)
        engines = [run.eng]
    eng, ev = lane0.eng, lane0.evaluator    # instrumentation: one lane's kernels
    # --serial-ranks (N ranks rehearsed on ONE shared card): the ranks take turns from here to the
    # end of the timed region, each with the card to itself (stagger, warm-up and timed plies:
    # four persistent fused launches of 512 workgroups each on one card would time-slice and trip
    # the task queue's bounded wait), so the per-rank values compare the shards and sum / max
    # predicts N cards. Rank r waits for rounds 0..r-1 (ranks 0..r-1 done), runs, then joins the
    # remaining rounds: `world` barrier calls per rank in all.
    serial = args.serial_ranks and world > 1
    if serial:
        for _ in range(rank):
            rdist.barrier()
    run.start()
    tag = "" if getattr(args, "label", None) is None else args.label + "."
    stagger_plies = 0.0
    if not args.no_stagger:
        stagger_plies = stagger(args, [lane0] if args.fused else
                                (run.runners if args.lanes > 1 else [run]), tag, device,
                                first_game)

    # warmup: the first ply eager, then capture the ply graph with lane 0's trunk launches
    # stamping a ring of per-workgroup device wall-clock stamps, one row per launch (the heads
    # launch advances the ring's device counter): read after the timed replays, the dominant
    # kernel's duration over every lane-0 launch of the timed region
    graph_events = []
    cap_kw = {"free_run": not args.joined_lanes} if args.lanes > 1 else {}
    ppg = args.plies_per_graph or (args.steps if args.fused else 1)
    ppg = 1 if args.no_graph else ppg
    if args.steps % ppg:
        raise SystemExit(f"--steps {args.steps} is not a multiple of --plies-per-graph {ppg}")
    cap_kw["plies"] = ppg
    warm = max(args.warmup, 0 if args.no_graph else 1)
    wdisp = Dispatches(play_kernel(args.board, args.filters), device) if args.fused else None
    for i in range(warm):
        if i == 0 and not args.no_graph and not args.no_stamps and not args.fused:
            run.ply()
            grid = _lib.load().rvz_resnet_h2_grid(args.board, args.filters, eng.n_games)
            ring = max(1, args.steps) * eng.n_batches
            stamps = torch.zeros(ring, grid, 2, dtype=torch.int64, device=device)
            ctr = torch.zeros(1, dtype=torch.int32, device=device)
            ev.trunk_stamps = (stamps, ctr)
            run.capture(**cap_kw)
            graph_events = [stamps, ctr]
            ev.trunk_stamps = None
            continue
        if i == 0 and args.fused:
            # a first launch of the same size as the timed one (every warm-up and timed k_play
            # dispatch covers ppg plies)
            wdisp(f"{tag}warmup", lambda: run._body(ppg))
        elif args.fused:
            wdisp(f"{tag}warmup", run.ply)
        else:
            run.ply()
        if i == 0 and not args.no_graph:
            run.capture(**cap_kw)
    torch.cuda.synchronize(device)
    if wdisp is not None:
        wdisp.flush()
    # fused: every warm-up launch plays ppg plies; pull-style: one eager ply, then graph replays
    warm_plies = warm * ppg if args.fused else (1 + (warm - 1) * ppg if warm else 0)

    def rows_now():
        if args.fused:
            return sum(int(e.play_rows.item()) for e in engines)
        return sum(e.rows_total() for e in engines)

    rows0 = rows_now()
    tab0 = eng.table_stats.clone() if args.fused else None
    if graph_events:
        graph_events[1].zero_()            # the ring starts with the timed region
    if not serial:
        rdist.barrier()
    torch.cuda.synchronize(device)
    s0 = int(run.steps.item())
    n_rep = args.steps // ppg
    # fused: HIP events (no system fence) around every replay on its stream = the k_play
    # launches' durations (a replay is one launch)
    ftimer = _lib.Timer(2 * n_rep) if args.fused else None
    fstream = _lib.stream_handle(device)

    def timed():
        torch.cuda.synchronize(device)
        ta = time.perf_counter()
        enq = []
        for i in range(n_rep):                 # one replay plays ppg plies
            if ftimer is not None:
                ftimer.record(fstream)
            run.ply()
            if ftimer is not None:
                ftimer.record(fstream)
            enq.append(time.perf_counter())
        torch.cuda.synchronize(device)
        return ta, time.perf_counter(), enq

    t0, t1, t_enq = timed()
    if os.environ.get("RVZ_BENCH_ENQ"):
        iv = np.diff(np.array([t0] + t_enq)) * 1e3
        print(f"[bench] {args.config}: host enqueue ms per ply: {np.round(iv, 3).tolist()}; "
              f"device total {(t1 - t0) * 1e3:.1f} ms", file=sys.stderr)
    if serial:
        for _ in range(world - rank):      # this rank's turn is over; the later ranks' turns
            rdist.barrier()
    else:
        rdist.barrier()
    s1 = int(run.steps.item())
    rows1 = rows_now()
    tab_d = (eng.table_stats - tab0).tolist() if tab0 is not None else None
    for e in engines:
        e.check()
    total, dt, value = rdist.aggregate_rate(s1 - s0, t1 - t0)
    # leaf rows evaluated per NN call in the timed region (compaction on), else the full batch
    # (a last batch left to the memo, --evals lazy, is not an NN call)
    # (a one-batch search evaluates its batch even with skip_last_eval: Engine.search, rvz_play)
    calls_per_search = [e.n_batches - (1 if args.skip_last_eval and e.n_batches > 1 else 0)
                        for e in engines]
    nn_calls = args.steps * sum(calls_per_search)
    rows = rows1 - rows0 if not args.no_compact else nn_calls * eng.n_games
    # every rank's own plies, seconds, rate and rows per ply, and their spread (rank 0 prints)
    ranks = rdist.rank_report(
        rank_fields(rank, first_game, first_game + args.games, s1 - s0, t1 - t0,
                    round(rows / max(1, s1 - s0), 3), device, **stagger_fields(args),
                    table_hits_per_ply=(round(tab_d[0] / max(1, s1 - s0), 3)
                                        if tab_d is not None and args.table else None)),
        keys=("value", "seconds", "nn_rows_per_ply", "table_hits_per_ply"))
    trunk_live = None
    if graph_events:
        trunk_live = trunk_spans(graph_events[0], int(graph_events[1].item()))
        if args.stamps_dump and rank == 0:
            n_st = min(int(graph_events[1].item()), graph_events[0].shape[0])
            np.save(args.stamps_dump, graph_events[0][:n_st].cpu().numpy())

    ms = n = bytes_ = None
    if full:
        ms, n, bytes_ = instrumented(lane0, eng, ev, args.instrument_plies)
        eng.check()
    t_iso = ms["nn_trunk"] if ms else isolated_trunk_ms(ev, eng.leaf_x)

    # roofline of the dominant kernel, the NN trunk k_resnet_h2 (MFMA-bound): FLOPs per row x
    # rows per launch / launch duration. Executed = the 16-bit MFMA products the kernel issues (3
    # per fp32 product, stem K 27 -> 32, skipped edge taps); useful = SURVEY §8(d)'s 2 x MACs.
    fpr, upr = ev.mfma_flops_per_row(), ev.useful_flops_per_row()
    peak = MFMA16_PEAK_TFLOPS
    lane_games = eng.n_games
    iso = {"avg_ms_per_launch": round(t_iso, 4), "rows_per_launch": lane_games,
           "achieved": round(fpr * lane_games / (t_iso * 1e-3) / 1e12, 2),
           "frac": round(fpr * lane_games / (t_iso * 1e-3) / 1e12 / peak, 4),
           "useful_frac": round(upr * lane_games / (t_iso * 1e-3) / 1e12 / peak, 4),
           "timing": "HIP events over 10 back-to-back launches of one full batch, no other "
                     "lane running"}
    if ftimer is not None:
        durs = [ftimer.elapsed(2 * i, 2 * i + 1) for i in range(n_rep)]
        DISPATCHES.extend((play_kernel(args.board, args.filters), f"{tag}timed", d) for d in durs)
        t_tr, rows_tr = sum(durs) / n_rep, rows / n_rep
        timing = (f"in the timed region: all {n_rep} k_play launches (one per graph replay, "
                  f"{ppg} plies each), HIP events without system fence around each replay on "
                  "its stream")
    elif trunk_live:
        t_tr, rows_tr = trunk_live["ms"], trunk_live["rows"]
        timing = (f"in the timed region: all {trunk_live['launches']} trunk launches of lane 0, "
                  "first workgroup start to last end (device s_memrealtime stamps)")
    else:
        t_tr, rows_tr, timing = t_iso, lane_games, iso["timing"]
    ach = fpr * rows_tr / (t_tr * 1e-3) / 1e12
    ach_u = upr * rows_tr / (t_tr * 1e-3) / 1e12
    region = fpr * rows / (t1 - t0) / 1e12      # every lane's evaluated rows / timed wall time
    traffic, traffic_src = (stored_traffic(args, "play", ppg) if args.fused else
                            stored_traffic(args, "nn_trunk") if full else (None, None))
    roof = {"kernel": "k_play" if args.fused else ev.trunk_kernel_name, "bound": "mfma",
            "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4),
            "flops": "executed 16-bit MFMA FLOPs (mfma_flops_per_row x rows_per_launch)" +
                     ("; k_play's MFMA work is its h2 trunk passes (the search, act and FC "
                      "heads phases run in the same launch and count as time only)"
                      if args.fused else ""),
            "mfma_flops_per_row": fpr,
            "useful_flops_per_row": upr,
            "useful_achieved": round(ach_u, 2), "useful_frac": round(ach_u / peak, 4),
            "traffic": traffic, "traffic_source": traffic_src,
            "pmc_clock": stored_pmc_clock(args) if args.fused else None,
            "avg_ms_per_launch": round(t_tr, 4), "rows_per_launch": round(rows_tr, 1),
            "timing": timing, "isolated": iso,
            "live_rows_per_launch_timed": round(rows / nn_calls, 1),
            "timed_region_trunk_tflops": round(region, 2),
            "timed_region_trunk_frac": round(region / peak, 4),
            "timed_region_useful_frac": round(upr * rows / (t1 - t0) / 1e12 / peak, 4)}
    plies_local = s1 - s0
    if world > 1:
        ranks["timing"] = ("serial: the ranks took turns on a shared card (--serial-ranks)"
                           if args.serial_ranks else "concurrent")
    out = {"value": value, "dt": dt, "total": total, "roofline": roof, "net": net, "ranks": ranks,
           "eng": eng, "ev": ev, "lanes": args.lanes,
           "nn_rows_per_ply": round(rows / max(1, plies_local), 3),
           "table": ({"slots": args.table_slots, "max_discs": args.table_discs,
                      "hits_per_ply": round(tab_d[0] / max(1, plies_local), 3),
                      "inserts_per_ply": round(tab_d[1] / max(1, plies_local), 3)}
                     if tab_d is not None and args.table else None),
           "nn_calls_per_ply": sum(calls_per_search),
           # host time to enqueue the timed plies (graph replays): below ms_per_step, the device
           # never waits for the host
           "host_enqueue_ms_per_step": round((t_enq[-1] - t0) / max(1, args.steps) * 1e3, 3),
           "plies_per_graph": ppg,
           "play_group": args.play_group if args.fused else None,
           "play_gate": (args.play_gate if args.fused and args.filters >= 128 and args.board == 8
                         else None),
           "warmup_plies": {"stagger_mean": round(stagger_plies, 2),
                            "stagger": None if args.no_stagger else
                            f"game g of N at ply " + (
                                f"floor(g * {args.board ** 2 - 4} / N)"
                                if args.stagger_order == "blocked" else
                                f"g mod {args.board ** 2 - 4}") +
                            " of its game (one budgeted rvz_play launch)",
                            "after_stagger": warm_plies,
                            "total_mean": round(stagger_plies + warm_plies, 2)}}
    if full:
        kernels = {}
        for k in ("step", "act"):
            per_launch = bytes_[k] / max(1, n[k])
            kernels[k] = {"avg_us": ms[k] * 1e3, "launches_per_ply": n[k] // args.instrument_plies,
                          "alg_bytes_per_launch": per_launch,
                          "achieved_GBs": per_launch / (ms[k] * 1e-3) / 1e9}
        dom = max(("step", "act"),
                  key=lambda k: kernels[k]["avg_us"] * kernels[k]["launches_per_ply"])
        roof["avg_ms_per_call"] = round(ms["nn"], 4)
        roof["avg_ms_in_eager_plies"] = (round(ms["nn_trunk_in_ply"], 4)
                                         if "nn_trunk_in_ply" in ms else None)
        straffic, ssrc = stored_traffic(args, dom)
        a = kernels[dom]["achieved_GBs"]
        out["search_roofline"] = {"kernel": f"k_{dom}", "bound": "hbm", "achieved": round(a, 2),
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(a / HBM_PEAK_GBS, 5), "traffic": straffic,
                                  "traffic_source": ssrc}
        out["kernels"] = {k: {kk: round(vv, 3) for kk, vv in v.items()}
                          for k, v in kernels.items()}
        # the env + tree path as a whole — the search kernels' own algorithmic-byte
        # counters per committed board-step (lane 0's instrumented plies) x the job's rate
        bps = (bytes_["step"] + bytes_["act"]) / max(1, args.instrument_plies * eng.n_games)
        out["path_roofline"] = {
            "what": "env + tree (k_step + k_act algorithmic bytes per board-step, from the "
                    "kernels' counters) x board-steps/s", "bound": "hbm",
            "bytes_per_board_step": round(bps, 1), "achieved": round(value * bps / 1e9, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(value * bps / 1e9 / HBM_PEAK_GBS, 5)}
        # the NN must dominate for "roofline" to name the trunk (else the search kernel)
        search_ms = kernels[dom]["avg_us"] * kernels[dom]["launches_per_ply"] / 1e3
        out["nn_dominant"] = t_iso * n["nn"] / max(1, args.instrument_plies) > search_ms
    return out


def sub_config(base, name, device, rank, world):
    """A preset measured beside the headline: the same harness, its own net and engines."""
    a = copy.copy(base)
    for k in ("games", "sims", "blocks", "filters", "board", "lanes", "fused", "play_group"):
        setattr(a, k, None)
    a.config = name
    a.stamps_dump = None
    a.label = name
    apply_preset(a, name)
    r = selfplay(a, device, rank, world, full=False)
    out = {"value": round(r["value"], 2), "unit": "board-steps/s",
           "ms_per_step": round(r["dt"] / a.steps * 1e3, 3), "steps": a.steps,
           "workload": f"{name}: {a.games} games/GPU x {a.sims} sims, {a.blocks}x{a.filters} "
                       f"ResNet, {a.board}x{a.board}, {a.lanes} lane(s)",
           "games_per_gpu": a.games, "sims": a.sims, "nn": f"{a.blocks}x{a.filters}",
           "board": a.board, "lanes": a.lanes, "nn_rows_per_ply": r["nn_rows_per_ply"],
           "warmup_plies": r["warmup_plies"], "table": r["table"], "roofline": r["roofline"],
           "play_gate": r.get("play_gate")}
    del r
    torch.cuda.empty_cache()
    return out


def main_c4(args, rank, world, device):
    """BASELINE.json config 4: self-play + training, one process per GPU (rvz.pipeline;
    reference pipeline.py:114-150). A bench step is one ITERATION: every game of the rank from
    the start position to its end (60 plies, captured ply graph), the device records turned into
    training arrays, then --train-steps DDP steps whose gradient all-reduce runs over RCCL. value
    = board-steps of all ranks / max-over-ranks wall time of the K iterations, training included.
    The process group exists even at one rank (backend nccl = RCCL), so DDP's all-reduce runs
    at every N."""
    import torch.distributed as tdist

    from rvz import dist as rdist
    from rvz.pipeline import SelfPlayTrainer

    net = make_net(args, device)
    n_params = sum(p.numel() for p in net.parameters())
    spt = SelfPlayTrainer(net, args.games, args.sims, args.batch, 1.0, 1.0, seed=args.seed,
                          train_steps=args.train_steps, train_batch=args.train_batch,
                          graph=not args.no_graph, compact_leaves=not args.no_compact,
                          memo=not args.no_memo, fused=args.fused,
                          table_slots=args.table_slots if args.table else 0,
                          table_discs=args.table_discs)
    spt.runner.play_group = args.play_group
    # warm-up (untimed): two plies (fused: one launch; else one eager ply and the ply graph
    # captured), two DDP steps on stand-in data
    run = spt.runner
    run.start()
    if args.fused:
        run.play_record(2)
    else:
        run.ply()
        if not args.no_graph:
            run.capture()
    g = torch.Generator(device=device).manual_seed(rank)
    warm = {"states": (torch.rand(4 * args.train_batch, 3, args.board, args.board, device=device,
                                  generator=g) > 0.6).float(),
            "policy_targets": torch.rand(4 * args.train_batch, args.board ** 2 + 1,
                                         device=device, generator=g),
            "value_targets": torch.zeros(4 * args.train_batch, 1, device=device)}
    spt.trainer.train_epoch(warm, seed=0, max_steps=2, local_data=True)
    spt.trainer.sync_buffers()
    spt.evaluator.refresh()
    for _ in range(args.warmup):
        spt.run_iteration()
    rdist.barrier()
    torch.cuda.synchronize(device)
    rows0 = int(spt.eng.play_rows.item()) if args.fused else 0
    hits0 = int(spt.eng.table_stats[0].item()) if args.fused else 0
    t0 = time.perf_counter()
    its = [spt.run_iteration() for _ in range(args.steps)]
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    rows_sp = (int(spt.eng.play_rows.item()) - rows0) if args.fused else 0
    rdist.barrier()
    steps = sum(r["board_steps"] for r in its)
    total, dt, value = rdist.aggregate_rate(steps, t1 - t0)
    sp_s = rdist.reduce_max(sum(r["selfplay_s"] for r in its))
    tr_s = rdist.reduce_max(sum(r["train_s"] for r in its))
    n_train = sum(r["steps"] for r in its)
    sp_rate = rdist.reduce_sum(steps) / sp_s
    a0 = rank * args.games
    loc = rank_fields(rank, a0, a0 + args.games, steps, t1 - t0,
                      round(rows_sp / max(1, steps), 3) if args.fused else None, device)
    loc["selfplay_s"] = round(sum(r["selfplay_s"] for r in its), 4)
    loc["train_s"] = round(sum(r["train_s"] for r in its), 4)
    ranks = rdist.rank_report(loc, keys=("value", "seconds", "selfplay_s", "train_s",
                                         "nn_rows_per_ply"))
    # the gradient all-reduce alone: one flat fp32 bucket of every parameter (what DDP's single
    # 25 MB bucket carries), HIP events on the current stream, 20 back-to-back collectives
    buf = torch.randn(n_params, device=device)
    tdist.all_reduce(buf)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rdist.barrier()
    a.record()
    for _ in range(20):
        tdist.all_reduce(buf)
    b.record()
    torch.cuda.synchronize(device)
    ar_ms = rdist.reduce_max(a.elapsed_time(b) / 20)
    ev, eng = spt.evaluator, spt.eng
    if args.fused:
        # the dominant kernel is the iteration's one k_play launch (self-play of every game);
        # its duration is the self-play phase's device-synchronised wall time
        t_tr = sp_s / max(1, args.steps) * 1e3
        rows_l = rows_sp / max(1, args.steps)
        timing = ("the iteration's k_play launch: rows it evaluated (its own counter) over the "
                  "self-play phase's device-synchronised wall time")
    else:   # the trunk in isolation: HIP events over 10 back-to-back launches
        t_tr = isolated_trunk_ms(ev, eng.leaf_x)
        rows_l = eng.n_games
        timing = "HIP events over 10 back-to-back full-batch launches after the timed region"
    ach = ev.mfma_flops_per_row() * rows_l / (t_tr * 1e-3) / 1e12
    uach = ev.useful_flops_per_row() * rows_l / (t_tr * 1e-3) / 1e12
    roof = {"kernel": "k_play" if args.fused else ev.trunk_kernel_name, "bound": "mfma",
            "achieved": round(ach, 2), "peak": MFMA16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / MFMA16_PEAK_TFLOPS, 4),
            "mfma_flops_per_row": ev.mfma_flops_per_row(),
            "useful_flops_per_row": ev.useful_flops_per_row(),
            "useful_frac": round(uach / MFMA16_PEAK_TFLOPS, 4), "traffic": None,
            "avg_ms_per_launch": round(t_tr, 4), "rows_per_launch": round(rows_l, 1),
            "timing": timing}
    spt.eng.check()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, net)
    if rank == 0:
        out = {
            "metric": f"self-play board-steps/sec @ {args.sims} sims/move, "
                      f"{args.board}x{args.board} Reversi",
            "value": round(value, 2), "unit": "board-steps/s", "n_gpus": world,
            "rccl_world": tdist.get_world_size(), "dist_backend": tdist.get_backend(),
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u64 rules + f32 NN (fp32 as 2-part f16 split on MFMA); fp32 training",
            "data": "synthetic (start position, per-game seeds, random-init net trained in the "
                    "loop)",
            "config": {"workload": f"c4: self-play + training; {args.games} games/GPU x "
                                   f"{args.sims} sims, {args.blocks}x{args.filters} ResNet, "
                                   f"{args.board}x{args.board}; a step = one iteration "
                                   f"(whole games, then {args.train_steps} DDP steps)",
                       "games_per_gpu": args.games, "global_games": args.games * world,
                       "sims": args.sims, "batch": args.batch,
                       "nn": f"{args.blocks}x{args.filters}",
                       "train_steps_per_iter": args.train_steps,
                       "train_batch_per_rank": args.train_batch,
                       "parallelism": f"games sharded x{world}; DDP x{world} "
                                      f"({tdist.get_backend()})"},
            "selfplay_board_steps_per_s": round(sp_rate, 2),
            "selfplay": ("fused: one rvz_play launch per iteration with device records, memo, "
                         "deferred last batch and the cross-game table (a new generation per "
                         "weight refresh)" if args.fused else "pull-style ply graph"),
            "table": ({"hits_per_ply": round((int(spt.eng.table_stats[0].item()) - hits0) /
                                            max(1, steps), 3),
                       "nn_rows_per_ply": round(rows_sp / max(1, steps), 3)}
                      if args.fused and args.table else None),
            "selfplay_s": round(sp_s, 3), "train_s": round(tr_s, 3), "ranks": ranks,
            "ms_per_train_step": round(tr_s / max(1, n_train) * 1e3, 3),
            "allreduce": {"backend": tdist.get_backend(), "world": world,
                          "bytes": n_params * 4, "ms": round(ar_ms, 4),
                          "algbw_GBs": round(n_params * 4 / (ar_ms * 1e-3) / 1e9, 1)},
            "train_loss": [round(r["train/loss"], 4) for r in its],
            "roofline": roof, "cpu_baseline": cpu,
        }
        emit(out)
    tdist.destroy_process_group()


def main():
    args = parse()
    launch(args)                               # exits here when it started the ranks itself
    quiet_stdout()
    rank, world, device, backend = setup(args)
    if args.dry_run:
        return dry_run(args, rank, world, backend)
    if args.config == "c4":
        return main_c4(args, rank, world, device)
    import torch.distributed as tdist

    r = selfplay(args, device, rank, world, full=True)
    value, dt, net = r["value"], r["dt"], r["net"]
    evals_ab = {}
    if not args.no_evals_ab and not args.no_compact:
        # the same workload with the other --evals modes: the games are identical
        # (tests/test_gpu_memo.py, test_bench_configuration_at_full_size_plays_the_plain_games), so
        # the row differences are the memo's hits and the deferred last batches
        for mode in ("reference", "memo", "lazy", "table"):
            if mode == args.evals:
                continue
            a = copy.copy(args)
            set_evals(a, mode)
            a.stamps_dump = None
            a.label = f"evals_{mode}"
            o = selfplay(a, device, rank, world, full=False)
            evals_ab[mode] = {"value": round(o["value"], 2),
                              "ms_per_step": round(o["dt"] / args.steps * 1e3, 3),
                              "nn_rows_per_ply": o["nn_rows_per_ply"],
                              "speedup_of_headline": round(value / o["value"], 4)}
            del o
            torch.cuda.empty_cache()
    subs = {}
    names = (args.sub_configs.split(",") if args.sub_configs not in (None, "none") else
             (SUB_CONFIGS if args.sub_configs is None and world == 1 and args.config == "c2"
              else ()))
    for name in names:
        if name and name != args.config:
            subs[name] = sub_config(args, name, device, rank, world)
    envb = env_bench(device, args.board) if rank == 0 else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, net)

    if rank == 0:
        roof = r["roofline"]
        nn_dom = r["nn_dominant"]
        out = {
            "metric": f"self-play board-steps/sec @ {args.sims} sims/move, "
                      f"{args.board}x{args.board} Reversi",
            "value": round(value, 2), "unit": "board-steps/s",
            "n_gpus": world, "rccl_world": tdist.get_world_size(), "dist_backend": backend,
            "steps": args.steps, "warmup": args.warmup,
            "warmup_plies": r["warmup_plies"],
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u64 rules + f32 NN (fp32 as 2-part f16 split on MFMA)",
            "data": "synthetic (start position, per-game seeds, random-init net)",
            "config": {"workload": f"{args.config}: {args.games} games/GPU x {args.sims} sims, "
                                   f"{args.blocks}x{args.filters} ResNet, {args.board}x{args.board}",
                       "games_per_gpu": args.games, "global_games": args.games * world,
                       "sims": args.sims, "batch": args.batch,
                       "nn": f"{args.blocks}x{args.filters}",
                       "nn_kernel": ("k_play (h2_pass + heads_fc16 inside the fused self-play "
                                     "launch)" if args.fused else "rvz_resnet_fwd_h2"),
                       "fused": args.fused, "plies_per_graph": r["plies_per_graph"],
                       "graph": not args.no_graph, "lanes": args.lanes,
                       "lane_graphs": ("joined" if args.joined_lanes else "free")
                       if args.lanes > 1 else None,
                       "evals": args.evals, "skip_last_eval": args.skip_last_eval,
                       "memo": not args.no_memo,
                       "table": ({"slots": args.table_slots, "max_discs": args.table_discs}
                                 if args.table and args.fused else None),
                       "parallelism": f"games sharded x{world}"},
            "nn_rows_per_ply": r["nn_rows_per_ply"],
            "ranks": r["ranks"],
            "table": r["table"],
            "nn_calls_per_ply": r["nn_calls_per_ply"],
            "host_enqueue_ms_per_step": r["host_enqueue_ms_per_step"],
            "evals_ab": evals_ab or None,
            "nn_rows_frac_of_reference": (round(r["nn_rows_per_ply"] /
                                                max(1e-9, evals_ab["reference"]["nn_rows_per_ply"]),
                                                4) if "reference" in evals_ab else None),
            # the dominant kernel of a ply (by time per ply) carries "roofline"
            "roofline": roof if nn_dom else r["search_roofline"],
            "search_roofline" if nn_dom else "nn_roofline":
                r["search_roofline"] if nn_dom else roof,
            "kernels": r["kernels"],
            "path_roofline": r["path_roofline"],
            "env_roofline": envb,
            "configs": subs or None,
            "k_play_dispatches": dispatch_summary(),
            "cpu_baseline": cpu,
        }
        emit(out)
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
