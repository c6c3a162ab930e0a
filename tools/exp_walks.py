"""Select-phase walk counters per ply over whole games (instrumented build, -DRVZ_WALK_STATS):
walks from the root, tree levels read, known-terminal hits (memory / register fast path) and new
terminals, per game and launch; with k_step's mean launch time beside them.

    RVZ_LIB=tools/_ab/librvz_walks.so CONFIG=c2 python tools/exp_walks.py
(build: hipcc ... -DRVZ_WALK_STATS -shared -o tools/_ab/librvz_walks.so csrc/*.hip)"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402
from rvz import _lib  # noqa: E402

CFG = {"c2": (4096, 800, 8, 6, 64), "c5": (16384, 400, 6, 6, 64)}[os.environ.get("CONFIG", "c2")]
G, S, BS, NB, F = CFG
PLIES = int(os.environ.get("PLIES", 62 if BS == 8 else 34))
lib = _lib.load()
lib.rvz_walk_stats.argtypes = [C.c_int32, C.POINTER(C.c_int64)]
lib.rvz_walk_times.argtypes = [C.c_int32, C.POINTER(C.c_int64)]
CATS = ("expand", "walk_levels", "term_backup_mem", "fast_path", "leaf")
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(BS, NB, F).cuda().eval()
eng = rvz.Engine(G, S, 64, 1.0, board_size=BS, compact_leaves=True)
run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=42)
run.start()
out10 = (C.c_int64 * 10)()
out11 = (C.c_int64 * 11)()
torch.cuda.synchronize()
lib.rvz_walk_stats(G, out10)                       # zero
lib.rvz_walk_times(G, out11)
rows = []
for p in range(PLIES):
    eng.timing_enable(True)
    run.ply()
    torch.cuda.synchronize()
    t = eng.timing_read()
    eng.timing_enable(False)
    assert lib.rvz_walk_stats(G, out10) == 0
    assert lib.rvz_walk_times(G, out11) == 0
    s, mx = list(out10[:5]), list(out10[5:])
    launches0 = eng.n_batches
    tslow = {k: round(out11[i] / launches0) for i, k in enumerate(CATS)}
    tmean = {k: round(out11[5 + i] / launches0) for i, k in enumerate(CATS)}
    launches = eng.n_batches                        # k_step launches per ply
    rows.append({"ply": p, "step_us": round(t["step"][0] * 1e3, 1),
                 "walks_per_game_launch": round(s[0] / G / launches, 2),
                 "levels_per_walk": round(s[1] / max(1, s[0]), 2),
                 "term_mem": round(s[2] / G / launches, 2), "term_fast": round(s[3] / G / launches, 2),
                 "new_term": round(s[4] / G / launches, 3),
                 "max_walks_game_ply": mx[0], "max_levels_game_ply": mx[1],
                 "cycles_per_launch_slowest_game": tslow, "cycles_per_launch_mean_game": tmean})
print(json.dumps({"config": CFG, "plies": rows}))
