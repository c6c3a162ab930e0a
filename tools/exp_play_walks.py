"""Where a game's turn in k_play's search phase goes (instrumented build:
tools/ab_lib_build.sh walks "-DRVZ_WALK_STATS"; RVZ_LIB=tools/_ab/librvz_walks.so): mean shader
clocks per game step of the expand, the select's walk levels / terminal backups / register fast
path / leaf, act + autoreset, and the whole step, over PLIES plies of the C2 workload.
GAMES (4096), SIMS (800), PLIES (20), WARM (3), GROUP (-6), TABLE (1: bench.py's cross-game
table), STAGGER (1: bench.py's blocked stagger first)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

G = int(os.environ.get("GAMES", 4096))
S = int(os.environ.get("SIMS", 800))
PLIES = int(os.environ.get("PLIES", 20))
WARM = int(os.environ.get("WARM", 3))
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
eng = rvz.Engine(G, S, 64, memo=True)
if int(os.environ.get("TABLE", 1)):        # bench.py's default --evals table
    eng.table(1 << 20, 14)
run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=42,
                         skip_last_eval=True, fused=True)
run.play_group = int(os.environ.get("GROUP", -6))
run.start()
if int(os.environ.get("STAGGER", 1)):      # bench.py's blocked phase stagger
    bud = ((run.seeds - 42) * 60 // G).to(torch.int32).contiguous()
    eng.play(run.evaluator, 59, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
             reset=True, skip_last_eval=True, games_per_workgroup=run.play_group, budget=bud)
lib = rvz.load()
lib.rvz_play_walk_read.argtypes = [C.c_int32, C.c_void_p]
buf = np.zeros((G, 9), dtype=np.uint64)
for _ in range(WARM):
    run.ply()
torch.cuda.synchronize()
lib.rvz_play_walk_read(G, buf.ctypes.data)
eng.play(run.evaluator, PLIES, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
         reset=True, skip_last_eval=True, games_per_workgroup=run.play_group)
torch.cuda.synchronize()
assert lib.rvz_play_walk_read(G, buf.ctypes.data) == 0
b = buf.astype(np.float64)
steps = b[:, 8].sum()
names = ("table_lookup", "walk_levels", "term_backup_mem", "fast_path", "leaf")
out = {"games": G, "plies": PLIES, "steps_per_game_ply": round(steps / G / PLIES, 2)}
per = {n: round(b[:, i].sum() / steps) for i, n in enumerate(names)}
per["expand"] = round(b[:, 5].sum() / steps)
per["act_autoreset"] = round(b[:, 6].sum() / steps)
per["step_total"] = round(b[:, 7].sum() / steps)
per["unattributed"] = per["step_total"] - sum(v for k, v in per.items() if k != "step_total")
out["cycles_per_step"] = per
print(json.dumps(out))
