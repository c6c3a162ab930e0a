"""k_step / k_act mean launch time per ply over whole games (eager, engine timing events), to see
how the endgame's known-terminal re-walks load the search kernels.

    CONFIG=c5 python tools/exp_kstep_plies.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

CFG = {"c2": (4096, 800, 8, 6, 64), "c5": (16384, 400, 6, 6, 64)}[os.environ.get("CONFIG", "c5")]
G, S, BS, NB, F = CFG
PLIES = int(os.environ.get("PLIES", 66 if BS == 8 else 38))
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(BS, NB, F).cuda().eval()
eng = rvz.Engine(G, S, 64, 1.0, board_size=BS, compact_leaves=True)
run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=42)
run.start()
out = []
for p in range(PLIES):
    eng.timing_enable(True)
    t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t[0].record()
    run.ply()
    t[1].record()
    torch.cuda.synchronize()
    tm = eng.timing_read()
    eng.timing_enable(False)
    out.append({"ply": p, "ply_ms": round(t[0].elapsed_time(t[1]), 3),
                "step_us": round(tm["step"][0] * 1e3, 1), "act_us": round(tm["act"][0] * 1e3, 1)})
tot_ply = sum(o["ply_ms"] for o in out)
tot_step = sum(o["step_us"] * eng.n_batches for o in out) / 1e3
print(json.dumps({"config": CFG, "step_share": round(tot_step / tot_ply, 4), "plies": out}))
