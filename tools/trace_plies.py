"""Eager self-play plies at C2 for a roctx marker timeline (the C-ABI's ranges: rvz.search.step,
rvz.eval.trunk / .heads, rvz.search.submit, rvz.act, rvz.env.*; csrc/rvz_trace.h):

    RVZ_ROCTX=1 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/trace -o run \
        -- python tools/trace_plies.py [plies] [games]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

plies = int(sys.argv[1]) if len(sys.argv) > 1 else 3
games = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
eng = rvz.Engine(games, 800, 64, compact_leaves=True)
run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=42)
run.start()
for _ in range(plies):
    run.ply()
torch.cuda.synchronize()
eng.check()
print("plies", plies, "steps", int(run.steps.item()))
