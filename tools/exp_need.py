"""How many rows of each NN batch need an evaluation at all (need[g] > 0)? C2 self-play, eager,
63 plies (3 warm-up + 60). Rows with need == 0 are games whose traversal ended on a terminal."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

G = int(os.environ.get("GAMES", 4096))
BS = int(os.environ.get("BOARD", 8))
SIMS = int(os.environ.get("SIMS", 800))
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(BS, 6, 64).cuda().eval()
ev = rvz.LeafEvaluator(net)
eng = rvz.Engine(G, SIMS, 64, 1.0, board_size=BS, device=torch.device("cuda"))
tot, live, per_ply = [], [], []


def evaluator(x):
    live.append(int((eng.need > 0).sum()))
    tot.append(G)
    return ev(x)


run = rvz.SelfPlayRunner(eng, evaluator, temperature=1.0, fused_softmax=True, autoreset=True,
                         seed_base=42)
for p in range(63):
    n0 = len(live)
    run.ply()
    torch.cuda.synchronize()
    if p >= 3:
        per_ply.append(round(sum(live[n0:]) / sum(tot[n0:]), 4))
live, tot = live[3 * eng.n_batches:], tot[3 * eng.n_batches:]
print(json.dumps({"games": G, "frac_rows_needed": round(sum(live) / sum(tot), 4),
                  "per_ply": per_ply}))
