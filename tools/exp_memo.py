"""How many NN rows of a search repeat a position the SAME game evaluated in its previous search?
(CPU, the oracle's literal search + the fp32 torch net; VERDICT r02 'next' item 5.)

The reference rebuilds the tree every move (mcts.py:334), so the new root — the child the move
went to, always visited, hence evaluated — and often some of its children were leaves of the
previous search. A row's NN output depends only on the position, so such a row is a repeat.
Counts per ply: rows evaluated, rows whose position (black, white, side) was evaluated in the
previous search of the same game (an upper bound of what a tree-linked memo can find), and the
root-only share. GAMES (64), PLIES (60), SIMS (800), NET (6x64)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
from oracle import oracle as O  # noqa: E402
from rvz.network import AlphaZeroNetwork  # noqa: E402

G = int(os.environ.get("GAMES", 64))
PLIES = int(os.environ.get("PLIES", 60))
SIMS = int(os.environ.get("SIMS", 800))
BS = int(os.environ.get("BOARD", 8))
blocks, filters = (int(x) for x in os.environ.get("NET", "6x64").split("x"))
torch.manual_seed(0)
net = AlphaZeroNetwork(BS, blocks, filters).eval()
torch.set_num_threads(int(os.environ.get("THREADS", 8)))

games = [O.new_game(BS) for _ in range(G)]
mts = [O.MT(42 + g) for g in range(G)]
srch = O.Search(G, SIMS, 64, 1.0, bs=BS)
npol = BS * BS + 1
prev = [set() for _ in range(G)]
per_ply = []
for ply in range(PLIES):
    live = [g for g in range(G) if not games[g].over]
    if not live:
        break
    cur = [set() for _ in range(G)]
    rows = hits = root_hits = 0
    srch.begin(games)
    k = 0
    while (r := srch.step()) is not None:
        leaves, ncop = r
        for g in range(G):
            if ncop[g] > 0 and not games[g].over:
                key = (int(leaves[g].black), int(leaves[g].white), int(leaves[g].side))
                rows += 1
                if key in prev[g]:
                    hits += 1
                    root_hits += k == 0
                cur[g].add(key)
        x = torch.from_numpy(O.leaf_planes(leaves, BS))
        with torch.no_grad():
            lg, v = net(x)
        srch.submit(torch.softmax(lg, 1).numpy(), v.numpy())
        k += 1
    vis = srch.visits()
    for g in live:
        nd = O.action_needs_draw(vis[g], 1.0)
        idx, _, _ = O.action(vis[g], 1.0, mts[g].random_sample() if nd else 0.0)
        O.make_move(games[g], -1 if idx == npol - 1 else idx, BS)
    prev = cur
    per_ply.append((rows, hits, root_hits, len(live)))
    print(ply, rows / max(1, len(live)), hits / max(1, len(live)), file=sys.stderr)

R = sum(p[0] for p in per_ply)
H = sum(p[1] for p in per_ply)
RH = sum(p[2] for p in per_ply)
L = sum(p[3] for p in per_ply)
print(json.dumps({"games": G, "plies": len(per_ply), "sims": SIMS, "net": f"{blocks}x{filters}",
                  "rows_per_ply": round(R / L, 3), "repeat_rows_per_ply": round(H / L, 3),
                  "root_repeats_per_ply": round(RH / L, 3), "repeat_frac": round(H / R, 4),
                  "per_ply_repeats": [round(p[1] / max(1, p[3]), 2) for p in per_ply]}))
