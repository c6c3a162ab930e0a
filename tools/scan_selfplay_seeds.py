"""Find np.random seeds whose self-play games exercise SelfPlay's draw-order passes: a game that
ends before the board is full (its successors' stream offsets move) and a pass.

  python tools/scan_selfplay_seeds.py table 12 200 0 300     # CPU oracle, the table evaluator
  python tools/scan_selfplay_seeds.py h2 12 200 0 40         # rvz.SelfPlay on the GPU, 1x64 net

Prints per seed the game lengths (moves), the passes per game and the distinct openings. The
seeds in tests/test_selfplay_order_cpu.py and tests/test_gpu_dropin.py come from here."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "alphazero-reversi_amd")]

import numpy as np  # noqa: E402


def main():
    kind, n, sims, lo, hi = sys.argv[1], *map(int, sys.argv[2:6])
    if kind == "table":
        from oracle import oracle as O
        from oracle_play import reference_generate_games
        from test_selfplay_order_cpu import table_eval

        def play(seed):
            gs = reference_generate_games(O, n, sims, 1.0, np.random.RandomState(seed), table_eval)
            return [g["current_players"] for g in gs], None
    else:
        import tempfile
        import torch
        import rvz
        torch.manual_seed(0)
        net = rvz.AlphaZeroNetwork(8, 1, 64).cuda().eval()
        sp = rvz.SelfPlay(net, {"num_simulations": sims, "save_dir": tempfile.mkdtemp()})

        def play(seed):
            np.random.seed(seed)
            gs = sp.generate_games(n)
            return [g["current_players"] for g in gs], sp.reference_order_passes
    for s in range(lo, hi):
        t = time.time()
        players, npass = play(s)
        lens = [len(p) for p in players]
        passes = [sum(a == b for a, b in zip(p, p[1:])) for p in players]
        print(s, lens, passes, "replay passes", npass, f"{time.time() - t:.1f}s", flush=True)


if __name__ == "__main__":
    main()
