"""Replay of the F-mcts fixtures (tests/golden/mcts_*.npz) through a pull-style search.

Shared by the CPU oracle tests and the GPU parity tests: the search under test asks for leaf
evaluations, the replay checks each leaf against the reference's recorded NN call (as planes
bitmasks) and answers with the reference's own recorded softmax row and value. Visits, the f64
policy vector and the sampled action are then compared per ply with what the reference produced.
"""
from __future__ import annotations

import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_paths(pattern: str = "mcts_*.npz"):
    return sorted(glob.glob(os.path.join(GOLDEN, pattern)))


def load(path):
    d = np.load(path)
    return {k: d[k] for k in d.files}


def games(fx):
    """Yield per-game dicts: seed, plies (state, visits, p, action), calls (masks, probs, value)."""
    for gi, seed in enumerate(fx["seeds"]):
        pm = fx["game"] == gi
        cm = fx["call_game"] == gi
        yield {
            "seed": int(seed),
            "ply_black": fx["ply_black"][pm], "ply_white": fx["ply_white"][pm],
            "ply_side": fx["ply_side"][pm], "ply_visits": fx["ply_visits"][pm],
            "ply_p": fx["ply_p"][pm], "ply_action": fx["ply_action"][pm],
            "call_ply": fx["call_ply"][cm], "call_masks": fx["call_masks"][cm],
            "call_probs": fx["call_probs"][cm], "call_value": fx["call_value"][cm],
            "winner": int(fx["winners"][gi]),
        }


def planes_to_masks(x: np.ndarray):
    """[3, S, S] 0/1 planes -> three python-int bitmasks (square s = bit s)."""
    out = []
    for p in range(3):
        bits = np.flatnonzero(np.asarray(x[p], np.float32).reshape(-1) > 0.5)
        out.append(sum(1 << int(b) for b in bits))
    return out


class ReplayEvaluator:
    """A leaf evaluator that answers with the reference's recorded NN outputs.

    Plugs into rvz.SelfPlay / rvz.Engine.search (``outputs_probs``: it hands over the
    reference's own F.softmax rows, mcts.py:596, so the expand uses them bit for bit). Each live
    leaf row (need > 0; uncompacted batches, row g = game g) must be the reference's next
    recorded NN input of that game (checked as plane bitmasks). Eager only (host round trip).
    """

    outputs_probs = True

    def __init__(self, games):
        self.games = list(games)
        self.eng = None

    def bind(self, eng):
        import torch
        if eng.n_games != len(self.games) or eng.compact_leaves:
            raise ValueError("replay needs one engine game per fixture game, uncompacted")
        self.eng, self.ci = eng, [0] * len(self.games)
        self.probs = torch.zeros(eng.n_games, eng.npol, dtype=torch.float32, device=eng.device)
        self.value = torch.zeros(eng.n_games, dtype=torch.float32, device=eng.device)

    def __call__(self, x):
        import torch
        need = self.eng.need.cpu().numpy()
        xs = x.cpu().numpy()
        G = len(self.games)
        pr = np.zeros((G, self.eng.npol), np.float32)
        va = np.zeros(G, np.float32)
        for gi, g in enumerate(self.games):
            if need[gi] == 0:
                continue
            c = self.ci[gi]
            if c >= len(g["call_ply"]):
                raise AssertionError(f"game {gi}: more NN calls than the reference made")
            got = planes_to_masks(xs[gi])
            want = [int(v) for v in g["call_masks"][c]]
            if got != want:
                raise AssertionError(f"game {gi} call {c}: leaf {got} != reference {want}")
            pr[gi], va[gi] = g["call_probs"][c], g["call_value"][c]
            self.ci[gi] += 1
        self.probs.copy_(torch.from_numpy(pr))
        self.value.copy_(torch.from_numpy(va))
        return self.probs, self.value

    def all_calls_used(self) -> bool:
        return all(c == len(g["call_ply"]) for c, g in zip(self.ci, self.games))


def expected_records(oracle, g):
    """The reference's game_data dict for one fixture game (self_play.py:72-126): canonical
    planes of the position before each move (game.py:131-162, via the oracle), the f64 policy
    vectors, the player to move, and values +1/-1/0 from the final winner's perspective."""
    n = len(g["ply_action"])
    states, players = [], []
    for k in range(n):
        st = oracle.Game(int(g["ply_black"][k]), int(g["ply_white"][k]), int(g["ply_side"][k]))
        states.append(oracle.canonical(st))
        players.append(int(g["ply_side"][k]))
    w = g["winner"]
    values = [0.0 if w == 0 else (1.0 if p == w else -1.0) for p in players]
    return {"states": states, "action_probs": [g["ply_p"][k] for k in range(n)],
            "current_players": players, "values": values}
