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
