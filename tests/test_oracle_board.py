"""The CPU oracle's board rules against the reference (tests/golden/board_vectors.npz) and the
reference's own known-answer tests (test_game.py:7-126), restated on the oracle."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "board_vectors.npz")


def load_vectors():
    with np.load(GOLDEN) as z:     # materialise once: NpzFile re-inflates on every access
        return {k: z[k] for k in z.files}


def _game(O, d, i):
    g = O.Game()
    g.black, g.white = int(d["black"][i]), int(d["white"][i])
    g.side, g.over, g.winner, g.passed = (int(d[k][i]) for k in ("side", "over", "winner", "passed"))
    return g


def test_legal_masks_match_reference(oracle):
    d = load_vectors()
    bad = 0
    for i in range(len(d["black"])):
        b, w, s = int(d["black"][i]), int(d["white"][i]), int(d["side"][i])
        P, Q = (b, w) if s == 1 else (w, b)
        bad += oracle.legal(P, Q) != int(d["legal"][i])
    assert bad == 0 and len(d["black"]) > 10000


def test_make_move_matches_reference(oracle):
    d = load_vectors()
    n_illegal = n_pass = 0
    for i in range(len(d["black"])):
        g = _game(oracle, d, i)
        ok = oracle.make_move(g, int(d["move"][i]))
        exp = tuple(int(d[k][i]) for k in ("black_after", "white_after", "side_after",
                                            "over_after", "winner_after", "passed_after"))
        assert ok == bool(d["ok"][i]), i
        assert g.astuple() == exp, i
        n_illegal += not ok
        n_pass += int(d["move"][i]) == -1
    assert n_illegal > 100 and n_pass > 100   # the fixture covers the False paths too


# ---- test_game.py restated (the reference's only known-answer tests for the board)
def test_initial_board(oracle):
    g = oracle.new_game()
    assert g.white == (1 << 27) | (1 << 36) and g.black == (1 << 28) | (1 << 35)
    assert bin(g.black | g.white).count("1") == 4


def test_valid_moves(oracle):
    g = oracle.new_game()
    m = oracle.legal(g.black, g.white)
    assert {divmod(s, 8) for s in range(64) if m >> s & 1} == {(2, 3), (3, 2), (4, 5), (5, 4)}


def test_make_move(oracle):
    g = oracle.new_game()
    assert oracle.make_move(g, 2 * 8 + 3)
    assert g.black >> (2 * 8 + 3) & 1 and g.black >> (3 * 8 + 3) & 1
    assert g.side == 2


def test_game_over(oracle):
    g = oracle.new_game()
    black, white = 0x2, 0
    for i in range(8):
        for j in range(8):
            if i > 0 or j > 1:
                pos = i * 8 + j
                if (i + j) % 2 == 0:
                    white |= 1 << pos
                else:
                    black |= 1 << pos
    black &= ~1
    white &= ~2
    black |= 2
    g.black, g.white, g.side = black, white, 2
    assert oracle.make_move(g, 0)
    assert g.over and g.winner == 2


def test_6x6_rules_are_consistent(oracle):
    """Build-defined 6x6 variant: start position, 4 legal moves, games end within 32 plies."""
    rng = np.random.default_rng(0)
    for _ in range(50):
        g = oracle.new_game(6)
        assert bin(g.black).count("1") == 2 and bin(g.white).count("1") == 2
        plies = 0
        while not g.over:
            P, Q = (g.black, g.white) if g.side == 1 else (g.white, g.black)
            m = oracle.legal(P, Q, 6)
            assert m and m < (1 << 36)
            moves = [s for s in range(36) if m >> s & 1]
            assert oracle.make_move(g, int(rng.choice(moves)), 6)
            plies += 1
        assert plies <= 32 and (g.black | g.white) < (1 << 36)
