"""rvz.arena.ELORatingSystem against the reference's (tests/golden/elo_sequence.json)."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "elo_sequence.json")


def test_elo_sequence_matches_reference(tmp_path):
    from rvz.arena import ELORatingSystem
    fx = json.load(open(GOLDEN))
    elo = ELORatingSystem(k=32, initial_rating=1500.0)
    for (a, b, s), after in zip(fx["updates"], fx["ratings_after"]):
        elo.update_ratings(a, b, s)
        assert [elo.ratings.get(p, 1500.0) for p in fx["players"]] == after   # bitwise floats
    assert [(r["player_id"], r["rating"], r["games_played"]) for r in elo.get_leaderboard()] == \
        [(r["player_id"], r["rating"], r["games_played"]) for r in fx["leaderboard"]]
    path = tmp_path / "elo.json"
    elo.save_ratings(str(path))
    again = ELORatingSystem.load_ratings(str(path))
    assert again.ratings == elo.ratings and again.games_played == elo.games_played


def _fake_game(g, mcts_side, u_of, choice_of, mcts_ends=True):
    """A stand-in for one game's moves that consumes draws like an arena game: up to 12 moves,
    sides alternate; an MCTS move takes one uniform and (mcts_ends) ends the game below 0.15, a
    random move chooses among 1 + (7 t + g) mod 9 squares and ends the game on square 0. Returns
    a result that depends on every draw. mcts_ends False: an MCTS-only game always makes 12
    moves, as 8x8 games (60 plies, 30 moves a side, bar passes) nearly always do."""
    h = 0
    for t in range(12):
        if mcts_side[t % 2]:
            u = u_of()
            h = (h * 31 + int(u * 1e6)) % 1000003
            if u < 0.15 and mcts_ends:
                break
        else:
            m = choice_of(list(range(1 + (7 * t + g) % 9)))
            h = (h * 31 + m) % 1000003
            if m == 0:
                break
    return [0.0, 0.5, 1.0][h % 3]


def test_reference_draw_order_passes_reproduce_sequential_draws(monkeypatch):
    """Arena._play_reference_order's lockstep passes against the sequential loop, with the
    game replaced by _fake_game (no GPU): same results and both generators end in the same
    state, for MCTS-only, mixed and random-only schedules."""
    import random
    import types
    import numpy as np
    from rvz.arena import Arena

    played = []
    ends = [True]

    def fake_lockstep(self, black_ids, white_ids, games, draws, cache=None):
        played.extend(games)
        G = len(black_ids)
        draws.begin_ply(G)
        res = [None] * G
        for g in games:
            side = (self.players[black_ids[g]].model is not None,
                    self.players[white_ids[g]].model is not None)
            res[g] = _fake_game(g, side, lambda: float(draws.uniforms(np.array([g]))[g]),
                                lambda sq: draws.choice(g, sq), ends[0])
        return res

    monkeypatch.setattr(Arena, "_lockstep", fake_lockstep)
    mixed = [("a", "r"), ("r", "b"), ("a", "b"), ("r", "r")] * 4
    for pairs, ends[0] in (([("a", "b")] * 5, True), (mixed, True), ([("r", "r")] * 6, True),
                           ([("a", "b")] * 12, False), (mixed, False)):
        arena = Arena(seed=5)
        played.clear()
        for pid in "abr":
            arena.players[pid] = types.SimpleNamespace(
                model=None if pid == "r" else object(), board_size=8, device="cpu")
        black = [p[0] for p in pairs]
        white = [p[1] for p in pairs]
        got = arena.play_games(black, white)
        np_rng, py_rng = np.random.RandomState(5), random.Random(5)
        want = [_fake_game(g, (b != "r", w != "r"), lambda: float(np_rng.random_sample()),
                           py_rng.choice, ends[0]) for g, (b, w) in enumerate(pairs)]
        assert got == want
        assert arena.np_rng.random_sample() == np_rng.random_sample()
        assert arena.py_rng.random() == py_rng.random()
        assert arena.reference_order_passes <= len(pairs) + 1
        if not ends[0]:
            # cost when MCTS move counts are fixed, as in real games: one pass per
            # game with a random player plus at most three, and every game played a bounded
            # number of times (round 4 replayed the whole rest of the tournament every pass)
            n_rand = sum(1 for b, w in pairs if "r" in (b, w))
            assert arena.reference_order_passes <= n_rand + 3
            assert len(played) <= 3 * len(pairs), len(played)
        print(pairs[:2], "passes", arena.reference_order_passes, "plays", len(played))
