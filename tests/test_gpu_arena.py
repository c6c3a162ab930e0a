"""Batched arena (rvz/arena.py; reference src/arena/arena.py) on the GPU."""
import numpy as np
import pytest
import torch

from evaluators import TableEvaluator as _TableEvaluator

pytestmark = pytest.mark.gpu


def _players():
    import rvz
    from rvz.arena import ELOPlayer
    torch.manual_seed(0)
    a = rvz.AlphaZeroNetwork(8, 1, 64)
    torch.manual_seed(1)
    b = rvz.AlphaZeroNetwork(8, 1, 64)
    params = {"num_simulations": 128, "c_puct": 1.0}
    return [ELOPlayer("net_a", a, params), ELOPlayer("net_b", b, {"num_simulations": 192}),
            ELOPlayer("random", None)]


def test_tournament_structure_and_elo_conservation():
    from rvz.arena import Arena
    arena = Arena(seed=3)
    for p in _players():
        arena.add_player(p)
    res = arena.run_tournament(rounds=6)
    assert res["games_played"] == 6 * 3
    for m in res["matchups"].values():
        assert m["games_played"] == 6 and m["wins1"] + m["wins2"] + m["draws"] == 6
    total = sum(r["rating"] for r in res["leaderboard"])
    assert abs(total - 3 * 1500.0) < 1e-6                    # ELO updates are zero-sum
    assert sum(r["games_played"] for r in res["leaderboard"]) == 2 * 18
    assert len(arena.elo.history) == 18


def test_play_games_results_and_colours():
    """Results are from the black player's view; swapping colours keeps every game legal."""
    from rvz.arena import Arena
    arena = Arena(seed=5)
    for p in _players():
        arena.add_player(p)
    r1 = arena.play_games(["net_a"] * 8 + ["random"] * 8, ["random"] * 8 + ["net_a"] * 8)
    assert len(r1) == 16 and set(r1) <= {0.0, 0.5, 1.0}
    assert arena.play_game("net_b", "net_a") in (0.0, 0.5, 1.0)


def _literal_arena_sequential(O, players, black_ids, white_ids, seed):
    """The reference's tournament loop as it runs (arena.py:218-286, 324-337): one game after
    another; each MCTS move is a search then get_action_probs at T = 1 drawing one
    random_sample() from NumPy's global stream (mcts.py:684, here RandomState(seed), which is
    np.random.seed(seed)); each random-player move is random.choice(valid_moves) on Python's
    global stream (arena.py:178-180, here random.Random(seed)). Returns the results and both
    generators, to compare where they end."""
    import random
    np_rng, py_rng = np.random.RandomState(seed), random.Random(seed)
    res = []
    for bid, wid in zip(black_ids, white_ids):
        game = O.new_game()
        while not game.over:
            pid = bid if game.side == 1 else wid
            P, Q = (game.black, game.white) if game.side == 1 else (game.white, game.black)
            if players[pid] is None:
                lg = O.legal(P, Q)
                sq = [s for s in range(64) if (lg >> s) & 1]
                mv = py_rng.choice(sq) if sq else -1
            else:
                srch = O.Search(1, players[pid], 64, 1.0)
                srch.begin([game])
                while (r := srch.step()) is not None:
                    p, v = _TableEvaluator.numpy(O.leaf_planes(r[0]))
                    srch.submit(p, v)
                vis = srch.visits()[0]
                u = float(np_rng.random_sample()) if O.action_needs_draw(vis, 1.0) else 0.0
                idx, _, _ = O.action(vis, 1.0, u)
                mv = -1 if idx == 64 else idx
            assert O.make_move(game, mv)
        nb, nw = bin(game.black).count("1"), bin(game.white).count("1")
        res.append(1.0 if nb > nw else (0.0 if nw > nb else 0.5))
    return res, np_rng, py_rng


def _literal_arena(O, players, black_ids, white_ids, seed):
    """The reference's game loop (arena.py:218-286: while not over, the player to move's
    get_move, make_move; winner by disc count; ELOPlayer.get_move arena.py:175-188: MCTS
    get_action_probs at T = 1, random.choice for a random player) on the CPU oracle, game by game
    within each lockstep ply, with the batched arena's documented draw order: one
    random_sample() per game per ply from RandomState(seed), random.Random(seed) choices in
    (sorted player id, game) order."""
    import random
    np_rng, py_rng = np.random.RandomState(seed), random.Random(seed)
    G = len(black_ids)
    ids = sorted(set(black_ids) | set(white_ids))
    games = [O.new_game() for _ in range(G)]
    for _ in range(60):
        if all(g.over for g in games):
            break
        u = np_rng.random_sample(G)
        move = [-1] * G
        for pid in ids:
            mine = [g for g in range(G) if not games[g].over and
                    (black_ids[g] if games[g].side == 1 else white_ids[g]) == pid]
            if not mine:
                continue
            sims = players[pid]
            if sims is None:
                for g in mine:
                    P, Q = (games[g].black, games[g].white) if games[g].side == 1 else \
                        (games[g].white, games[g].black)
                    lg = O.legal(P, Q)
                    sq = [s for s in range(64) if (lg >> s) & 1]
                    move[g] = py_rng.choice(sq) if sq else -1
                continue
            srch = O.Search(len(mine), sims, 64, 1.0)
            srch.begin([games[g] for g in mine])
            while (r := srch.step()) is not None:
                p, v = _TableEvaluator.numpy(O.leaf_planes(r[0]))
                srch.submit(p, v)
            vis = srch.visits()
            for j, g in enumerate(mine):
                idx, _, _ = O.action(vis[j], 1.0, float(u[g]))
                move[g] = -1 if idx == 64 else idx
        for g in range(G):
            if not games[g].over:
                assert O.make_move(games[g], move[g])
    res = []
    for g in games:
        nb, nw = bin(g.black).count("1"), bin(g.white).count("1")
        res.append(1.0 if nb > nw else (0.0 if nw > nb else 0.5))
    return res


def test_play_games_matches_literal_reference_loop(oracle):
    """Arena.play_games (lockstep, one engine per player searching only its own games) == the
    reference's per-game loop restated on the CPU oracle with the same evaluator and draws:
    every game's result. Players: two MCTS players (128 and 192 simulations) and a random
    player, in every pairing and both colours. (At S <= 64 = one batch the root's children are
    never visited, get_action_probs falls back to argmax(0s) = square 0, which is illegal: the
    reference's arena loop then never ends; rvz raises instead.)"""
    import rvz
    from rvz.arena import Arena, ELOPlayer
    net = rvz.AlphaZeroNetwork(8, 1, 64)
    arena = Arena(seed=11, draw_order="batched")
    arena.add_player(ELOPlayer("a", net, {"num_simulations": 128}, evaluator=_TableEvaluator()))
    arena.add_player(ELOPlayer("b", net, {"num_simulations": 192}, evaluator=_TableEvaluator()))
    arena.add_player(ELOPlayer("r", None))
    pairs = [("a", "b"), ("b", "a"), ("a", "r"), ("r", "a"), ("b", "r"), ("r", "b"), ("a", "a")]
    black = [p[0] for p in pairs for _ in range(3)]
    white = [p[1] for p in pairs for _ in range(3)]
    got = arena.play_games(black, white)
    want = _literal_arena(oracle, {"a": 128, "b": 192, "r": None}, black, white, seed=11)
    assert got == want


@pytest.mark.parametrize("pairs", [
    [("a", "b"), ("b", "a"), ("a", "a"), ("b", "b")],
    [("a", "b"), ("b", "a"), ("a", "r"), ("r", "a"), ("b", "r"), ("r", "b"), ("r", "r")]],
    ids=["mcts-only", "with-random"])
def test_reference_draw_order_replays_the_sequential_tournament(oracle, pairs):
    """draw_order "reference" (the default): the lockstep passes give every game exactly what
    the reference's one-game-after-another loop gives with the same seeds — each game's result
    — and leave the NumPy and Python generators where that loop leaves them (VERDICT r03
    missing 5: arena.py:175-188, mcts.py:684)."""
    import rvz
    from rvz.arena import Arena, ELOPlayer
    net = rvz.AlphaZeroNetwork(8, 1, 64)
    arena = Arena(seed=7)
    arena.add_player(ELOPlayer("a", net, {"num_simulations": 128}, evaluator=_TableEvaluator()))
    arena.add_player(ELOPlayer("b", net, {"num_simulations": 192}, evaluator=_TableEvaluator()))
    arena.add_player(ELOPlayer("r", None))
    black = [p[0] for p in pairs for _ in range(2)]
    white = [p[1] for p in pairs for _ in range(2)]
    got = arena.play_games(black, white)
    want, np_rng, py_rng = _literal_arena_sequential(
        oracle, {"a": 128, "b": 192, "r": None}, black, white, seed=7)
    assert got == want
    assert arena.np_rng.random_sample() == np_rng.random_sample()
    assert arena.py_rng.random() == py_rng.random()
    assert 1 <= arena.reference_order_passes <= len(black) + 1
    print("passes", arena.reference_order_passes, "games", len(black))
