"""The CPU oracle's MCTS + action selection against the reference's recorded games
(tests/golden/mcts_*.npz) and its RNG / reductions against live NumPy."""
import numpy as np
import pytest

import golden_replay as R


@pytest.mark.parametrize("path", R.fixture_paths(), ids=lambda p: p.split("/")[-1])
def test_oracle_replays_reference_games(oracle, path):
    fx = R.load(path)
    sims, T = int(fx["sims"]), float(fx["temperature"])
    for g in R.games(fx):
        mt = oracle.MT(g["seed"])
        game, ci = oracle.new_game(), 0
        srch = oracle.Search(1, sims, int(fx["batch"]), float(fx["c_puct"]))
        for k in range(len(g["ply_action"])):
            assert (int(g["ply_black"][k]), int(g["ply_white"][k]), int(g["ply_side"][k])) == \
                (game.black, game.white, game.side)
            srch.begin([game])
            while (r := srch.step()) is not None:
                leaves, nc = r
                if nc[0] == 0:
                    continue
                assert R.planes_to_masks(oracle.canonical(leaves[0])) == \
                    [int(x) for x in g["call_masks"][ci]]
                srch.submit(g["call_probs"][ci][None], g["call_value"][ci:ci + 1])
                ci += 1
            vis = srch.visits()[0]
            np.testing.assert_array_equal(vis, g["ply_visits"][k])
            u = mt.random_sample() if oracle.action_needs_draw(vis, T) else 0.0
            idx, p, _ = oracle.action(vis, T, u)
            assert np.array_equal(p.view(np.int64), g["ply_p"][k].view(np.int64))  # bitwise f64
            assert idx == g["ply_action"][k]
            assert oracle.make_move(game, -1 if idx == 64 else idx)
        assert ci == len(g["call_ply"])
        assert game.winner == g["winner"]


def test_mt19937_matches_numpy(oracle):
    for seed in (0, 1, 42, 2**31 + 5, 2**32 - 1):
        np.random.seed(seed)
        mt = oracle.MT(seed)
        for _ in range(700):   # crosses the 624-word regeneration
            assert mt.random_sample() == np.random.random_sample()


def test_choice_matches_numpy(oracle):
    rng = np.random.default_rng(1)
    for t in range(300):
        vis = (rng.integers(0, 40, 65) * (rng.random(65) < 0.2)).astype(np.int32)
        vis[rng.integers(0, 64)] += 1
        seed = int(rng.integers(0, 2**31))
        for T in (1.0, 0.5, 2.0, 0.7):
            p = vis / vis.sum()
            p = p ** (1.0 / T)
            p = p / np.sum(p)
            np.random.seed(seed)
            ref_idx = np.random.choice(len(p), p=p)
            idx, pp, drew = oracle.action(vis, T, oracle.MT(seed).random_sample())
            assert drew
            if T in (1.0, 0.5, 2.0):   # numpy fast_scalar_power paths: copy / sqrt / square
                assert idx == ref_idx
                assert np.array_equal(pp.view(np.int64), p.view(np.int64))
            else:
                # general exponents: numpy's array power runs a SIMD kernel that differs from
                # libm pow by a few ulp on this host ("T outside the fast paths")
                assert np.abs(pp.view(np.int64) - p.view(np.int64)).max() <= 4
                assert abs(idx - ref_idx) <= 64


def test_pairwise_sum_matches_numpy(oracle):
    rng = np.random.default_rng(2)
    for n in (1, 5, 8, 9, 37, 64, 65, 127, 128, 300):
        for _ in range(50):
            a = rng.random(n) * (rng.random(n) < 0.5)
            assert oracle.np_sum(a) == np.sum(a)


def test_dedup_invariant_holds_in_literal_search(oracle):
    """Every batch of the literal reference search queues copies of ONE leaf per game
    (the engine's exact dedup relies on it); Search.step raises otherwise."""
    G = 16
    srch = oracle.Search(G, 800, 64, 1.0)
    games = [oracle.new_game() for _ in range(G)]
    rng = np.random.default_rng(3)
    for ply in range(12):
        srch.begin(games)
        while (r := srch.step()) is not None:
            probs = rng.dirichlet(np.ones(65), G).astype(np.float32)
            srch.submit(probs, rng.uniform(-1, 1, G).astype(np.float32))
        vis = srch.visits()
        for g in range(G):
            assert vis[g].sum() == 800 - 64   # root absorbs the first batch as its own leaf
            assert oracle.make_move(games[g], int(np.argmax(vis[g])))
