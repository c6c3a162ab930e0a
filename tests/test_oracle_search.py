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


_POW_SCRIPT = r"""
import sys, numpy as np
rng = np.random.default_rng(5)
out = []
for t in range(400):
    vis = (rng.integers(0, 800, 65) * (rng.random(65) < 0.3)).astype(np.int32)
    vis[rng.integers(0, 64)] += 1
    for T in (0.7, 0.3, 1.5, 0.25, 3.0, 0.9):
        p = vis / vis.sum()
        p = p ** (1.0 / T)
        out.append(p / np.sum(p))
np.save(sys.argv[1], np.stack(out))
"""


def test_numpy_power_scalar_dispatch_is_libm_pow(oracle, tmp_path):
    """get_action_probs' `p ** (1/T)` for general T: NumPy's array power is host-dependent —
    with AVX512 it dispatches to a SIMD kernel (differs from libm by a few ulp, see
    test_choice_matches_numpy), otherwise it calls libm pow. Run NumPy with its AVX512 dispatch
    disabled (NPY_DISABLE_CPU_FEATURES) and the oracle's libm pow matches it bitwise. k_act
    computes the correctly rounded power instead (test_pow_cr_is_correctly_rounded)."""
    import os
    import subprocess
    import sys
    from numpy._core._multiarray_umath import __cpu_features__ as feats
    off = " ".join(k for k, v in feats.items() if v and k.startswith("AVX512"))
    path = tmp_path / "p.npy"
    env = dict(os.environ, NPY_DISABLE_CPU_FEATURES=off)
    subprocess.run([sys.executable, "-c", _POW_SCRIPT, str(path)], check=True, env=env)
    got = np.load(path)
    rng = np.random.default_rng(5)
    i = 0
    for t in range(400):
        vis = (rng.integers(0, 800, 65) * (rng.random(65) < 0.3)).astype(np.int32)
        vis[rng.integers(0, 64)] += 1
        for T in (0.7, 0.3, 1.5, 0.25, 3.0, 0.9):
            _, p, _ = oracle.action(vis, T, 0.5)
            assert np.array_equal(p.view(np.int64), got[i].view(np.int64)), (t, T)
            i += 1


def test_pow_cr_is_correctly_rounded():
    """k_act's power (csrc/rvz_pow.hip.h pow_cr, host build in tools/alt) is the correctly rounded
    x ** e: equal to 60-digit decimal exp(e ln x) rounded once, on the p = n / total inputs k_act
    sees at eight temperatures and on a wide range (including overflow and subnormal results).
    glibc's pow (0.52-ulp bound) misses it on a small fraction, counted as a bound."""
    import math
    from decimal import Decimal, getcontext
    import alt_eval
    getcontext().prec = 60

    def cr(x, e):
        try:
            return float((Decimal(x).ln() * Decimal(e)).exp())
        except OverflowError:
            return math.inf

    lib = alt_eval.load()
    rng = np.random.default_rng(1)
    N = 2000
    n = rng.integers(1, 800, N)
    x = n / (n + rng.integers(0, 2200, N))
    xs = [np.repeat(x, 8), np.exp(rng.uniform(-700, 700, 4000)), rng.uniform(0.5, 2, 2000)]
    es = [np.tile(1.0 / np.array([0.7, 0.3, 1.5, 0.25, 3.0, 0.9, 0.05, 7.0]), N),
          rng.uniform(-3, 3, 4000), rng.uniform(-50, 50, 2000)]
    x, e = np.concatenate(xs), np.concatenate(es)
    out = np.empty_like(x)
    assert lib.rvz_alt_pow_host(x.size, x.ctypes.data, e.ctypes.data, out.ctypes.data) == 0
    want = np.array([cr(a, b) for a, b in zip(x, e)])
    assert np.array_equal(out.view(np.int64), want.view(np.int64))
    assert (np.abs(want) < 2.3e-308).sum() > 100        # subnormal / zero results covered
    glibc = np.array([math.pow(a, b) for a, b in zip(x[:16000], e[:16000])])
    assert (glibc != want[:16000]).mean() < 0.005
    for a, b, r in [(0.0, 1.5, 0.0), (0.0, -1.5, math.inf), (1.0, 37.0, 1.0), (0.3, 0.0, 1.0),
                    (math.inf, 2.5, math.inf), (0.5, math.inf, 0.0)]:
        xa, ea, o = np.array([a]), np.array([b]), np.empty(1)
        lib.rvz_alt_pow_host(1, xa.ctypes.data, ea.ctypes.data, o.ctypes.data)
        assert o[0] == r, (a, b, o[0])
