"""Batched arena (rvz/arena.py; reference src/arena/arena.py) on the GPU."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _players():
    import rvz
    from rvz.arena import ELOPlayer
    torch.manual_seed(0)
    a = rvz.AlphaZeroNetwork(8, 1, 16)
    torch.manual_seed(1)
    b = rvz.AlphaZeroNetwork(8, 1, 16)
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
