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
