"""Batched arena / ELO evaluation (reference src/arena/arena.py:19-389).

``ELORatingSystem`` mirrors arena.py:19-135 (K-factor, expected score, sequential updates,
leaderboard, JSON save/load). ``ELOPlayer`` and ``Arena`` keep the reference's API
(``add_player``, ``play_game``, ``run_tournament``, ``print_leaderboard``, ``save_results``), but
the games of a matchup are played in lockstep on the GPU: one rvz engine per player (its own MCTS
parameters and evaluator) searches, each ply, exactly the games in which that player is to move
(the others are handed to its engine as finished, so they cost no search and, with compacted leaf
batches, no NN rows), and applies its moves — the reference's ``current_player.get_move(game)``
(arena.py:244-262) for a whole batch.
Results are then folded into the ratings in exactly the reference's game order, so the ELO
history is what the sequential tournament would record for the same game outcomes.

Randomness (round 4): by default every game draws exactly what the reference's sequential
tournament draws — one ``random_sample()`` per MCTS move from the NumPy stream and one
``random.choice()`` per random-player move from the Python stream, game after game
(arena.py:175-188, mcts.py:684) — so the same seeds give the reference's tournament; lockstep
passes find each game's place in the streams (``Arena._play_reference_order``).
``draw_order="batched"`` keeps round 3's cheaper order (one draw per game per ply).
"""
from __future__ import annotations

import json
import os
import random
import time
from datetime import datetime
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .engine import Engine
from .network import leaf_evaluator


class ELORatingSystem:
    def __init__(self, k: float = 32, initial_rating: float = 1500.0):
        self.k = k
        self.initial_rating = initial_rating
        self.ratings: Dict[str, float] = {}
        self.games_played: Dict[str, int] = {}
        self.history: List[Dict] = []

    def add_player(self, player_id: str, rating: Optional[float] = None):
        if player_id not in self.ratings:
            self.ratings[player_id] = self.initial_rating if rating is None else rating
            self.games_played[player_id] = 0

    def get_rating(self, player_id: str) -> float:
        return self.ratings.get(player_id, self.initial_rating)

    @staticmethod
    def get_expected_score(rating_a: float, rating_b: float) -> float:
        return 1.0 / (1.0 + 10.0 ** ((rating_b - rating_a) / 400.0))

    def update_ratings(self, player_a: str, player_b: str, score_a: float) -> Dict:
        self.add_player(player_a)
        self.add_player(player_b)
        ra, rb = self.ratings[player_a], self.ratings[player_b]
        ea = self.get_expected_score(ra, rb)
        eb = 1.0 - ea
        na = ra + self.k * (score_a - ea)
        nb = rb + self.k * ((1 - score_a) - eb)
        self.ratings[player_a], self.ratings[player_b] = na, nb
        self.games_played[player_a] += 1
        self.games_played[player_b] += 1
        rec = {"timestamp": time.time(), "player_a": player_a, "player_b": player_b,
               "score_a": score_a, "score_b": 1.0 - score_a, "rating_a_before": ra,
               "rating_b_before": rb, "rating_a_after": na, "rating_b_after": nb}
        self.history.append(rec)
        return rec

    def get_leaderboard(self) -> List[Dict]:
        board = [{"player_id": p, "rating": r, "games_played": self.games_played[p]}
                 for p, r in self.ratings.items()]
        return sorted(board, key=lambda x: x["rating"], reverse=True)

    def save_ratings(self, filepath: str):
        with open(filepath, "w") as f:
            json.dump({"k": self.k, "initial_rating": self.initial_rating,
                       "ratings": self.ratings, "games_played": self.games_played,
                       "history": self.history, "last_updated": datetime.now().isoformat()},
                      f, indent=2)

    @classmethod
    def load_ratings(cls, filepath: str) -> "ELORatingSystem":
        with open(filepath) as f:
            d = json.load(f)
        elo = cls(k=d["k"], initial_rating=d["initial_rating"])
        elo.ratings = {k: float(v) for k, v in d["ratings"].items()}
        elo.games_played = {k: int(v) for k, v in d["games_played"].items()}
        elo.history = d.get("history", [])
        return elo


class ELOPlayer:
    """A model player (MCTS with its own parameters) or, with model None, a random player."""

    def __init__(self, player_id: str, model=None, mcts_params: Optional[Dict] = None,
                 device: str = "cuda", nn_dtype=torch.float32, evaluator=None):
        """evaluator: the leaf evaluator of a model player (default leaf_evaluator(model): the h2
        kernels); any callable leaf_x -> (logits, value) works (``outputs_probs = True``:
        softmaxed rows)."""
        self.player_id = player_id
        self.model = model
        self.device = torch.device(device)
        params = mcts_params or {"num_simulations": 800, "c_puct": 1.0, "temperature": 1.0}
        self.num_simulations = int(params.get("num_simulations", 800))
        self.c_puct = float(params.get("c_puct", 1.0))
        self.batch_size = int(params.get("batch_size", 64))
        self.evaluator = None
        self.board_size = int(getattr(model, "board_size", 8))
        if model is not None:
            model.eval()
            model.to(self.device)
            self.evaluator = evaluator if evaluator is not None else leaf_evaluator(
                model, dtype=nn_dtype, device=self.device)

    def reset(self):
        """Searches start from a fresh root every move (mcts.py:334): nothing to reset."""


class _BatchedDraws:
    """draw_order "batched": one random_sample() per game per ply from the arena's NumPy
    generator (used by the games whose mover searches), random choices in (sorted player id,
    game) order from its Python generator."""

    def __init__(self, arena: "Arena"):
        self.arena = arena
        self.u = None

    def begin_ply(self, G: int):
        self.u = self.arena.np_rng.random_sample(G)

    def uniforms(self, games: np.ndarray) -> np.ndarray:
        u = np.zeros(len(self.u))
        u[games] = self.u[games]
        return u

    def choice(self, g: int, sq: List[int]) -> int:
        return self.arena.py_rng.choice(sq) if sq else -1


class _ReferenceDraws:
    """draw_order "reference", one pass: game g's MCTS moves take stream[offsets[g]],
    stream[offsets[g] + 1], ...; its random moves use a Python generator started at states[g].
    Counts what each game drew."""

    def __init__(self, stream: np.ndarray, offsets: np.ndarray, states: List):
        G = len(offsets)
        self.stream = stream
        self.ptr = [int(o) for o in offsets]
        self.n_mcts = [0] * G
        self.calls: List[List[int]] = [[] for _ in range(G)]
        self.rng = []
        for st in states:
            r = random.Random()
            r.setstate(st)
            self.rng.append(r)

    def begin_ply(self, G: int):
        pass

    def uniforms(self, games: np.ndarray) -> np.ndarray:
        u = np.zeros(len(self.ptr))
        for g in games:
            if self.ptr[g] >= len(self.stream):
                raise RuntimeError("Arena: draw stream exhausted (more MCTS moves than plies)")
            u[g] = self.stream[self.ptr[g]]
            self.ptr[g] += 1
            self.n_mcts[g] += 1
        return u

    def choice(self, g: int, sq: List[int]) -> int:
        if not sq:                      # arena.py:180: (-1, -1) without a draw
            return -1
        self.calls[g].append(len(sq))
        return self.rng[g].choice(sq)


class Arena:
    def __init__(self, elo_system: Optional[ELORatingSystem] = None, seed: int = 0,
                 draw_order: str = "reference"):
        """seed: the arena's NumPy and Python generators start as np.random.seed(seed) and
        random.seed(seed) would leave the reference's global ones (the reference draws from
        those, arena.py:178-188). draw_order: see ``play_games``."""
        self.elo = elo_system if elo_system is not None else ELORatingSystem()
        self.players: Dict[str, ELOPlayer] = {}
        self.np_rng = np.random.RandomState(seed)
        self.py_rng = random.Random(seed)
        self.draw_order = draw_order
        self.reference_order_passes = 0

    def add_player(self, player: ELOPlayer):
        self.players[player.player_id] = player
        self.elo.add_player(player.player_id)

    # ------------------------------------------------------------------ batched games
    def play_games(self, black_ids: Sequence[str], white_ids: Sequence[str],
                   draw_order: Optional[str] = None) -> List[float]:
        """Play len(black_ids) games in lockstep; game g has black_ids[g] (moves first) against
        white_ids[g]. Returns each game's result for its black player: 1.0 / 0.5 / 0.0
        (arena.py:264-282). Every player that appears gets one engine over all games.

        draw_order (default: the arena's): "reference" draws exactly what the reference's
        sequential loop draws (game after game from the global streams, arena.py:175-188,
        mcts.py:684; see ``_play_reference_order``); "batched" draws one random_sample() per
        game per ply and the random players' choices in (sorted player id, game) order."""
        order = draw_order or self.draw_order
        if order not in ("reference", "batched"):
            raise ValueError(f"draw_order must be 'reference' or 'batched', got {order!r}")
        G = len(black_ids)
        if G == 0:
            return []
        for pid in set(black_ids) | set(white_ids):
            if pid not in self.players:
                raise ValueError(f"One or both players not found: {pid}")
        if order == "batched":
            return self._lockstep(black_ids, white_ids, range(G), _BatchedDraws(self))
        return self._play_reference_order(black_ids, white_ids)

    def _play_reference_order(self, black_ids, white_ids) -> List[float]:
        """The reference plays its games one after another, and every MCTS move draws one
        random_sample() from NumPy's global stream (np.random.choice, mcts.py:684; none when all
        visits are 0, mcts.py:679, which the engine refuses anyway), every random-player move one
        random.choice() from Python's (arena.py:178-180). So game k's draws are a contiguous
        piece of each stream, starting after everything games 0..k-1 drew.

        Lockstep passes reproduce that exactly. A game's inputs are its NumPy offset (the draws
        of the earlier games as the latest pass counted them) and its Python generator state
        (the earlier games' choice() calls replayed in game order from the arena's state); its
        moves are a function of those inputs alone (searches are per game, bit for bit), so a
        game whose inputs did not change keeps its result. A pass plays the games whose inputs
        changed since they were last played, except that of the games with a random player only
        the FIRST such changed game is played: its choice() calls set the generator state of
        every later random-player game, so their replays in the same pass would be thrown away
        (round 4 replayed them all: one pass per random-player game, each over the whole rest
        of the tournament with full MCTS). Game 0's inputs are exact from the start,
        and once games 0..k are exact, game k+1's are, so the passes end. Cost: MCTS-only
        tournaments take two or three passes (the offsets depend only on the earlier games'
        MCTS move counts, guessed right for most games); each game with a random player takes
        one pass of its own (the reference plays every game one after another, and a random
        game's generator state depends on the previous random game's moves), i.e. about
        (random-player games + 2) passes, each as long as one game, with every other game
        played about once. `reference_order_passes` reports the count; the engines are built
        once per call. Both generators end where the sequential loop leaves them.
        """
        G = len(black_ids)
        nsq = self._board_size(black_ids, white_ids) ** 2
        mcts = {p: self.players[p].model is not None for p in set(black_ids) | set(white_ids)}
        mcts_only = [mcts[black_ids[g]] and mcts[white_ids[g]] for g in range(G)]
        cache: Dict = {}
        rs = np.random.RandomState()
        rs.set_state(self.np_rng.get_state())
        stream = rs.random_sample(G * (nsq - 4) + nsq)
        py0 = self.py_rng.getstate()
        # first guess: an MCTS player moves (nsq - 4) / 2 times per game
        n_mcts = [(mcts[black_ids[g]] + mcts[white_ids[g]]) * (nsq - 4) // 2 for g in range(G)]
        calls: List[List[int]] = [[] for _ in range(G)]
        prev = [None] * G
        results: List[Optional[float]] = [None] * G
        self.reference_order_passes = 0
        while True:
            offsets = np.concatenate([[0], np.cumsum(n_mcts)[:-1]]).astype(np.int64)
            r = random.Random()
            r.setstate(py0)
            states = []
            for g in range(G):
                states.append(r.getstate())
                for n in calls[g]:
                    r.choice(range(n))
            inputs = [(int(offsets[g]), states[g]) for g in range(G)]
            todo, rand_seen = [], False
            for g in range(G):
                if inputs[g] == prev[g]:
                    continue
                if not mcts_only[g]:          # one random-player game per pass (docstring)
                    if rand_seen:
                        continue
                    rand_seen = True
                todo.append(g)
            if not todo:
                break
            draws = _ReferenceDraws(stream, offsets, states)
            res = self._lockstep(black_ids, white_ids, todo, draws, cache=cache)
            for g in todo:
                results[g] = res[g]
                n_mcts[g] = draws.n_mcts[g]
                calls[g] = draws.calls[g]
                prev[g] = inputs[g]
            self.reference_order_passes += 1
        total = int(sum(n_mcts))
        if total:
            self.np_rng.random_sample(total)
        for g in range(G):
            for n in calls[g]:
                self.py_rng.choice(range(n))
        return results

    def _board_size(self, black_ids, white_ids) -> int:
        sizes = {self.players[p].board_size for p in set(black_ids) | set(white_ids)
                 if self.players[p].model is not None}
        if len(sizes) > 1:
            raise ValueError(f"players of one batch play on one board size, got {sorted(sizes)}")
        return sizes.pop() if sizes else 8

    def _lockstep(self, black_ids, white_ids, games, draws,
                  cache: Optional[Dict] = None) -> List[Optional[float]]:
        """Play `games` (indices into black_ids / white_ids) to their end in lockstep; the other
        games start finished. draws supplies each MCTS move's uniform and each random move.
        cache: a dict that keeps the engines between calls over the same schedule."""
        G = len(black_ids)
        ids = sorted(set(black_ids) | set(white_ids))
        dev = next(iter(self.players[p].device for p in ids))
        bs = self._board_size(black_ids, white_ids)
        nsq = bs * bs
        cache = {} if cache is None else cache
        if not cache:
            for pid in ids:
                pl = self.players[pid]
                if pl.model is not None:
                    cache[pid] = Engine(G, pl.num_simulations, pl.batch_size, pl.c_puct,
                                        board_size=bs, device=dev, compact_leaves=True)
            cache[None] = Engine(G, 64, 64, board_size=bs, device=dev)   # the boards (env only)
        engines = {pid: e for pid, e in cache.items() if pid is not None}
        env = cache[None]
        env.reset(range(G))
        active = np.zeros(G, bool)
        active[list(games)] = True
        if not active.all():
            b, w, st = env.get_state()
            st = st.clone()
            st[:, 1] = torch.where(torch.from_numpy(active).to(dev), st[:, 1],
                                   torch.ones_like(st[:, 1]))
            env.set_state(b.clone(), w.clone(), st)
        black = np.asarray([ids.index(b) for b in black_ids])
        white = np.asarray([ids.index(w) for w in white_ids])
        for _ in range(nsq - 4):                       # every move places a disc
            b, w, st = env.get_state()
            status = st.cpu().numpy()
            if status[:, 1].all():
                break
            side = status[:, 0]
            mover = np.where(side == 1, black, white)  # index into ids per game
            draws.begin_ply(G)
            move = np.full(G, -1, np.int64)
            for k, pid in enumerate(ids):
                games_k = (mover == k) & (status[:, 1] == 0)
                if not games_k.any():
                    continue
                pl = self.players[pid]
                if pl.model is None:                   # random player: random.choice(valid)
                    legal = env.legal().cpu().numpy().view(np.uint64)
                    for g in np.flatnonzero(games_k):
                        sq = [s for s in range(nsq) if (int(legal[g]) >> s) & 1]
                        move[g] = draws.choice(g, sq)
                    continue
                eng = engines[pid]
                # this player's games only: the others enter its engine as finished (no search)
                st_k = st.clone()
                st_k[:, 1] = torch.where(torch.from_numpy(games_k).to(dev), st[:, 1],
                                         torch.ones_like(st[:, 1]))
                eng.set_state(b, w, st_k)
                eng.search(pl.evaluator)
                u = torch.from_numpy(draws.uniforms(np.flatnonzero(games_k)))
                idx, _ = eng.act(1.0, u=u, apply=False)   # arena.py:183-186 uses T = 1.0
                idx = idx.cpu().numpy()
                move[games_k] = np.where(idx[games_k] == nsq, -1, idx[games_k])
            over = status[:, 1] != 0
            sq = torch.from_numpy(np.where(over, nsq, move).astype(np.int32)).to(dev)
            env.apply(sq)                              # make_move; finished games reject it
        for eng in engines.values():
            eng.check()                                # device error words / evaluator overflow
        b, w, st = env.get_state()
        if not bool(st[:, 1].all()):
            raise RuntimeError("Arena.play_games: a game is not over after its last ply")
        bb = b.cpu().numpy().view(np.uint64)
        ww = w.cpu().numpy().view(np.uint64)
        res: List[Optional[float]] = [None] * G
        for g in np.flatnonzero(active):
            nb, nw = bin(int(bb[g])).count("1"), bin(int(ww[g])).count("1")
            res[g] = 1.0 if nb > nw else (0.0 if nw > nb else 0.5)
        return res

    def play_game(self, player1_id: str, player2_id: str, verbose: bool = False,
                  print_games: bool = False) -> float:
        """One game, player1 Black (arena.py:218-282)."""
        r = self.play_games([player1_id], [player2_id])[0]
        if verbose or print_games:
            print(f"{player1_id} (Black) vs {player2_id} (White): {r}")
        return r

    def run_tournament(self, rounds: int = 100, verbose: bool = False,
                       print_games: bool = False) -> Dict:
        """Round robin (arena.py:288-389): every pair meets `rounds` times, colours alternating
        by (i + j + round) % 2; all games of a pair are played in one lockstep batch, then the
        ratings are updated in the reference's game order."""
        pids = list(self.players.keys())
        if len(pids) < 2:
            raise ValueError("Need at least 2 players for a tournament")
        results = {"games_played": 0, "matchups": {}, "start_time": time.time(),
                   "end_time": None, "rounds": []}
        schedule: List[Tuple[int, str, str]] = []     # (round, black, white) in reference order
        for i in range(len(pids)):
            for j in range(i + 1, len(pids)):
                results["matchups"][f"{pids[i]}_vs_{pids[j]}"] = {
                    "player1": pids[i], "player2": pids[j], "games_played": 0,
                    "wins1": 0, "wins2": 0, "draws": 0}
        for rnd in range(rounds):
            for i in range(len(pids)):
                for j in range(i + 1, len(pids)):
                    p1, p2 = pids[i], pids[j]
                    if (i + j + rnd) % 2 == 0:
                        p1, p2 = p2, p1
                    schedule.append((rnd, p1, p2))
        outcome = self.play_games([s[1] for s in schedule], [s[2] for s in schedule])
        for rnd in range(rounds):
            results["rounds"].append({"round": rnd + 1, "games": []})
        for n, ((rnd, p1, p2), r) in enumerate(zip(schedule, outcome)):
            self.elo.update_ratings(p1, p2, r)
            key = f"{p1}_vs_{p2}" if f"{p1}_vs_{p2}" in results["matchups"] else f"{p2}_vs_{p1}"
            m = results["matchups"][key]
            m["games_played"] += 1
            results["games_played"] += 1
            # wins1 counts wins of the game's first player, as arena.py:346-351 does
            if r == 1.0:
                m["wins1"] += 1
            elif r == 0.0:
                m["wins2"] += 1
            else:
                m["draws"] += 1
            a1, a2 = self.elo.get_rating(p1), self.elo.get_rating(p2)
            k, ex = self.elo.k, self.elo.get_expected_score
            # arena.py:361-362 reconstructs the "before" ratings from the updated ones (with the
            # expected score of the AFTER ratings), not the ratings the update started from;
            # the reference's values are kept for drop-in results
            results["rounds"][rnd]["games"].append({
                "player1": p1, "player2": p2, "result": r,
                "elo1_before": a1 - (k * (r - ex(a1, a2))),
                "elo2_before": a2 - (k * ((1 - r) - ex(a2, a1))),
                "elo1_after": a1, "elo2_after": a2})
            if verbose or print_games:
                if n + 1 == len(schedule) or schedule[n + 1][0] != rnd:
                    print(f"\n--- After Round {rnd + 1} ---")
                    self.print_leaderboard()
        if not verbose and not print_games:
            print("\n--- Tournament Complete ---")
            self.print_leaderboard()
        results["end_time"] = time.time()
        results["duration"] = results["end_time"] - results["start_time"]
        results["leaderboard"] = self.elo.get_leaderboard()
        return results

    def print_leaderboard(self):
        print("\nCurrent Leaderboard:")
        print("Rank  Player ID               Rating  Games Played")
        print("----  ---------------------  -------  ------------")
        for i, p in enumerate(self.elo.get_leaderboard(), 1):
            print(f"{i:4d}  {p['player_id']:22s}  {p['rating']:7.1f}  {p['games_played']:12d}")

    def save_results(self, filepath: str):
        self.elo.save_ratings(os.path.splitext(filepath)[0] + "_elo.json")
        with open(filepath, "w") as f:
            json.dump(self.elo.get_leaderboard(), f, indent=2)
