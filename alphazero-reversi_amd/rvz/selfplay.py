"""Batched self-play: the reference's SelfPlay (src/self_play/self_play.py:21-219) over the engine.

``SelfPlayRunner`` advances every game of an ``Engine`` by one ply per call (one MCTS search +
one move per live game, self_play.py:80-101), optionally captured once into a HIP graph and
replayed (the 13 select / NN / expand rounds and the act of a ply are one graph launch).
With ``autoreset`` a finished game restarts at once with the next seed of its slot
(seed_g, seed_g + G, ...), which keeps every slot busy for steady-state measurement.

``SelfPlay`` is the drop-in for the reference class: same constructor ``(model, args)``, same
``generate_games(n)`` / ``generate_training_data(n)`` outputs (per-game dict of canonical states,
action_probs, current_players, values; self_play.py:117-131), with the n games played in
lockstep instead of one after another.
"""
from __future__ import annotations

import os
import time
from datetime import datetime
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from .engine import Engine, board_canonical


class SelfPlayRunner:
    def __init__(self, engine: Engine, evaluator: Callable, temperature: float = 1.0,
                 fused_softmax: bool = True, autoreset: bool = False, seed_base: int = 42,
                 record: bool = False, max_plies: int = 60, seed_stride: int = None,
                 skip_last_eval: bool = False, fused_bookkeeping: bool = True,
                 fused: bool = False):
        self.eng = engine
        self.skip_last_eval = bool(skip_last_eval)
        # fused: each ply() is ONE rvz_play launch (Engine.play: search + the h2 evaluator +
        # act + autoreset per workgroup) instead of the per-batch launches; same games
        self.fused = bool(fused)
        self.play_group = 0       # Engine.play's games_per_workgroup (0: the task queue default)
        if self.fused and not fused_softmax:
            raise ValueError("the fused runner plays with fused_softmax")
        if self.fused and record and autoreset:
            raise ValueError("a recording fused runner plays whole games (no autoreset)")
        # fused_bookkeeping: ply counting and autoreset in one engine kernel (rvz_env_autoreset)
        # instead of ~12 small torch kernels per ply; the games are the same either way
        self.fused_bookkeeping = bool(fused_bookkeeping)
        self.evaluator = evaluator
        self.temperature = float(temperature)
        self.fused_softmax = fused_softmax
        self.autoreset = autoreset
        self.seed_base = seed_base
        self.seed_stride = engine.n_games if seed_stride is None else int(seed_stride)
        self.record = record
        G, dev = engine.n_games, engine.device
        self.seeds = (torch.arange(G, dtype=torch.int64, device=dev) + seed_base)
        self._plies = torch.zeros(G, dtype=torch.int64, device=dev)   # committed plies per slot
        self._done = torch.zeros(G, dtype=torch.int64, device=dev)    # finished games per slot
        self.pre_black = torch.zeros(G, dtype=torch.int64, device=dev)
        self.pre_white = torch.zeros(G, dtype=torch.int64, device=dev)
        self.pre_status = torch.zeros(G, 4, dtype=torch.int32, device=dev)
        self.post_status = torch.zeros(G, 4, dtype=torch.int32, device=dev)
        self._seed32 = torch.zeros(G, dtype=torch.int32, device=dev)
        self._mask = torch.zeros(G, dtype=torch.uint8, device=dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        if record:
            self.rec_black = torch.zeros(max_plies, G, dtype=torch.int64, device=dev)
            self.rec_white = torch.zeros(max_plies, G, dtype=torch.int64, device=dev)
            self.rec_side = torch.zeros(max_plies, G, dtype=torch.int32, device=dev)
            self.rec_idx = torch.full((max_plies, G), -2, dtype=torch.int32, device=dev)
            self.rec_p = torch.zeros(max_plies, G, engine.npol, dtype=torch.float64, device=dev)
            self.rec_over = torch.zeros(max_plies, G, 4, dtype=torch.int32, device=dev)
        self.ply_index = 0
        if self.fused:       # play()'s buffers exist before any capture (Engine.play_buffers)
            engine.play_buffers(evaluator)

    @property
    def steps(self) -> torch.Tensor:
        """Committed plies (board-steps) over all slots, a 0-d device tensor."""
        return self._plies.sum()

    @property
    def games_done(self) -> torch.Tensor:
        return self._done.sum()

    def start(self):
        self.eng.reset(self.seeds)
        self.ply_index = 0

    def check(self):
        """Synchronise; raise RvzError on a device error word or an evaluator overflow
        (Engine.check)."""
        self.eng.check()

    # one ply for every game; graph-capturable (no host sync)
    def _body(self, plies: int = 1):
        eng = self.eng
        if self.fused:
            rec, hist = None, None
            if self.record:   # plies [ply_index, ply_index + plies) of the records, in place
                k, n = self.ply_index, plies
                if k + n > self.rec_idx.shape[0]:
                    raise ValueError("records are full (max_plies)")
                rec = (self.rec_black[k:k + n], self.rec_white[k:k + n], self.rec_side[k:k + n],
                       self.rec_p[k:k + n])
                hist = self.rec_idx[k:k + n]
            eng.play(self.evaluator, plies, self.temperature, self.seeds, self.seed_stride,
                     self._plies, self._done, reset=self.autoreset,
                     skip_last_eval=self.skip_last_eval, hist=hist,
                     games_per_workgroup=self.play_group, records=rec)
            if self.record:
                self.post_status.copy_(eng.get_state()[2])
            return
        if self.record:          # the states before the move, for the game records
            b, w, st = eng.get_state()
            self.pre_black.copy_(b)
            self.pre_white.copy_(w)
            self.pre_status.copy_(st)
        eng.search(self.evaluator, fused_softmax=self.fused_softmax,
                   skip_last_eval=self.skip_last_eval)
        idx, _ = eng.act(self.temperature, apply=True)
        if self.record:
            self.post_status.copy_(eng.get_state()[2])
        if self.fused_bookkeeping:
            eng.autoreset(idx, self.seeds, self.seed_stride, self._plies, self._done,
                          reset=self.autoreset)
            return
        self._plies += (idx >= 0).to(torch.int64)
        if self.autoreset:
            self.restart_finished(eng.get_state()[2])

    def restart_finished(self, status: torch.Tensor):
        """Restart games that just ended with the next seed of their slot (graph-capturable;
        the torch form of rvz_env_autoreset's reset)."""
        over = status[:, 1]
        self._done += over.to(torch.int64)
        self.seeds += over.to(torch.int64) * self.seed_stride
        self._mask.copy_(over.to(torch.uint8))
        self._seed32.copy_(self.seeds.bitwise_and(0xFFFFFFFF).to(torch.int32))
        self.eng.reset_device(self._seed32, self._mask)

    def capture(self, plies: int = 1):
        """Capture `plies` plies into one HIP graph (call after at least one eager ply warmed the
        kernels); ply() then replays them all (plies_per_call)."""
        if plies < 1 or (plies > 1 and self.record and not self.fused) or (self.record and
                                                                          self.fused):
            raise ValueError("plies >= 1; a recording runner captures one ply per graph (the "
                             "fused recording runner writes to the ply's record slice: use "
                             "play_record)")
        torch.cuda.synchronize(self.eng.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            if self.fused:
                self._body(plies)          # one launch plays them all
            else:
                for _ in range(plies):
                    self._body()
        self.graph = g
        self.plies_per_call = int(plies)
        torch.cuda.synchronize(self.eng.device)

    plies_per_call = 1        # plies one ply() call plays (a captured multi-ply graph: more)

    def play_record(self, plies: int):
        """Fused recording runner: `plies` plies of every game in one rvz_play launch, recorded
        into plies [ply_index, ply_index + plies) of the records."""
        if not (self.fused and self.record):
            raise ValueError("play_record is the fused recording runner's")
        self._body(plies)
        self.ply_index += plies

    def ply(self):
        """One ply of every game (a captured graph: plies_per_call plies)."""
        if self.graph is not None:
            self.graph.replay()
        else:
            self._body()
        if self.record and self.fused:
            self.ply_index += 1
            return
        if self.record:
            k = self.ply_index
            self.rec_black[k].copy_(self.pre_black)
            self.rec_white[k].copy_(self.pre_white)
            self.rec_side[k].copy_(self.pre_status[:, 0])
            self.rec_idx[k].copy_(self.eng.idx_buf)
            self.rec_p[k].copy_(self.eng.p_buf)
            self.rec_over[k].copy_(self.post_status)
        self.ply_index += 1


class LaneRunner:
    """``lanes`` independent SelfPlayRunners ("lanes"), one stream per lane, captured into ONE HIP
    graph with a fork / join (or one graph per lane, capture(free_run=True)). The lanes share
    nothing, so while one lane runs its FC heads, k_step or the tail of its trunk kernel, the
    other lanes' trunk workgroups fill the CUs (tools/exp_lanes.py: two 2048-board evaluator
    chains in one graph take 0.443 ms per call against 0.458 for one 4096-board chain).
    The games are split in order into lanes whose sizes differ by at most one (the first
    n_games % lanes lanes hold one more); game g of a lane starting at global game o is global
    game o + g with the same seed as in one runner of n_games: the games, trees and moves are
    those of the single-lane run.

    make_engine(n) -> Engine, make_evaluator() -> a callable owning its own output buffers."""

    def __init__(self, make_engine: Callable[[int], Engine], make_evaluator: Callable,
                 n_games: int, lanes: int = 2, temperature: float = 1.0,
                 fused_softmax: bool = True, autoreset: bool = False, seed_base: int = 42,
                 seed_stride: int = None, skip_last_eval: bool = False, fused: bool = False):
        if lanes < 1 or n_games < lanes:
            raise ValueError("need 1 <= lanes <= n_games")
        sizes = [n_games // lanes + (1 if k < n_games % lanes else 0) for k in range(lanes)]
        offsets = [sum(sizes[:k]) for k in range(lanes)]
        stride = n_games if seed_stride is None else int(seed_stride)
        self.runners = [SelfPlayRunner(make_engine(gl), make_evaluator(), temperature,
                                       fused_softmax, autoreset, seed_base + o,
                                       seed_stride=stride, skip_last_eval=skip_last_eval,
                                       fused=fused)
                        for gl, o in zip(sizes, offsets)]
        dev = self.runners[0].eng.device
        self.streams = [torch.cuda.Stream(dev) for _ in range(lanes)]
        self.temperature = float(temperature)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.lane_graphs = []         # capture(free_run=True): one graph per lane

    @property
    def steps(self) -> torch.Tensor:
        self.join()
        return torch.stack([r.steps for r in self.runners]).sum()

    @property
    def games_done(self) -> torch.Tensor:
        self.join()
        return torch.stack([r.games_done for r in self.runners]).sum()

    def join(self):
        """Make the current stream wait for every lane (free-running lanes are not joined per
        ply)."""
        main = torch.cuda.current_stream(self.runners[0].eng.device)
        for s in self.streams:
            main.wait_stream(s)

    def start(self):
        for r in self.runners:
            r.start()

    def check(self):
        self.join()
        for r in self.runners:
            r.check()

    def _body(self):
        main = torch.cuda.current_stream(self.runners[0].eng.device)
        for r, s in zip(self.runners, self.streams):
            s.wait_stream(main)
            with torch.cuda.stream(s):
                r._body()
        for s in self.streams:
            main.wait_stream(s)

    def capture(self, free_run: bool = False, plies: int = 1):
        """One graph holding every lane with a fork / join per ply, or (free_run) one graph per
        lane replayed on the lane's own stream: the lanes then drift freely against each other
        (no per-ply join bubble) and meet only at join() / a device synchronisation. `plies`
        plies go into each graph (ply() then plays them all): fewer graph launch boundaries."""
        if plies < 1:
            raise ValueError("plies >= 1")
        dev = self.runners[0].eng.device
        torch.cuda.synchronize(dev)
        if free_run:
            self.lane_graphs = []
            for r, s in zip(self.runners, self.streams):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    if r.fused:
                        r._body(plies)
                    else:
                        for _ in range(plies):
                            r._body()
                self.lane_graphs.append(g)
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(plies):
                    self._body()
            self.graph = g
        self.plies_per_call = int(plies)
        torch.cuda.synchronize(dev)

    plies_per_call = 1

    def ply(self):
        if self.lane_graphs:
            main = torch.cuda.current_stream(self.runners[0].eng.device)
            for g, s in zip(self.lane_graphs, self.streams):
                s.wait_stream(main)
                with torch.cuda.stream(s):
                    g.replay()
        elif self.graph is not None:
            self.graph.replay()
        else:
            self._body()


class SelfPlay:
    """self_play.py:21-219 with the games of one call played in lockstep on the GPU.

    Randomness. The reference samples every move with np.random.choice (mcts.py:684), i.e. one
    random_sample() from NumPy's GLOBAL stream per move at temperature > 0, and plays the games
    of one generate_games call one after another (self_play.py:66-101); the stream is seeded once
    per pipeline (pipeline.py:74-80) and SelfPlay takes no seed (pipeline.py:152-168). By default
    this class draws exactly that: game k's moves take the k-th contiguous piece of the caller's
    np.random stream, and np.random is left where the sequential loop leaves it. The lockstep
    games cannot know in advance where their piece starts (it depends on the earlier games'
    lengths), so the call plays passes (as rvz.arena does for tournaments): every game first
    assumes that each earlier game drew bs*bs - 4 values (a full board; true of all but ~0.1 %
    of games), the games are played in lockstep with their pieces handed to the engine
    (Engine.set_draws), each game's actual draw count is read back (Engine.draws), and only the
    games whose start offset changed are played again. A game's moves are a function of its
    piece alone (searches are per game, bit for bit), game 0's offset is always exact, and once
    games 0..k are exact so is game k + 1, so the passes end; `reference_order_passes` reports
    the count (1 unless an earlier game ended before the board was full).

    args["seed"] (opt-in, the round 1-5 behaviour): game i of the j-th game played by this
    object instead draws from its own np.random.seed(seed + j) stream, and np.random is not
    touched.
    """

    def __init__(self, model, args: dict, evaluator: Optional[Callable] = None):
        """evaluator: the leaf evaluator (default: rvz.network.leaf_evaluator(model): the fp32 h2
        kernels, or for a net they do not cover the module on the GPU, ModuleEvaluator).
        Any callable leaf_x -> (logits, value) works; with ``outputs_probs = True`` it returns
        softmaxed rows instead of logits, and a ``bind(engine)`` method is called with each new
        engine (tests replay the reference's recorded NN outputs this way).
        args["fused"] (default: True with the h2 LeafEvaluator, the default evaluator): every game
        of a pass is played to its end in ONE rvz_play launch (Engine.play: search, the h2 trunk
        and heads, act, records) instead of the pull-style ply loop; the same games, bit for bit
        (tests/test_gpu_dropin.py). Another evaluator always runs pull-style."""
        from .network import LeafEvaluator, leaf_evaluator
        self.model = model
        self.device = next(model.parameters()).device
        if self.device.type != "cuda":
            self.device = torch.device("cuda", torch.cuda.current_device())
            self.model = model.to(self.device)
        self.model.eval()
        self.args = args
        self.evaluator = evaluator if evaluator is not None else leaf_evaluator(
            self.model, dtype=args.get("nn_dtype", torch.float32), device=self.device)
        self.board_size = int(getattr(model, "board_size", 8))
        self.save_dir = args.get("save_dir", "self_play_data")
        os.makedirs(self.save_dir, exist_ok=True)
        self.seed = None if args.get("seed") is None else int(args["seed"])
        self.fused = bool(args.get("fused", isinstance(self.evaluator, LeafEvaluator)))
        if self.fused and not isinstance(self.evaluator, LeafEvaluator):
            raise ValueError("SelfPlay: args['fused'] plays the h2 LeafEvaluator inside the "
                             "launch; another evaluator goes through the pull-style loop")
        self.games_played = 0
        self.reference_order_passes = 0

    def _run(self, num_games: int, seed_base: int, draws: Optional[np.ndarray] = None):
        """Play num_games fresh games to their end; draws (float64 [num_games, RVZ_DRAWS]):
        each game's move-sampling values (None: game i draws from np.random.seed(seed_base + i)).
        Returns the records (rec_black, rec_white, rec_side, rec_idx [P, G], rec_p [P, G, npol],
        final status [G, 4]) and the draws each game consumed (int32 [G], host)."""
        # compacted leaf batches: only the live leaves are evaluated (as _process_batch does);
        # the NN-output memo (Engine.memo) with the default evaluator, whose rows depend only on
        # the position; the games are identical either way
        from .network import LeafEvaluator
        bs = self.board_size
        eng = Engine(num_games, self.args.get("num_simulations", 800),
                     self.args.get("batch_size", 64), self.args.get("c_puct", 1.0),
                     board_size=bs, device=self.device,
                     compact_leaves=bool(self.args.get("compact_leaves", True)),
                     memo=bool(self.args.get("memo", isinstance(self.evaluator, LeafEvaluator)
                                             and self.args.get("fused_softmax", True))))
        if hasattr(self.evaluator, "bind"):
            self.evaluator.bind(eng)
        max_plies = bs * bs - 4         # every ply places a disc (passes are inside make_move)
        run = SelfPlayRunner(eng, self.evaluator, self.args.get("temperature", 1.0),
                             fused_softmax=self.args.get("fused_softmax", True),
                             seed_base=seed_base, record=True, max_plies=max_plies,
                             fused=self.fused)
        run.start()
        if draws is not None:
            eng.set_draws(torch.from_numpy(np.ascontiguousarray(draws, np.float64)))
        if self.fused:
            run.play_record(max_plies)
        else:
            for _ in range(max_plies):
                run.ply()
        run.check()
        if not bool(run.post_status[:, 1].all()):
            raise RuntimeError(f"SelfPlay: a game is not over after {max_plies} plies")
        used = eng.draws().cpu().numpy()
        return (run.rec_black, run.rec_white, run.rec_side, run.rec_idx, run.rec_p,
                run.post_status.clone()), used

    def _play_reference_order(self, num_games: int):
        """The passes of the class docstring over NumPy's global stream. Returns (records of
        every pass, game -> (pass, column))."""
        from ._lib import RVZ_DRAWS
        T = float(self.args.get("temperature", 1.0))
        passes, where, _ = sequential_draw_passes(
            num_games, self.board_size ** 2 - 4, RVZ_DRAWS, T > 0, np.random,
            lambda U: self._run(len(U), 0, draws=U))
        self.reference_order_passes = len(passes)
        return passes, where


    def _play(self, num_games: int) -> List[Dict]:
        if num_games <= 0:
            self._last_records = None
            return []
        if self.seed is not None:
            recs, _ = self._run(num_games, self.seed + self.games_played)
            passes, where = [recs], [(0, g) for g in range(num_games)]
            self.reference_order_passes = 0
        else:
            passes, where = self._play_reference_order(num_games)
        # one record set in game order: the columns of the pass that last played each game
        base = np.concatenate([[0], np.cumsum([r[3].shape[1] for r in passes])[:-1]])
        col = torch.tensor([int(base[p]) + j for p, j in where], device=self.device)
        recs = [torch.cat([r[i] for r in passes], dim=1).index_select(1, col)
                for i in range(5)]
        recs.append(torch.cat([r[5] for r in passes], dim=0).index_select(0, col))
        self._last_records = recs
        bs = self.board_size
        G, P = num_games, bs * bs - 4
        black, white, side, idx_t, p_t, final_t = recs
        st = torch.stack([side, torch.zeros_like(side), torch.full_like(side, -1),
                          torch.zeros_like(side)], dim=-1).reshape(-1, 4).contiguous()
        planes = board_canonical(black.reshape(-1).contiguous(), white.reshape(-1).contiguous(),
                                 st, bs).reshape(P, G, 3, bs, bs)
        planes, idx, p = planes.cpu().numpy(), idx_t.cpu().numpy(), p_t.cpu().numpy()
        side_h, final = side.cpu().numpy(), final_t.cpu().numpy()
        games = []
        for g in range(G):
            live = np.flatnonzero(idx[:, g] >= 0)
            winner = int(final[g, 2]) if final[g, 1] else None
            players = [int(side_h[k, g]) for k in live]
            values = [0.0 if winner == 0 else (1.0 if pl == winner else -1.0) for pl in players]
            games.append({"states": [planes[k, g] for k in live],
                          "action_probs": [p[k, g] for k in live],
                          "current_players": players, "values": values, "winner": winner})
        self.games_played += G
        return games

    def training_tensors(self) -> Dict[str, torch.Tensor]:
        """The last call's games as device training arrays (rvz.trainer.records_to_training)."""
        from .trainer import records_to_training
        if getattr(self, "_last_records", None) is None:
            raise ValueError("SelfPlay.training_tensors: no games played by the last call")
        return records_to_training(*self._last_records, self.board_size)

    def generate_games(self, num_games: int) -> List[Dict]:
        t0 = time.time()
        games = self._play(num_games)
        stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
        for i, gd in enumerate(games):
            rec = {k: gd[k] for k in ("states", "action_probs", "current_players", "values")}
            torch.save(rec, os.path.join(self.save_dir, f"game_{stamp}_{i}.pt"))
        print(f"SelfPlay: {num_games} games in {time.time() - t0:.1f}s")
        return games

    def generate_training_data(self, num_games: int) -> Optional[Dict[str, np.ndarray]]:
        """self_play.py:161-219: states (n,3,S,S), action_probs (n,S*S+1), values (n,1), float32,
        built on the device from the engine's records (games in order, plies in order)."""
        games = self.generate_games(num_games)
        if not any(g["states"] for g in games):
            return None
        t = self.training_tensors()
        return {"states": t["states"].cpu().numpy(),
                "action_probs": t["policy_targets"].cpu().numpy(),
                "values": t["value_targets"].cpu().numpy()}


def sequential_draw_passes(num_games: int, max_draws: int, piece: int, draws_on: bool, rng,
                           play: Callable):
    """Lockstep passes that give every game the piece of ONE random_sample() stream it would
    draw if the games ran one after another (SelfPlay's class docstring; self_play.py:66-101
    with mcts.py:684). rng: a NumPy RandomState or the np.random module (its state is read once
    and advanced at the end by exactly the values the sequential loop draws). A game draws at
    most max_draws values (one per move; none when draws_on is False, i.e. temperature 0,
    mcts.py:679-681). play(U float64 [k, piece]) plays k fresh games, game j drawing U[j, 0],
    U[j, 1], ... in order, and returns (payload, used int [k]: the values each game drew).
    Returns (payloads of every pass, game -> (pass, index in that pass), draws per game)."""
    G = int(num_games)
    rs = np.random.RandomState()
    rs.set_state(rng.get_state())
    stream = rs.random_sample(G * max_draws + piece)
    n = np.full(G, max_draws if draws_on else 0, np.int64)   # first guess: the longest game
    prev: List[Optional[int]] = [None] * G
    where: List = [None] * G
    payloads = []
    while True:
        off = np.concatenate([[0], np.cumsum(n)[:-1]]).astype(np.int64)
        todo = [g for g in range(G) if prev[g] != int(off[g])]
        if not todo:
            break
        payload, used = play(np.stack([stream[off[g]:off[g] + piece] for g in todo]))
        for j, g in enumerate(todo):
            if not 0 <= int(used[j]) <= max_draws:
                raise RuntimeError(f"game drew {int(used[j])} values (at most {max_draws})")
            n[g], prev[g], where[g] = int(used[j]), int(off[g]), (len(payloads), j)
        payloads.append(payload)
    total = int(n.sum())
    if total:                       # leave the stream where the sequential loop leaves it
        rng.random_sample(total)
    return payloads, where, n
