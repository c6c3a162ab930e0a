"""Host mirror of the rvz engine: owns one C-ABI engine (include/rvz.h) and its device buffers.

One ``Engine`` = ``n_games`` Reversi games resident in HBM, each with its own MCTS tree.
It is what the reference's per-game ``ReversiGame`` + ``MCTS`` pair becomes when all games of a
self-play batch are advanced in lockstep (self_play.py:80-101, mcts.py:322-694):

    eng.reset(seeds)                      # ReversiGame() x n + np.random.seed per game
    eng.search(evaluator)                 # MCTS.search for every live game
    idx, p = eng.act(temperature)         # get_action_probs tail + game.make_move

Every tensor handed to the library is a device tensor on ``eng.device``; all work is enqueued on
the current torch stream of that device (graph-capturable: no host syncs inside ``search``/``act``).
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import RVZ_DONE, RVZ_LEAF_BF16, RVZ_LEAF_F32, RvzError, check, ptr

U64 = 0xFFFFFFFFFFFFFFFF


def to_signed64(x: int) -> int:
    x &= U64
    return x - (1 << 64) if x >> 63 else x


def to_unsigned64(x: int) -> int:
    return int(x) & U64


class Engine:
    def __init__(self, n_games: int, num_simulations: int = 800, batch_size: int = 64,
                 c_puct: float = 1.0, board_size: int = 8, device=None,
                 leaf_dtype: torch.dtype = torch.float32, compact_leaves: bool = False,
                 memo: bool = False):
        if not torch.cuda.is_available():
            raise RvzError("rvz needs a HIP device (MI355X); there is no CPU fallback")
        self.lib = _lib.load()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.n_games, self.board_size = int(n_games), int(board_size)
        self.num_simulations, self.batch_size = int(num_simulations), int(batch_size)
        self.c_puct = float(c_puct)
        self.nsq = board_size * board_size
        self.npol = self.nsq + 1
        if leaf_dtype not in (torch.float32, torch.bfloat16):
            raise RvzError("leaf_dtype must be torch.float32 or torch.bfloat16")
        self.leaf_dtype = leaf_dtype
        cfg = _lib.Config(board_size, n_games, num_simulations, batch_size, c_puct,
                          self.device.index,
                          RVZ_LEAF_F32 if leaf_dtype == torch.float32 else RVZ_LEAF_BF16)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            check(self.lib.rvz_create(C.byref(cfg), C.byref(h)), None, "rvz_create")
        self._h = h
        G, dev = self.n_games, self.device
        self.leaf_x = torch.zeros(G, 3, board_size, board_size, dtype=leaf_dtype, device=dev)
        self.need = torch.zeros(G, dtype=torch.int32, device=dev)
        self.visits_buf = torch.zeros(G, self.npol, dtype=torch.int32, device=dev)
        self.p_buf = torch.zeros(G, self.npol, dtype=torch.float64, device=dev)
        self.idx_buf = torch.zeros(G, dtype=torch.int32, device=dev)
        self.black = torch.zeros(G, dtype=torch.int64, device=dev)
        self.white = torch.zeros(G, dtype=torch.int64, device=dev)
        self.status = torch.zeros(G, 4, dtype=torch.int32, device=dev)
        self.n_batches = -(-num_simulations // batch_size)
        self.compact_leaves = False
        if compact_leaves:
            self.compact(True)
        self.memo_on = False
        if memo:
            self.memo(True)

    # ------------------------------------------------------------------ plumbing
    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self.lib.rvz_destroy(h)
            self._h = None

    def _stream(self):
        s = _lib.stream_handle(self.device)
        check(self.lib.rvz_set_stream(self._h, s), self._h, "rvz_set_stream")

    def _call(self, name: str, *args) -> int:
        return check(getattr(self.lib, name)(self._h, *args), self._h, name)

    def check(self) -> None:
        """Synchronise and raise RvzError if a kernel set the device error word (node pool, path
        depth, RNG stream, non-finite NN output) or an evaluator this engine's searches used
        reports an activation overflow (LeafEvaluator.overflowed: h2's sticky device word).
        Both are accumulated on the device and read only here, so graph replays stay sync-free."""
        self._stream()
        err = C.c_int32(0)
        self._call("rvz_check", C.byref(err))
        for ev in getattr(self, "_evaluators", ()):
            of = getattr(ev, "overflowed", None)
            if of is not None and of():
                raise RvzError(f"leaf evaluator ({getattr(ev, 'kernel', type(ev).__name__)}) "
                               "overflowed its f16 activation range (|x| >= 65520) even in the "
                               "ranged re-run: the NN outputs of the searches are not valid")

    def counters(self) -> Tuple[int, int]:
        out = (C.c_int64 * 2)()
        self.lib.rvz_counters(self._h, out)
        return int(out[0]), int(out[1])

    def footprint(self) -> Tuple[int, int]:
        a, b = C.c_int64(), C.c_int64()
        self.lib.rvz_footprint(self._h, C.byref(a), C.byref(b))
        return a.value, b.value

    def stats_enable(self, on: bool = True):
        self._stream()
        self._call("rvz_stats_enable", int(bool(on)))

    def stats_read(self):
        """Algorithmic bytes moved since stats_enable: (select, expand_backup, act)."""
        self._stream()
        out = (C.c_int64 * 3)()
        self._call("rvz_stats_read", out)
        return int(out[0]), int(out[1]), int(out[2])

    def timing_enable(self, on: bool = True):
        self._call("rvz_timing_enable", int(bool(on)))

    def timing_read(self):
        """Mean ms per launch and launch counts of k_step / k_act since timing_enable."""
        self._stream()
        ms, n = (C.c_double * 2)(), (C.c_int32 * 2)()
        self._call("rvz_timing_read", ms, n)
        return {"step": (ms[0], n[0]), "act": (ms[1], n[1])}

    def tree(self):
        """(nodes int32[G, M, 4] = {N, W, P, C} (W/P/C as float32 bits), meta uint32-as-int32[G, M])."""
        self._stream()
        M = self.lib.rvz_tree_nodes(self._h)
        nodes = torch.empty(self.n_games, M, 4, dtype=torch.int32, device=self.device)
        meta = torch.empty(self.n_games, M, dtype=torch.int32, device=self.device)
        self._call("rvz_tree_export", ptr(nodes), ptr(meta))
        return nodes, meta

    # ------------------------------------------------------------------ env
    def reset(self, seeds: Optional[Sequence[int]] = None, mask: Optional[torch.Tensor] = None):
        """ReversiGame() for every (masked) game + np.random.seed(seeds[g]) per game."""
        self._stream()
        if seeds is None:
            seeds = range(self.n_games)
        if not isinstance(seeds, torch.Tensor):
            seeds = torch.tensor([int(s) & 0xFFFFFFFF for s in seeds], dtype=torch.int64)
        s = seeds.to(self.device).to(torch.int64).bitwise_and(0xFFFFFFFF).to(torch.int32)
        if s.numel() != self.n_games:
            raise RvzError("one seed per game")
        m = None if mask is None else mask.to(self.device, torch.uint8).contiguous()
        self._seeds = s.contiguous()
        self._call("rvz_env_reset", ptr(self._seeds), ptr(m) if m is not None else None)

    def reset_device(self, seeds_i32: torch.Tensor, mask_u8: Optional[torch.Tensor] = None):
        """Graph-capturable reset: persistent int32 seeds / uint8 mask device tensors."""
        self._stream()
        self._call("rvz_env_reset", ptr(seeds_i32), ptr(mask_u8) if mask_u8 is not None else None)

    def autoreset(self, idx: torch.Tensor, seeds: torch.Tensor, stride: int,
                  plies: torch.Tensor, done: torch.Tensor, reset: bool = True):
        """rvz_env_autoreset: count committed plies per game; restart finished games with their
        slot's next seed (seeds int64 [G] advanced in place by stride). Graph-capturable."""
        for t, dt in ((idx, torch.int32), (seeds, torch.int64), (plies, torch.int64),
                      (done, torch.int64)):
            if t.dtype != dt or t.numel() != self.n_games or not t.is_contiguous():
                raise RvzError("autoreset: idx int32, seeds/plies/done int64, [n_games]")
        self._stream()
        self._call("rvz_env_autoreset", ptr(idx), ptr(seeds), int(stride), ptr(plies), ptr(done),
                   int(bool(reset)))

    def set_draws(self, u: torch.Tensor):
        """rvz_env_set_draws: game g's move-sampling draws become u[g] (float64 [G, RVZ_DRAWS],
        the values np.random.random_sample() would return), each game rewound to its first."""
        uu = u.to(self.device, torch.float64).contiguous()
        if uu.shape != (self.n_games, _lib.RVZ_DRAWS):
            raise RvzError(f"set_draws: u must be float64 [{self.n_games}, {_lib.RVZ_DRAWS}]")
        self._stream()
        self._call("rvz_env_set_draws", ptr(uu))
        self._draws_keep = uu          # the copy is stream-ordered: keep the source alive

    def draws(self) -> torch.Tensor:
        """rvz_env_draws: the draws each game consumed since its reset / set_draws (int32 [G])."""
        out = torch.empty(self.n_games, dtype=torch.int32, device=self.device)
        self._stream()
        self._call("rvz_env_draws", ptr(out))
        return out

    def get_state(self):
        """(black int64[G], white int64[G], status int32[G,4]) device tensors (bit patterns)."""
        self._stream()
        self._call("rvz_env_get", ptr(self.black), ptr(self.white), ptr(self.status))
        return self.black, self.white, self.status

    def set_state(self, black: torch.Tensor, white: torch.Tensor, status: torch.Tensor):
        self._stream()
        b = black.to(self.device, torch.int64).contiguous()
        w = white.to(self.device, torch.int64).contiguous()
        st = status.to(self.device, torch.int32).contiguous()
        self._call("rvz_env_set", ptr(b), ptr(w), ptr(st))
        torch.cuda.current_stream(self.device).synchronize()  # b, w, st are temporaries

    def legal(self) -> torch.Tensor:
        self._stream()
        out = torch.empty(self.n_games, dtype=torch.int64, device=self.device)
        self._call("rvz_env_legal", ptr(out))
        return out

    def apply(self, sq: torch.Tensor) -> torch.Tensor:
        self._stream()
        s = sq.to(self.device, torch.int32).contiguous()
        ok = torch.empty(self.n_games, dtype=torch.int32, device=self.device)
        self._call("rvz_env_apply", ptr(s), ptr(ok))
        return ok

    # ------------------------------------------------------------------ fused self-play
    def play_buffers(self, evaluator=None):
        """Allocate what play() needs (the row counter, the launch scratch, the evaluator's
        overflow word) outside any graph capture: allocated inside one, their zero-fill would be
        recorded into the graph and every replay would reset the counter."""
        if getattr(self, "play_rows", None) is None:   # rows evaluated by play() calls
            self.play_rows = torch.zeros(1, dtype=torch.int64, device=self.device)
            # {table hits, table inserts} of play() calls (rvz_play_table)
            self.table_stats = torch.zeros(2, dtype=torch.int64, device=self.device)
        n = self.lib.rvz_play_scratch_size(self._h)
        sc = getattr(self, "_play_scratch", None)
        if sc is None or sc.numel() < n:
            self._play_scratch = torch.zeros(n, dtype=torch.float32, device=self.device)
        if evaluator is not None and hasattr(evaluator, "ovf_word"):
            evaluator.ovf_word()

    def play(self, evaluator, plies: int, temperature: float, seeds: torch.Tensor, stride: int,
             plies_done: torch.Tensor, games_done: torch.Tensor, reset: bool = True,
             skip_last_eval: bool = False, hist: Optional[torch.Tensor] = None,
             games_per_workgroup: int = 0, budget: Optional[torch.Tensor] = None,
             records=None):
        """rvz_play: every game commits `plies` plies (search of num_simulations + move + the
        autoreset bookkeeping of autoreset()) in ONE launch, the h2 LeafEvaluator's trunk and
        heads inside it; the same games, moves and counters as search() + act() + autoreset()
        with that evaluator (fused_softmax). idx_buf / p_buf: each game's last act. hist: int32
        [plies, n_games] for every act's index, or None. budget: int32 [n_games], game g commits
        min(plies, budget[g]) plies (the others stay as they are), or None. records: (black
        int64 [plies, G], white int64 [plies, G], side int32 [plies, G], p float64
        [plies, G, npol]): the position before every act and its policy vector (hist: the move;
        p_buf is then not written), or None. Graph-capturable once play_buffers() ran outside
        the capture (it runs here on the first eager call)."""
        from .network import LeafEvaluator
        if not isinstance(evaluator, LeafEvaluator):
            raise RvzError("play() runs the h2 LeafEvaluator inside the launch; another "
                           "evaluator goes through search() / act()")
        if evaluator.board_size != self.board_size or evaluator.device != self.device:
            raise RvzError("play(): the evaluator's board size / device differ from the engine's")
        for t, dt in ((seeds, torch.int64), (plies_done, torch.int64), (games_done, torch.int64)):
            if t.dtype != dt or t.numel() != self.n_games or not t.is_contiguous():
                raise RvzError("play: seeds / plies_done / games_done int64 [n_games]")
        if hist is not None and (hist.dtype != torch.int32 or hist.shape != (plies, self.n_games)
                                 or not hist.is_contiguous()):
            raise RvzError("play: hist int32 [plies, n_games]")
        if budget is not None and (budget.dtype != torch.int32 or budget.numel() != self.n_games
                                   or not budget.is_contiguous()
                                   or budget.device != self.device):
            raise RvzError("play: budget int32 [n_games] on the engine's device")
        rec = (None,) * 4
        if records is not None and hist is None:
            # the C-ABI's record contract: hist holds each recorded act's move (out_p is not
            # written when records are given), so records without hist would lose the moves
            raise RvzError("play: records need hist (the moves of the recorded plies)")
        if records is not None:
            rb, rw, rs, rp = records
            G = self.n_games
            if not (rb.dtype == rw.dtype == torch.int64 and rs.dtype == torch.int32
                    and rp.dtype == torch.float64 and rb.shape == rw.shape == rs.shape
                    == (plies, G) and rp.shape == (plies, G, self.npol)
                    and all(t.is_contiguous() and t.device == self.device
                            for t in (rb, rw, rs, rp))):
                raise RvzError("play: records = (black int64, white int64 [plies, G], side int32 "
                               "[plies, G], p float64 [plies, G, npol]) on the engine's device")
            rec = tuple(t.data_ptr() for t in records)
        n = self.lib.rvz_play_scratch_size(self._h)
        ready = (getattr(self, "play_rows", None) is not None and
                 getattr(self, "_play_scratch", None) is not None and
                 self._play_scratch.numel() >= n and getattr(evaluator, "_ovf", None) is not None)
        if not ready:
            if torch.cuda.is_current_stream_capturing():
                raise RvzError("play() inside a graph capture before its buffers exist: call "
                               "Engine.play_buffers(evaluator) (or one eager play) first")
            self.play_buffers(evaluator)
        sc = self._play_scratch
        self._bind(evaluator)
        a = _lib.PlayArgs(evaluator.params.data_ptr(), evaluator.wsplit.data_ptr(),
                          evaluator.filters, evaluator.n_blocks, sc.data_ptr(),
                          evaluator.ovf_word().data_ptr(), int(plies), int(bool(skip_last_eval)),
                          int(bool(reset)), int(games_per_workgroup), float(temperature),
                          seeds.data_ptr(), int(stride), plies_done.data_ptr(),
                          games_done.data_ptr(), self.idx_buf.data_ptr(), self.p_buf.data_ptr(),
                          hist.data_ptr() if hist is not None else None,
                          self.play_rows.data_ptr(),
                          budget.data_ptr() if budget is not None else None,
                          self.table_stats.data_ptr(), *rec)
        self._stream()
        self._call("rvz_play", C.byref(a))

    def _bind(self, evaluator):
        """Remember the evaluator (check() reads its overflow word) and register this engine with
        it: LeafEvaluator.refresh() (new weights) then drops this engine's memo links itself."""
        evs = self.__dict__.setdefault("_evaluators", [])
        if not any(e is evaluator for e in evs):
            evs.append(evaluator)
            reg = getattr(evaluator, "bind_engine", None)
            if reg is not None:
                reg(self)

    def table(self, slots: int = 1 << 20, max_discs: int = 14):
        """rvz_play_table: the cross-game NN-output table of play() (slots = 0: off). A leaf whose
        position has at most max_discs discs takes the logits and value an earlier evaluation of
        the same position stored (any game of this engine, same weights): the same games, fewer
        evaluated rows. New weights: memo_reset() / LeafEvaluator.refresh() start a new
        generation. Call before capturing a graph."""
        self._stream()
        self._call("rvz_play_table", int(slots), int(max_discs))
        self.table_slots = int(slots)

    def play_gate(self, fraction: float = -1.0, timeout_us: float = 0.0, late_us: float = 0.0):
        """rvz_play_gate: the per-XCD pass gate of play()'s 8x8 forms of 128 / 256 filters (fraction 0: off; < 0:
        the default 0.8 / 400 us / 200 us). Timing only: the same games with any setting."""
        self._call("rvz_play_gate", float(fraction), float(timeout_us), float(late_us))

    # ------------------------------------------------------------------ search
    def search_begin(self):
        self._call("rvz_search_begin")

    def search_step(self) -> bool:
        """One batch up to the NN call. False once every batch of this search was issued."""
        self._stream()
        rc = self._call("rvz_search_step", ptr(self.leaf_x), ptr(self.need))
        return rc != RVZ_DONE

    def compact(self, on: bool = True):
        """Compacted leaf batches (rvz_search_compact): the leaves that need an evaluation go to
        rows [0, U) of leaf_x, U on the device (live_count()); an evaluator with
        ``accepts_live_count`` evaluates only those rows (mcts.py:544-623 evaluates U leaves).
        Same visits, p and moves as the uncompacted search."""
        self._call("rvz_search_compact", int(bool(on)))
        self.compact_leaves = bool(on)

    def memo(self, on: bool = True):
        """NN-output memo across consecutive searches (rvz_search_memo): a leaf whose position
        the game's previous search expanded takes that expansion's priors and value instead of
        a new evaluation (the reference re-evaluates it: it rebuilds the tree every move,
        mcts.py:334). Same visits, p and moves; fewer evaluated rows. The evaluator must be
        row-deterministic and unchanged between searches: memo_reset() after new weights."""
        self._stream()
        self._call("rvz_search_memo", int(bool(on)))
        self.memo_on = bool(on)

    def memo_reset(self):
        """Forget the carried expansions (new evaluator weights); graph-capturable."""
        self._stream()
        self._call("rvz_search_memo_reset")

    def live_count(self) -> int:
        """Device address of the int32 live-row count of the most recently issued batch."""
        a = self.lib.rvz_search_live_count(self._h)
        if not a:
            raise RvzError("no live count: compaction off or no batch issued")
        return int(a)

    def rows_total(self) -> int:
        """Live rows evaluated over all completed searches (compaction on; the rows of a last
        batch left by skip_last_eval are not counted)."""
        out = C.c_int64()
        self._call("rvz_search_rows_total", C.byref(out))
        return int(out.value)

    def search_submit(self, policy: torch.Tensor, value: torch.Tensor, is_logits: bool):
        if policy.dtype != torch.float32 or value.dtype != torch.float32:
            raise RvzError("policy/value must be float32")
        if policy.shape != (self.n_games, self.npol) or value.shape != (self.n_games,):
            raise RvzError(f"policy must be [{self.n_games},{self.npol}], value [{self.n_games}]")
        self._stream()
        self._call("rvz_search_submit", ptr(policy), int(bool(is_logits)), ptr(value))
        # the expand + backup is deferred into the next launch: keep the rows alive until then
        self._keep = (policy, value)

    def search_skip(self):
        """Leave the last batch unevaluated (rvz_search_skip): same visits, p and move."""
        self._stream()
        self._call("rvz_search_skip")

    def search(self, evaluator: Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]],
               fused_softmax: bool = True, skip_last_eval: bool = False):
        """MCTS.search for every live game. evaluator(leaf_x) -> (logits, value), or
        (probabilities, value) when the evaluator has ``outputs_probs = True``.

        fused_softmax=False applies torch's F.softmax (the reference's mcts.py:596) before the
        expand kernel instead of the kernel's fused softmax. skip_last_eval=True does not
        evaluate the last batch (rvz_search_skip; bit-identical visits, one NN call fewer) when
        a search has two batches or more: a single batch's leaf is the root, which the act needs
        expanded, so it is evaluated."""
        self._bind(evaluator)
        self.search_begin()
        k = 0
        while self.search_step():
            k += 1
            if skip_last_eval and k == self.n_batches > 1:
                self.search_skip()
                break
            if self.compact_leaves and getattr(evaluator, "accepts_live_count", False):
                logits, value = evaluator(self.leaf_x, n_live=self.live_count())
            else:
                logits, value = evaluator(self.leaf_x)
            logits = logits.float().contiguous()
            value = value.float().contiguous()
            if getattr(evaluator, "outputs_probs", False):
                # the evaluator hands over softmaxed rows (e.g. recorded reference outputs)
                self.search_submit(logits, value, False)
            elif fused_softmax:
                self.search_submit(logits, value, True)
            else:
                self.search_submit(torch.softmax(logits, dim=1).contiguous(), value, False)

    def visits(self) -> torch.Tensor:
        self._stream()
        self._call("rvz_search_visits", ptr(self.visits_buf))
        return self.visits_buf

    def act(self, temperature: float = 1.0, u: Optional[torch.Tensor] = None,
            apply: bool = True):
        """get_action_probs tail (+ make_move): returns (idx int32[G], p float64[G,npol])."""
        self._stream()
        uu = None
        if u is not None:
            uu = u.to(self.device, torch.float64).contiguous()
            self._u_keep = uu
        self._call("rvz_act", float(temperature), ptr(uu) if uu is not None else None,
                   int(bool(apply)), ptr(self.idx_buf), ptr(self.p_buf))
        return self.idx_buf, self.p_buf


# -------------------------------------------------------------------------- board kernels
def board_legal(black: torch.Tensor, white: torch.Tensor, status: torch.Tensor,
                board_size: int = 8) -> torch.Tensor:
    lib = _lib.load()
    n = black.numel()
    out = torch.empty(n, dtype=torch.int64, device=black.device)
    check(lib.rvz_board_legal(board_size, n, ptr(black), ptr(white), ptr(status), ptr(out),
                              _lib.stream_handle(black.device)), None, "rvz_board_legal")
    return out


def board_apply(black: torch.Tensor, white: torch.Tensor, status: torch.Tensor, sq: torch.Tensor,
                board_size: int = 8) -> torch.Tensor:
    """In place on (black, white, status); returns make_move's bool per board."""
    lib = _lib.load()
    n = black.numel()
    ok = torch.empty(n, dtype=torch.int32, device=black.device)
    check(lib.rvz_board_apply(board_size, n, ptr(black), ptr(white), ptr(status),
                              ptr(sq.to(torch.int32).contiguous()), ptr(ok),
                              _lib.stream_handle(black.device)), None, "rvz_board_apply")
    return ok


def board_canonical(black: torch.Tensor, white: torch.Tensor, status: torch.Tensor,
                    board_size: int = 8) -> torch.Tensor:
    lib = _lib.load()
    n = black.numel()
    out = torch.empty(n, 3, board_size, board_size, dtype=torch.float32, device=black.device)
    check(lib.rvz_board_canonical(board_size, n, ptr(black), ptr(white), ptr(status), ptr(out),
                                  _lib.stream_handle(black.device)), None, "rvz_board_canonical")
    return out


def policy_softmax(logits: torch.Tensor, board_size: int = 8) -> torch.Tensor:
    """rvz_policy_softmax: F.softmax(logits, dim=1) (mcts.py:596) exactly as the engine's expand
    computes it from logits (the fused softmax of search_submit(is_logits=True) and of play())."""
    lib = _lib.load()
    lg = logits.float().contiguous()
    n = lg.shape[0]
    if lg.shape != (n, board_size * board_size + 1):
        raise RvzError(f"logits must be [n, {board_size * board_size + 1}]")
    out = torch.empty_like(lg)
    check(lib.rvz_policy_softmax(board_size, n, ptr(lg), ptr(out), _lib.stream_handle(lg.device)),
          None, "rvz_policy_softmax")
    return out
