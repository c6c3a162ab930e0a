"""ctypes wrapper of the CPU oracle (oracle/rvz_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the checker) and
bench.py's cpu_baseline leg. The product package (alphazero-reversi_amd/rvz) never imports it.

Mirrors the reference's Python surface closely enough that tests read like the reference's own:
``legal``/``flips``/``Game.make_move`` follow src/game/board.py + src/game/game.py, ``Search``
follows src/mcts/mcts.py (MCTS.search / get_action_probs), ``MT`` follows numpy's legacy
RandomState seeding + random_sample.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "librvz_oracle.so")
# RVZ_ORACLE_LIB: load another build of the same sources instead (tests/test_oracle_sanitize.py
# points it at the ASan/UBSan build, librvz_oracle_san.so)
_LIB_OVERRIDE = os.environ.get("RVZ_ORACLE_LIB")


class Game(C.Structure):
    _fields_ = [("black", C.c_uint64), ("white", C.c_uint64), ("side", C.c_int32),
                ("over", C.c_int32), ("winner", C.c_int32), ("passed", C.c_int32)]

    def copy(self) -> "Game":
        g = Game()
        C.pointer(g)[0] = self
        return g

    def astuple(self):
        return (int(self.black), int(self.white), int(self.side), int(self.over),
                int(self.winner), int(self.passed))


class _MT(C.Structure):
    _fields_ = [("key", C.c_uint32 * 624), ("pos", C.c_int32)]


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "rvz_oracle.c"))):
        subprocess.run(["make", "-C", _HERE, "librvz_oracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(_LIB_OVERRIDE or build())
        L = _lib
        u64, i32, f64 = C.c_uint64, C.c_int32, C.c_double
        L.rvzo_legal.restype = u64
        L.rvzo_legal.argtypes = [C.c_int, u64, u64]
        L.rvzo_flips.restype = u64
        L.rvzo_flips.argtypes = [C.c_int, C.c_int, u64, u64]
        L.rvzo_game_init.argtypes = [C.c_int, C.POINTER(Game)]
        L.rvzo_make_move.restype = C.c_int
        L.rvzo_make_move.argtypes = [C.c_int, C.POINTER(Game), C.c_int]
        L.rvzo_canonical.argtypes = [C.c_int, C.POINTER(Game), C.c_void_p]
        L.rvzo_mt_seed.argtypes = [C.POINTER(_MT), C.c_uint32]
        L.rvzo_mt_next32.restype = C.c_uint32
        L.rvzo_mt_next32.argtypes = [C.POINTER(_MT)]
        L.rvzo_mt_res53.restype = f64
        L.rvzo_mt_res53.argtypes = [C.POINTER(_MT)]
        L.rvzo_np_sum.restype = f64
        L.rvzo_np_sum.argtypes = [C.c_void_p, C.c_int]
        L.rvzo_action.restype = C.c_int
        L.rvzo_action.argtypes = [C.c_int, C.c_void_p, f64, f64, C.c_void_p, C.POINTER(i32)]
        L.rvzo_action_needs_draw.restype = C.c_int
        L.rvzo_action_needs_draw.argtypes = [C.c_int, C.c_void_p, f64]
        L.rvzo_create.restype = C.c_void_p
        L.rvzo_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, f64]
        L.rvzo_destroy.argtypes = [C.c_void_p]
        L.rvzo_search_begin.restype = C.c_int
        L.rvzo_search_begin.argtypes = [C.c_void_p, C.c_void_p]
        L.rvzo_search_step.restype = C.c_int
        L.rvzo_search_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.rvzo_search_submit.restype = C.c_int
        L.rvzo_search_submit.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.rvzo_search_visits.restype = C.c_int
        L.rvzo_search_visits.argtypes = [C.c_void_p, C.c_void_p]
        L.rvzo_stats.argtypes = [C.c_void_p, C.c_void_p]
    return _lib


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


# ---------------------------------------------------------------- rules (board.py / game.py)
def legal(P: int, O: int, bs: int = 8) -> int:
    return int(lib().rvzo_legal(bs, P, O))


def flips(sq: int, P: int, O: int, bs: int = 8) -> int:
    return int(lib().rvzo_flips(bs, sq, P, O))


def new_game(bs: int = 8) -> Game:
    g = Game()
    lib().rvzo_game_init(bs, C.byref(g))
    return g


def make_move(g: Game, sq: int, bs: int = 8) -> bool:
    return bool(lib().rvzo_make_move(bs, C.byref(g), sq))


def canonical(g: Game, bs: int = 8) -> np.ndarray:
    out = np.zeros((3, bs, bs), np.float32)
    lib().rvzo_canonical(bs, C.byref(g), _ptr(out))
    return out


# ---------------------------------------------------------------- numpy legacy RNG
class MT:
    """np.random.seed(s) + random_sample() restated (legacy MT19937)."""

    def __init__(self, seed: int):
        self._s = _MT()
        lib().rvzo_mt_seed(C.byref(self._s), seed & 0xFFFFFFFF)

    def next32(self) -> int:
        return int(lib().rvzo_mt_next32(C.byref(self._s)))

    def random_sample(self) -> float:
        return float(lib().rvzo_mt_res53(C.byref(self._s)))


def np_sum(a: np.ndarray) -> float:
    a = np.ascontiguousarray(a, np.float64)
    return float(lib().rvzo_np_sum(_ptr(a), a.size))


def action(visits: np.ndarray, temperature: float, u: float = 0.0):
    """mcts.py:656-692 tail. Returns (index, p[npol] f64, consumed_draw)."""
    v = np.ascontiguousarray(visits, np.int32)
    p = np.zeros(v.size, np.float64)
    nd = C.c_int32(0)
    idx = lib().rvzo_action(v.size, _ptr(v), float(temperature), float(u), _ptr(p), C.byref(nd))
    return int(idx), p, bool(nd.value)


def action_needs_draw(visits: np.ndarray, temperature: float) -> bool:
    v = np.ascontiguousarray(visits, np.int32)
    return bool(lib().rvzo_action_needs_draw(v.size, _ptr(v), float(temperature)))


# ---------------------------------------------------------------- batched reference search
class Search:
    """G independent reference-semantics searches (mcts.py MCTS.search), pull-style evaluator."""

    def __init__(self, n_games: int, num_simulations: int = 800, batch_size: int = 64,
                 c_puct: float = 1.0, bs: int = 8):
        self.bs, self.G, self.npol = bs, n_games, bs * bs + 1
        self._h = lib().rvzo_create(bs, n_games, num_simulations, batch_size, float(c_puct))
        if not self._h:
            raise ValueError("rvzo_create rejected the configuration")
        self._leaf = (Game * n_games)()
        self.n_copies = np.zeros(n_games, np.int32)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().rvzo_destroy(self._h)
            self._h = None

    def begin(self, roots):
        arr = (Game * self.G)(*roots)
        lib().rvzo_search_begin(self._h, C.cast(arr, C.c_void_p))

    def step(self):
        """Returns None when the search is done, else (leaf games list, n_copies[G])."""
        r = lib().rvzo_search_step(self._h, C.cast(self._leaf, C.c_void_p), _ptr(self.n_copies))
        if r == 1:
            return None
        if r < 0:
            raise RuntimeError("oracle search step: distinct leaves inside one batch")
        return [self._leaf[g] for g in range(self.G)], self.n_copies.copy()

    def submit(self, probs: np.ndarray, values: np.ndarray):
        p = np.ascontiguousarray(probs, np.float32).reshape(self.G, self.npol)
        v = np.ascontiguousarray(values, np.float32).reshape(self.G)
        lib().rvzo_search_submit(self._h, _ptr(p), _ptr(v))

    def visits(self) -> np.ndarray:
        out = np.zeros((self.G, self.npol), np.int32)
        lib().rvzo_search_visits(self._h, _ptr(out))
        return out

    def stats(self) -> np.ndarray:
        out = np.zeros(4, np.int64)
        lib().rvzo_stats(self._h, _ptr(out))
        return out


def leaf_planes(leaves, bs: int = 8) -> np.ndarray:
    return np.stack([canonical(g, bs) for g in leaves])
