"""ctypes binding of librvz.so (the C-ABI declared in include/rvz.h).

The library is built in-tree (``make -C alphazero-reversi_amd`` or ``__graft_entry__.build()``)
and is the ONLY implementation of the hot path: there is no CPU fallback. Loading fails loudly
when the library is missing, and every call that returns an error code raises ``RvzError``.

torch is imported first so that librvz.so binds to the HIP runtime torch already loaded (both
carry the soname libamdhip64.so.7): torch streams and tensors are then valid in our launches.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RVZ_LIB", os.path.join(_HERE, "librvz.so"))   # RVZ_LIB: experiments

RVZ_OK, RVZ_DONE = 0, 1
RVZ_LEAF_F32, RVZ_LEAF_BF16 = 0, 1
RVZ_DRAWS = 64          # move-sampling draws held per game (rvz_env_set_draws)


class RvzError(RuntimeError):
    pass


class Config(C.Structure):
    _fields_ = [("board_size", C.c_int32), ("n_games", C.c_int32),
                ("num_simulations", C.c_int32), ("batch_size", C.c_int32),
                ("c_puct", C.c_double), ("device", C.c_int32), ("leaf_dtype", C.c_int32)]


# name -> (restype, argtypes); kept in the order of include/rvz.h
_P = C.c_void_p
SIGNATURES = {
    "rvz_version": (C.c_int, []),
    "rvz_create": (C.c_int, [C.POINTER(Config), C.POINTER(_P)]),
    "rvz_destroy": (None, [_P]),
    "rvz_last_error": (C.c_char_p, [_P]),
    "rvz_set_stream": (C.c_int, [_P, _P]),
    "rvz_sync": (C.c_int, [_P]),
    "rvz_check": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "rvz_env_reset": (C.c_int, [_P, _P, _P]),
    "rvz_env_set_draws": (C.c_int, [_P, _P]),
    "rvz_env_draws": (C.c_int, [_P, _P]),
    "rvz_env_get": (C.c_int, [_P, _P, _P, _P]),
    "rvz_env_set": (C.c_int, [_P, _P, _P, _P]),
    "rvz_env_legal": (C.c_int, [_P, _P]),
    "rvz_env_apply": (C.c_int, [_P, _P, _P]),
    "rvz_board_legal": (C.c_int, [C.c_int32, C.c_int32, _P, _P, _P, _P, _P]),
    "rvz_board_apply": (C.c_int, [C.c_int32, C.c_int32, _P, _P, _P, _P, _P, _P]),
    "rvz_board_canonical": (C.c_int, [C.c_int32, C.c_int32, _P, _P, _P, _P, _P]),
    "rvz_policy_softmax": (C.c_int, [C.c_int32, C.c_int32, _P, _P, _P]),
    "rvz_search_begin": (C.c_int, [_P]),
    "rvz_search_step": (C.c_int, [_P, _P, _P]),
    "rvz_search_submit": (C.c_int, [_P, _P, C.c_int32, _P]),
    "rvz_env_autoreset": (C.c_int, [_P, _P, _P, C.c_int64, _P, _P, C.c_int32]),
    "rvz_resnet_h2_grid": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32]),
    "rvz_resnet_trunk_h2_ex": (C.c_int, [C.c_int32, _P, C.c_int32, _P, _P, C.c_int32,
                                         C.c_int32, _P, _P, _P, _P, C.c_int32, _P]),
    "rvz_resnet_heads_fc_ex": (C.c_int, [C.c_int32, _P, C.c_int32, _P, C.c_int32, C.c_int32, _P,
                                         _P, _P, _P, _P]),
    "rvz_resnet_fwd_h2_ex": (C.c_int, [C.c_int32, _P, C.c_int32, _P, _P, C.c_int32, C.c_int32,
                                       _P, _P, _P, _P, _P]),
    "rvz_search_compact": (C.c_int, [_P, C.c_int32]),
    "rvz_search_memo": (C.c_int, [_P, C.c_int32]),
    "rvz_search_memo_reset": (C.c_int, [_P]),
    "rvz_search_live_count": (C.c_void_p, [_P]),
    "rvz_search_rows_total": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "rvz_timer_create": (C.c_int, [C.c_int32, C.POINTER(C.c_void_p)]),
    "rvz_timer_record": (C.c_int, [_P, C.c_int32, _P]),
    "rvz_timer_elapsed": (C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(C.c_float)]),
    "rvz_timer_destroy": (None, [_P]),
    "rvz_search_skip": (C.c_int, [_P]),
    "rvz_search_visits": (C.c_int, [_P, _P]),
    "rvz_act": (C.c_int, [_P, C.c_double, _P, C.c_int32, _P, _P]),
    "rvz_play_scratch_size": (C.c_int64, [_P]),
    "rvz_play": (C.c_int, [_P, _P]),
    "rvz_play_table": (C.c_int, [_P, C.c_int64, C.c_int32]),
    "rvz_play_gate": (C.c_int, [_P, C.c_double, C.c_double, C.c_double]),
    "rvz_counters": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "rvz_stats_enable": (C.c_int, [_P, C.c_int32]),
    "rvz_stats_read": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "rvz_timing_enable": (C.c_int, [_P, C.c_int32]),
    "rvz_timing_read": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_int32)]),
    "rvz_tree_nodes": (C.c_int, [_P]),
    "rvz_tree_export": (C.c_int, [_P, _P, _P]),
    "rvz_footprint": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "rvz_resnet_params_size": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "rvz_resnet_work_size": (C.c_int64, [C.c_int32]),
    "rvz_resnet_heads_fc": (C.c_int, [C.c_int32, _P, C.c_int32, _P, C.c_int32, C.c_int32, _P, _P,
                                      _P]),
    "rvz_resnet_h2_size": (C.c_int64, [C.c_int32, C.c_int32]),
    "rvz_resnet_h2_weights": (C.c_int, [_P, C.c_int32, C.c_int32, _P, _P]),
    "rvz_resnet_trunk_h2": (C.c_int, [C.c_int32, _P, C.c_int32, _P, _P, C.c_int32, C.c_int32,
                                      _P, _P]),
    "rvz_resnet_fwd_h2": (C.c_int, [C.c_int32, _P, C.c_int32, _P, _P, C.c_int32, C.c_int32, _P,
                                    _P, _P, _P]),
}

_lib = None


class PlayArgs(C.Structure):
    """include/rvz.h rvz_play_args (pointers as integers: device addresses)."""
    _fields_ = [("params", C.c_void_p), ("blob", C.c_void_p), ("filters", C.c_int32),
                ("blocks", C.c_int32), ("scratch", C.c_void_p), ("ovf", C.c_void_p),
                ("plies", C.c_int32), ("skip_last_eval", C.c_int32), ("reset", C.c_int32),
                ("games_per_workgroup", C.c_int32), ("temperature", C.c_double),
                ("seeds", C.c_void_p), ("seed_stride", C.c_int64), ("plies_done", C.c_void_p),
                ("games_done", C.c_void_p), ("out_idx", C.c_void_p), ("out_p", C.c_void_p),
                ("hist", C.c_void_p), ("rows_evaluated", C.c_void_p),
                ("ply_budget", C.c_void_p), ("table_stats", C.c_void_p),
                ("rec_black", C.c_void_p), ("rec_white", C.c_void_p), ("rec_side", C.c_void_p),
                ("rec_p", C.c_void_p)]


def load() -> C.CDLL:
    """Load librvz.so (no GPU needed to load; calls that launch kernels need one)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RvzError(f"{LIB_PATH} is missing: build it with `make -C alphazero-reversi_amd` "
                           "(there is no CPU fallback for the rvz hot path)")
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, handle=None, what: str = "") -> int:
    if rc < 0:
        msg = load().rvz_last_error(handle)
        raise RvzError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


def ptr(t) -> int:
    """Device pointer of a contiguous CUDA (HIP) tensor; 16-byte aligned as the kernels assume."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RvzError("rvz buffers must be device tensors (no host fallback)")
    if not t.is_contiguous():
        raise RvzError("rvz buffers must be contiguous")
    p = t.data_ptr()
    if p % 16:
        raise RvzError("rvz buffers must be 16-byte aligned")
    return p


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class Timer:
    """rvz_timer: stream-ordered HIP events without system fence (eager timing)."""

    def __init__(self, n_events: int):
        self.capacity = int(n_events)
        h = C.c_void_p()
        check(load().rvz_timer_create(self.capacity, C.byref(h)), None, "rvz_timer_create")
        self.h = h
        self.used = 0

    def record(self, stream_handle) -> int:
        if self.used >= self.capacity:
            raise RvzError("timer full")
        check(load().rvz_timer_record(self.h, self.used, stream_handle), None, "rvz_timer_record")
        self.used += 1
        return self.used - 1

    def elapsed(self, i: int, j: int) -> float:
        ms = C.c_float()
        check(load().rvz_timer_elapsed(self.h, i, j, C.byref(ms)), None, "rvz_timer_elapsed")
        return float(ms.value)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                load().rvz_timer_destroy(h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
