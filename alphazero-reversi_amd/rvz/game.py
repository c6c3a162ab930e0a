"""Drop-in ``Board`` / ``ReversiGame`` (reference: src/game/board.py, src/game/game.py).

Same attributes, method names, argument meaning, return values and error behaviour as the
reference classes, but every rule evaluation (move generation, flips, auto-pass, terminal and
winner, canonical planes) runs in the rvz HIP kernels (rvz_board_legal / rvz_board_apply /
rvz_board_canonical) on a one-board batch. The Python objects only mirror the state (two
bitboards + counters) so attribute access works as in the reference; they never evaluate a rule.

``Board.is_valid_move`` (board.py:253-285, a file-masked rule nothing in the reference calls)
and the unused private helpers ``_get_flipped_pieces`` / ``_check_game_over`` are not mirrored.

These classes are the single-game API. The batched self-play path keeps all games in HBM
(``rvz.engine.Engine``) and never round-trips through them.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .engine import board_apply, board_canonical, board_legal, to_signed64, to_unsigned64

_DEVICE = None


def _device():
    global _DEVICE
    if _DEVICE is None:
        if not torch.cuda.is_available():
            raise RuntimeError("rvz.game needs a HIP device: its rules run only in the HIP kernels")
        _DEVICE = torch.device("cuda", torch.cuda.current_device())
    return _DEVICE


def _upload(black: int, white: int, side: int, over: int, winner: int, passed: int):
    dev = _device()
    b = torch.tensor([to_signed64(black)], dtype=torch.int64, device=dev)
    w = torch.tensor([to_signed64(white)], dtype=torch.int64, device=dev)
    st = torch.tensor([[side, over, winner, passed]], dtype=torch.int32, device=dev)
    return b, w, st


def _moves_from_mask(mask: int, size: int) -> List[Tuple[int, int]]:
    return [divmod(s, size) for s in range(size * size) if (mask >> s) & 1]


class Board:
    """Bitboard Reversi board (board.py:10-431). Bit i <-> square (i // 8, i % 8)."""

    SIZE = 8
    BOARD_SIZE = SIZE * SIZE
    EMPTY, BLACK, WHITE = 0, 1, 2

    def __init__(self, size: int = 8):
        if size != 8:
            raise ValueError("Only 8x8 board is supported")
        self.size = size
        self.black = 0x0000000810000000
        self.white = 0x0000001008000000
        self.current_player = self.BLACK
        self.game_over = False
        self.winner = None
        self.move_history = []
        self.passed_moves_in_a_row = 0
        self._board = np.zeros((size, size), dtype=int)
        self._update_board_state()

    # -- mirror of the bitboards as the (8, 8) int array the reference keeps (board.py:45-55)
    def _update_board_state(self) -> None:
        bits = np.arange(self.size * self.size, dtype=np.uint64)
        b = (np.uint64(self.black & 0xFFFFFFFFFFFFFFFF) >> bits) & np.uint64(1)
        w = (np.uint64(self.white & 0xFFFFFFFFFFFFFFFF) >> bits) & np.uint64(1)
        self._board = np.where(b == 1, self.BLACK, np.where(w == 1, self.WHITE, self.EMPTY)) \
            .astype(int).reshape(self.size, self.size)

    def _ensure_board_updated(self) -> None:
        self._update_board_state()

    def copy(self) -> "Board":
        nb = Board(self.size)
        nb.black, nb.white = self.black, self.white
        nb.current_player = self.current_player
        nb.game_over, nb.winner = self.game_over, self.winner
        nb.move_history = self.move_history.copy()
        nb.passed_moves_in_a_row = self.passed_moves_in_a_row
        nb._update_board_state()
        return nb

    def _legal_mask(self, player: int) -> int:
        b, w, st = _upload(self.black, self.white, player, 0, -1, 0)
        return to_unsigned64(int(board_legal(b, w, st)[0].item()))

    def get_valid_moves(self, player: int = None) -> List[Tuple[int, int]]:
        if player is None:
            player = self.current_player
        return _moves_from_mask(self._legal_mask(player), self.size)

    def make_move(self, row: int, col: int, player: int = None) -> bool:
        """board.py:135-251 (no game_over check at board level, as the reference)."""
        if player is None:
            player = self.current_player
        if row == -1 and col == -1:
            sq = -1
        else:
            sq = row * 8 + col
            if sq < 0:
                raise ValueError("negative shift count")  # `1 << (row * 8 + col)`, board.py:170
            if sq >= 64:
                return False
        b, w, st = _upload(self.black, self.white, player, 0, -1, self.passed_moves_in_a_row)
        ok = bool(board_apply(b, w, st, torch.tensor([sq], dtype=torch.int32,
                                                     device=b.device))[0].item())
        if not ok:
            return False
        side, over, winner, passed = (int(x) for x in st[0].tolist())
        self.black, self.white = to_unsigned64(int(b[0].item())), to_unsigned64(int(w[0].item()))
        self.move_history.append((row, col, player))
        self.current_player = side
        self.passed_moves_in_a_row = passed
        if over:
            self.game_over = True
            self.winner = winner
        self._update_board_state()
        return True

    def has_any_valid_move(self, player: int = None) -> bool:
        return self._legal_mask(self.current_player if player is None else player) != 0

    def get_board_state(self) -> np.ndarray:
        self._ensure_board_updated()
        return self._board.copy()

    def get_score(self) -> Tuple[int, int]:
        return self.bit_count(self.black), self.bit_count(self.white)

    @staticmethod
    def bit_count(x: int) -> int:
        return bin(x & 0xFFFFFFFFFFFFFFFF).count("1")

    def __call__(self, row: int, col: int, player: int = None) -> bool:
        return self.make_move(row, col, player)

    def __str__(self) -> str:
        sym = {self.EMPTY: ".", self.BLACK: "B", self.WHITE: "W"}
        self._update_board_state()
        rows = [" ".join(sym[int(v)] for v in r) for r in self._board]
        out = ["\n".join(rows),
               f"Current player: {'Black' if self.current_player == self.BLACK else 'White'}"]
        b, w = self.get_score()
        out.append(f"Score - Black: {b}, White: {w}")
        if self.game_over:
            out.append("Game over! It's a draw!" if self.winner == 0 else
                       f"Game over! {'Black' if self.winner == self.BLACK else 'White'} wins!")
        return "\n".join(out)


class ReversiGame:
    """Game wrapper (game.py:9-192): move history, game-level over/winner/current_player."""

    def __init__(self, size: int = 8):
        self.board = Board(size)
        self.size = size
        self.current_player = Board.BLACK
        self.game_over = False
        self.winner = None
        self.move_history: List[Dict[str, Any]] = []

    def reset(self) -> None:
        self.__init__(self.size)

    def make_move(self, row: int, col: int) -> bool:
        if self.game_over:
            return False
        before = self.board.copy()
        ok = self.board.make_move(row, col, self.current_player)
        if ok:
            self.move_history.append({"player": self.current_player, "move": (row, col),
                                      "board_before": before, "board_after": self.board.copy()})
            self.game_over = self.board.game_over
            self.winner = self.board.winner
            self.current_player = self.board.current_player
        return ok

    def get_valid_moves(self) -> List[Tuple[int, int]]:
        return self.board.get_valid_moves(self.current_player)

    def is_game_over(self) -> bool:
        return self.board.game_over

    def get_winner(self) -> Optional[int]:
        return self.board.winner if self.game_over else None

    def get_score(self) -> Tuple[int, int]:
        return self.board.get_score()

    def get_board_state(self) -> np.ndarray:
        return self.board.get_board_state()

    def get_current_player(self) -> int:
        return self.current_player

    def get_move_history(self) -> List[Dict[str, Any]]:
        return self.move_history.copy()

    def get_canonical_state(self) -> np.ndarray:
        """[current player's discs, opponent's discs, legal moves] float32 (game.py:131-162)."""
        b, w, st = _upload(self.board.black, self.board.white, self.current_player, 0, -1, 0)
        return board_canonical(b, w, st)[0].cpu().numpy()

    def copy(self) -> "ReversiGame":
        g = ReversiGame(self.size)
        g.board = self.board.copy()
        g.current_player = self.current_player
        g.game_over = self.game_over
        g.winner = self.winner
        g.move_history = self.move_history.copy()
        return g

    # engine interop: the state tuple the batched engine stores per game
    def state_tuple(self):
        b = self.board
        return (b.black, b.white, self.current_player, int(bool(b.game_over)),
                -1 if b.winner is None else int(b.winner), int(b.passed_moves_in_a_row))

    def __str__(self) -> str:
        return str(self.board)
