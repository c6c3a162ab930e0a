"""Drop-in ``MCTS`` (reference: src/mcts/mcts.py:191-719).

Same constructor, ``search(game) -> {move: visit_count}``,
``get_action_probs(game, temperature) -> ((row, col), float64[65])`` and
``update_with_move(move)`` as the reference; the tree, the traversals, expansion, backup and
action selection run in the rvz HIP kernels on a one-game engine. The model is the reference's
model protocol (``parameters()``, ``eval()``, ``predict(x) -> (logits, value)``, mcts.py:211,235,
501), called once per batch of ``batch_size`` simulations exactly where the reference calls it.

Randomness: the reference samples with the global NumPy RNG (``np.random.choice``, mcts.py:684);
this class draws that same ``np.random.random_sample()`` value on the host and hands it to the
act kernel, so a caller's ``np.random.seed`` drives both identically. Within one batch the
reference evaluates ``batch_size`` identical copies of the same leaf; rvz evaluates
that leaf once and backs its value up ``copies`` times, which is exact.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .engine import Engine, to_signed64


class MCTS:
    def __init__(self, model, c_puct: float = 1.0, num_simulations: int = 800,
                 batch_size: int = 64, num_threads: int = 1, use_transposition: bool = True):
        self.model = model
        self.device = next(model.parameters()).device
        self.c_puct = c_puct
        self.num_simulations = num_simulations
        self.batch_size = batch_size
        self.num_threads = num_threads            # unused, as in the reference (mcts.py:207)
        self.use_transposition = use_transposition  # inert in the reference (no zobrist hash)
        self.root = None
        self._engines: Dict[int, Engine] = {}
        self.model.eval()

    def _engine(self, size: int) -> Engine:
        eng = self._engines.get(size)
        if eng is None:
            eng = Engine(1, self.num_simulations, self.batch_size, self.c_puct, board_size=size)
            self._engines[size] = eng
        return eng

    def _predict(self, x: torch.Tensor):
        with torch.no_grad():
            logits, value = self.model.predict(x.to(self.device))   # mcts.py:500-501
        return logits, value

    def _run_search(self, game) -> Engine:
        eng = self._engine(game.size)
        b = game.board
        dev = eng.device
        eng.set_state(
            torch.tensor([to_signed64(b.black)], dtype=torch.int64, device=dev),
            torch.tensor([to_signed64(b.white)], dtype=torch.int64, device=dev),
            torch.tensor([[game.current_player, int(bool(b.game_over)),
                           -1 if b.winner is None else int(b.winner),
                           int(b.passed_moves_in_a_row)]], dtype=torch.int32, device=dev))

        def evaluate(x):
            logits, value = self._predict(x)
            # the reference's softmax (mcts.py:596), applied on the model's device
            probs = F.softmax(logits, dim=1)
            return probs.to(dev, torch.float32), value.reshape(-1).to(dev, torch.float32)

        eng.search_begin()
        while eng.search_step():
            probs, value = evaluate(eng.leaf_x)
            eng.search_submit(probs.contiguous(), value.contiguous(), is_logits=False)
        self.root = "rvz"
        return eng

    def search(self, game) -> Dict[Tuple[int, int], int]:
        eng = self._run_search(game)
        return self._visit_dict(eng, game.size)

    def _visit_dict(self, eng: Engine, size: int) -> Dict[Tuple[int, int], int]:
        vis = eng.visits()[0].cpu().numpy()
        legal = int(eng.legal()[0].item()) & 0xFFFFFFFFFFFFFFFF
        if vis.sum() == 0 and legal == 0:
            return {}
        # the root's children are its legal moves in row-major order (mcts.py:605-618)
        return {divmod(s, size): int(vis[s]) for s in range(size * size) if (legal >> s) & 1}

    def get_action_probs(self, game, temperature: float = 1.0):
        eng = self._run_search(game)
        vis = eng.visits()[0].cpu().numpy()
        # np.random.choice consumes one random_sample() unless the argmax branch is taken
        needs_draw = temperature != 0.0 and int(vis.sum()) > 0
        u = None
        if needs_draw:
            u = torch.tensor([np.random.random_sample()], dtype=torch.float64)
        idx, p = eng.act(temperature, u=u if u is not None else torch.zeros(1, dtype=torch.float64),
                         apply=False)
        i = int(idx[0].item())
        probs = p[0].cpu().numpy().copy()
        size = game.size
        action = (-1, -1) if i == size * size else divmod(i, size)
        return action, probs

    def update_with_move(self, move: Optional[Tuple[int, int]] = None):
        """mcts.py:696-719. search() always builds a fresh root, so this has no effect there."""
        if move is None:
            self.root = None
