"""The self-play + training loop of one rank: BASELINE.json config 4 (C4).

Counterpart of ``AlphaZeroPipeline.train``'s iteration (src/trainer/pipeline.py:114-150):
generate self-play games with the current net (``_generate_self_play_data``, :152-246), train on
them (``_train_epoch``, :272-366), repeat. One process per GPU:

* self-play: this rank's ``games`` games from the start position, lockstep on its own engine,
  recorded on the device (``SelfPlayRunner(record=True)``), one ply = one HIP-graph replay;
  global game g of iteration i is seeded ``seed + i * games * world + g`` (games sharded by rank,
  no collective);
* records -> training arrays on the device (``records_to_training``; no host round trip);
* training: ``DDPTrainer`` steps; DDP's bucketed gradient all-reduce over RCCL (backend "nccl"
  on ROCm) during backward is the only collective of the loop; then rank 0's BN statistics are
  broadcast and the evaluator re-reads the weights in place (``LeafEvaluator.refresh``), so the
  captured self-play graph evaluates the new net at its next replay.

The reference's evaluation tournament and checkpointing (:128-140) are out of scope.
"""
from __future__ import annotations

import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

from .engine import Engine
from .network import LeafEvaluator, leaf_evaluator
from .selfplay import SelfPlayRunner
from .trainer import DDPTrainer, records_to_training


class SelfPlayTrainer:
    def __init__(self, model, games: int, num_simulations: int = 800, batch_size: int = 64,
                 c_puct: float = 1.0, temperature: float = 1.0, seed: int = 42,
                 train_steps: Optional[int] = None, train_batch: int = 64, lr: float = 1e-3,
                 weight_decay: float = 1e-4, gradient_clip: float = 1.0,
                 graph: bool = True, compact_leaves: bool = True, lr_milestones=(),
                 lr_gamma: float = 0.1, memo: bool = True, fused: bool = True,
                 table_slots: Optional[int] = None, table_discs: int = 14):
        """table_slots: slots of the fused launch's cross-game NN-output table (0: no table;
        None: the next power of two >= 32 x games, within [2^12, 2^22]: 2^20 for C4's 32,768
        games per rank). Each slot is 576 B of granules + a 4-B claim word on 8x8 (48 granules
        on 6x6): 2^20 slots = 608 MB, 2^12 = 2.4 MB."""
        self.model = model.eval()
        self.device = next(model.parameters()).device
        self.distributed = dist.is_available() and dist.is_initialized()
        self.rank, self.world = ((dist.get_rank(), dist.get_world_size()) if self.distributed
                                 else (0, 1))
        self.games, self.seed = int(games), int(seed)
        self.train_steps = train_steps
        self.trainer = DDPTrainer(model, lr=lr, weight_decay=weight_decay,
                                  gradient_clip=gradient_clip, batch_size=train_batch,
                                  lr_milestones=lr_milestones, lr_gamma=lr_gamma)
        # the h2 kernels when they cover the net, else the module itself on the GPU
        # (ModuleEvaluator: pull-style, eager plies; it reads the live module, so refresh() only
        # drops the memo)
        self.evaluator = leaf_evaluator(model, device=self.device)
        h2 = isinstance(self.evaluator, LeafEvaluator)
        bs = int(getattr(model, "board_size", 8))
        self.eng = Engine(games, num_simulations, batch_size, c_puct, board_size=bs,
                          device=self.device, compact_leaves=compact_leaves, memo=memo)
        self.max_plies = bs * bs - 4
        # fused: every game of the iteration in ONE rvz_play launch with device records, the
        # memo's deferred last batch and the cross-game table (a new generation per refresh());
        # else the pull-style ply graph (per-batch launches, records copied per ply)
        self.fused = bool(fused) and h2
        if table_slots is None:
            table_slots = 1 << min(22, max(12, (32 * self.games - 1).bit_length()))
        if self.fused and table_slots:
            self.eng.table(table_slots, table_discs)
        self.runner = SelfPlayRunner(self.eng, self.evaluator, temperature, record=True,
                                     max_plies=self.max_plies,
                                     seed_base=self.seed + self.rank * self.games,
                                     fused=self.fused, skip_last_eval=self.fused and memo)
        self.graph = bool(graph) and h2
        self.iteration = 0

    def _seeds(self):
        base = self.seed + self.iteration * self.games * self.world + self.rank * self.games
        self.runner.seeds.copy_(torch.arange(self.games, dtype=torch.int64,
                                             device=self.device) + base)

    def generate(self) -> Dict[str, torch.Tensor]:
        """One iteration's self-play: every game of this rank from the start to its end.
        Returns the training arrays (states, policy_targets, value_targets) on the device."""
        run = self.runner
        self._seeds()
        run.start()
        if self.fused:
            run.play_record(self.max_plies)     # one launch: whole games, records on the device
        else:
            for k in range(self.max_plies):
                if self.graph and run.graph is None and k == 1:
                    run.capture()               # after one eager ply (kernel warm-up)
                run.ply()
        run.check()
        if not bool(run.post_status[:, 1].all()):
            raise RuntimeError(f"a game is not over after {self.max_plies} plies")
        return records_to_training(run.rec_black, run.rec_white, run.rec_side, run.rec_idx,
                                   run.rec_p, run.post_status, self.eng.board_size)

    def train(self, data: Dict[str, torch.Tensor]) -> Dict[str, float]:
        """_train_epoch over this iteration's data (each rank walks its own games; DDP averages
        the gradients), then the evaluator picks up the new weights."""
        out = self.trainer.train_epoch(data, seed=self.seed + self.iteration,
                                       max_steps=self.train_steps, local_data=True)
        self.trainer.sync_buffers()
        self.trainer.scheduler_step()          # pipeline.py:131, once per iteration
        self.model.eval()
        self.evaluator.refresh()               # also drops the engine's memo (the old net's outputs)
        return out

    def run_iteration(self) -> Dict[str, float]:
        """generate + train; wall times of both phases (device-synchronised) in the result."""
        dev = self.device
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        steps0 = int(self.runner.steps.item())
        data = self.generate()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        plies = int(self.runner.steps.item()) - steps0
        out = self.train(data)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        self.iteration += 1
        out.update({"selfplay_s": t1 - t0, "train_s": t2 - t1, "board_steps": plies,
                    "samples": int(data["states"].shape[0])})
        return out
