"""Data-parallel training of the policy/value net on self-play records.

Counterpart of the reference's ``AlphaZeroPipeline._train_epoch`` (src/trainer/pipeline.py:272-366):
AdamW(lr, weight_decay) (:91-97), CrossEntropy against ``argmax`` of the MCTS policy target plus
MSE on the value (:305-327, criterion :107-113), weighted sum, ``clip_grad_norm_`` (:333-337),
optimizer step. Differences by design:

* one process per GPU; the model is wrapped in DistributedDataParallel, whose bucketed gradient
  all-reduce runs over RCCL (backend "nccl" on ROCm) and overlaps the backward pass — the only
  collective of the whole self-play + training loop (config 4 of BASELINE.json);
* every rank trains on its own shard of the global sample order, drawn from one seeded
  permutation, so the global batch of a step is world_size x batch_size;
* the training arrays come straight from the engine's device-side records
  (``records_to_training``): no host round trip, no per-state Python lists.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from .engine import board_canonical


def records_to_training(rec_black: torch.Tensor, rec_white: torch.Tensor, rec_side: torch.Tensor,
                        rec_idx: torch.Tensor, rec_p: torch.Tensor, final_status: torch.Tensor,
                        board_size: int = 8, canonical=None) -> Dict[str, torch.Tensor]:
    """Self-play records [plies, G] -> training arrays in the reference's layout and order.

    states f32 [n,3,S,S] (get_canonical_state of the position before each move), policy_targets
    f32 [n,S*S+1] (get_action_probs' p), value_targets f32 [n,1] = +1/-1/0 from the final winner
    relative to the player to move (self_play.py:117-126); games in order, plies in order
    (pipeline.py:179-246). Only plies that committed a move (rec_idx >= 0) are kept.
    canonical(black, white, status, board_size) -> planes: default the rvz_board_canonical HIP
    kernel (tests on a host without a GPU pass the oracle's restatement).
    """
    if canonical is None:
        canonical = board_canonical
    P, G = rec_idx.shape
    live = (rec_idx >= 0).t().reshape(-1)                    # game-major order
    black = rec_black.t().reshape(-1)[live].contiguous()
    white = rec_white.t().reshape(-1)[live].contiguous()
    side = rec_side.t().reshape(-1)[live]
    st = torch.stack([side, torch.zeros_like(side), torch.full_like(side, -1),
                      torch.zeros_like(side)], dim=1).to(torch.int32).contiguous()
    states = canonical(black, white, st, board_size)
    policy = rec_p.permute(1, 0, 2).reshape(P * G, -1)[live].to(torch.float32)
    winner = final_status[:, 2].to(torch.int32).unsqueeze(0).expand(P, G).t().reshape(-1)[live]
    over = final_status[:, 1].unsqueeze(0).expand(P, G).t().reshape(-1)[live]
    v = torch.where(winner == side.to(torch.int32), 1.0, -1.0)
    v = torch.where(winner == 0, torch.zeros_like(v), v)
    v = torch.where(over != 0, v, -torch.ones_like(v))      # winner None -> -1 (self_play.py:121-126)
    return {"states": states, "policy_targets": policy, "value_targets": v.reshape(-1, 1).float()}


class DDPTrainer:
    def __init__(self, model: nn.Module, lr: float = 1e-3, weight_decay: float = 1e-4,
                 gradient_clip: float = 1.0, policy_loss_weight: float = 1.0,
                 value_loss_weight: float = 1.0, batch_size: int = 64, bucket_cap_mb: int = 25,
                 lr_milestones=(), lr_gamma: float = 0.1):
        """Defaults = the reference's TrainingConfig (config.py:46-60): AdamW(lr 1e-3, weight decay
        1e-4), clip 1.0, loss weights 1, batch 64, MultiStepLR(milestones [], gamma 0.1)
        (pipeline.py:91-105), stepped once per iteration (scheduler_step, pipeline.py:131)."""
        self.model = model
        self.device = next(model.parameters()).device
        self.distributed = dist.is_available() and dist.is_initialized()
        if self.distributed:
            kw = {"device_ids": [self.device.index]} if self.device.type == "cuda" else {}
            # gradients of ~3 M parameters (10x128) = 11.9 MB: one 25 MB bucket, one all-reduce
            self.net = nn.parallel.DistributedDataParallel(model, bucket_cap_mb=bucket_cap_mb,
                                                           broadcast_buffers=True, **kw)
        else:
            self.net = model
        self.opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=weight_decay)
        self.scheduler = torch.optim.lr_scheduler.MultiStepLR(self.opt, milestones=list(lr_milestones),
                                                              gamma=lr_gamma)
        self.clip = gradient_clip
        self.wp, self.wv = policy_loss_weight, value_loss_weight
        self.batch_size = batch_size

    @torch.no_grad()
    def sync_buffers(self):
        """Broadcast rank 0's BN running statistics: DDP broadcasts buffers before each forward,
        but the last forward of an epoch updates them locally, so without this the ranks would
        self-play with slightly different nets."""
        if not self.distributed:
            return
        for b in self.model.buffers():
            dist.broadcast(b, 0)

    def scheduler_step(self):
        """The per-iteration learning-rate step of the reference's train loop (pipeline.py:131)."""
        self.scheduler.step()

    def rank_world(self):
        return (dist.get_rank(), dist.get_world_size()) if self.distributed else (0, 1)

    def train_step(self, states, policy_targets, value_targets):
        """One optimizer step (pipeline.py:297-340); returns (loss, policy_loss, value_loss)."""
        self.net.train()
        self.opt.zero_grad()
        logits, value = self.net(states)
        policy_loss = F.cross_entropy(logits.view(-1, logits.size(-1)),
                                      policy_targets.argmax(dim=1))
        value_loss = F.mse_loss(value.squeeze(-1), value_targets.reshape(-1))
        loss = self.wp * policy_loss + self.wv * value_loss
        loss.backward()                      # DDP: bucketed RCCL all-reduce during backward
        if self.clip > 0:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.clip)
        self.opt.step()
        return loss.detach(), policy_loss.detach(), value_loss.detach()

    def train_epoch(self, data: Dict[str, torch.Tensor], seed: int = 0,
                    max_steps: Optional[int] = None, local_data: bool = False
                    ) -> Dict[str, float]:
        """One pass over the data. local_data=False: `data` is identical on every rank and each
        rank takes every world-th batch of one seeded permutation. local_data=True: every rank
        holds its own data (its own self-play games, rvz.pipeline) and walks its own permutation
        (seed * world + rank). Either way each step's global batch is world x batch_size, and
        every rank runs the same number of steps (the minimum over ranks). Returns the
        reference's averaged loss dict (pipeline.py:342-366), averaged over ranks too.
        Order: the permutation the reference's DataLoader(shuffle=True) draws when handed a
        generator seeded with `seed` (its base-seed draw, then randperm(n)). On one
        process the last partial batch is trained too, as the reference's DataLoader (no
        drop_last) does; across ranks every step is a full world x batch_size batch."""
        rank, world = self.rank_world()
        ranks = world
        n = data["states"].shape[0]
        # local data: one stream per (seed, rank) pair, seed * world + rank, so rank r at seed s
        # never repeats rank r + 1's shuffle at seed s - 1 (the pipeline passes seed + iteration)
        g = torch.Generator().manual_seed(seed * world + rank if local_data else seed)
        # DataLoader(shuffle=True, generator=g) first draws its workers' base seed from g, then
        # the RandomSampler's permutation: the same two draws give the same batches
        torch.empty((), dtype=torch.int64).random_(generator=g)
        order = torch.randperm(n, generator=g)
        if local_data:
            rank, world = 0, 1        # indexing within this rank's own permutation
        per_step = self.batch_size * world
        partial = not self.distributed and world == 1
        steps = -(-n // per_step) if partial else n // per_step
        if max_steps is not None:
            steps = min(steps, max_steps)
        if self.distributed:          # every rank must run the same number of DDP steps
            t = torch.tensor([steps], dtype=torch.int64,
                             device=self.device if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            steps = int(t.item())
        tot = torch.zeros(3, dtype=torch.float64, device=self.device)
        for s in range(steps):
            idx = order[s * per_step + rank * self.batch_size:
                        s * per_step + (rank + 1) * self.batch_size].to(self.device)
            losses = self.train_step(data["states"][idx], data["policy_targets"][idx],
                                     data["value_targets"][idx])
            tot += torch.stack([x.double() for x in losses])
        tot /= max(1, steps)
        if self.distributed and ranks > 1:   # the job's loss: the mean over ranks
            t = tot.to(self.device if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t)
            tot = t / ranks
        return {"train/loss": float(tot[0]), "train/policy_loss": float(tot[1]),
                "train/value_loss": float(tot[2]), "train/lr": self.opt.param_groups[0]["lr"],
                "steps": steps}
