"""DDPTrainer (rvz/trainer.py; reference pipeline.py:272-366) on CPU with gloo, world_size 2:
after DDP steps every rank holds identical parameters, equal to a single process that averages
the two ranks' per-shard gradients (what DDP's all-reduce computes; BN stays per-shard)."""
import copy
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=512, seed=0):
    g = torch.Generator().manual_seed(seed)
    states = (torch.rand(n, 3, 8, 8, generator=g) > 0.6).float()
    policy = torch.rand(n, 65, generator=g)
    policy = policy / policy.sum(1, keepdim=True)
    values = torch.randint(-1, 2, (n, 1), generator=g).float()
    return {"states": states, "policy_targets": policy, "value_targets": values}


def _model():
    import rvz
    torch.manual_seed(0)
    return rvz.AlphaZeroNetwork(8, 1, 16)


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-reversi_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from rvz import dist as rd
    from rvz.trainer import DDPTrainer
    rd.init("gloo")
    tr = DDPTrainer(_model(), batch_size=64)
    out = tr.train_epoch(_data(), seed=1, max_steps=3)
    # numpy copies: torch tensors would travel as shared-memory handles that die with the worker
    q.put((rank, {k: v.detach().numpy().copy() for k, v in tr.model.state_dict().items()}, out))
    dist.destroy_process_group()


def test_ddp_two_ranks_match_gradient_averaging():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-reversi_amd"))
    import torch.nn.functional as F
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd0 = {k: torch.from_numpy(v) for k, v in res[0][1].items()}
    sd1 = {k: torch.from_numpy(v) for k, v in res[1][1].items()}
    for k in sd0:
        if "running" in k or "num_batches" in k:
            continue
        assert torch.equal(sd0[k], sd1[k]), k          # DDP keeps the replicas identical

    # single-process emulation: per-shard forward/backward (BN on each 64-sample shard),
    # averaged gradients, clip, AdamW step
    model = _model()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    data = _data()
    g = torch.Generator().manual_seed(1)
    torch.empty((), dtype=torch.int64).random_(generator=g)   # DataLoader's base-seed draw
    order = torch.randperm(512, generator=g)
    shadow = copy.deepcopy(model)
    for s in range(3):
        grads = None
        for r in range(world):
            idx = order[s * 128 + r * 64: s * 128 + (r + 1) * 64]
            shadow.load_state_dict(model.state_dict())
            shadow.train()
            shadow.zero_grad()
            logits, v = shadow(data["states"][idx])
            loss = F.cross_entropy(logits, data["policy_targets"][idx].argmax(1)) + \
                F.mse_loss(v, data["value_targets"][idx].reshape(-1))
            loss.backward()
            g = [p.grad.clone() for p in shadow.parameters()]
            grads = g if grads is None else [a + b for a, b in zip(grads, g)]
        for p, g in zip(model.parameters(), grads):
            p.grad = g / world
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
    for k, v in model.state_dict().items():
        if "running" in k or "num_batches" in k:
            continue
        assert torch.allclose(v, sd0[k], rtol=1e-4, atol=1e-5), k
    assert res[0][2]["steps"] == 3 and res[0][2]["train/loss"] > 0


def _reference_train_epoch(model, optimizer, data, batch_size, generator, clip=1.0, wp=1.0,
                           wv=1.0):
    """The reference's AlphaZeroPipeline._train_epoch (src/trainer/pipeline.py:272-366) restated
    line by line: TensorDataset + DataLoader(shuffle=True) (:277-289; its generator made explicit
    so the permutation is reproducible, workers and pinning do not change the math), per batch
    zero_grad, model.predict, CrossEntropyLoss against argmax of the policy target (:305-309,
    criterion :107-113), MSELoss on the squeezed value (:312-320), weighted sum (:323-326),
    backward, clip_grad_norm_ (:333-337), AdamW step (:340), averaged .item() losses (:342-366)."""
    import torch.nn as nn
    from torch.utils.data import DataLoader, TensorDataset
    model.train()
    ds = TensorDataset(torch.FloatTensor(data["states"]), torch.FloatTensor(data["policy_targets"]),
                       torch.FloatTensor(data["value_targets"]))
    loader = DataLoader(ds, batch_size=batch_size, shuffle=True, generator=generator)
    crit = {"policy": nn.CrossEntropyLoss(), "value": nn.MSELoss()}
    tl = tp = tv = 0.0
    for states, pt, vt in loader:
        optimizer.zero_grad()
        logits, vp = model.predict(states)
        pl = crit["policy"](logits.view(-1, logits.size(-1)), pt.argmax(dim=1))
        vp = vp.squeeze(-1)
        if vt.dim() > 1:
            vt = vt.squeeze(-1)
        vl = crit["value"](vp, vt)
        loss = wp * pl + wv * vl
        loss.backward()
        if clip > 0:
            torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
        optimizer.step()
        tl += loss.item()
        tp += pl.item()
        tv += vl.item()
    n = len(loader)
    return {"train/loss": tl / n, "train/policy_loss": tp / n, "train/value_loss": tv / n,
            "train/lr": optimizer.param_groups[0]["lr"]}


def test_trainer_equals_reference_train_epoch_restatement():
    """DDPTrainer on one process == the reference's _train_epoch restated (above) with the
    reference's TrainingConfig defaults (config.py:46-60) and MultiStepLR stepped once per
    iteration (pipeline.py:99-105, :131): bitwise-equal parameters and BN statistics after two
    epochs (200 samples: three full batches and a partial one each, the partial one trained as
    the reference's DataLoader does), equal averaged losses, equal learning rate."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "alphazero-reversi_amd"))
    from rvz.trainer import DDPTrainer
    data = _data(n=200, seed=3)
    a, b = _model(), _model()
    tr = DDPTrainer(a, lr_milestones=[1], lr_gamma=0.1)
    opt = torch.optim.AdamW(b.parameters(), lr=1e-3, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.MultiStepLR(opt, milestones=[1], gamma=0.1)
    for ep in range(2):
        got = tr.train_epoch(data, seed=10 + ep)
        tr.scheduler_step()
        want = _reference_train_epoch(b, opt, data, 64, torch.Generator().manual_seed(10 + ep))
        sched.step()
        assert got["steps"] == 4
        for k in ("train/loss", "train/policy_loss", "train/value_loss", "train/lr"):
            assert abs(got[k] - want[k]) <= 1e-12 * max(1.0, abs(want[k])), (k, got[k], want[k])
    assert tr.opt.param_groups[0]["lr"] == opt.param_groups[0]["lr"] == 1e-4
    sa, sb = a.state_dict(), b.state_dict()
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
