"""C4's loop on one GPU (rvz.pipeline.SelfPlayTrainer; reference pipeline.py:114-150): self-play
with a captured graph -> device records -> DDPTrainer -> the evaluator re-reads the trained net.
The next iteration's self-play must be exactly what a fresh SelfPlay of the trained net plays."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_selfplay_trainer_iterations_use_the_trained_net(tmp_path):
    import rvz
    from rvz.pipeline import SelfPlayTrainer
    torch.manual_seed(0)
    G, S = 64, 200        # four batches: distinct games (asserted below; mcts.py:96-97)
    net = rvz.AlphaZeroNetwork(8, 2, 64).cuda()
    spt = SelfPlayTrainer(net, G, num_simulations=S, seed=7, train_steps=40, train_batch=64)
    r0 = spt.run_iteration()
    assert r0["board_steps"] == r0["samples"] and r0["steps"] == 40
    assert np.isfinite(r0["train/loss"])
    # refresh(): the evaluator (same buffers the graph holds) == a freshly built evaluator
    x = (torch.rand(G, 3, 8, 8, device="cuda") > 0.6).float()
    l1, v1 = spt.evaluator(x)
    l1, v1 = l1.clone(), v1.clone()
    l2, v2 = rvz.LeafEvaluator(net.eval())(x)
    assert torch.equal(l1, l2) and torch.equal(v1, v2)
    # iteration 1 self-play (graph replays) == eager SelfPlay of the trained net, same seeds
    data = spt.generate()
    sp = rvz.SelfPlay(net, {"num_simulations": S, "seed": 7 + G, "save_dir": str(tmp_path)})
    games = sp.generate_games(G)
    t = sp.training_tensors()
    assert torch.equal(t["states"], data["states"])
    assert torch.equal(t["policy_targets"], data["policy_targets"])
    assert torch.equal(t["value_targets"], data["value_targets"])
    assert sum(len(g["states"]) for g in games) == data["states"].shape[0]
    assert len({g["states"][4].tobytes() for g in games}) > 1   # not one game in every slot


def test_c4_shaped_iteration_over_rccl_world1(tmp_path):
    """C4's shape at world 1 (BASELINE.json configs[3]: 10x128 net, 800 sims; 2,048 games on the
    one GPU instead of 32,768): one SelfPlayTrainer iteration with its DDP steps' gradients going
    through RCCL (backend "nccl"), then the next iteration's captured self-play must equal an
    eager SelfPlay of the trained net with the same seeds (reference pipeline.py:114-150)."""
    import socket
    import torch.distributed as dist
    import rvz
    from rvz.pipeline import SelfPlayTrainer
    G, S = 2048, 800
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        net = rvz.AlphaZeroNetwork(8, 10, 128).cuda()
        init = {k: v.clone() for k, v in net.state_dict().items()}
        spt = SelfPlayTrainer(net, G, num_simulations=S, seed=11, train_steps=20, train_batch=64)
        assert spt.distributed and spt.world == 1
        r0 = spt.run_iteration()
        assert r0["board_steps"] == r0["samples"] >= 9 * G and r0["steps"] == 20
        assert np.isfinite(r0["train/loss"])
        moved = max((net.state_dict()[k].float() - init[k].float()).abs().max().item()
                    for k in init if init[k].is_floating_point())
        assert moved > 1e-4                     # the DDP steps changed the weights
        data = spt.generate()                   # iteration 1: graph replays, memo reset
    finally:
        dist.destroy_process_group()
    sp = rvz.SelfPlay(net, {"num_simulations": S, "seed": 11 + G, "save_dir": str(tmp_path)})
    games = sp.generate_games(G)
    t = sp.training_tensors()
    assert sum(len(g["states"]) for g in games) == data["states"].shape[0]
    assert torch.equal(t["states"], data["states"])
    assert torch.equal(t["policy_targets"], data["policy_targets"])
    assert torch.equal(t["value_targets"], data["value_targets"])


@pytest.mark.parametrize("filters", [32, 256])
def test_pipeline_with_other_net_widths(tmp_path, filters):
    """SelfPlayTrainer with a 32- and a 256-filter net (the reference's pipeline takes any
    num_filters, network.py:33). 32: the h2 kernels do not cover it, so the evaluator is the
    module on the GPU (ModuleEvaluator, with a warning), the plies run pull-style and eager;
    256: the h2 kernels and the fused launch with the table. Training changes the weights, and the
    next iteration's games (ModuleEvaluator reads the live module, LeafEvaluator re-reads the
    weights; refresh() drops the memo / table) equal an eager SelfPlay of the trained net with the
    same seeds."""
    import contextlib
    import rvz
    from rvz.pipeline import SelfPlayTrainer
    G, S = 64, 200          # four batches: the games differ
    torch.manual_seed(2)
    net = rvz.AlphaZeroNetwork(8, 2, filters).cuda()
    init = {k: v.clone() for k, v in net.state_dict().items()}
    module = filters == 32
    warn = (lambda: pytest.warns(UserWarning, match="ModuleEvaluator")) if module else \
        contextlib.nullcontext
    with warn():
        spt = SelfPlayTrainer(net, G, num_simulations=S, seed=11, train_steps=5, train_batch=64)
    if module:
        assert isinstance(spt.evaluator, rvz.ModuleEvaluator) and not spt.fused and not spt.graph
    else:
        assert isinstance(spt.evaluator, rvz.LeafEvaluator) and spt.fused
    r0 = spt.run_iteration()
    assert r0["board_steps"] == r0["samples"] >= 9 * G and np.isfinite(r0["train/loss"])
    moved = max((net.state_dict()[k].float() - init[k].float()).abs().max().item()
                for k in init if init[k].is_floating_point())
    assert moved > 1e-4
    data = spt.generate()                       # iteration 1, the trained net
    with warn():
        sp = rvz.SelfPlay(net, {"num_simulations": S, "seed": 11 + G, "save_dir": str(tmp_path)})
    games = sp.generate_games(G)
    assert len({g["states"][4].tobytes() for g in games}) > 1
    t = sp.training_tensors()
    assert torch.equal(t["states"], data["states"])
    assert torch.equal(t["policy_targets"], data["policy_targets"])
    assert torch.equal(t["value_targets"], data["value_targets"])


def test_ddp_trainer_over_rccl_world1_equals_plain_training():
    """DDPTrainer with a torch.distributed process group on the 'nccl' backend (RCCL on ROCm) at
    world size 1: every step's gradients go through DDP's bucketed RCCL all-reduce, and the
    trained parameters equal those of the same steps without a process group, to the run-to-run
    noise of the plain path itself. Deterministic convolution algorithms are requested; where
    MIOpen's backward kernels still differ run to run, the plain path runs three times and its
    own spread sets the bound (x4). The comparison is over the trainable parameters (the BN
    running statistics follow the same updates and would only repeat the check at a larger
    scale)."""
    import socket
    import torch.distributed as dist
    import rvz
    from rvz.trainer import DDPTrainer
    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        _ddp_vs_plain(socket, dist, rvz, DDPTrainer)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det


def _ddp_vs_plain(socket, dist, rvz, DDPTrainer):
    torch.manual_seed(3)
    n = 512
    data = {"states": (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float(),
            "policy_targets": torch.softmax(torch.randn(n, 65, device="cuda"), 1),
            "value_targets": torch.rand(n, device="cuda") * 2 - 1}
    nets = []
    for distributed in (False, False, False, True):
        torch.manual_seed(0)
        net = rvz.AlphaZeroNetwork(8, 2, 64).cuda()
        if distributed:
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                    world_size=1)
        try:
            tr = DDPTrainer(net, batch_size=64)
            assert tr.distributed == distributed
            for epoch in range(2):
                out = tr.train_epoch(data, seed=epoch)
                assert out["steps"] == n // 64
            torch.cuda.synchronize()
        finally:
            if distributed:
                dist.destroy_process_group()
        nets.append(net)
    sd = [dict(m.named_parameters()) for m in nets]
    torch.manual_seed(0)
    init = dict(rvz.AlphaZeroNetwork(8, 2, 64).cuda().named_parameters())

    def diff(a, b):
        return max((a[k].detach().float() - b[k].detach().float()).abs().max().item() for k in init)

    moved = diff(sd[0], init)
    noise = max(diff(sd[0], sd[1]), diff(sd[0], sd[2]), diff(sd[1], sd[2]))
    ddp = min(diff(sd[i], sd[3]) for i in range(3))
    assert moved > 1e-3                       # the nets trained
    assert ddp <= 4 * noise + 1e-6 * moved, (ddp, noise, moved)


@pytest.mark.timeout(900)
def test_c4_per_rank_shard_over_rccl_world1(oracle):
    """C4's per-rank shard as configured (BASELINE.json configs[3]: 32,768 games x 800 sims per
    GPU, 10x128 net): one SelfPlayTrainer iteration (whole games, records ->
    training arrays, 100 DDP steps whose gradients go through RCCL at world 1, evaluator refresh),
    then the next iteration's self-play. 16 sampled games of that iteration are replayed by the
    literal oracle fed the TRAINED net's h2 outputs (reference pipeline.py:114-150 plays the new
    iteration with the updated model): every ply's move and f64 policy, and their rows of the
    training arrays (states, policy_targets, value_targets; self_play.py:117-126)."""
    import socket
    import torch.distributed as dist
    import rvz
    from oracle_play import OracleGames
    from rvz.pipeline import SelfPlayTrainer
    G, S, seed = 32768, 800, 11
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        net = rvz.AlphaZeroNetwork(8, 10, 128).cuda()
        init = {k: v.clone() for k, v in net.state_dict().items()}
        spt = SelfPlayTrainer(net, G, num_simulations=S, seed=seed, train_steps=100,
                              train_batch=64)
        assert spt.distributed and spt.world == 1
        r0 = spt.run_iteration()
        assert r0["board_steps"] == r0["samples"] >= 59 * G and r0["steps"] == 100
        assert np.isfinite(r0["train/loss"])
        moved = max((net.state_dict()[k].float() - init[k].float()).abs().max().item()
                    for k in init if init[k].is_floating_point())
        assert moved > 1e-4
        data = spt.generate()                   # iteration 1: the trained net, graph replays
    finally:
        dist.destroy_process_group()
    run = spt.runner
    rec_idx = run.rec_idx.cpu().numpy()
    counts = (rec_idx >= 0).sum(0)
    assert int(counts.sum()) == data["states"].shape[0]
    first = np.concatenate([[0], np.cumsum(counts)[:-1]])
    sample = np.linspace(0, G - 1, 16).astype(int)
    orc = OracleGames(oracle, [seed + G + int(g) for g in sample], S)
    ev = spt.evaluator                          # refreshed in place: the trained weights
    ev_fresh = rvz.LeafEvaluator(net.eval())
    x = (torch.rand(64, 3, 8, 8, device="cuda") > 0.6).float()
    assert all(torch.equal(a, b) for a, b in zip(ev(x), ev_fresh(x)))
    states = data["states"].cpu().numpy()
    pol = data["policy_targets"].cpu().numpy()
    val = data["value_targets"].cpu().numpy().reshape(-1)
    rec_p = run.rec_p.cpu().numpy()
    sides = []
    for ply in range(spt.max_plies):
        if orc.over():
            break
        live = np.array([not g.over for g in orc.games])
        sd = [g.side for g in orc.games]
        _, oi, op, planes = orc.ply(ev)
        for j, g in enumerate(sample):
            if not live[j]:
                continue
            assert oi[j] == rec_idx[ply, g], (ply, g)
            assert np.array_equal(op[j].view(np.int64), rec_p[ply, g].view(np.int64)), (ply, g)
            row = first[g] + ply
            assert np.array_equal(states[row], planes[j]), (ply, g)
            assert np.array_equal(pol[row], op[j].astype(np.float32)), (ply, g)
            sides.append((row, sd[j], j))
    assert orc.over()
    for j, g in enumerate(sample):
        assert counts[g] == sum(1 for r, _, jj in sides if jj == j)
    win = orc.winners()
    for row, side, j in sides:
        want = 0.0 if win[j] == 0 else (1.0 if side == win[j] else -1.0)
        assert val[row] == want, (row, side, win[j])


@pytest.mark.parametrize("table", [False, True])
def test_fused_records_equal_the_pull_style_records(table):
    """The fused recording runner (one rvz_play launch with device records: the position before
    every act, its policy vector, the move) records exactly what the pull-style recording runner
    copies out ply by ply (self_play.py:88-101), and the trainer arrays built from them are
    equal (pipeline.py:179-246)."""
    import rvz
    from rvz.trainer import records_to_training
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 2, 64).cuda().eval()
    G, S, P = 160, 200, 60     # four batches: distinct games per slot
    runs = []
    for fused in (False, True):
        eng = rvz.Engine(G, S, 64, compact_leaves=True, memo=True)
        if fused and table:
            eng.table(1 << 14, 14)
        run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), record=True, max_plies=P,
                                 seed_base=5, fused=fused, skip_last_eval=fused)
        run.start()
        if fused:
            run.play_record(20)
            run.play_record(P - 20)              # two launches: records land in their slices
        else:
            for _ in range(P):
                run.ply()
        run.check()
        assert bool(run.post_status[:, 1].all())
        runs.append(run)
    a, b = runs
    for name in ("rec_black", "rec_white", "rec_side", "rec_idx", "rec_p", "post_status"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    ta = records_to_training(a.rec_black, a.rec_white, a.rec_side, a.rec_idx, a.rec_p,
                             a.post_status)
    tb = records_to_training(b.rec_black, b.rec_white, b.rec_side, b.rec_idx, b.rec_p,
                             b.post_status)
    assert all(torch.equal(ta[k], tb[k]) for k in ta)


def _trainer_gap(cudnn: bool):
    """DDPTrainer on the GPU vs the reference's _train_epoch restated on the CPU in float32 and
    vs a float64 run of the same algorithm (DDPTrainer on the CPU in float64): two epochs of 4
    AdamW steps on tests/test_trainer_cpu.py's seeded data, MultiStepLR stepped between them."""
    import copy
    import rvz
    from rvz.trainer import DDPTrainer
    from test_trainer_cpu import _data, _reference_train_epoch
    torch.manual_seed(0)
    cpu_net = rvz.AlphaZeroNetwork(8, 2, 64)
    gpu_net = copy.deepcopy(cpu_net).cuda()
    f64_net = copy.deepcopy(cpu_net).double()
    init = {k: v.clone() for k, v in cpu_net.state_dict().items()}
    data = _data(n=200, seed=3)
    tr = DDPTrainer(gpu_net, lr_milestones=[1], lr_gamma=0.1)
    t64 = DDPTrainer(f64_net, lr_milestones=[1], lr_gamma=0.1)
    opt = torch.optim.AdamW(cpu_net.parameters(), lr=1e-3, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.MultiStepLR(opt, milestones=[1], gamma=0.1)
    gdata = {k: v.cuda() for k, v in data.items()}
    ddata = {k: v.double() for k, v in data.items()}
    rep = {"miopen": cudnn, "loss_rel": []}
    with torch.backends.cudnn.flags(enabled=cudnn):
        for ep in range(2):
            got = tr.train_epoch(gdata, seed=10 + ep)
            tr.scheduler_step()
            t64.train_epoch(ddata, seed=10 + ep)
            t64.scheduler_step()
            want = _reference_train_epoch(cpu_net, opt, data, 64,
                                          torch.Generator().manual_seed(10 + ep))
            sched.step()
            assert got["steps"] == 4 and got["train/lr"] == want["train/lr"]
            rep["loss_rel"].append(max(abs(got[k] - want[k]) / max(1e-12, abs(want[k]))
                                       for k in ("train/loss", "train/policy_loss",
                                                 "train/value_loss")))
    sg, sc, sd = gpu_net.state_dict(), cpu_net.state_dict(), f64_net.state_dict()
    keys = [k for k in sc if sc[k].is_floating_point() and "running" not in k]

    def dist(a):
        return max((a[k].detach().cpu().double() - sd[k].double()).abs().max().item() for k in keys)

    rep["gpu_vs_f64"], rep["cpu_vs_f64"] = dist(sg), dist(sc)
    rep["moved_max_abs"] = max((sc[k].double() - init[k].double()).abs().max().item() for k in keys)
    return rep


def test_gpu_trainer_tracks_the_reference_train_epoch_restatement():
    """the trainer on the GPU (DDPTrainer, one process: the C4 loop's
    optimizer step) against the reference's _train_epoch restated on the CPU
    (tests/test_trainer_cpu.py::_reference_train_epoch, pipeline.py:272-366, bitwise equal to
    DDPTrainer on the CPU): same init, data and batch order (the DataLoader's seeded permutation).
    The GPU's kernels round differently from the CPU's, so the check is fp32-class against a
    float64 run of the same algorithm. With PyTorch's own GPU convolutions (MIOpen off) the
    algorithm is held tightly: each epoch's averaged losses within 1e-5 relative of the CPU
    restatement's, and the GPU's parameters no further from the float64 ones than 2x the CPU
    float32 run's distance (measured: 0.7x). With MIOpen (the trainer's default) the solver
    MIOpen picks decides the rounding; measured on MI355X boxes: loss gaps 1e-7-4e-6 and 2.7x
    the CPU's parameter distance on three boxes, 9.3e-4 / 24x on one (a less exact weight-gradient
    or Winograd solver), so that run is bounded loosely (5e-3, 50x) and reported in
    gpurun_out/trainer_gpu_vs_cpu.json. (AdamW divides by sqrt(v): near-zero gradients turn
    rounding into visible parameter differences on either device.)"""
    import json
    import os
    exact, miopen = _trainer_gap(False), _trainer_gap(True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
        with open(os.path.join(root, "gpurun_out", "trainer_gpu_vs_cpu.json"), "w") as f:
            json.dump({"miopen_off": exact, "miopen_on": miopen}, f, indent=1)
    except OSError:
        pass
    print(exact, miopen)
    for rep in (exact, miopen):
        assert rep["moved_max_abs"] > 1e-3, rep
    assert max(exact["loss_rel"]) <= 1e-5, exact
    assert exact["gpu_vs_f64"] <= 2 * exact["cpu_vs_f64"] + 1e-7, exact
    assert max(miopen["loss_rel"]) <= 5e-3, miopen
    assert miopen["gpu_vs_f64"] <= 50 * miopen["cpu_vs_f64"], miopen
