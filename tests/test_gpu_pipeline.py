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
    G, S = 64, 128
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
