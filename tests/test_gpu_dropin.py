"""The drop-in Python classes (rvz.MCTS, rvz.SelfPlay) — the reference's API on the HIP engine."""
import numpy as np
import pytest
import torch

import golden_replay as R

pytestmark = pytest.mark.gpu


class _Recorder:
    """Model protocol of mcts.py (parameters / eval / predict) recording every call."""

    def __init__(self, net):
        self.net, self.calls = net, []

    def parameters(self):
        return self.net.parameters()

    def eval(self):
        self.net.eval()
        return self

    def predict(self, x):
        with torch.no_grad():
            logits, value = self.net.predict(x)
        self.calls.append((x.detach().clone(), logits.detach().clone(), value.detach().clone()))
        return logits, value


def test_mcts_dropin_matches_oracle(oracle):
    import rvz
    torch.manual_seed(0)
    rec = _Recorder(rvz.AlphaZeroNetwork(8, 2, 32).cuda())
    mcts = rvz.MCTS(rec, c_puct=1.0, num_simulations=200)
    game, og = rvz.ReversiGame(), oracle.new_game()
    np.random.seed(5)
    mt = oracle.MT(5)
    for ply in range(12):
        rec.calls.clear()
        action, probs = mcts.get_action_probs(game, temperature=1.0)
        srch = oracle.Search(1, 200, 64, 1.0)
        srch.begin([og])
        ci = 0
        while (r := srch.step()) is not None:
            leaves, nc = r
            if nc[0] == 0:
                continue
            x, logits, value = rec.calls[ci]
            ci += 1
            assert R.planes_to_masks(x[0].cpu().numpy()) == \
                R.planes_to_masks(oracle.canonical(leaves[0]))
            srch.submit(torch.softmax(logits, 1).cpu().numpy(), value.cpu().numpy())
        assert ci == len(rec.calls)
        vis = srch.visits()[0]
        idx, p, _ = oracle.action(vis, 1.0, mt.random_sample())
        assert action == divmod(idx, 8)
        assert np.array_equal(p.view(np.int64), probs.view(np.int64))
        visits = mcts.search(game)
        assert {divmod(s, 8): int(vis[s]) for s in range(64) if vis[s]} == \
            {k: v for k, v in visits.items() if v}
        assert game.make_move(*action) and oracle.make_move(og, idx)
        mcts.update_with_move(action)
    assert (game.board.black, game.board.white) == (og.black, og.white)


def test_selfplay_dropin_records(tmp_path):
    import rvz
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 2, 64).cuda()
    sp = rvz.SelfPlay(net, {"num_simulations": 128, "c_puct": 1.0, "temperature": 1.0,
                            "save_dir": str(tmp_path), "seed": 3})
    games = sp.generate_games(8)
    assert len(games) == 8
    assert len(list(tmp_path.glob("game_*.pt"))) == 8
    for g in games:
        n = len(g["states"])
        assert 9 <= n <= 60 and len(g["action_probs"]) == n == len(g["values"])
        assert g["winner"] in (0, 1, 2)
        for st, pl, v in zip(g["states"], g["current_players"], g["values"]):
            assert st.shape == (3, 8, 8) and st.dtype == np.float32
            assert st[2].sum() >= 1                       # the side to move had a legal move
            assert v == (0.0 if g["winner"] == 0 else (1.0 if pl == g["winner"] else -1.0))
        for p in g["action_probs"]:
            assert p.shape == (65,) and abs(p.sum() - 1.0) < 1e-12
        assert g["states"][0][0].sum() == 2 and g["states"][0][1].sum() == 2
    # the device-side training arrays == the per-game dicts, concatenated (pipeline.py:179-246)
    t = sp.training_tensors()
    st = np.concatenate([np.stack(g["states"]) for g in games])
    pr = np.concatenate([np.stack(g["action_probs"]) for g in games]).astype(np.float32)
    va = np.concatenate([np.asarray(g["values"], np.float32) for g in games]).reshape(-1, 1)
    assert np.array_equal(t["states"].cpu().numpy(), st)
    assert np.array_equal(t["policy_targets"].cpu().numpy(), pr)
    assert np.array_equal(t["value_targets"].cpu().numpy(), va)
    data = sp.generate_training_data(4)
    assert data["states"].shape[1:] == (3, 8, 8) and data["values"].shape[1] == 1
    assert data["action_probs"].shape[1] == 65 and len(data["states"]) == len(data["values"])


def test_selfplay_dropin_compaction_is_exact(tmp_path):
    """SelfPlay compacts its leaf batches by default (only live leaves reach the h2 evaluator);
    the recorded games equal the uncompacted run's."""
    import rvz
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 1, 64).cuda()
    out = []
    for compact in (True, False):
        sp = rvz.SelfPlay(net, {"num_simulations": 128, "seed": 5, "compact_leaves": compact,
                                "save_dir": str(tmp_path / str(compact))})
        assert sp.evaluator.accepts_live_count
        out.append(sp.generate_games(16))
    for a, b in zip(*out):
        assert a["winner"] == b["winner"] and len(a["states"]) == len(b["states"])
        for pa, pb in zip(a["action_probs"], b["action_probs"]):
            assert np.array_equal(pa, pb)


def test_ddp_trainer_single_gpu_step_on_records():
    """DDPTrainer (no process group) consumes the engine's records directly and learns."""
    import rvz
    from rvz.trainer import DDPTrainer
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 2, 64).cuda()
    sp = rvz.SelfPlay(net, {"num_simulations": 128, "save_dir": "/tmp/rvz_sp_test", "seed": 9})
    sp.generate_games(16)
    data = sp.training_tensors()
    tr = DDPTrainer(net, batch_size=64)
    first = tr.train_epoch(data, seed=0)
    for _ in range(4):
        last = tr.train_epoch(data, seed=1)
    assert first["steps"] >= 10 and last["train/loss"] < first["train/loss"]


def test_selfplay_runner_graph_replay_equals_eager():
    """One ply captured in a HIP graph and replayed == the same plies run eagerly (bit-exact)."""
    import rvz
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 2, 64).cuda().eval()
    ev = rvz.LeafEvaluator(net)
    outs = []
    for graph in (False, True):
        eng = rvz.Engine(256, 128, 64)
        run = rvz.SelfPlayRunner(eng, ev, autoreset=True, seed_base=11)
        run.start()
        run.ply()
        if graph:
            run.capture()
        for _ in range(5):
            run.ply()
        b, w, st = eng.get_state()
        torch.cuda.synchronize()
        outs.append((b.clone(), w.clone(), st.clone(), int(run.steps.item())))
        eng.check()
    assert all(torch.equal(a, b) for a, b in zip(outs[0][:3], outs[1][:3]))
    assert outs[0][3] == outs[1][3] == 6 * 256
