"""C4's data path on CPU (no GPU): self-play records -> training arrays -> DDP training, world
size 2 over gloo (rvz/trainer.py, rvz/pipeline.py; reference pipeline.py:114-150, :179-246,
:272-366).

Synthetic records come from random playouts on the oracle (the engine's record layout: plies x
games of black / white / side / move / policy, plus each game's final status); the canonical
planes come from the oracle too, since rvz_board_canonical needs the GPU. Checked:
records_to_training against per-game dicts built as self_play.py:72-126 builds them, and two
DDP ranks training on their shards end with identical weights and BN buffers.
"""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _paths():
    for p in (ROOT, os.path.join(ROOT, "alphazero-reversi_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_canonical(black, white, status, bs):
    from oracle import oracle as O
    out = np.zeros((black.numel(), 3, bs, bs), np.float32)
    b = black.numpy().view(np.uint64)
    w = white.numpy().view(np.uint64)
    s = status.numpy()
    for i in range(len(b)):
        out[i] = O.canonical(O.Game(int(b[i]), int(w[i]), int(s[i, 0])), bs)
    return torch.from_numpy(out)


def synthetic_records(G=24, seed=0):
    """Random legal playouts on the oracle, recorded like SelfPlayRunner(record=True)."""
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    P = 60
    black = np.zeros((P, G), np.uint64)
    white = np.zeros((P, G), np.uint64)
    side = np.zeros((P, G), np.int32)
    idx = np.full((P, G), -2, np.int32)
    p = np.zeros((P, G, 65))
    final = np.zeros((G, 4), np.int32)
    games = []
    for g in range(G):
        game = O.new_game()
        rows = []
        for k in range(P):
            if game.over:
                break
            black[k, g], white[k, g], side[k, g] = game.black, game.white, game.side
            legal = O.legal(game.black, game.white) if game.side == 1 else \
                O.legal(game.white, game.black)
            sqs = [s for s in range(64) if legal >> s & 1]
            pv = rng.random(65)
            pv[64] = 0.0
            pv /= pv.sum()
            p[k, g] = pv
            mv = int(rng.choice(sqs))
            idx[k, g] = mv
            rows.append((O.canonical(game), pv, int(game.side)))
            assert O.make_move(game, mv)
        final[g] = (game.side, game.over, game.winner, game.passed)
        w = int(game.winner)
        games.append({"states": [r[0] for r in rows], "action_probs": [r[1] for r in rows],
                      "current_players": [r[2] for r in rows],
                      "values": [0.0 if w == 0 else (1.0 if r[2] == w else -1.0) for r in rows]})
    t = {"rec_black": torch.from_numpy(black.view(np.int64)),
         "rec_white": torch.from_numpy(white.view(np.int64)),
         "rec_side": torch.from_numpy(side), "rec_idx": torch.from_numpy(idx),
         "rec_p": torch.from_numpy(p), "final_status": torch.from_numpy(final)}
    return t, games


def test_records_to_training_equals_selfplay_dicts():
    _paths()
    from rvz.trainer import records_to_training
    rec, games = synthetic_records()
    t = records_to_training(rec["rec_black"], rec["rec_white"], rec["rec_side"],
                            rec["rec_idx"], rec["rec_p"], rec["final_status"], 8,
                            canonical=_oracle_canonical)
    st = np.concatenate([np.stack(g["states"]) for g in games])
    pr = np.concatenate([np.stack(g["action_probs"]) for g in games]).astype(np.float32)
    va = np.concatenate([np.asarray(g["values"], np.float32) for g in games]).reshape(-1, 1)
    assert np.array_equal(t["states"].numpy(), st)
    assert np.array_equal(t["policy_targets"].numpy(), pr)
    assert np.array_equal(t["value_targets"].numpy(), va)


def _worker(rank, world, port, q):
    _paths()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from rvz import dist as rd
    from rvz.network import AlphaZeroNetwork
    from rvz.trainer import DDPTrainer, records_to_training
    rd.init("gloo")
    rec, _ = synthetic_records(G=16, seed=10 + rank)     # each rank its own games
    data = records_to_training(rec["rec_black"], rec["rec_white"], rec["rec_side"],
                               rec["rec_idx"], rec["rec_p"], rec["final_status"], 8,
                               canonical=_oracle_canonical)
    torch.manual_seed(rank)                                # DDP syncs rank 0's init
    net = AlphaZeroNetwork(8, 1, 16)
    tr = DDPTrainer(net, batch_size=32)
    out = tr.train_epoch(data, seed=3, max_steps=4 if rank == 0 else None, local_data=True)
    tr.sync_buffers()
    q.put((rank, {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}, out))
    dist.destroy_process_group()


def test_records_to_ddp_two_ranks_identical_nets():
    _paths()
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd0, sd1 = res[0][1], res[1][1]
    for k in sd0:                 # weights via the all-reduce, BN buffers via sync_buffers
        assert np.array_equal(sd0[k], sd1[k]), k
    assert res[0][2]["steps"] == 4 and np.isfinite(res[0][2]["train/loss"])
    # the loss dict is the job's: the mean over ranks, identical on every rank
    assert res[0][2]["train/loss"] == res[1][2]["train/loss"]
    assert res[0][2]["train/value_loss"] == res[1][2]["train/value_loss"]
