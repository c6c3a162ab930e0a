"""Generate the committed golden fixtures from the Python reference at /root/reference.

Run in the build container only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py

Outputs (all plain npz, no pickles):
  board_vectors.npz   F-board: seeded random-playout positions -> reference legal mask, and one
                      make_move per position (legal, illegal or pass) -> resulting state + bool.
  mcts_<tag>.npz      F-mcts:  full reference games (src/mcts/mcts.py get_action_probs driving
                      src/game/game.py), every NN call recorded (leaf planes as bitmasks, the
                      reference's own softmax row and value), every ply's visits / p / action.
  net_tiny.npz        F-net:   a 1x16 AlphaZeroNetwork state_dict (keys as the reference names
                      them), a batch of inputs and the reference's outputs (CPU fp32).

What the reference calls is cited per block: board.py:70-251, game.py:36-162, mcts.py:322-694,
network.py:30-158, self_play.py:80-126.
"""
from __future__ import annotations

import os
import random
import sys
import time

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import torch  # noqa: F401
    from src.game.game import ReversiGame  # type: ignore
    from src.mcts.mcts import MCTS  # type: ignore
    from src.model.network import AlphaZeroNetwork  # type: ignore
    return ReversiGame, MCTS, AlphaZeroNetwork


def _mask(moves) -> int:
    m = 0
    for r, c in moves:
        m |= 1 << (r * 8 + c)
    return m


def _planes_to_masks(x: np.ndarray):
    out = []
    for p in range(3):
        bits = np.flatnonzero(x[p].reshape(-1) > 0.5)
        out.append(sum(1 << int(b) for b in bits))
    return out


# ---------------------------------------------------------------------------------- F-board
def make_board_vectors(n_games: int = 300, seed: int = 1234):
    ReversiGame, _, _ = _import_reference()
    rng = random.Random(seed)
    pre, legal, mv, ok, post = [], [], [], [], []
    for _ in range(n_games):
        game = ReversiGame()
        while not game.is_game_over():
            b = game.board
            state = (b.black, b.white, game.current_player, int(b.passed_moves_in_a_row),
                     int(game.game_over), -1 if game.winner is None else int(game.winner))
            moves = game.get_valid_moves()
            lm = _mask(moves)
            # mostly legal moves (drives the playout), sometimes an illegal square or a pass
            roll = rng.random()
            if roll < 0.08:
                sq = rng.randrange(64)
            elif roll < 0.10:
                sq = -1
            else:
                r, c = rng.choice(moves)
                sq = r * 8 + c
            trial = game.copy()
            res = trial.make_move(*(divmod(sq, 8) if sq >= 0 else (-1, -1)))
            tb = trial.board
            after = (tb.black, tb.white, trial.current_player, int(tb.passed_moves_in_a_row),
                     int(trial.game_over), -1 if trial.winner is None else int(trial.winner))
            pre.append(state); legal.append(lm); mv.append(sq); ok.append(int(res)); post.append(after)
            # advance the playout with a legal move
            r, c = rng.choice(moves)
            game.make_move(r, c)
    u64 = lambda rows, i: np.array([r[i] for r in rows], dtype=np.uint64)  # noqa: E731
    i32 = lambda rows, i: np.array([r[i] for r in rows], dtype=np.int32)  # noqa: E731
    np.savez_compressed(
        os.path.join(OUT, "board_vectors.npz"),
        black=u64(pre, 0), white=u64(pre, 1), side=i32(pre, 2), passed=i32(pre, 3),
        over=i32(pre, 4), winner=i32(pre, 5), legal=np.array(legal, dtype=np.uint64),
        move=np.array(mv, dtype=np.int32), ok=np.array(ok, dtype=np.int32),
        black_after=u64(post, 0), white_after=u64(post, 1), side_after=i32(post, 2),
        passed_after=i32(post, 3), over_after=i32(post, 4), winner_after=i32(post, 5))
    print(f"board_vectors: {len(pre)} positions")


# ---------------------------------------------------------------------------------- F-mcts
class _Recorder:
    """Duck-typed model (mcts.py:211,235,501) that records every predict() call."""

    def __init__(self, net):
        self.net = net
        self.calls = []

    def parameters(self):
        return self.net.parameters()

    def eval(self):
        self.net.eval()
        return self

    def predict(self, x):
        import torch
        import torch.nn.functional as F
        logits, value = self.net.predict(x)
        probs = F.softmax(logits, dim=1).cpu().numpy()       # exactly mcts.py:596
        vals = value.cpu().numpy()                            # mcts.py:597
        xs = x.cpu().numpy()
        same_in = bool(np.all(xs == xs[:1]))
        same_out = bool(np.all(probs == probs[:1]) and np.all(vals == vals[:1]))
        self.calls.append((xs[0].copy(), probs[0].copy(), np.float32(vals[0]), len(xs),
                           same_in, same_out))
        return logits, value


def make_mcts_games(tag: str, blocks: int, filters: int, sims: int, seeds, temperature: float,
                    net_seed: int = 0, max_plies: int = 60, threads: int = 8):
    import torch
    ReversiGame, MCTS, AlphaZeroNetwork = _import_reference()
    torch.set_num_threads(threads)
    torch.manual_seed(net_seed)
    net = AlphaZeroNetwork(board_size=8, num_res_blocks=blocks, num_filters=filters)
    rec = _Recorder(net)
    mcts = MCTS(rec, c_puct=1.0, num_simulations=sims)      # batch_size=64 default (mcts.py:198)
    orig_search = mcts.search
    visits_log = []

    def search_spy(game):
        v = orig_search(game)
        visits_log.append(dict(v))
        return v

    mcts.search = search_spy
    data = {k: [] for k in ("game", "ply_black", "ply_white", "ply_side", "ply_visits", "ply_p",
                            "ply_action", "call_game", "call_ply", "call_masks", "call_probs",
                            "call_value", "call_rows", "call_same_in", "call_same_out")}
    winners = []
    t0 = time.time()
    for gi, seed in enumerate(seeds):
        np.random.seed(seed)                                 # the RNG behind np.random.choice
        game = ReversiGame()
        ply = 0
        while not game.is_game_over() and ply < max_plies:
            b = game.board
            n_before = len(rec.calls)
            action, probs = mcts.get_action_probs(game, temperature=temperature)
            vis = np.zeros(65, np.int32)
            for (r, c), cnt in visits_log[-1].items():
                vis[64 if (r, c) == (-1, -1) else r * 8 + c] = cnt
            data["game"].append(gi)
            data["ply_black"].append(b.black); data["ply_white"].append(b.white)
            data["ply_side"].append(game.current_player)
            data["ply_visits"].append(vis); data["ply_p"].append(np.asarray(probs, np.float64))
            data["ply_action"].append(64 if action == (-1, -1) else action[0] * 8 + action[1])
            for xs, pr, v, nrows, si, so in rec.calls[n_before:]:
                data["call_game"].append(gi); data["call_ply"].append(ply)
                data["call_masks"].append(_planes_to_masks(xs)); data["call_probs"].append(pr)
                data["call_value"].append(v); data["call_rows"].append(nrows)
                data["call_same_in"].append(si); data["call_same_out"].append(so)
            # np.argmax (T == 0) returns np.int64 indices, which make the reference's own
            # board.make_move raise OverflowError (board.py:170,213); a caller passes ints.
            game.make_move(int(action[0]), int(action[1]))
            ply += 1
        winners.append(-1 if game.get_winner() is None else int(game.get_winner()))
        print(f"  {tag}: game {gi} seed {seed}: {ply} plies, winner {winners[-1]}, "
              f"{time.time() - t0:.1f}s")
    np.savez_compressed(
        os.path.join(OUT, f"mcts_{tag}.npz"),
        seeds=np.array(seeds, np.int64), sims=np.int32(sims), batch=np.int32(64),
        c_puct=np.float64(1.0), temperature=np.float64(temperature),
        blocks=np.int32(blocks), filters=np.int32(filters), winners=np.array(winners, np.int32),
        game=np.array(data["game"], np.int32),
        ply_black=np.array(data["ply_black"], np.uint64),
        ply_white=np.array(data["ply_white"], np.uint64),
        ply_side=np.array(data["ply_side"], np.int32),
        ply_visits=np.stack(data["ply_visits"]), ply_p=np.stack(data["ply_p"]),
        ply_action=np.array(data["ply_action"], np.int32),
        call_game=np.array(data["call_game"], np.int32),
        call_ply=np.array(data["call_ply"], np.int32),
        call_masks=np.array(data["call_masks"], np.uint64),
        call_probs=np.stack(data["call_probs"]).astype(np.float32),
        call_value=np.array(data["call_value"], np.float32),
        call_rows=np.array(data["call_rows"], np.int32),
        call_same_in=np.array(data["call_same_in"], bool),
        call_same_out=np.array(data["call_same_out"], bool))
    n_calls = len(data["call_game"])
    print(f"mcts_{tag}: {len(data['game'])} plies, {n_calls} NN calls, "
          f"all-rows-identical inputs {all(data['call_same_in'])}, "
          f"outputs {all(data['call_same_out'])}")


# ---------------------------------------------------------------------------------- F-net
def make_net_fixture():
    import torch
    _, _, AlphaZeroNetwork = _import_reference()
    torch.manual_seed(7)
    net = AlphaZeroNetwork(board_size=8, num_res_blocks=1, num_filters=16)
    # non-trivial BN statistics so the eval-mode BN path is exercised
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.1, 0.1)
    net.eval()
    g = torch.Generator().manual_seed(3)
    x = (torch.rand(32, 3, 8, 8, generator=g) > 0.6).float()
    with torch.no_grad():
        logits, value = net.predict(x)
    sd = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()
          if not k.startswith("_script_module.")}
    np.savez_compressed(os.path.join(OUT, "net_tiny.npz"), x=x.numpy(), logits=logits.numpy(),
                        value=value.numpy(), **{"sd/" + k: v for k, v in sd.items()})
    print(f"net_tiny: {len(sd)} tensors")


# ---------------------------------------------------------------------------------- F-elo
def make_elo_fixture(n_updates: int = 200, seed: int = 11):
    """arena.py:19-135 ELORatingSystem on a seeded sequence of (a, b, score) updates."""
    import json
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import types
    # src.arena imports tqdm at module level; the ELO class itself needs nothing else
    from src.arena.arena import ELORatingSystem  # type: ignore
    rng = random.Random(seed)
    players = ["p0", "p1", "p2", "p3"]
    elo = ELORatingSystem(k=32, initial_rating=1500.0)
    seq, after = [], []
    for _ in range(n_updates):
        a, b = rng.sample(players, 2)
        score = rng.choice([0.0, 0.5, 1.0])
        elo.update_ratings(a, b, score)
        seq.append([a, b, score])
        after.append([elo.ratings.get(p, 1500.0) for p in players])
    json.dump({"players": players, "updates": seq, "ratings_after": after,
               "leaderboard": elo.get_leaderboard()},
              open(os.path.join(OUT, "elo_sequence.json"), "w"))
    print(f"elo_sequence: {n_updates} updates")


if __name__ == "__main__":
    which = sys.argv[1:] or ["board", "net", "mcts", "elo"]
    if "elo" in which:
        make_elo_fixture()
    if "board" in which:
        make_board_vectors()
    if "net" in which:
        make_net_fixture()
    runs = {"s100_t1": (2, 32, 100, [0, 1, 2, 3], 1.0),
            "s100_t0": (2, 32, 100, [4], 0.0),
            "s100_t05": (2, 32, 100, [5], 0.5),
            "s100_t07": (2, 32, 100, [6], 0.7),
            "s100_t2": (2, 32, 100, [7], 2.0),
            "s800_6x64": (6, 64, 800, [0, 1], 1.0)}
    for tag, args in runs.items():
        if "mcts" in which or tag in which:
            make_mcts_games(tag, *args)
