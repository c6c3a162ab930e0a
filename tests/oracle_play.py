"""The literal CPU oracle (oracle/, reference semantics) driven like the fused self-play launch:
for a sample of games, one MCTS search per ply (mcts.py:322-407) whose leaves are evaluated by
the same h2 LeafEvaluator on the GPU and softmaxed by rvz.policy_softmax — bitwise the softmax
the expand inside rvz_play applies to its logits (one device function, csrc/rvz_engine.hip) —
then get_action_probs' tail (mcts.py:642-694) with each game's numpy MT19937 stream and
make_move. Test infrastructure only: the checker of tests/ and __graft_entry__.smoke()."""
from __future__ import annotations

import numpy as np
import torch


class OracleGames:
    def __init__(self, O, seeds, sims: int, temperature: float = 1.0, bs: int = 8,
                 batch: int = 64):
        self.O, self.bs, self.S, self.T, self.B = O, bs, int(sims), float(temperature), batch
        self.games = [O.new_game(bs) for _ in seeds]
        self.mts = [O.MT(int(s)) for s in seeds]

    def ply(self, ev):
        """One ply of every sampled game: returns (visits int32 [n, npol], idx [n], p f64
        [n, npol], planes f32 [n, 3, bs, bs] of the positions before the move)."""
        import rvz
        O, bs = self.O, self.bs
        planes = np.stack([O.canonical(g, bs) for g in self.games])
        srch = O.Search(len(self.games), self.S, self.B, 1.0, bs=bs)
        srch.begin(self.games)
        dev = ev.device
        while (r := srch.step()) is not None:
            x = torch.from_numpy(O.leaf_planes(r[0], bs)).to(dev)
            logits, value = ev(x)
            probs = rvz.policy_softmax(logits, bs)
            srch.submit(probs.cpu().numpy(), value.cpu().numpy())
        vis = srch.visits()
        idx, ps = [], []
        for j, g in enumerate(self.games):
            if g.over:
                idx.append(-2)
                ps.append(np.zeros(bs * bs + 1))
                continue
            u = self.mts[j].random_sample() if O.action_needs_draw(vis[j], self.T) else 0.0
            a, p, _ = O.action(vis[j], self.T, u)
            assert O.make_move(g, -1 if a == bs * bs else a, bs)
            idx.append(a)
            ps.append(p)
        return vis, np.array(idx), np.stack(ps), planes

    def over(self):
        return all(g.over for g in self.games)

    def winners(self):
        return [g.winner if g.over else None for g in self.games]


def reference_generate_games(O, num_games: int, sims: int, temperature: float, rng, evaluate,
                             bs: int = 8, batch: int = 64, c_puct: float = 1.0):
    """SelfPlay.generate_games as the reference runs it (self_play.py:66-126), on the CPU oracle:
    one game after another, each ply one MCTS search (mcts.py:322-407) whose leaves `evaluate`
    answers (planes f32 [n, 3, bs, bs] -> (softmaxed rows f32 [n, npol], values f32 [n])), then
    get_action_probs' tail (mcts.py:642-694) drawing its np.random.choice value from ONE stream
    `rng` (a RandomState standing in for NumPy's global state, seeded once as pipeline.py:74-80
    seeds it), the record of the position before the move, make_move. Returns the per-game dicts
    (states, action_probs, current_players, values, winner, moves)."""
    out = []
    for _ in range(num_games):
        game = O.new_game(bs)
        d = {"states": [], "action_probs": [], "current_players": [], "moves": []}
        while not game.over:
            srch = O.Search(1, sims, batch, c_puct, bs=bs)
            srch.begin([game])
            while (r := srch.step()) is not None:
                p, v = evaluate(O.leaf_planes(r[0], bs))
                srch.submit(p, v)
            vis = srch.visits()[0]
            u = float(rng.random_sample()) if O.action_needs_draw(vis, temperature) else 0.0
            a, p, _ = O.action(vis, temperature, u)
            d["states"].append(O.canonical(game, bs))
            d["current_players"].append(int(game.side))
            d["action_probs"].append(p)
            d["moves"].append(a)
            assert O.make_move(game, -1 if a == bs * bs else a, bs)
        w = int(game.winner)
        d["winner"] = w
        d["values"] = [0.0 if w == 0 else (1.0 if pl == w else -1.0)
                       for pl in d["current_players"]]
        out.append(d)
    return out
