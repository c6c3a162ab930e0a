"""Cross-game redundancy of the NN rows: how many evaluated leaf rows repeat
a position some earlier evaluation (any game, any earlier batch, same net) already computed.

Plays the C2 workload (4,096 games x 800 sims, 6x64 random-init net, memo + the deferred last
batch, i.e. exactly the rows the headline evaluates) with the pull-style engine, eagerly, for
--plies plies from the lockstep start (every game restarts at once when it ends), and records the
key of every evaluated row: the NN input is a function of three bitboards (canonical planes:
mover, opponent, legal moves), so (P, O, V) is the exact cache key. Reports, per ply of a game:
rows, rows repeating an earlier batch's row (what a persistent position -> output table saves),
rows duplicating another row of the same batch (in-flight duplicates), by disc count too.

    python tools/exp_xgame.py --plies 180 --out gpurun_out/xgame.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))

import torch  # noqa: E402


def pack(planes):
    """[n, 3, S, S] 0/1 float planes -> int64 [n, 3] bitboards (bit s = square s)."""
    n = planes.shape[0]
    b = (planes.reshape(n, 3, planes.shape[-1] * planes.shape[-2]) > 0.5).long()
    w = torch.ones(b.shape[-1], dtype=torch.long, device=b.device) << torch.arange(
        b.shape[-1], device=b.device)
    return (b * w).sum(-1)      # distinct bits: the sum is the OR (wraps into bit 63 correctly)


def main():
    import rvz
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--plies", type=int, default=180)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--filters", type=int, default=64)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, a.blocks, a.filters).to(dev).eval()
    ev = rvz.LeafEvaluator(net)
    G = a.games
    eng = rvz.Engine(G, a.sims, 64, device=dev, memo=True)
    run = rvz.SelfPlayRunner(eng, ev, autoreset=True, seed_base=42, skip_last_eval=True)
    run.start()
    keys, batch_id, ply_of, gply = [], [], [], []
    plies_in_game = torch.zeros(G, dtype=torch.long, device=dev)
    bid = 0
    for ply in range(a.plies):
        eng.search_begin()
        k = 0
        while eng.search_step():
            k += 1
            if k == eng.n_batches:
                eng.search_skip()
                break
            live = eng.need > 0
            logits, value = ev(eng.leaf_x)
            rows = torch.nonzero(live).squeeze(1)
            if rows.numel() == 0:
                eng.search_submit(logits, value, True)
                bid += 1
                continue
            keys.append(pack(eng.leaf_x[rows]))
            batch_id.append(torch.full((rows.numel(),), bid, dtype=torch.long, device=dev))
            ply_of.append(torch.full((rows.numel(),), ply, dtype=torch.long, device=dev))
            gply.append(plies_in_game[rows].clone())
            bid += 1
            eng.search_submit(logits, value, True)
        idx, _ = eng.act(1.0, apply=True)
        over = eng.get_state()[2][:, 1].long()
        eng.autoreset(idx, run.seeds, run.seed_stride, run._plies, run._done, reset=True)
        plies_in_game = torch.where(over > 0, torch.zeros_like(plies_in_game), plies_in_game + 1)
    eng.check()
    K = torch.cat(keys)
    B = torch.cat(batch_id)
    P = torch.cat(ply_of)
    GP = torch.cat(gply)
    n = K.shape[0]
    uniq, inv = torch.unique(K, dim=0, return_inverse=True)
    first_b = torch.full((uniq.shape[0],), 1 << 62, dtype=torch.long, device=dev)
    first_b.scatter_reduce_(0, inv, B, reduce="amin")
    pos = torch.arange(n, device=dev)
    first_i = torch.full((uniq.shape[0],), 1 << 62, dtype=torch.long, device=dev)
    first_i.scatter_reduce_(0, inv, pos, reduce="amin")
    earlier = B > first_b[inv]                              # an earlier batch evaluated it
    same = (B == first_b[inv]) & (pos != first_i[inv])      # another row of the same batch
    discs = torch.stack([((K[:, 0] >> i) & 1) + ((K[:, 1] >> i) & 1) for i in range(64)]).sum(0)
    out = {"games": G, "sims": a.sims, "plies": a.plies, "rows": n,
           "rows_per_ply": n / a.plies / G, "distinct": int(uniq.shape[0]),
           "repeat_earlier_batch": int(earlier.sum()), "dup_same_batch": int(same.sum())}
    for lo in (0, 60):
        m = P >= lo
        out[f"from_ply{lo}"] = {"rows": int(m.sum()), "repeat_earlier": int((earlier & m).sum()),
                                "dup_same": int((same & m).sum()),
                                "frac_repeat_earlier": float((earlier & m).sum() / max(1, m.sum())),
                                "frac_dup_same": float((same & m).sum() / max(1, m.sum()))}
    per = {}
    for q in range(61):
        m = (GP == q) & (P >= 60)
        if m.any():
            per[q] = [int(m.sum()), int((earlier & m).sum()), int((same & m).sum())]
    out["per_game_ply_after60"] = per
    byd = {}
    for d in range(4, 65):
        m = (discs == d) & (P >= 60)
        if m.any():
            byd[d] = [int(m.sum()), int((earlier & m).sum()), int((same & m).sum())]
    out["by_discs_after60"] = byd
    # distinct positions a table keyed up to a disc threshold must hold
    out["distinct_by_max_discs"] = {d: int((torch.stack([((uniq[:, 0] >> i) & 1) +
                                                          ((uniq[:, 1] >> i) & 1)
                                                          for i in range(64)]).sum(0) <= d).sum())
                                    for d in (8, 10, 12, 14, 16, 20)}
    s = json.dumps(out)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
