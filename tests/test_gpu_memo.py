"""The NN-output memo across consecutive searches (rvz_search_memo, include/rvz.h).

The reference rebuilds the tree at every move (mcts.py:334), so the next search's root (the
child the move went to) and often some of its descendants are positions the game's previous
search already evaluated; with the memo on they are expanded from that earlier output. These
tests hold the memo to the contract that matters: whole games (moves, f64 policy vectors,
boards, counters) bit-identical to the engine without the memo — itself pinned to the
reference's recorded games and the literal oracle (test_gpu_search.py) — with fewer evaluated
rows, across autoreset, compaction, lanes / graphs, the skipped last batch, the 6x6 variant and
the host-side env edits that must drop the carried links."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _play(memo, G, sims, plies, board=8, net=None, compact=True, skip=False, lanes=1,
          graph=False, seed_base=11):
    import rvz

    def make_eng(n):
        return rvz.Engine(n, num_simulations=sims, batch_size=64, board_size=board,
                          compact_leaves=compact, memo=memo)

    if lanes > 1:
        run = rvz.LaneRunner(make_eng, lambda: rvz.LeafEvaluator(net), G, lanes, autoreset=True,
                             seed_base=seed_base, seed_stride=1000, skip_last_eval=skip)
        engines = [r.eng for r in run.runners]
    else:
        run = rvz.SelfPlayRunner(make_eng(G), rvz.LeafEvaluator(net), autoreset=True,
                                 seed_base=seed_base, seed_stride=1000, skip_last_eval=skip)
        engines = [run.eng]
    run.start()
    trace = []
    for k in range(plies):
        run.ply()
        if graph and k == 0:
            run.capture(**({"free_run": True} if lanes > 1 else {}))
        if lanes > 1:
            run.join()
        idx = torch.cat([e.idx_buf for e in engines]).clone()
        p = torch.cat([e.p_buf for e in engines]).clone()
        st = [e.get_state() for e in engines]
        trace.append((idx, p, torch.cat([s[0] for s in st]).clone(),
                      torch.cat([s[1] for s in st]).clone(),
                      torch.cat([s[2] for s in st]).clone()))
    for e in engines:
        e.check()
    rows = sum(e.rows_total() for e in engines) if compact else None
    return trace, int(run.steps.item()), int(run.games_done.item()), rows


def _same(a, b):
    (ta, sa, da, _), (tb, sb, db, _) = a, b
    assert sa == sb and da == db
    for k, (x, y) in enumerate(zip(ta, tb)):
        for u, v in zip(x, y):
            assert torch.equal(u, v), k


def _net(board, blocks=2, filters=64, seed=0):
    import rvz
    torch.manual_seed(seed)
    return rvz.AlphaZeroNetwork(board, blocks, filters).cuda().eval()


@pytest.mark.parametrize("board,sims,plies,G", [(8, 800, 66, 256), (8, 100, 66, 256),
                                                 (6, 400, 40, 300)],
                         ids=["8x8-s800", "8x8-s100", "6x6-s400"])
def test_memo_plays_the_same_games(board, sims, plies, G):
    """Whole games and their restarts: bit-identical with and without the memo; the memo
    evaluates fewer rows (SURVEY §8c-style size-independent property: same games, fewer rows)."""
    net = _net(board)
    off = _play(False, G, sims, plies, board, net)
    on = _play(True, G, sims, plies, board, net)
    _same(off, on)
    assert off[2] > 0                                  # games ended and restarted
    saved = 1 - on[3] / off[3]
    print(f"board {board} sims {sims}: rows {off[3]} -> {on[3]} ({saved:.1%} fewer)")
    assert on[3] < off[3] and saved > 0.05


def test_memo_uncompacted_and_skip_last_eval():
    """Memo with every row handed to the evaluator (no compaction), and with the last batch
    skipped (its leaves are not expanded, so they never become memo sources)."""
    net = _net(8, seed=2)
    base = _play(False, 128, 800, 64, net=net, compact=False)
    _same(base, _play(True, 128, 800, 64, net=net, compact=False))
    _same(base, _play(True, 128, 800, 64, net=net, compact=True, skip=True))


def test_memo_with_lanes_and_graphs():
    """The bench's form: free-running lane graphs (the memo's carried links and pool halves live
    on the device, so captured plies replay correctly)."""
    net = _net(8, seed=4)
    base = _play(False, 192, 800, 64, net=net)
    _same(base, _play(True, 192, 800, 64, net=net, lanes=2, graph=True))
    _same(base, _play(True, 192, 800, 64, net=net, lanes=3, graph=True))


def test_memo_drops_links_on_host_edits():
    """rvz_env_set / rvz_env_apply / act without apply / an abandoned search / memo_reset all drop
    the carried links: the following searches equal a memo-less engine's on the same states."""
    import rvz
    G, S = 64, 800
    net = _net(8, seed=5)
    ev = rvz.LeafEvaluator(net)
    a = rvz.Engine(G, S, 64, compact_leaves=True)
    b = rvz.Engine(G, S, 64, compact_leaves=True, memo=True)
    for e in (a, b):
        e.reset(range(100, 100 + G))

    def ply(e, apply=True):
        e.search(ev)
        v = e.visits().clone()
        idx, p = e.act(1.0, apply=apply)
        return v, idx.clone(), p.clone()

    def both(apply=True):
        ra, rb = ply(a, apply), ply(b, apply)
        for x, y in zip(ra, rb):
            assert torch.equal(x, y)

    for _ in range(4):
        both()
    # positions edited from the host: another game's state in every slot
    st = [t.clone() for t in a.get_state()]
    perm = torch.randperm(G, generator=torch.Generator().manual_seed(0)).cuda()
    for e in (a, b):
        e.set_state(st[0][perm], st[1][perm], st[2][perm])
    both()
    # a move applied from the host (the first legal square of each game)
    legal = a.legal().cpu().numpy().view(np.uint64)
    sq = torch.tensor([(int(m) & -int(m)).bit_length() - 1 if int(m) else -1 for m in legal],
                      dtype=torch.int32)
    for e in (a, b):
        e.apply(sq)
    both()
    both(apply=False)                                 # act without a move: no carry
    both()
    for e in (a, b):                                  # an abandoned search
        e.search_begin()
        assert e.search_step()
    both()
    b.memo_reset()
    both()
    a.check()
    b.check()


def test_memo_reset_after_new_weights():
    """The memo is only valid for an unchanged net: after LeafEvaluator.refresh() with new
    weights, memo_reset() makes the next searches those of a memo-less engine."""
    import rvz
    G, S = 96, 800
    net = _net(8, seed=6)
    ev = rvz.LeafEvaluator(net)
    a = rvz.Engine(G, S, 64, compact_leaves=True)
    b = rvz.Engine(G, S, 64, compact_leaves=True, memo=True)
    for e in (a, b):
        e.reset(range(G))
    for k in range(6):
        if k == 3:
            with torch.no_grad():
                for prm in net.parameters():
                    prm.mul_(1.5)
            ev.refresh()
            b.memo_reset()
        outs = []
        for e in (a, b):
            e.search(ev)
            idx, p = e.act(1.0, apply=True)
            outs.append((idx.clone(), p.clone()))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), k


def test_memo_api_errors():
    import rvz
    eng = rvz.Engine(8, 128, 64)
    eng.reset(range(8))
    eng.search_begin()
    assert eng.search_step()
    with pytest.raises(rvz.RvzError):
        eng.memo(True)                                # inside a search
