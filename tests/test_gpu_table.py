"""The cross-game NN-output table of the fused self-play launch (rvz_play_table, VERDICT r03 item
5): a leaf whose position an earlier evaluation (any game, same weights) stored is expanded from
the stored logits and value instead of a new NN row. An h2 row's outputs depend only on its
input planes, which are a function of the (mover, opponent, legal) bitboards the table is keyed
on, so every game must be bit-identical with and without the table; only the evaluated rows
change. The reference carries an inert transposition table for this purpose
(mcts.py:228-320,368-385)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net(board, blocks, filters, seed=0):
    import rvz
    torch.manual_seed(seed)
    return rvz.AlphaZeroNetwork(board, blocks, filters).cuda().eval()


def _run(net, G, S, plies, table=None, gpw=-6, memo=True, skip=True, chunks=None, seed_base=42):
    """Fused self-play; table = (slots, max_discs) or None. Returns (runner, moves [plies, G])."""
    import rvz
    eng = rvz.Engine(G, S, 64, board_size=net.board_size, memo=memo)
    if table:
        eng.table(*table)
    run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=seed_base,
                             skip_last_eval=skip, fused=True)
    run.play_group = gpw
    run.start()
    hs = []
    for n in (chunks or [plies]):
        h = torch.full((n, G), -9, dtype=torch.int32, device="cuda")
        eng.play(run.evaluator, n, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
                 reset=True, skip_last_eval=skip, hist=h, games_per_workgroup=gpw)
        hs.append(h)
    eng.check()
    return run, torch.cat(hs)


def _same(a, b):
    (ra, ma), (rb, mb) = a, b
    for k in range(ma.shape[0]):
        assert torch.equal(ma[k], mb[k]), f"ply {k}: {int((ma[k] != mb[k]).sum())} games differ"
    for x, y in zip(ra.eng.get_state(), rb.eng.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(ra._plies, rb._plies) and torch.equal(ra.seeds, rb.seeds)
    assert torch.equal(ra.eng.p_buf, rb.eng.p_buf)


def test_table_plays_the_same_games_at_full_c2_size():
    """bench.py's C2 headline (4,096 games x 800 sims, 6x64, memo + deferred last batch, groups
    of 6) for 64 plies (whole games and restarts), with and without the table (2^20 slots,
    positions of <= 14 discs): identical games; the table saves rows."""
    net = _net(8, 6, 64)
    G, S, P = 4096, 800, 64
    with_t = _run(net, G, S, P, table=(1 << 20, 14))
    plain = _run(net, G, S, P)
    _same(with_t, plain)
    hits, ins = with_t[0].eng.table_stats.tolist()
    rows_t, rows_p = int(with_t[0].eng.play_rows.item()), int(plain[0].eng.play_rows.item())
    assert hits > 0 and ins > 0
    assert rows_t + hits == rows_p, (rows_t, hits, rows_p)   # every hit is one row not evaluated


@pytest.mark.parametrize("slots,discs,gpw", [(1024, 64, -4), (1024, 10, 7), (1 << 16, 20, -1)])
def test_table_tiny_full_or_static(slots, discs, gpw):
    """A 1,024-slot table asked to hold every position (it fills, probe chains end, inserts are
    dropped), a static schedule, groups of one: the same games."""
    net = _net(8, 2, 64, seed=3)
    G, S, P = 203, 160, 30
    _same(_run(net, G, S, P, table=(slots, discs), gpw=gpw), _run(net, G, S, P, gpw=gpw))


@pytest.mark.parametrize("board,blocks,filters", [(6, 2, 64), (8, 2, 128)])
def test_table_other_geometries(board, blocks, filters):
    net = _net(board, blocks, filters, seed=1)
    G, S, P = 160, 200, 34     # four batches: distinct games per slot
    _same(_run(net, G, S, P, table=(1 << 14, 14), chunks=[10, 24]), _run(net, G, S, P))


def test_table_generations_follow_the_weights():
    """New weights in place (LeafEvaluator.refresh) start a new table generation; another
    evaluator's blob on the same engine does too. The games equal those of an engine without the
    table (neither has the memo, whose links would need their own reset for the second net)."""
    import rvz
    G, S = 96, 192
    out = []
    for table in (True, False):
        net = _net(8, 2, 64, seed=6)
        net2 = _net(8, 2, 64, seed=7)
        eng = rvz.Engine(G, S, 64)                     # no memo: only the table carries rows
        if table:
            eng.table(1 << 14, 20)
        ev = rvz.LeafEvaluator(net)
        run = rvz.SelfPlayRunner(eng, ev, autoreset=True, seed_base=9, fused=True)
        run.start()
        moves = []

        def ply(e):
            h = torch.full((1, G), -9, dtype=torch.int32, device="cuda")
            eng.play(e, 1, 1.0, run.seeds, run.seed_stride, run._plies, run._done, reset=True,
                     hist=h)
            moves.append(h[0])

        for _ in range(3):
            ply(ev)
        with torch.no_grad():
            for prm in net.parameters():
                prm.mul_(1.5)
        ev.refresh()
        for _ in range(3):
            ply(ev)
        ev2 = rvz.LeafEvaluator(net2)                 # another blob: a new generation
        for _ in range(3):
            ply(ev2)
        eng.check()
        out.append(torch.stack(moves))
    assert torch.equal(out[0], out[1])


def test_table_blob_switch_is_refused_inside_a_capture():
    """a play with another weight blob bumps the table generation with a kernel on
    the stream; inside a graph capture that kernel would be recorded and invalidate the table on
    every replay, so rvz_play refuses it there. After one eager play with the new evaluator the
    capture goes through, and its replays keep the table (hits accumulate)."""
    import rvz
    G, S = 4096, 128                  # openings: the same positions in many games (hits)
    eng = rvz.Engine(G, S, 64, memo=True)
    eng.table(1 << 16, 14)
    ev_a = rvz.LeafEvaluator(_net(8, 1, 64, seed=1))
    ev_b = rvz.LeafEvaluator(_net(8, 1, 64, seed=2))
    run = rvz.SelfPlayRunner(eng, ev_a, autoreset=True, seed_base=3, skip_last_eval=True,
                             fused=True)
    run.start()
    run._body(1)                      # the table's generation belongs to ev_a's blob
    eng.play_buffers(ev_b)
    run.evaluator = ev_b
    g = torch.cuda.CUDAGraph()
    with pytest.raises(rvz.RvzError, match="capturing"):
        with torch.cuda.graph(g):
            run._body(1)
    torch.cuda.synchronize()
    run._body(1)                      # eager: the generation moves to ev_b's blob
    run.capture(plies=1)
    h0, p0 = int(eng.table_stats[0].item()), int(run._plies.sum())
    for _ in range(3):
        run.ply()
    torch.cuda.synchronize()
    eng.check()
    assert int(run._plies.sum()) - p0 == 3 * G
    assert int(eng.table_stats[0].item()) > h0


def test_play_records_need_hist():
    """the C-ABI writes a recorded act's move only to hist (out_p is not written
    with records), so Engine.play refuses records without hist instead of losing the moves."""
    import rvz
    G, S, n = 16, 64, 2
    eng = rvz.Engine(G, S, 64, memo=True)
    ev = rvz.LeafEvaluator(_net(8, 1, 64))
    z = torch.zeros(G, dtype=torch.int64, device="cuda")
    rec = (torch.zeros(n, G, dtype=torch.int64, device="cuda"),
           torch.zeros(n, G, dtype=torch.int64, device="cuda"),
           torch.zeros(n, G, dtype=torch.int32, device="cuda"),
           torch.zeros(n, G, eng.npol, dtype=torch.float64, device="cuda"))
    with pytest.raises(rvz.RvzError, match="hist"):
        eng.play(ev, n, 1.0, z + 5, G, z.clone(), z.clone(), records=rec)
