"""The fused self-play launch (rvz_play / Engine.play / SelfPlayRunner(fused=True)): each
workgroup plays its own games — search, h2 trunk + FC heads, act, autoreset — in one launch.
Held bit for bit against the pull-style runner (per-batch k_step / trunk / heads launches, k_act,
k_autoreset), which the other GPU tests pin to the oracle and the reference's recorded games:
every ply's move of every game, the final boards, statuses, RNG-driven restarts and counters."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net(board, blocks, filters, seed=0):
    import rvz
    torch.manual_seed(seed)
    return rvz.AlphaZeroNetwork(board, blocks, filters).cuda().eval()


def _plain(net, G, S, plies, memo, skip, seed_base=42):
    import rvz
    run = rvz.SelfPlayRunner(rvz.Engine(G, S, 64, board_size=net.board_size, compact_leaves=True,
                                        memo=memo),
                             rvz.LeafEvaluator(net), autoreset=True, seed_base=seed_base,
                             skip_last_eval=skip)
    run.start()
    moves = []
    for _ in range(plies):
        run.ply()
        moves.append(run.eng.idx_buf.clone())
    return run, torch.stack(moves)


def _fused(net, G, S, plies, memo, skip, seed_base=42, gpw=0, chunks=(None,), gate=None):
    import rvz
    eng = rvz.Engine(G, S, 64, board_size=net.board_size, memo=memo)
    if gate is not None:                  # rvz_play_gate (fraction, us, late_us); default: on
        eng.play_gate(*gate)
    run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=seed_base,
                             skip_last_eval=skip, fused=True)
    run.start()
    hs, done = [], 0
    for c in chunks:              # plies per launch (None: all of them)
        n = plies - done if c is None else c
        hist = torch.full((n, G), -9, dtype=torch.int32, device="cuda")
        eng.play(run.evaluator, n, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
                 reset=True, skip_last_eval=skip, hist=hist, games_per_workgroup=gpw)
        hs.append(hist)
        done += n
    assert done == plies
    return run, torch.cat(hs)


def _same(a, b):
    (ra, ma), (rb, mb) = a, b
    assert ma.shape == mb.shape
    for k in range(ma.shape[0]):
        assert torch.equal(ma[k], mb[k]), f"ply {k}: {int((ma[k] != mb[k]).sum())} games differ"
    for x, y in zip(ra.eng.get_state(), rb.eng.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(ra._plies, rb._plies) and torch.equal(ra._done, rb._done)
    assert torch.equal(ra.seeds, rb.seeds)
    assert torch.equal(ra.eng.p_buf, rb.eng.p_buf)
    ra.eng.check()
    rb.eng.check()


@pytest.mark.parametrize("memo,skip", [(False, False), (True, False), (True, True)])
def test_fused_plays_the_runner_games(memo, skip):
    """8x8, 6x64 net, 300 games x 200 sims over 70 plies (whole games and restarts)."""
    net = _net(8, 6, 64)
    G, S, plies = 300, 200, 70
    _same(_fused(net, G, S, plies, memo, skip), _plain(net, G, S, plies, memo, skip))


@pytest.mark.parametrize("gpw,chunks", [(1, (None,)), (3, (5, 1, 14)), (7, (20,)), (64, (20,)),
                                        (-1, (None,)), (-2, (20,)), (-3, (7, 13)), (-4, (9, 11)),
                                        (-6, (20,)), (-8, (20,)), (-16, (9, 11)), (-64, (20,))])
def test_fused_workgroup_sizes_and_launch_splits(gpw, chunks):
    """Static schedule with 1 / 3 / 7 / 64 games per workgroup (a partial last workgroup, odd
    queues) and the task queue with groups of 1 / 2 / 3 / 4 / 6 / 8 / 16 (C3's) / 64 games (a group's
    consecutive plies on different workgroups, published by agent-scope release / acquire), the
    plies split over several launches: the same games."""
    net = _net(8, 2, 64, seed=3)
    G, S = 203, 200       # four batches: the games' sampled moves diverge (with two, every copy
    # of the second batch takes the first unvisited child and the slots play one game)
    a = _fused(net, G, S, 20, True, True, gpw=gpw, chunks=chunks)
    assert len(set(a[1][3].tolist())) > 1                  # distinct games by the fourth ply
    _same(a, _plain(net, G, S, 20, True, True))


@pytest.mark.parametrize("board,blocks,filters,gpw", [(8, 2, 128, 0), (8, 2, 128, -16),
                                                     (6, 2, 64, 0), (6, 1, 128, 0),
                                                     (8, 2, 256, 0), (8, 1, 256, 5)])
def test_fused_other_geometries(board, blocks, filters, gpw):
    """The C3 trunk shape (128 filters, one board per pass; with the default queue groups and
    with bench.py's C3 groups of 16, play_group -16), the packed 6x6 geometry (C5) and the
    256-filter trunk (k_play<256, 1, 4, 4, 8, 1>, one workgroup per CU; queue and static)."""
    net = _net(board, blocks, filters, seed=1)
    # three (8x8) / four (6x6) leaf batches: the visits spread over two or three root children,
    # so the games diverge (with two batches every slot plays one game, mcts.py:96-97)
    G, S, plies = 160, 160 if board == 8 else 200, 24
    a = _fused(net, G, S, plies, True, True, gpw=gpw)
    assert len(set(a[1][3].tolist())) > 1                  # distinct games by the fourth ply
    _same(a, _plain(net, G, S, plies, True, True))


def test_fused_headline_configuration_at_full_size():
    """bench.py's C2 workload at full size: 4,096 games x 800 sims, the 6x64 net, memo and the
    last batch left to it, 64 plies (a whole game and its restarts): identical to the runner."""
    net = _net(8, 6, 64)
    G, S, plies = 4096, 800, 64
    _same(_fused(net, G, S, plies, True, True), _plain(net, G, S, plies, True, True))


def test_fused_graph_capture_and_errors():
    """A captured fused ply replays the same games; play() refuses non-h2 evaluators and a
    call inside a pull-style search."""
    import rvz
    net = _net(8, 1, 64)
    G, S = 64, 200        # four batches: distinct games (asserted below)
    eng = rvz.Engine(G, S, 64, memo=True)
    run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=5, fused=True)
    run.start()
    run.ply()
    run.capture(plies=3)
    for _ in range(4):
        run.ply()
    ref, _ = _plain(net, G, S, 13, True, False, seed_base=5)
    for x, y in zip(run.eng.get_state(), ref.eng.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(run._plies, ref._plies)
    assert len(set(run.eng.get_state()[0].tolist())) > 1   # not one game in every slot
    with pytest.raises(rvz.RvzError):
        eng.play(lambda x: net(x), 1, 1.0, run.seeds, G, run._plies, run._done)
    eng.search_begin()
    eng.search_step()
    with pytest.raises(rvz.RvzError):
        eng.play(run.evaluator, 1, 1.0, run.seeds, G, run._plies, run._done)


@pytest.mark.parametrize("board,filters", [(8, 64), (6, 64), (8, 128), (8, 256)])
def test_fused_ranged_rerun_is_per_board(board, filters):
    """The activation range's re-run inside k_play (h2_pass: an unscaled trunk, then the boards
    that overflowed again with their images scaled) keeps every board's outputs a function of
    its own position: stem channels 0-7 fire at 2e5 (past f16's 65520) exactly where the mover
    has >= 7 discs in a 3x3 window (and feed nothing but the skip path, so the games stay
    ordinary), so mid-game passes mix overflowing and ordinary boards, and
    the fused launch (queue groups, its own pass grouping) plays the same games, bit for bit, as
    the pull-style runner (k_resnet_h2's pass grouping). Geometries: the 8x8 pair (C2), three
    packed 6x6 boards (C5), one 8x8 board at F = 128 (C3)."""
    net = _net(board, 2, filters, seed=2)
    W = 2e5
    with torch.no_grad():
        net.conv.weight[:8].zero_()
        net.conv.weight[:8, 0] = W
        if net.conv.bias is not None:
            net.conv.bias[:8].zero_()
        net.bn.running_mean[:8] = 0.0
        net.bn.running_var[:8] = 1.0 - net.bn.eps
        net.bn.weight[:8] = 1.0
        net.bn.bias[:8] = -6.5 * W
        # the loud channels reach no other channel and no head (they ride the skip path): the
        # games stay ordinary, only the stored images carry the large values
        for blk in net.res_blocks:
            blk.conv1.weight[:, :8] = 0.0
        for m in (net.policy_conv, net.value_conv):
            m.weight[:, :8] = 0.0
    # S = 320: five batches, so a search's visits spread over several root children (with two,
    # every copy of the second batch takes the first unvisited child: mcts.py's +inf for N = 0)
    # and the games' sampled moves diverge
    G, S, plies = 192, 320, (56 if board == 8 else 28)
    n = board * board
    bits = np.arange(n, dtype=np.uint64)

    def loud_boards(eng):      # boards whose mover has a window of >= 7 discs (stem past 65520)
        state = eng.get_state()
        torch.cuda.synchronize()                  # (copied on the engine's stream)
        bl, wh, st = (t.cpu().numpy() for t in state)
        mover = np.where((st[:, 0] == 1)[:, None], bl.view(np.uint64)[:, None],
                         wh.view(np.uint64)[:, None])
        grid = ((mover >> bits) & np.uint64(1)).astype(np.int32).reshape(G, board, board)
        pad = np.pad(grid, ((0, 0), (1, 1), (1, 1)))
        win = sum(pad[:, 1 + dr:1 + dr + board, 1 + dc:1 + dc + board]
                  for dr in (-1, 0, 1) for dc in (-1, 0, 1))
        return int((win >= 7).any(axis=(1, 2)).sum())

    import rvz
    run = rvz.SelfPlayRunner(rvz.Engine(G, S, 64, board_size=board, compact_leaves=True, memo=True),
                             rvz.LeafEvaluator(net), autoreset=True, seed_base=42,
                             skip_last_eval=True)
    run.start()
    moves, counts = [], []
    for _ in range(plies):
        run.ply()
        moves.append(run.eng.idx_buf.clone())
        counts.append(loud_boards(run.eng))       # roots of the next search: some loud, some not
    assert sum(0 < c < G for c in counts) >= 3, str(counts)
    a = _fused(net, G, S, plies, True, True)
    _same(a, (run, torch.stack(moves)))
    for r in (a[0], run):
        assert not r.evaluator.overflowed()


@pytest.mark.parametrize("gate,filters", [((-1.0, 0.0, 0.0), 128), ((0.05, 20.0, 0.0), 128),
                                          ((1.0, 5.0, 0.0), 128), ((0.5, 20.0, 10.0), 128),
                                          ((-1.0, 0.0, 0.0), 256)],
                         ids=["default", "low", "timeout", "late", "default-256"])
def test_pass_gate_keeps_the_games(gate, filters):
    """The per-XCD pass gate (rvz_play_gate, rvz_play.hip.h play_gate; the 8x8 forms of 128 and
    256 filters) changes when a workgroup starts a trunk pass, never what it computes: the same
    games with the gate off and with the default setting (on), rounds opened by a low arrival
    fraction, by the timeout (every running workgroup of an XCD never arrives together), and with
    the late-join window."""
    net = _net(8, 2, filters, seed=1)
    G, S, plies = 160, 200, 12
    a = _fused(net, G, S, plies, True, True, gpw=-4, gate=(0.0, 0.0, 0.0))
    b = _fused(net, G, S, plies, True, True, gpw=-4, gate=gate)
    assert len(set(a[1][3].tolist())) > 1
    _same(a, b)


def test_pass_gate_setting_is_checked():
    import rvz
    eng = rvz.Engine(8, 64, 64)
    for bad in ((1.5, 10.0, 0.0), (0.5, -1.0, 0.0), (0.5, 10.0, -1.0), (0.5, 2e6, 0.0)):
        with pytest.raises(rvz.RvzError, match="rvz_play_gate"):
            eng.play_gate(*bad)
    eng.play_gate(0.0)                    # off
    eng.play_gate()                       # the default
