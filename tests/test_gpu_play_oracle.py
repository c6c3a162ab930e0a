"""The fused self-play launch (rvz_play, kernel k_play) held DIRECTLY against the literal oracle
(VERDICT r03 item 3), at the configurations bench.py runs it with, plus the launch's own
contracts: per-game ply budgets (the bench's phase stagger), the bounded queue wait, evaluator
refresh vs the memo, and capture before any eager call.

Oracle side (tests/oracle_play.py): for sampled games, the reference-semantics search of
oracle/ (mcts.py:322-407, 64 traversals per batch, virtual loss) with its leaves evaluated by the
same h2 evaluator and softmaxed by rvz.policy_softmax (the expand's own softmax), then
get_action_probs' tail (mcts.py:642-694) with the game's MT19937 stream. Compared: every ply's
f64 policy vector (bitwise; p = N / sum N, so equal p means equal visit counts) and move."""
import os

import numpy as np
import pytest
import torch

from oracle_play import OracleGames

pytestmark = pytest.mark.gpu


def _net(board, blocks, filters, seed=0):
    import rvz
    torch.manual_seed(seed)
    return rvz.AlphaZeroNetwork(board, blocks, filters).cuda().eval()


def _fused_runner(net, G, S, memo=True, skip=True, seed_base=42, gpw=0, table=None):
    import rvz
    eng = rvz.Engine(G, S, 64, board_size=net.board_size, memo=memo)
    if table:
        eng.table(*table)
    run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=seed_base,
                             skip_last_eval=skip, fused=True)
    run.play_group = gpw
    run.start()
    return run


def _play(run, plies, budget=None):
    G = run.eng.n_games
    hist = torch.full((plies, G), -9, dtype=torch.int32, device="cuda")
    run.eng.play(run.evaluator, plies, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
                 reset=True, skip_last_eval=run.skip_last_eval, hist=hist,
                 games_per_workgroup=run.play_group, budget=budget)
    return hist


def _vs_oracle(oracle, net, G, S, plies, gpw, sample_n=16, memo=True, skip=True, table=None):
    run = _fused_runner(net, G, S, memo=memo, skip=skip, gpw=gpw, table=table)
    sample = np.linspace(0, G - 1, sample_n).astype(int)
    orc = OracleGames(oracle, [42 + int(g) for g in sample], S, bs=net.board_size)
    compared = 0
    for ply in range(plies):
        hist = _play(run, 1)                       # one k_play launch per ply
        run.eng.check()
        idx = hist[0].cpu().numpy()
        p = run.eng.p_buf.cpu().numpy()
        live = np.array([not g.over for g in orc.games])   # an ended game restarted (autoreset)
        _, oi, op, _ = orc.ply(run.evaluator)
        s = sample[live]
        assert np.array_equal(oi[live], idx[s]), (ply, oi[live], idx[s])
        assert np.array_equal(op[live].view(np.int64), p[s].view(np.int64)), ply
        compared += int(live.sum())
    assert compared >= sample_n * plies * 0.9
    assert not run.evaluator.overflowed()
    return run


def test_k_play_c2_headline_form_vs_oracle(oracle):
    """bench.py's C2 headline form at full size: 4,096 games x 800 sims, the 6x64 net, memo and
    the last batch left to it, the cross-game table (--evals table), the task queue with groups
    of 6 (play_group -6); 16 sampled games, 3 plies, each ply one k_play launch. In these plies
    every game's leaves are opening positions that other games evaluated: table hits."""
    net = _net(8, 6, 64)
    run = _vs_oracle(oracle, net, 4096, 800, 3, -6, table=(1 << 20, 14))
    assert int(run.eng.table_stats[0].item()) > 0


def test_k_play_c5_preset_vs_oracle(oracle):
    """C5's fused preset at full size: 16,384 6x6 games x 400 sims, the 6x64 net on packed 6x6
    boards (three per workgroup), groups of 24; 16 sampled games, 2 plies (parity of the 6x6
    variant is unpinned by design: the reference's Board rejects size != 8, board.py:27-28)."""
    net = _net(6, 6, 64)
    _vs_oracle(oracle, net, 16384, 400, 2, -24, table=(1 << 20, 14))


def test_k_play_c3_shape_vs_oracle_whole_games(oracle):
    """The 10x128 trunk inside k_play (one board per pass), 96 games x 800 sims played to their
    end (60 plies), 12 sampled games against the oracle in every ply."""
    net = _net(8, 10, 128, seed=2)
    _vs_oracle(oracle, net, 96, 800, 60, -4, sample_n=12)


def test_k_play_c3_bench_form_at_full_size(oracle):
    """C3 exactly as bench.py runs it: 32,768 games x 800 sims, the 10x128
    net, memo + the last batch left to it + the cross-game table, the task queue with groups of
    16 (play_group -16), autoreset; one k_play launch per ply. Every ply: 16 sampled games equal
    the oracle (f64 policy bitwise, move), and every game's move equals the pull-style runner's
    (per-batch launches, no table); at the end boards / statuses / counters / seeds / p equal."""
    import rvz
    net = _net(8, 10, 128)
    G, S, plies = 32768, 800, 2
    run = _fused_runner(net, G, S, gpw=-16, table=(1 << 20, 14))
    ref = rvz.SelfPlayRunner(rvz.Engine(G, S, 64, compact_leaves=True, memo=True),
                             rvz.LeafEvaluator(net), autoreset=True, seed_base=42,
                             skip_last_eval=True)
    ref.start()
    sample = np.linspace(0, G - 1, 16).astype(int)
    orc = OracleGames(oracle, [42 + int(g) for g in sample], S)
    for ply in range(plies):
        hist = _play(run, 1)
        run.eng.check()
        ref.ply()
        assert torch.equal(hist[0], ref.eng.idx_buf), f"ply {ply}: fused != pull-style"
        _, oi, op, _ = orc.ply(run.evaluator)
        idx = hist[0].cpu().numpy()
        p = run.eng.p_buf.cpu().numpy()
        assert np.array_equal(oi, idx[sample]), (ply, oi, idx[sample])
        assert np.array_equal(op.view(np.int64), p[sample].view(np.int64)), ply
    for x, y in zip(run.eng.get_state(), ref.eng.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(run._plies, ref._plies) and torch.equal(run._done, ref._done)
    assert torch.equal(run.seeds, ref.seeds) and torch.equal(run.eng.p_buf, ref.eng.p_buf)
    assert int(run.eng.table_stats[0].item()) > 0      # opening positions: table hits
    ref.eng.check()
    assert not run.evaluator.overflowed()


def test_k_play_c1_preset_vs_oracle_whole_game(oracle):
    """C1's fused preset (round 6): one game, 100 sims, the ModelConfig default 5x128 net, the
    memo + the last batch left to it + the cross-game table, one workgroup playing the game:
    61 plies (a whole game of at most 60 moves, then the next one, autoreset), each ply's f64
    policy and move equal to the oracle's; the same game, move for move, as the pull-style runner
    (per-batch launches, no table), which the preset ran until round 6. Table hits come from
    positions the game's earlier searches evaluated. (At 100 sims a search is two batches of 64:
    the second goes whole to the first unvisited root child, mcts.py:96-97, so this pins the
    launch's mechanics at C1's shape; the RNG and the net's outputs are pinned by the other
    tests.)"""
    import rvz
    net = _net(8, 5, 128, seed=3)
    G, S, plies = 1, 100, 61
    run = _vs_oracle(oracle, net, G, S, plies, 0, sample_n=1, table=(1 << 20, 14))
    assert int(run.eng.table_stats[0].item()) > 0
    ref = rvz.SelfPlayRunner(rvz.Engine(G, S, 64, compact_leaves=True, memo=True),
                             rvz.LeafEvaluator(net), autoreset=True, seed_base=42,
                             skip_last_eval=True)
    ref.start()
    for _ in range(plies):
        ref.ply()
    for x, y in zip(run.eng.get_state(), ref.eng.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(run._plies, ref._plies) and torch.equal(run._done, ref._done)
    assert torch.equal(run.seeds, ref.seeds)
    ref.eng.check()


def test_k_play_c5_preset_equals_runner_at_full_size():
    """C5 as bench.py runs it (16,384 games, 400 sims, groups of 24, three 6x6 boards per
    workgroup), 34 plies (every 6x6 game ends within 32, so restarts are included): every ply's
    moves, the final boards / statuses / seeds / counters / p equal the pull-style runner's."""
    import rvz
    net = _net(6, 6, 64)
    G, S, plies = 16384, 400, 34
    run = _fused_runner(net, G, S, gpw=-24)
    hist = _play(run, plies)
    ref = rvz.SelfPlayRunner(rvz.Engine(G, S, 64, board_size=6, compact_leaves=True, memo=True),
                             rvz.LeafEvaluator(net), autoreset=True, seed_base=42,
                             skip_last_eval=True)
    ref.start()
    for k in range(plies):
        ref.ply()
        assert torch.equal(hist[k], ref.eng.idx_buf), f"ply {k}"
    for x, y in zip(run.eng.get_state(), ref.eng.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(run._plies, ref._plies) and torch.equal(run._done, ref._done)
    assert torch.equal(run.seeds, ref.seeds) and torch.equal(run.eng.p_buf, ref.eng.p_buf)
    run.eng.check()
    ref.eng.check()


@pytest.mark.parametrize("gpw", [-6, 5])
def test_ply_budget_plays_prefixes(gpw):
    """rvz_play's ply_budget: game g commits min(plies, budget[g]) plies and is otherwise left
    alone; its moves are the first budget[g] of an unbudgeted run, and topping the budgets up to
    the same total afterwards gives the unbudgeted run's games exactly (queue and static)."""
    net = _net(8, 2, 64, seed=5)
    G, S, P = 203, 200, 9      # four batches: distinct games per slot
    full = _fused_runner(net, G, S, gpw=gpw)
    hf = _play(full, P)
    bud = torch.arange(G, dtype=torch.int32, device="cuda") % (P + 2) - 1   # -1 .. P
    part = _fused_runner(net, G, S, gpw=gpw)
    hb = _play(part, P, budget=bud)
    b = bud.clamp(min=0).long().cpu()
    assert torch.equal(part._plies.cpu(), torch.minimum(b, torch.tensor(P)))
    hf, hb = hf.cpu(), hb.cpu()
    for g in range(G):
        n = min(int(b[g]), P)
        assert torch.equal(hb[:n, g], hf[:n, g]), g
        assert (hb[n:, g] == -9).all(), g
    rest = (P - torch.minimum(b, torch.tensor(P))).to(torch.int32).cuda()
    _play(part, P, budget=rest)
    for x, y in zip(part.eng.get_state(), full.eng.get_state()):
        assert torch.equal(x, y)
    assert torch.equal(part._plies, full._plies) and torch.equal(part.seeds, full.seeds)
    part.eng.check()


def test_stagger_then_pull_style_equals_fused():
    """bench.py staggers a pull-style preset's games (C3) with one budgeted rvz_play launch and
    then runs its per-batch launches on the same engine: the games must be those of the fused
    launch continuing instead (the engine state k_play leaves is the pull-style path's)."""
    import rvz
    net = _net(8, 2, 128, seed=4)
    G, S, P = 160, 160, 12
    bud = (torch.arange(G, dtype=torch.int32, device="cuda") * 7) % 13
    outs = []
    for pull in (True, False):
        eng = rvz.Engine(G, S, 64, compact_leaves=True, memo=True)
        run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=3,
                                 skip_last_eval=True, fused=not pull)
        run.start()
        eng.play(run.evaluator, 13, 1.0, run.seeds, run.seed_stride, run._plies, run._done,
                 reset=True, skip_last_eval=True, budget=bud)
        if pull:
            moves = []
            for _ in range(P):
                run.ply()
                moves.append(eng.idx_buf.clone())
            moves = torch.stack(moves)
        else:
            moves = _play(run, P)
        eng.check()
        outs.append((moves, [t.clone() for t in eng.get_state()], run._plies.clone()))
    (ma, sa, pa), (mb, sb, pb) = outs
    assert torch.equal(ma, mb)
    assert all(torch.equal(x, y) for x, y in zip(sa, sb)) and torch.equal(pa, pb)


def test_queue_wait_timeout_drains_and_reports():
    """The bounded queue wait: a wait that times out sets device error 16; the other
    workgroups stop drawing tasks and the launch ends (no hang); after a reset the engine plays
    normally again. RVZ_PLAY_SPIN_LIMIT=0 makes every wait time out at once."""
    import rvz
    net = _net(8, 1, 64)
    G, S = 256, 64
    run = _fused_runner(net, G, S, gpw=-1)
    os.environ["RVZ_PLAY_SPIN_LIMIT"] = "0"
    try:
        _play(run, 4)
        torch.cuda.synchronize()
    finally:
        del os.environ["RVZ_PLAY_SPIN_LIMIT"]
    with pytest.raises(rvz.RvzError, match="16"):
        run.eng.check()
    run.start()
    ok = _fused_runner(net, G, S, gpw=-1)
    run._plies.zero_()
    h1, h2 = _play(run, 3), _play(ok, 3)
    run.eng.check()
    assert torch.equal(h1, h2)


def test_evaluator_refresh_drops_the_memo():
    """after LeafEvaluator.refresh() (new weights) an engine with the memo must not
    expand from the old net's carried outputs: the games equal those of an engine without the
    memo, with refresh() alone (no explicit memo_reset)."""
    import rvz
    out = []
    for memo in (True, False):
        net = _net(8, 2, 64, seed=6)
        eng = rvz.Engine(96, 192, 64, compact_leaves=True, memo=memo)
        ev = rvz.LeafEvaluator(net)
        run = rvz.SelfPlayRunner(eng, ev, autoreset=True, seed_base=9, skip_last_eval=memo)
        run.start()
        for _ in range(3):
            run.ply()
        with torch.no_grad():
            for prm in net.parameters():
                prm.mul_(1.5)
        ev.refresh()
        moves = []
        for _ in range(5):
            run.ply()
            moves.append(eng.idx_buf.clone())
        eng.check()
        out.append(torch.stack(moves))
    assert torch.equal(out[0], out[1])


def test_fused_capture_without_an_eager_ply_counts_rows():
    """the fused runner's first call may be a graph capture; play()'s row counter and
    scratch are allocated before it (SelfPlayRunner(fused=True)), so replays accumulate rows as
    eager launches do."""
    import rvz
    net = _net(8, 1, 64)
    G, S = 64, 200        # four batches: distinct games (asserted below)
    runs = []
    for graph in (True, False):
        eng = rvz.Engine(G, S, 64, memo=True)
        run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=1,
                                 skip_last_eval=True, fused=True)
        run.start()
        if graph:
            run.capture(plies=2)
        for _ in range(3):
            run.ply() if graph else run._body(2)
        torch.cuda.synchronize()
        runs.append((int(eng.play_rows.item()), run._plies.clone(),
                     eng.get_state()[0].clone()))
    assert runs[0][0] == runs[1][0] > 0 and torch.equal(runs[0][1], runs[1][1])
    assert torch.equal(runs[0][2], runs[1][2]) and len(set(runs[0][2].tolist())) > 1


def test_play_refuses_to_allocate_inside_a_capture(monkeypatch):
    """Engine.play called inside a capture before its buffers exist raises instead of recording
    their zero-fill into the graph (the capture is simulated: no graph is left half-captured)."""
    import rvz
    eng = rvz.Engine(8, 64, 64)
    ev = rvz.LeafEvaluator(_net(8, 1, 64))
    z = torch.zeros(8, dtype=torch.int64, device="cuda")
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    with pytest.raises(rvz.RvzError, match="play_buffers"):
        eng.play(ev, 1, 1.0, z, 8, z, z)
    monkeypatch.undo()
    eng.play_buffers(ev)
    eng.play(ev, 1, 1.0, z.clone() + 5, 8, z, z.clone())
    eng.check()


def test_fused_graph_replays_keep_playing():
    """Regression (round 4): rvz_play's queue words were reset by a hipMemsetAsync node, whose
    graph replays left a device address in them (tools/diag_stagger.py), so every replay after
    the first drew no task and played nothing, silently. A fill kernel resets them now: every
    replay of a captured 20-ply launch at C2 size commits 20 plies of every game."""
    net = _net(8, 6, 64)
    G = 4096
    run = _fused_runner(net, G, 800, gpw=-6)
    run._body(20)
    run.capture(plies=20)
    for _ in range(4):
        p0 = int(run._plies.sum())
        run.ply()
        torch.cuda.synchronize()
        assert int(run._plies.sum()) - p0 == 20 * G
        run.eng.check()
