"""Search kernels (select / expand_backup / visits / act) through the C-ABI:

 * replay of the reference's recorded games (tests/golden/mcts_*.npz): the engine's leaves must be
   the reference's NN inputs, and with the reference's own softmax rows and values fed back the
   visits, the f64 policy vectors (bitwise) and the sampled actions must be the reference's;
 * lockstep against the literal CPU oracle (no dedup, virtual loss kept) at larger game counts
   with a real network's outputs shared by both, 8x8 and the 6x6 variant;
 * full-size (4,096 and 32,768 games) invariants.
"""
import numpy as np
import pytest
import torch

import golden_replay as R

pytestmark = pytest.mark.gpu


def _status_rows(games):
    return torch.tensor([[g.side, g.over, g.winner, g.passed] for g in games], dtype=torch.int32)


@pytest.mark.parametrize("path", R.fixture_paths(), ids=lambda p: p.split("/")[-1])
def test_engine_replays_reference_games(path):
    import rvz
    fx = R.load(path)
    games = list(R.games(fx))
    G, sims, T = len(games), int(fx["sims"]), float(fx["temperature"])
    eng = rvz.Engine(G, num_simulations=sims, batch_size=int(fx["batch"]),
                     c_puct=float(fx["c_puct"]))
    eng.reset([g["seed"] for g in games])
    ci = [0] * G
    n_ply = max(len(g["ply_action"]) for g in games)
    probs = torch.zeros(G, 65, dtype=torch.float32, device="cuda")
    value = torch.zeros(G, dtype=torch.float32, device="cuda")
    for k in range(n_ply):
        b, w, st = eng.get_state()
        b, st = b.cpu().numpy().view(np.uint64), st.cpu().numpy()
        for gi, g in enumerate(games):
            if k < len(g["ply_action"]):
                assert int(b[gi]) == int(g["ply_black"][k]) and st[gi, 0] == g["ply_side"][k]
        eng.search_begin()
        while eng.search_step():
            need = eng.need.cpu().numpy()
            x = eng.leaf_x.cpu().numpy()
            pr = np.zeros((G, 65), np.float32)
            va = np.zeros(G, np.float32)
            for gi, g in enumerate(games):
                if need[gi] == 0:
                    continue
                c = ci[gi]
                assert R.planes_to_masks(x[gi]) == [int(v) for v in g["call_masks"][c]], (k, gi, c)
                pr[gi], va[gi] = g["call_probs"][c], g["call_value"][c]
                ci[gi] += 1
            probs.copy_(torch.from_numpy(pr))
            value.copy_(torch.from_numpy(va))
            eng.search_submit(probs, value, is_logits=False)
        vis = eng.visits().cpu().numpy()
        idx, p = eng.act(T, apply=True)
        idx, p = idx.cpu().numpy(), p.cpu().numpy()
        for gi, g in enumerate(games):
            if k >= len(g["ply_action"]):
                assert idx[gi] == -2
                continue
            np.testing.assert_array_equal(vis[gi], g["ply_visits"][k])
            assert np.array_equal(p[gi].view(np.int64), g["ply_p"][k].view(np.int64)), (k, gi)
            assert idx[gi] == g["ply_action"][k]
    for gi, g in enumerate(games):
        assert ci[gi] == len(g["call_ply"])
    _, _, st = eng.get_state()
    st = st.cpu().numpy()
    assert [int(s) for s in st[:, 2]] == [g["winner"] for g in games]
    eng.check()


def _lockstep(oracle, G, sims, bs, n_plies, net, T=1.0, seed0=100, fused=False):
    """Play n_plies of G games on the engine and on the oracle with shared NN outputs."""
    import rvz
    eng = rvz.Engine(G, num_simulations=sims, batch_size=64, board_size=bs)
    seeds = [seed0 + g for g in range(G)]
    eng.reset(seeds)
    srch = oracle.Search(G, sims, 64, 1.0, bs=bs)
    games = [oracle.new_game(bs) for _ in range(G)]
    mts = [oracle.MT(s) for s in seeds]
    npol = bs * bs + 1
    for k in range(n_plies):
        srch.begin(games)
        eng.search_begin()
        while eng.search_step():
            r = srch.step()
            assert r is not None
            leaves, ncop = r
            need = eng.need.cpu().numpy()
            np.testing.assert_array_equal(need, ncop)   # same number of queued copies per game
            with torch.no_grad():
                logits, v = net(eng.leaf_x)
            probs = torch.softmax(logits, dim=1).float().contiguous()
            v = v.float().contiguous()
            x = eng.leaf_x.cpu().numpy()
            for g in np.flatnonzero(need):
                np.testing.assert_array_equal(x[g], oracle.canonical(leaves[g], bs))
            if fused:
                eng.search_submit(logits.float().contiguous(), v, is_logits=True)
            else:
                eng.search_submit(probs, v, is_logits=False)
            srch.submit(probs.cpu().numpy(), v.cpu().numpy())
        assert srch.step() is None
        vis_e = eng.visits().cpu().numpy()
        vis_o = srch.visits()
        if fused:
            return vis_e, vis_o
        np.testing.assert_array_equal(vis_e, vis_o)
        idx, p = eng.act(T, apply=True)
        idx, p = idx.cpu().numpy(), p.cpu().numpy()
        for g in range(G):
            if games[g].over:
                assert idx[g] == -2
                continue
            u = mts[g].random_sample() if oracle.action_needs_draw(vis_o[g], T) else 0.0
            oi, op, _ = oracle.action(vis_o[g], T, u)
            assert oi == idx[g], (k, g)
            assert np.array_equal(op.view(np.int64), p[g].view(np.int64))
            oracle.make_move(games[g], -1 if oi == npol - 1 else oi, bs)
        b, w, st = eng.get_state()
        b, w, st = b.cpu().numpy().view(np.uint64), w.cpu().numpy().view(np.uint64), st.cpu().numpy()
        for g in range(G):
            assert (int(b[g]), int(w[g]), *map(int, st[g])) == \
                (games[g].black, games[g].white, games[g].side, games[g].over,
                 games[g].winner, games[g].passed)
    eng.check()
    return None


def _net(bs, blocks=2, filters=32, seed=0):
    import rvz
    torch.manual_seed(seed)
    net = rvz.AlphaZeroNetwork(board_size=bs, num_res_blocks=blocks, num_filters=filters).cuda().eval()
    return lambda x: net(x.float())


def test_lockstep_vs_oracle_8x8_full_games(oracle):
    _lockstep(oracle, G=48, sims=800, bs=8, n_plies=60, net=_net(8))


def test_lockstep_vs_oracle_8x8_s100_t05(oracle):
    _lockstep(oracle, G=64, sims=100, bs=8, n_plies=60, net=_net(8, seed=3), T=0.5, seed0=7)


def test_lockstep_vs_oracle_6x6(oracle):
    _lockstep(oracle, G=64, sims=400, bs=6, n_plies=32, net=_net(6, seed=1))


def test_fused_softmax_within_tolerance():
    """The expand kernel's fused softmax vs torch.softmax (mcts.py:596): priors to rtol 2e-6."""
    import rvz
    G = 256
    eng = rvz.Engine(G, num_simulations=64, batch_size=64)
    eng.reset(range(G))
    eng.search_begin()
    assert eng.search_step()
    torch.manual_seed(0)
    logits = (torch.randn(G, 65, device="cuda") * 3).contiguous()
    eng.search_submit(logits, torch.zeros(G, device="cuda"), is_logits=True)
    nodes, meta = eng.tree()
    torch.cuda.synchronize()
    eng.check()
    pri = nodes[:, 1:5, 2].cpu().view(torch.float32).numpy()    # root children (4 legal moves)
    sq = (meta[:, 1:5].cpu().numpy() & 63)
    ref = torch.softmax(logits, 1).cpu().numpy()
    np.testing.assert_array_equal(sq[0], [19, 26, 37, 44])
    np.testing.assert_allclose(pri, np.take_along_axis(ref, sq, 1), rtol=2e-6, atol=0)


def test_full_size_invariants_4096():
    """C2 size: one full 800-sim ply over 4,096 games with the 6x64 net (fp32)."""
    import rvz
    G = 4096
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
    ev = rvz.LeafEvaluator(net)
    eng = rvz.Engine(G, num_simulations=800, batch_size=64)
    eng.reset(range(42, 42 + G))
    eng.search(ev)
    vis = eng.visits()
    idx, p = eng.act(1.0, apply=True)
    torch.cuda.synchronize()
    eng.check()
    v = vis.cpu().numpy()
    assert (v.sum(1) == 800 - 64).all()            # root absorbs the first batch itself
    pp = p.cpu().numpy()
    assert np.allclose(pp.sum(1), 1.0, atol=1e-12)
    ii = idx.cpu().numpy()
    assert ((ii >= 0) & (ii < 64)).all()
    assert (v[np.arange(G), ii] > 0).all()          # sampled moves were visited
    # all games start from the same position: the 4 legal first moves only
    assert set(np.unique(ii)) <= {19, 26, 37, 44}


def test_full_size_invariants_32768():
    """C3 size (32,768 games, 800 sims): a full ply with a cheap evaluator; no device errors."""
    import rvz
    G = 32768
    eng = rvz.Engine(G, num_simulations=800, batch_size=64)
    eng.reset(range(G))
    zl = torch.zeros(G, 65, device="cuda")
    zv = torch.zeros(G, device="cuda")
    for ply in range(3):
        eng.search(lambda x: (zl, zv))
        idx, p = eng.act(1.0, apply=True)
    torch.cuda.synchronize()
    eng.check()
    vis = eng.visits().cpu().numpy()
    assert (vis.sum(1) == 736).all()


def test_c3_workload_two_plies(oracle):
    """C3 as configured (BASELINE.json configs[2]): 32,768 games x 800 sims with the 10x128 h2
    evaluator, compacted leaf batches, two plies. Properties of every game (no device error, no
    activation overflow, 736 = 800 - 64 root-child visits in the opening, every move legal) and,
    for 16 sampled games, the visit counts and moves of the literal oracle search fed by the
    same evaluator (an h2 row's outputs do not depend on its batch position)."""
    import rvz
    G, S = 32768, 800
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 10, 128).cuda().eval()
    ev = rvz.LeafEvaluator(net)
    eng = rvz.Engine(G, num_simulations=S, batch_size=64, compact_leaves=True)
    eng.reset(range(G))
    sample = np.linspace(0, G - 1, 16).astype(int)
    games = [oracle.new_game() for _ in sample]
    mts = [oracle.MT(int(g)) for g in sample]
    for ply in range(2):
        b0, w0, st0 = (t.clone() for t in eng.get_state())
        eng.search(ev, fused_softmax=False)          # torch's F.softmax on both sides
        vis = eng.visits().cpu().numpy().copy()
        idx, _ = eng.act(1.0, apply=True)
        idx = idx.cpu().numpy()
        eng.check()
        assert (vis.sum(1) == S - 64).all()
        legal = rvz.board_legal(b0, w0, st0).cpu().numpy().view(np.uint64)
        assert all((int(legal[g]) >> int(idx[g])) & 1 for g in range(G))
        srch = oracle.Search(len(sample), S, 64, 1.0)
        srch.begin(games)
        while (r := srch.step()) is not None:
            x = torch.from_numpy(oracle.leaf_planes(r[0])).cuda()
            lo, vo = ev(x)
            srch.submit(torch.softmax(lo, 1).cpu().numpy(), vo.cpu().numpy())
        ov = srch.visits()
        assert np.array_equal(ov, vis[sample]), ply
        for j, g in enumerate(sample):
            a, _, _ = oracle.action(ov[j], 1.0, mts[j].random_sample())
            assert a == idx[g]
            assert oracle.make_move(games[j], a)
    assert not ev.overflowed()


def test_c5_workload_two_plies(oracle):
    """C5 as configured (BASELINE.json configs[4]): 16,384 6x6 games x 400 sims with the 6x64 h2
    evaluator on packed 6x6 boards, compacted leaf batches, two plies: no device error or
    overflow, every move legal, and 16 sampled games' visits and moves equal the literal oracle
    search fed by the same evaluator (parity of the 6x6 variant is unpinned by design: the
    reference's Board rejects size != 8, board.py:27-28; the oracle generalises its rules)."""
    import rvz
    G, S, BS = 16384, 400, 6
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(BS, 6, 64).cuda().eval()
    ev = rvz.LeafEvaluator(net)
    eng = rvz.Engine(G, num_simulations=S, batch_size=64, board_size=BS, compact_leaves=True)
    eng.reset(range(G))
    sample = np.linspace(0, G - 1, 16).astype(int)
    games = [oracle.new_game(BS) for _ in sample]
    mts = [oracle.MT(int(g)) for g in sample]
    for ply in range(2):
        b0, w0, st0 = (t.clone() for t in eng.get_state())
        eng.search(ev, fused_softmax=False)          # torch's F.softmax on both sides
        vis = eng.visits().cpu().numpy().copy()
        idx, _ = eng.act(1.0, apply=True)
        idx = idx.cpu().numpy()
        eng.check()
        legal = rvz.board_legal(b0, w0, st0, BS).cpu().numpy().view(np.uint64)
        assert all((int(legal[g]) >> int(idx[g])) & 1 for g in range(G))
        srch = oracle.Search(len(sample), S, 64, 1.0, bs=BS)
        srch.begin(games)
        while (r := srch.step()) is not None:
            x = torch.from_numpy(oracle.leaf_planes(r[0], BS)).cuda()
            lo, vo = ev(x)
            srch.submit(torch.softmax(lo, 1).cpu().numpy(), vo.cpu().numpy())
        ov = srch.visits()
        assert np.array_equal(ov, vis[sample]), ply
        for j, g in enumerate(sample):
            a, _, _ = oracle.action(ov[j], 1.0, mts[j].random_sample())
            assert a == idx[g]
            assert oracle.make_move(games[j], a, BS)
    assert not ev.overflowed()


def test_bf16_leaf_planes_equal_f32():
    import rvz
    G = 512
    a = rvz.Engine(G, 128, 64, leaf_dtype=torch.float32)
    b = rvz.Engine(G, 128, 64, leaf_dtype=torch.bfloat16)
    for e in (a, b):
        e.reset(range(G))
        e.search_begin()
        assert e.search_step()
    torch.cuda.synchronize()
    assert torch.equal(a.leaf_x, b.leaf_x.float())
    assert torch.equal(a.need, b.need)


@pytest.mark.parametrize("board,sims", [(8, 800), (8, 100), (6, 400)])
def test_skip_last_eval_bit_exact(board, sims):
    """rvz_search_skip leaves the last batch of every search unevaluated: the visit counts, the
    f64 policy vectors, the sampled moves and the boards must be bit-identical to the evaluated
    search over whole games (autoreset keeps every slot busy), with a real network's outputs."""
    import rvz
    G, plies = 256, 70
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(board, 2, 64).cuda().eval()
    runs = []
    for skip in (False, True):
        ev = rvz.LeafEvaluator(net)
        eng = rvz.Engine(G, num_simulations=sims, batch_size=64, board_size=board)
        run = rvz.SelfPlayRunner(eng, ev, temperature=1.0, autoreset=True, seed_base=7,
                                 skip_last_eval=skip)
        run.start()
        trace = []
        for _ in range(plies):
            run.ply()
            b, w, st = eng.get_state()
            trace.append((eng.idx_buf.clone(), eng.p_buf.clone(), b.clone(), w.clone(),
                          st.clone()))
        eng.check()
        runs.append((trace, int(run.steps.item()), int(run.games_done.item())))
    (ta, sa, da), (tb, sb, db) = runs
    assert sa == sb and da == db and da > 0
    for k, (x, y) in enumerate(zip(ta, tb)):
        for u, v in zip(x, y):
            assert torch.equal(u, v), k


@pytest.mark.parametrize("n_lanes", [2, 3])
def test_lanes_play_the_same_games(n_lanes):
    """rvz.LaneRunner (independent lanes on forked streams, captured into one HIP graph; 3 lanes
    of 86 / 85 / 85 games) plays exactly the games of one SelfPlayRunner over the same global
    game indices: moves, policy vectors and boards bit-identical ply by ply, autoreset
    included."""
    import rvz
    G, plies, sims = 256, 64, 200
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 2, 64).cuda().eval()

    def make_eng(n):
        return rvz.Engine(n, num_simulations=sims, batch_size=64)

    one = rvz.SelfPlayRunner(make_eng(G), rvz.LeafEvaluator(net), autoreset=True, seed_base=11)
    two = rvz.LaneRunner(make_eng, lambda: rvz.LeafEvaluator(net), G, lanes=n_lanes,
                         autoreset=True, seed_base=11)
    one.start()
    two.start()
    for k in range(plies):
        for r in (one, two):
            r.ply()
            if k == 0:
                r.capture()         # first ply eager, the rest replayed from the graph
        rs = two.runners
        assert torch.equal(one.eng.idx_buf, torch.cat([r.eng.idx_buf for r in rs])), k
        assert torch.equal(one.eng.p_buf, torch.cat([r.eng.p_buf for r in rs])), k
        b1 = one.eng.get_state()[0].clone()
        b2 = torch.cat([r.eng.get_state()[0] for r in rs])
        assert torch.equal(b1, b2), k
    assert int(one.steps.item()) == int(two.steps.item())
    assert int(one.games_done.item()) == int(two.games_done.item()) > 0


def test_fused_bookkeeping_matches_torch_path():
    """rvz_env_autoreset (ply counting + restart of finished games with their slot's next seed,
    one kernel) against the torch form (restart_finished + rvz_env_reset): the same games,
    seeds, boards and counters, over enough plies that many games end and restart."""
    import rvz
    G, plies, sims = 128, 75, 128     # 2 batches: at 64 the root's children stay unvisited
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 1, 64).cuda().eval()
    runs = []
    for fused in (True, False):
        eng = rvz.Engine(G, num_simulations=sims, batch_size=64)
        run = rvz.SelfPlayRunner(eng, rvz.LeafEvaluator(net), autoreset=True, seed_base=3,
                                 seed_stride=1000, fused_bookkeeping=fused)
        run.start()
        trace = []
        for _ in range(plies):
            run.ply()
            b, w, st = eng.get_state()
            trace.append((eng.idx_buf.clone(), b.clone(), w.clone(), st.clone(),
                          run.seeds.clone()))
        runs.append((trace, int(run.steps.item()), int(run.games_done.item())))
    (ta, sa, da), (tb, sb, db) = runs
    assert sa == sb and da == db and da >= G
    for k, (x, y) in enumerate(zip(ta, tb)):
        for u, v in zip(x, y):
            assert torch.equal(u, v), k


@pytest.mark.parametrize("board,live_aware,skip", [(8, True, False), (8, False, False),
                                                   (6, True, False), (8, True, True)],
                         ids=["8x8-n_live", "8x8-all_rows", "6x6-n_live", "8x8-n_live-skip"])
def test_compacted_leaves_play_the_same_games(board, live_aware, skip):
    """rvz_search_compact: the leaves that need an evaluation go to rows [0, U) of leaf_x and the
    h2 evaluator evaluates only those (mcts.py:544-623 evaluates the U live leaves); an evaluator
    that ignores the count evaluates every row. Either way the moves, p and boards equal the
    uncompacted run's over whole games (the endgame's terminal traversals leave rows dead), and
    the live-row total is what the need vectors say."""
    import rvz
    G, plies, sims = (96, 66, 128) if board == 8 else (300, 40, 128)
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(board, 1, 64).cuda().eval()
    runs, rows = [], None
    for compact in (False, True):
        eng = rvz.Engine(G, num_simulations=sims, batch_size=64, board_size=board,
                         compact_leaves=compact)
        ev = rvz.LeafEvaluator(net)
        live_counts = []

        def evaluator(x, n_live=None, ev=ev, eng=eng, live_counts=live_counts):
            live_counts.append(int((eng.need > 0).sum()))
            return ev(x, n_live=n_live)
        evaluator.accepts_live_count = live_aware
        run = rvz.SelfPlayRunner(eng, evaluator, autoreset=True, seed_base=11,
                                 seed_stride=1000, skip_last_eval=skip)
        run.start()
        trace = []
        for _ in range(plies):
            run.ply()
            b, w, st = eng.get_state()
            trace.append((eng.idx_buf.clone(), eng.p_buf.clone(), b.clone(), w.clone(),
                          st.clone()))
        runs.append((trace, int(run.games_done.item())))
        if compact:
            rows = (eng.rows_total(), sum(live_counts))
    (ta, da), (tb, db) = runs
    assert da == db and da >= G
    for k, (x, y) in enumerate(zip(ta, tb)):
        for u, v in zip(x, y):
            assert torch.equal(u, v), k
    # rows_total counts the evaluated rows: a skipped last batch's rows are not among them
    assert rows[0] == rows[1] and rows[0] < G * plies * 2


def test_free_running_lanes_play_the_same_games():
    """LaneRunner.capture(free_run=True): one graph per lane on its own stream, no per-ply join;
    after join() the boards, moves and counters equal the single-runner games."""
    import rvz
    G, plies, sims = 128, 12, 128
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 1, 64).cuda().eval()
    one = rvz.SelfPlayRunner(rvz.Engine(G, sims, 64, compact_leaves=True),
                             rvz.LeafEvaluator(net), autoreset=True, seed_base=5)
    lanes = rvz.LaneRunner(lambda n: rvz.Engine(n, sims, 64, compact_leaves=True),
                           lambda: rvz.LeafEvaluator(net), G, 2, autoreset=True, seed_base=5)
    one.start()
    lanes.start()
    one.ply()
    lanes.ply()
    one.capture()
    lanes.capture(free_run=True)
    for _ in range(plies):
        one.ply()
        lanes.ply()
    assert int(lanes.steps.item()) == int(one.steps.item())
    b1, w1, s1 = one.eng.get_state()
    parts = [r.eng.get_state() for r in lanes.runners]
    assert torch.equal(torch.cat([p[0] for p in parts]), b1)
    assert torch.equal(torch.cat([p[1] for p in parts]), w1)
    assert torch.equal(torch.cat([p[2] for p in parts]), s1)


def test_compact_api_errors():
    """rvz_search_compact / rvz_search_live_count / the _ex stamp arguments fail loudly on misuse
    (include/rvz.h): no live count before a batch or with compaction off, no toggling inside a
    search, a stamp ring counter without a ring."""
    import ctypes as C
    import rvz
    from rvz import _lib
    lib = _lib.load()
    eng = rvz.Engine(8, 128, 64)
    with pytest.raises(rvz.RvzError):
        eng.live_count()                                  # compaction off
    eng.compact(True)
    with pytest.raises(rvz.RvzError):
        eng.live_count()                                  # no batch issued yet
    eng.reset(list(range(8)))
    eng.search_begin()
    assert eng.search_step()
    assert eng.live_count() != 0
    with pytest.raises(rvz.RvzError):
        eng.compact(False)                                # inside a search
    torch.manual_seed(0)
    ev = rvz.LeafEvaluator(rvz.AlphaZeroNetwork(8, 1, 64).cuda().eval())
    logits, value = ev(eng.leaf_x, n_live=eng.live_count())
    eng.search_submit(logits, value, True)
    while eng.search_step():
        logits, value = ev(eng.leaf_x, n_live=eng.live_count())
        eng.search_submit(logits, value, True)
    eng.act(1.0, apply=True)
    eng.check()
    assert eng.rows_total() == 8 * 2                      # 2 batches, every game live
    x = torch.zeros(8, 3, 8, 8, device="cuda")
    work = torch.zeros(lib.rvz_resnet_work_size(8), device="cuda")
    ctr = torch.zeros(1, dtype=torch.int32, device="cuda")
    rc = lib.rvz_resnet_trunk_h2_ex(8, x.data_ptr(), 8, ev.params.data_ptr(),
                                    ev.wsplit.data_ptr(), 64, 1, work.data_ptr(), None, None,
                                    ctr.data_ptr(), 4, _lib.stream_handle())
    assert rc == -22                                      # RVZ_EINVAL: counter without a ring


@pytest.mark.parametrize("n_lanes,memo,skip", [(3, False, False), (2, True, True)])
def test_bench_configuration_at_full_size_plays_the_plain_games(n_lanes, memo, skip):
    """The bench's C2 configuration at full size (4,096 games x 800 sims, 6x64 net; free-running
    lane graphs of games split in order (3 lanes: 1,366 / 1,365 / 1,365), compacted leaf batches;
    the headline's form: 2 lanes, the NN-output memo and the last batch left to the memo) against
    the plain path (one runner, every row evaluated, no memo, every batch evaluated, eager) over a
    whole game and its restarts: every ply's moves and the final boards, statuses and ply counters
    are identical."""
    import rvz
    G, S, plies = 4096, 800, 64
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
    lanes = rvz.LaneRunner(lambda n: rvz.Engine(n, S, 64, compact_leaves=True, memo=memo),
                           lambda: rvz.LeafEvaluator(net), G, n_lanes, autoreset=True,
                           seed_base=42, skip_last_eval=skip)
    plain = rvz.SelfPlayRunner(rvz.Engine(G, S, 64), rvz.LeafEvaluator(net), autoreset=True,
                               seed_base=42)
    lanes.start()
    plain.start()
    lanes.ply()
    plain.ply()
    lanes.capture(free_run=True)
    moves_l, moves_p = [], []
    for _ in range(plies - 1):
        lanes.ply()
        plain.ply()
        lanes.join()
        moves_l.append(torch.cat([r.eng.idx_buf for r in lanes.runners]).clone())
        moves_p.append(plain.eng.idx_buf.clone())
    assert int(lanes.steps.item()) == int(plain.steps.item())
    assert int(lanes.games_done.item()) == int(plain.games_done.item()) > 0
    for k, (a, b) in enumerate(zip(moves_l, moves_p)):
        assert torch.equal(a, b), k
    parts = [r.eng.get_state() for r in lanes.runners]
    b, w, st = plain.eng.get_state()
    assert torch.equal(torch.cat([p[0] for p in parts]), b)
    assert torch.equal(torch.cat([p[1] for p in parts]), w)
    assert torch.equal(torch.cat([p[2] for p in parts]), st)


@pytest.mark.parametrize("T", [0.7, 0.3, 1.5, 0.25, 3.0, 0.9])
def test_act_general_temperature_correctly_rounded(oracle, T):
    """k_act's `p ** (1/T)` for T outside NumPy's fast paths is the correctly rounded power
    (csrc/rvz_pow.hip.h): on the visit vectors of real searches (3 plies x 512 games, 200 sims,
    random policies) its f64 policy vectors equal, bitwise, NumPy's own normalisation of the
    correctly rounded powers (host pow_cr, itself checked against 60-digit decimal arithmetic in
    test_oracle_search.py), and its sampled index is np.random.choice's for that vector and u.
    The oracle (glibc pow, NumPy's non-AVX512 result) agrees on all but the vectors holding one
    of glibc's misrounded entries (0.52-ulp bound; counted, < 10% of vectors)."""
    import alt_eval
    import rvz
    G = 512
    eng = rvz.Engine(G, num_simulations=200, batch_size=64)
    eng.reset(list(range(G)))
    gen = torch.Generator(device="cuda").manual_seed(3)
    lib = alt_eval.load()
    glibc_diff, total = 0, 0
    for k in range(3):
        eng.search_begin()
        while eng.search_step():
            pr = torch.rand(G, 65, device="cuda", generator=gen) ** 4
            eng.search_submit((pr / pr.sum(1, keepdim=True)).contiguous(),
                              (torch.rand(G, device="cuda", generator=gen) * 2 - 1).contiguous(),
                              is_logits=False)
        vis = eng.visits().cpu().numpy()
        u = torch.rand(G, dtype=torch.float64, generator=torch.Generator().manual_seed(k))
        idx, p = eng.act(T, u=u, apply=False)
        idx, p = idx.cpu().numpy(), p.cpu().numpy()
        for g in range(G):
            q = vis[g] / vis[g].sum()
            e = np.full(q.shape, 1.0 / T)
            t = np.empty_like(q)
            assert lib.rvz_alt_pow_host(q.size, q.ctypes.data, e.ctypes.data, t.ctypes.data) == 0
            want = t / np.sum(t)
            assert np.array_equal(p[g].view(np.int64), want.view(np.int64)), (k, g)
            cdf = want.cumsum()
            cdf /= cdf[-1]
            assert idx[g] == np.searchsorted(cdf, float(u[g]), side="right"), (k, g)
            _, op, _ = oracle.action(vis[g], T, float(u[g]))
            glibc_diff += int(not np.array_equal(op, want))
            total += 1
        eng.act(1.0, apply=True)
    eng.check()
    print(f"T={T}: oracle (glibc pow) differs in {glibc_diff}/{total} vectors")
    assert glibc_diff <= total // 10
