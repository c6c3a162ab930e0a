"""Board kernels (rvz_board_legal / rvz_board_apply / rvz_board_canonical, rvz_env_*) against the
reference's golden vectors, bit-exact, plus the reference's own test_game.py through the drop-in
ReversiGame (its rules run in the kernels)."""
import numpy as np
import pytest
import torch

from test_oracle_board import load_vectors

pytestmark = pytest.mark.gpu


def _s64(a):
    return torch.from_numpy(np.asarray(a, np.uint64).view(np.int64).copy()).cuda()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.fixture(scope="module")
def vec():
    return load_vectors()


def _status(d, pre=""):
    cols = [d[k + pre] for k in ("side", "over", "winner", "passed")]
    return torch.from_numpy(np.stack(cols, 1).astype(np.int32)).cuda().contiguous()


def test_legal_bit_exact(vec):
    import rvz
    d = vec
    out = rvz.board_legal(_s64(d["black"]), _s64(d["white"]), _status(d))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u64(out), d["legal"])


def test_apply_bit_exact(vec):
    import rvz
    d = vec
    b, w, st = _s64(d["black"]), _s64(d["white"]), _status(d)
    ok = rvz.board_apply(b, w, st, torch.from_numpy(d["move"]).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ok.cpu().numpy(), d["ok"])
    np.testing.assert_array_equal(_u64(b), d["black_after"])
    np.testing.assert_array_equal(_u64(w), d["white_after"])
    post = st.cpu().numpy()
    for j, k in enumerate(("side", "over", "winner", "passed")):
        np.testing.assert_array_equal(post[:, j], d[k + "_after"])


def test_canonical_matches_oracle(vec, oracle):
    import rvz
    d = vec
    n = 2000
    planes = rvz.board_canonical(_s64(d["black"][:n]), _s64(d["white"][:n]),
                                 _status(d)[:n].contiguous()).cpu().numpy()
    for i in range(0, n, 7):
        g = oracle.Game()
        g.black, g.white, g.side = int(d["black"][i]), int(d["white"][i]), int(d["side"][i])
        np.testing.assert_array_equal(planes[i], oracle.canonical(g))


def test_engine_env_roundtrip_and_apply(vec):
    import rvz
    d = vec
    n = 4096
    eng = rvz.Engine(n, num_simulations=64, batch_size=64)
    eng.set_state(_s64(d["black"][:n]), _s64(d["white"][:n]), _status(d)[:n].contiguous())
    np.testing.assert_array_equal(_u64(eng.legal()), d["legal"][:n])
    ok = eng.apply(torch.from_numpy(d["move"][:n]).cuda())
    b, w, st = eng.get_state()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ok.cpu().numpy(), d["ok"][:n])
    np.testing.assert_array_equal(_u64(b), d["black_after"][:n])
    np.testing.assert_array_equal(st.cpu().numpy()[:, 0], d["side_after"][:n])
    eng.check()


def test_board_6x6_matches_oracle(oracle):
    """Build-defined 6x6 variant: kernels vs the oracle's restatement over random playouts."""
    import rvz
    rng = np.random.default_rng(5)
    states, moves = [], []
    for _ in range(200):
        g = oracle.new_game(6)
        while not g.over:
            P, Q = (g.black, g.white) if g.side == 1 else (g.white, g.black)
            m = oracle.legal(P, Q, 6)
            mv = [s for s in range(36) if m >> s & 1]
            sq = int(rng.choice(mv)) if rng.random() > 0.1 else int(rng.integers(-1, 40))
            states.append(g.copy())
            moves.append(sq)
            if oracle.make_move(g, sq, 6) is False:
                oracle.make_move(g, int(rng.choice(mv)), 6)
    b = _s64([s.black for s in states])
    w = _s64([s.white for s in states])
    st = torch.tensor([[s.side, s.over, s.winner, s.passed] for s in states], dtype=torch.int32).cuda()
    legal = _u64(rvz.board_legal(b, w, st, board_size=6))
    ok = rvz.board_apply(b, w, st, torch.tensor(moves, dtype=torch.int32).cuda(), board_size=6)
    bb, ww, ss, okk = _u64(b), _u64(w), st.cpu().numpy(), ok.cpu().numpy()
    for i, s in enumerate(states):
        P, Q = (s.black, s.white) if s.side == 1 else (s.white, s.black)
        assert int(legal[i]) == oracle.legal(P, Q, 6)
        g = s.copy()
        r = oracle.make_move(g, moves[i], 6)
        assert bool(okk[i]) == r
        assert (int(bb[i]), int(ww[i]), *map(int, ss[i])) == \
            (g.black, g.white, g.side, g.over, g.winner, g.passed)


# ---- the reference's test_game.py, through the drop-in ReversiGame (rules on the GPU)
def test_reference_test_game_initial_board():
    from rvz import ReversiGame
    game = ReversiGame()
    board = game.get_board_state()
    assert board.shape == (8, 8)
    assert board[3][3] == 2 and board[4][4] == 2 and board[3][4] == 1 and board[4][3] == 1
    assert np.sum(board == 0) == 60


def test_reference_test_game_valid_moves():
    from rvz import ReversiGame
    assert set(ReversiGame().get_valid_moves()) == {(2, 3), (3, 2), (4, 5), (5, 4)}


def test_reference_test_game_make_move():
    from rvz import ReversiGame
    game = ReversiGame()
    assert game.make_move(2, 3)
    board = game.get_board_state()
    assert board[2][3] == 1 and board[3][3] == 1
    assert game.get_current_player() == 2


def test_reference_test_game_game_over():
    from rvz import ReversiGame
    game = ReversiGame(8)
    game.board.black = 0x2
    game.board.white = 0
    for i in range(8):
        for j in range(8):
            if i > 0 or j > 1:
                pos = i * 8 + j
                if (i + j) % 2 == 0:
                    game.board.white |= (1 << pos)
                else:
                    game.board.black |= (1 << pos)
    game.board.black &= ~0x1
    game.board.white &= ~0x2
    game.board.black |= 0x2
    game.current_player = game.board.WHITE
    game.board._update_board_state()
    assert game.make_move(0, 0)
    assert game.is_game_over()
    assert game.get_winner() == game.board.WHITE


def test_dropin_error_behaviour():
    from rvz import ReversiGame
    g = ReversiGame()
    assert g.make_move(0, 0) is False          # illegal: False, no raise (board.py:178-179)
    assert g.make_move(8, 0) is False          # off-board square
    assert g.make_move(-1, -1) is False        # pass while moves exist (board.py:153-154)
    with pytest.raises(ValueError):
        g.make_move(-1, 3)                     # `1 << negative` raises in the reference
    canon = g.get_canonical_state()
    assert canon.shape == (3, 8, 8) and canon.dtype == np.float32
    assert canon[2].sum() == 4
