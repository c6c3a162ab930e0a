"""The leaf evaluator on the GPU: the fused conv epilogue (rvz_nn_bias_act) against PyTorch ops,
and the whole evaluator against the reference-shaped module (fp32 tolerance; bf16 looser)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from evaluators import make_evaluator  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("relu", [False, True])
def test_bias_act_f32_bit_exact(res, relu):
    import alt_eval
    from rvz import _lib
    cl = torch.channels_last
    torch.manual_seed(1)
    x = torch.randn(1000, 64, 8, 8, device="cuda").contiguous(memory_format=cl)
    b = torch.randn(64, device="cuda")
    r = torch.randn(1000, 64, 8, 8, device="cuda").contiguous(memory_format=cl) if res else None
    ref = x + b.view(1, -1, 1, 1)
    if res:
        ref = ref + r
    if relu:
        ref = F.relu(ref)
    y = x.clone(memory_format=cl)
    _lib.check(alt_eval.load().rvz_nn_bias_act_f32(y.data_ptr(), b.data_ptr(),
                                              r.data_ptr() if res else None, 1000 * 64, 64,
                                              int(relu), _lib.stream_handle()), None, "bias_act")
    assert torch.equal(y, ref)


def test_bias_act_bf16_close():
    import alt_eval
    from rvz import _lib
    cl = torch.channels_last
    x = torch.randn(512, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    r = torch.randn(512, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    b = torch.randn(64, device="cuda")
    ref = F.relu(x.float() + b.view(1, -1, 1, 1) + r.float()).to(torch.bfloat16)
    y = x.clone(memory_format=cl)
    _lib.check(alt_eval.load().rvz_nn_bias_act_bf16(y.data_ptr(), b.data_ptr(), r.data_ptr(),
                                               512 * 64, 64, 1, _lib.stream_handle()), None, "b")
    assert (y.float() - ref.float()).abs().max().item() <= 2 ** -7 * ref.float().abs().max().item()


@pytest.mark.parametrize("blocks,filters", [(6, 64), (2, 32)])
def test_evaluator_fp32_matches_module(blocks, filters):
    import rvz
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, blocks, filters).cuda().eval()
    with torch.no_grad():   # non-trivial BN statistics
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    x = (torch.rand(2048, 3, 8, 8, device="cuda") > 0.6).float()
    with torch.no_grad():
        lr, vr = net(x)
    scale = lr.abs().max().item()
    kinds = ((True, "miopen"), (False, "miopen")) + (((True, "h2"),) if filters in (64, 128) else ())
    for fused, kern in kinds:
        ev = make_evaluator(net, kern, fused_epilogue=fused)
        l, v = ev(x)
        # fp32 throughout; only the summation order differs (BN folding, NHWC igemm vs NCHW)
        assert (l - lr).abs().max().item() <= 2e-5 * scale
        assert (v - vr).abs().max().item() <= 2e-3   # tanh of large random-init activations
        pr = torch.softmax(lr, 1)
        assert (torch.softmax(l, 1) - pr).abs().max().item() <= 1e-4
    evb = make_evaluator(net, "miopen", dtype=torch.bfloat16)     # throughput mode, not parity grade
    lb, vb = evb(x)
    # bf16 activations: ~3 significant digits on logits of a deep random-init net
    assert (lb - lr).abs().max().item() <= 0.05 * scale
    assert (lb.argmax(1) == lr.argmax(1)).float().mean().item() > 0.8
    assert (vb - vr).abs().mean().item() < 0.1      # tanh saturates: a few signs flip


def _bn_net(blocks, filters, seed=3, board=8):
    import rvz
    torch.manual_seed(seed)
    net = rvz.AlphaZeroNetwork(board, blocks, filters).cuda().eval()
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.1, 0.1)
    return net


@pytest.mark.parametrize("blocks,filters,n", [(6, 64, 1000), (2, 128, 33), (0, 64, 1)])
def test_split_kernel_6x6_matches_module(blocks, filters, n):
    """The split kernel on the 6x6 variant (config 5): the board sits in the top-left corner of
    the 8x8 pixel grid, taps past row/column 5 read zero, the heads see the 36 cells."""
    import rvz
    torch.manual_seed(4)
    net = rvz.AlphaZeroNetwork(6, blocks, filters).cuda().eval()
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    x = (torch.rand(n, 3, 6, 6, device="cuda") > 0.6).float()
    with torch.no_grad():
        lr, vr = net(x)
    assert rvz.LeafEvaluator(net).kernel == "h2"
    for kern in ("h2", "split"):
        l, v = make_evaluator(net, kern)(x)
        torch.cuda.synchronize()
        assert l.shape == (n, 37)
        scale = lr.abs().max().item()
        assert (l - lr).abs().max().item() <= 2e-5 * scale, kern
        assert (v - vr).abs().max().item() <= 2e-3, kern


@pytest.mark.parametrize("kernel", ["resnet", "split", "h2"])
@pytest.mark.parametrize("blocks,filters,n", [(6, 64, 4096), (10, 128, 515), (5, 128, 257), (1, 64, 3),
                                              (0, 128, 2)])
def test_resnet_kernel_matches_module(kernel, blocks, filters, n):
    """rvz_resnet_fwd_f32 (f32 MFMA), rvz_resnet_fwd_split (fp32 as 3 bf16 parts) and
    rvz_resnet_fwd_h2 (fp32 as 2 f16 parts), whole forward, vs the nn.Module (fp32): fp32-class
    arithmetic, different summation order; odd batch sizes cover the partial last workgroup."""
    import rvz
    net = _bn_net(blocks, filters)
    x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
    with torch.no_grad():
        lr, vr = net(x)
    ev = make_evaluator(net, kernel)
    assert ev.kernel == kernel
    l, v = ev(x)
    torch.cuda.synchronize()
    scale = lr.abs().max().item()
    assert (l - lr).abs().max().item() <= 2e-5 * scale
    assert (v - vr).abs().max().item() <= 2e-3


@pytest.mark.parametrize("blocks,filters,n", [(6, 64, 512), (10, 128, 128), (5, 128, 128)])
def test_split_error_is_fp32_class(blocks, filters, n):
    """Error against an fp64 evaluation of the same module: the split kernels' (3 bf16 parts, 2
    f16 parts) must be of the order of the fp32 paths' (f32 MFMA kernel, PyTorch fp32) — not
    bf16's (~1e-3 relative). tools/emu_split.py predicts h2 at 0.8-1.5x plain fp32."""
    import rvz
    net = _bn_net(blocks, filters, seed=5)
    x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
    with torch.no_grad():
        l64, v64 = net.double().cpu()(x.double().cpu())
        net.float().cuda()
        lm, vm = net(x)
    err = {}
    for kern in ("resnet", "split", "h2"):
        l, v = make_evaluator(net, kern)(x)
        err[kern] = (l.double().cpu() - l64).abs().max().item()
    err["module"] = (lm.double().cpu() - l64).abs().max().item()
    scale = l64.abs().max().item()
    fp32 = max(err["resnet"], err["module"])
    for kern in ("split", "h2"):
        assert err[kern] <= 4 * fp32 + 1e-7 * scale, (kern, err, scale)
        assert err[kern] <= 1e-5 * scale, (kern, err, scale)


@pytest.mark.parametrize("kernel", ["h2", "split", "resnet", "miopen"])
def test_evaluator_matches_reference_outputs(kernel):
    """Every NN call of the reference's S=800 6x64 self-play fixture (1,499 leaf positions):
    the GPU evaluator's softmax rows and values against the reference's own recorded outputs
    (CPU fp32 PyTorch). The net is the fixture's (seed 0, pinned bit-exactly on CPU by
    test_network_cpu.py). Tolerance: fp32 evaluation-order differences; measured max |dp| / |dv|:
    split 3.6e-6 / 8.8e-5, f32 MFMA 7.3e-6 / 1.2e-4, MIOpen 7.0e-6 / 1.8e-4 (the value head of
    a random-init 6x64 net amplifies rounding: its pre-tanh sums cancel heavily)."""
    import os
    import rvz
    from test_network_cpu import fixture_planes
    x, probs, value = fixture_planes(os.path.join(os.path.dirname(__file__), "golden",
                                                  "mcts_s800_6x64.npz"))
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
    ev = make_evaluator(net, kernel)
    logits, v = ev(torch.from_numpy(x).cuda())
    p = torch.softmax(logits, 1).cpu().numpy()
    dp = np.abs(p - probs).max()
    dv = np.abs(v.cpu().numpy() - value).max()
    assert dp <= 2e-5 and dv <= 5e-4, (dp, dv)
    assert (p.argmax(1) == probs.argmax(1)).mean() > 0.99


def _fp64_outputs(net, x):
    """The reference module's forward in fp64 on the CPU (ground truth for the range tests)."""
    import copy
    m = copy.deepcopy(net).double().cpu().eval()
    with torch.no_grad():
        lo, v = m(x.double().cpu())
    return lo, v.reshape(-1)


def _fp32_module_err(net, x, l64, v64):
    with torch.no_grad():
        lo, v = net(x)
    return ((lo.double().cpu() - l64).abs().max().item(),
            (v.reshape(-1).double().cpu() - v64).abs().max().item())


@pytest.mark.parametrize("where", ["stem_bias", "tower_weights"])
def test_h2_activation_range_is_scaled_not_overflowed(where):
    """h2 keeps activations as two f16 parts, which overflow at 65520. A pass
    whose unscaled trunk overflowed re-runs the boards that did with each board's activation
    image stored scaled by a power of two chosen from a bound on the layer's outputs (h2_pass,
    csrc/rvz_h2.hip.h), so a net whose activations reach ~1e5-1e7 evaluates fp32-class instead
    of raising: the stem bias at 1e5 (round 4's overflow case), or the tower's conv weights
    scaled up so that activations grow block after block."""
    import rvz
    net = _bn_net(2, 64, seed=6)
    x = (torch.rand(256, 3, 8, 8, device="cuda") > 0.6).float()
    with torch.no_grad():
        if where == "stem_bias":
            net.bn.bias.fill_(1e5)            # stem output ~1e5 > the f16 range
        else:
            for blk in net.res_blocks:
                blk.conv1.weight.mul_(12.0)
                blk.conv2.weight.mul_(12.0)
    l64, v64 = _fp64_outputs(net, x)
    ev = rvz.LeafEvaluator(net, kernel="h2")
    lo, v = ev(x)
    assert not ev.overflowed()
    scale = l64.abs().max().item()
    assert scale > 1e4                        # the activations are past f16's range
    e32, ev32 = _fp32_module_err(net, x, l64, v64)
    err = (lo.double().cpu() - l64).abs().max().item()
    verr = (v.double().cpu() - v64).abs().max().item()
    assert err <= 4 * e32 + 1e-6 * scale, (err, e32, scale)
    assert verr <= 4 * ev32 + 1e-6, (verr, ev32)


def test_h2_activation_range_leaves_ordinary_nets_bitwise():
    """Ordinary nets never overflow, so nothing is re-run or scaled: the outputs are those of the
    unscaled arithmetic, which the fixture and fp32-class tests pin; here: the blob's range
    table (the re-run's bounds) holds K = max over channels of sum |w| and Bb = max |bias| of
    every layer (BN folded), and a row's outputs do not depend on its pass partner."""
    import rvz
    from rvz.network import pack_resnet_params  # noqa: F401
    net = _bn_net(2, 64, seed=3)
    ev = rvz.LeafEvaluator(net, kernel="h2")
    blob = ev.wsplit.cpu().numpy().view(np.uint16)
    F, NB = 64, 2
    n_el = blob.size
    nl = 1 + 2 * NB
    rng = blob[n_el - ((4 * nl + 7) // 8 * 8):][:4 * nl].view(np.float32).reshape(nl, 2)
    folded = []
    with torch.no_grad():
        def fold(conv, bn):
            s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
            w = conv.weight * s.view(-1, 1, 1, 1)
            b = bn.bias - bn.running_mean * s + (conv.bias * s if conv.bias is not None else 0)
            return w.double().cpu(), b.double().cpu()
        folded.append(fold(net.conv, net.bn))
        for blk in net.res_blocks:
            folded.append(fold(blk.conv1, blk.bn1))
            folded.append(fold(blk.conv2, blk.bn2))
    for i, (w, b) in enumerate(folded):
        k = w.abs().reshape(w.shape[0], -1).sum(1).max().item()
        assert abs(rng[i, 0] - k) <= 1e-5 * k, (i, rng[i], k)
        assert abs(rng[i, 1] - b.abs().max().item()) <= 1e-6 * max(1.0, b.abs().max().item())
    assert rng[:, 0].max() * 2 + rng[:, 1].max() < 2 ** 15
    x = (torch.rand(64, 3, 8, 8, device="cuda") > 0.6).float()
    lo, v = (t.clone() for t in ev(x))             # (the evaluator reuses its output buffers)
    lo2, v2 = ev(x.flip(0).contiguous())
    assert torch.equal(lo, lo2.flip(0)) and torch.equal(v, v2.flip(0))


def test_h2_weight_blob():
    """rvz_resnet_h2_weights: every fragment element is the f16 split of the scaled weight
    (w * 2^s == h0 + h1 up to 2^-22 relative), max |w| of each channel scaled into [2^14, 2^15),
    inverse scales exact powers of two."""
    import rvz
    net = _bn_net(1, 64, seed=7)
    ev = rvz.LeafEvaluator(net, kernel="h2")
    blob = ev.wsplit.cpu().numpy().view(np.uint16)
    F, NB, K, TM = 64, 1, 32, 16
    layer = 9 * F * F * 2
    pad_ksteps = 4                       # h2_pad_ksteps: the weight prefetch past the last layer
    stem_off = 2 * NB * layer + pad_ksteps * 2 * F * K
    assert not blob[2 * NB * layer:stem_off].any()
    sc_off = stem_off + 2 * F * K
    isc = blob[sc_off:sc_off + 2 * (1 + 2 * NB) * F].view(np.float32).reshape(1 + 2 * NB, F)
    assert np.all(np.log2(isc) == np.round(np.log2(isc)))
    prm = ev.params.cpu().numpy()
    from rvz.network import _fold
    w1, _ = _fold(net.res_blocks[0].conv1, net.res_blocks[0].bn1)
    w1 = w1.cpu().numpy()                                     # [n][k][3][3]
    frag = blob[:layer].view(np.float16).reshape(9, F // K, 2, F // TM, 64, 8).astype(np.float64)
    # rebuild w[t][n][k] from the fragments: lane = ((k % K) / 8) * TM + n % TM
    t, n, k = np.meshgrid(np.arange(9), np.arange(F), np.arange(F), indexing="ij")
    ln = ((k % K) // 8) * TM + n % TM
    h = frag[t, k // K, :, n // TM, ln, k % 8]                # [..., part]
    rebuilt = (h[..., 0] + h[..., 1]) * isc[1][n]
    ref = w1.transpose(2, 3, 0, 1).reshape(9, F, F).astype(np.float64)
    assert np.abs(rebuilt - ref).max() <= 2 ** -21 * np.abs(ref).max()
    scaled_max = np.abs(ref).reshape(9, F, F).max(axis=(0, 2)) / isc[1]
    assert np.all((scaled_max >= 2 ** 14) & (scaled_max < 2 ** 15))
    assert prm.dtype == np.float32


def test_h2_timing_forms_are_bit_identical():
    """bench.py's instrumented forms of the h2 evaluator (trunk with per-workgroup wall-clock
    stamps; fence-less event pair around the trunk) produce the same bits as the plain
    rvz_resnet_fwd_h2, and the stamps are ordered (start <= end, nonzero)."""
    import rvz
    from rvz import _lib
    net = _bn_net(2, 64, seed=8)
    x = (torch.rand(96, 3, 8, 8, device="cuda") > 0.6).float()
    ev = rvz.LeafEvaluator(net, kernel="h2")
    l0, v0 = (t.clone() for t in ev(x))
    grid = _lib.load().rvz_resnet_h2_grid(8, 64, 96)
    assert grid > 0
    stamps = torch.zeros(2, grid, 2, dtype=torch.int64, device="cuda")
    ctr = torch.zeros(1, dtype=torch.int32, device="cuda")
    ev.trunk_stamps = (stamps, ctr)
    l1, v1 = (t.clone() for t in ev(x))
    ev.trunk_stamps = None
    assert int(ctr.item()) == 1                      # the heads launch advanced the ring
    ev.trunk_events = (_lib.Timer(2), [])
    l2, v2 = (t.clone() for t in ev(x))
    tm, pairs = ev.trunk_events
    ev.trunk_events = None
    torch.cuda.synchronize()
    assert torch.equal(l0, l1) and torch.equal(v0, v1)
    assert torch.equal(l0, l2) and torch.equal(v0, v2)
    s = stamps[0].cpu()
    end = s[:, 1] & ((1 << 52) - 1)
    assert bool((((s[:, 1] >> 52) & 0xF) < 8).all())      # the XCD id field
    assert bool((s > 0).all()) and bool((end >= s[:, 0]).all())
    assert int((s[:, 1] >> 56).sum()) == 96          # evaluated boards, per workgroup
    assert bool((stamps[1] == 0).all())
    assert len(pairs) == 1 and 0.0 < tm.elapsed(*pairs[0]) < 1000.0


@pytest.mark.parametrize("board,filters,n,lives", [(8, 64, 96, [37]), (8, 64, 96, [0]),
                                                   (8, 64, 300, [37, 128, 5]),
                                                   (6, 64, 300, [41, 0, 44]),
                                                   (8, 128, 140, [17, 12]),
                                                   (8, 256, 140, [17, 12])])
def test_h2_live_rows(board, filters, n, lives):
    """rvz_resnet_fwd_h2_ex with n_live (per-stripe live counts, include/rvz.h RVZ_LIVE_STRIPE):
    the live rows of every stripe are bit-identical to the full evaluation, rows past the last
    16-row heads group holding a live row of their stripe are left untouched, and a row's result
    does not depend on its position in the batch (a permuted batch gives the permuted outputs),
    which is what makes compacted leaf batches exact."""
    import rvz
    from rvz import _lib
    lib = _lib.load()
    S, PITCH = 128, 16          # RVZ_LIVE_STRIPE, RVZ_LIVE_PITCH
    torch.manual_seed(board + filters)
    net = rvz.AlphaZeroNetwork(board, 1, filters).cuda().eval()
    ev = rvz.LeafEvaluator(net, kernel="h2")
    x = (torch.rand(n, 3, board, board, device="cuda") > 0.6).float()
    l0, v0 = (t.clone() for t in ev(x))
    perm = torch.randperm(n, device="cuda")
    lp, vp = ev(x[perm].contiguous())
    assert torch.equal(lp, l0[perm]) and torch.equal(vp, v0[perm])
    logits, value = ev(x)
    logits.fill_(float("nan"))
    value.fill_(float("nan"))
    cnt = torch.zeros(len(lives) * PITCH, dtype=torch.int32, device="cuda")
    cnt[::PITCH] = torch.tensor(lives, dtype=torch.int32)
    assert lib.rvz_resnet_fwd_h2_ex(board, x.data_ptr(), n, ev.params.data_ptr(),
                                    ev.wsplit.data_ptr(), filters, 1, ev._outs[n][2].data_ptr(),
                                    logits.data_ptr(), value.data_ptr(), cnt.data_ptr(),
                                    _lib.stream_handle()) == 0
    torch.cuda.synchronize()
    for s, live in enumerate(lives):
        a, e = s * S, min(n, (s + 1) * S)
        assert torch.equal(logits[a:a + live], l0[a:a + live]), s
        assert torch.equal(value[a:a + live], v0[a:a + live]), s
        tail = a + -(-live // 16) * 16
        assert bool(torch.isnan(logits[tail:e]).all()) and bool(torch.isnan(value[tail:e]).all())


@pytest.mark.parametrize("board,filters,n", [(8, 64, 300), (6, 64, 97), (8, 128, 37),
                                             (8, 256, 37)])
def test_h2_unit_counter_any_start(board, filters, n):
    """The trunk deals its board units to workgroups in start order from a 64-bit counter in the
    workspace (words n*192 + 2, 3; RVZ_H2_DYN), never reset: whatever the counter holds (below
    2^63), every unit is evaluated exactly once per launch, so the outputs are bit-identical to a fresh
    workspace's, launch after launch."""
    import rvz
    torch.manual_seed(board * filters + n)
    net = rvz.AlphaZeroNetwork(board, 2, filters).cuda().eval()
    ev = rvz.LeafEvaluator(net, kernel="h2")
    x = (torch.rand(n, 3, board, board, device="cuda") > 0.6).float()
    l0, v0 = (t.clone() for t in ev(x))
    work = ev._outs[n][2]
    ctr = work[n * 192 + 2:n * 192 + 4].view(torch.int64)
    for start in (1, 12345678901, 2 ** 62 + 7):
        ctr.fill_(start)
        for _ in range(3):
            lg, vl = ev(x)
            assert torch.equal(lg, l0) and torch.equal(vl, v0), start
    assert not ev.overflowed()


@pytest.mark.parametrize("board,blocks,filters", [(8, 2, 64), (6, 2, 64), (8, 1, 128),
                                                  (8, 1, 256)])
def test_h2_range_rerun_is_per_board(board, blocks, filters):
    """Passes that mix boards that overflow with boards that do not (every geometry: the 8x8
    pair, three packed 6x6 boards, one 8x8 board at F = 128). The stem's weights on input plane
    0 are scaled by 1e6, so a row overflows exactly when its plane 0 has a disc; half the rows
    have an empty plane 0. Only the overflowed boards are re-run scaled: a quiet row's outputs
    are bit for bit those of a batch of quiet rows only, a loud row's those of any other
    pairing (the table and memo need a row's outputs to depend on its position alone), and the
    loud rows are fp32-class against fp64."""
    import rvz
    net = _bn_net(blocks, filters, seed=9, board=board)
    with torch.no_grad():
        net.conv.weight[:, 0].mul_(1e6)
    n = 96
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.rand(n, 3, board, board, device="cuda", generator=g) > 0.6).float()
    loud = torch.arange(n, device="cuda") % 4 < 2                 # rows 0,1 4,5 ...: loud
    x[~loud, 0] = 0.0
    x[loud, 0, 0, 0] = 1.0                                        # at least one disc
    ev = rvz.LeafEvaluator(net, kernel="h2")
    lo, v = (t.clone() for t in ev(x))
    assert not ev.overflowed()
    q = torch.nonzero(~loud).flatten()
    lq, vq = (t.clone() for t in ev(x[q].contiguous()))
    assert torch.equal(lo[q], lq) and torch.equal(v[q], vq)
    perm = torch.randperm(n, device="cuda", generator=g)
    lp, vp = (t.clone() for t in ev(x[perm].contiguous()))
    inv = torch.argsort(perm)
    assert torch.equal(lp[inv], lo) and torch.equal(vp[inv], v)
    l64, v64 = _fp64_outputs(net, x)
    with torch.no_grad():                                         # the stems past f16's range
        stem = torch.relu(net.bn(net.conv(x))).amax(dim=(1, 2, 3))
    assert (stem[loud] > 65520).all() and (stem[~loud] < 100).all()
    e32, ev32 = _fp32_module_err(net, x, l64, v64)
    err = (lo.double().cpu() - l64).abs().max().item()
    verr = (v.double().cpu() - v64).abs().max().item()
    scale = l64.abs().max().item()
    assert err <= 4 * e32 + 1e-6 * scale, (err, e32, scale)
    assert verr <= 4 * ev32 + 1e-6, (verr, ev32)


@pytest.mark.parametrize("blocks,n", [(3, 200), (0, 5), (1, 1)])
def test_h2_f256_is_fp32_class(blocks, n):
    """The 8x8 trunk at 256 filters (k_resnet_h2<256, 1, 4, 4, 8, 1>: one board per workgroup,
    4 channel tiles per wave, the k-loop in chunks of 24 k-steps over ring slots): outputs
    fp32-class against an fp64 evaluation of the module — within 4x the PyTorch fp32 module's own
    error and 1e-5 of the logit scale — and a row's outputs independent of its batch."""
    import rvz
    net = _bn_net(blocks, 256, seed=11)
    ev = rvz.LeafEvaluator(net)
    assert ev.kernel == "h2" and rvz.network.h2_covers(net)
    x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
    lo, v = (t.clone() for t in ev(x))
    assert not ev.overflowed()
    l64, v64 = _fp64_outputs(net, x)
    e32, ev32 = _fp32_module_err(net, x, l64, v64)
    err = (lo.double().cpu() - l64).abs().max().item()
    verr = (v.double().cpu() - v64).abs().max().item()
    scale = l64.abs().max().item()
    assert err <= 4 * e32 + 1e-7 * scale, (err, e32, scale)
    assert err <= 1e-5 * scale, (err, scale)
    # the value (tanh of a 256-wide 1x1 conv -> fc1 -> fc2 chain whose pre-tanh sums cancel):
    # the maximum over a few rows of two independent rounding sequences is noisy (measured: 4.8e-5
    # vs the module's 1.1e-5 at 3 blocks), so its RMS over the rows is held to the module's and
    # its maximum to an absolute fp32-class bound
    with torch.no_grad():
        vm = net(x)[1].reshape(-1).double().cpu()
    rms = (v.double().cpu() - v64).pow(2).mean().sqrt().item()
    rms32 = (vm - v64).pow(2).mean().sqrt().item()
    assert rms <= 4 * rms32 + 1e-7, (rms, rms32, verr, ev32)
    assert verr <= 1e-4, (verr, ev32)
    perm = torch.randperm(n, device="cuda")
    lp, vp = ev(x[perm].contiguous())
    assert torch.equal(lp, lo[perm]) and torch.equal(vp, v[perm])


def test_h2_f256_is_8x8_only():
    """256 filters have an h2 instantiation on 8x8 only: a 6x6 net of that width is refused by
    the C-ABI and by LeafEvaluator, and the default evaluator falls back to ModuleEvaluator."""
    import rvz
    from rvz import _lib
    lib = _lib.load()
    assert lib.rvz_resnet_h2_grid(8, 256, 10) == 10 + 8      # one board per unit + spares
    assert lib.rvz_resnet_h2_grid(6, 256, 10) < 0
    net = rvz.AlphaZeroNetwork(6, 1, 256).cuda().eval()
    assert not rvz.network.h2_covers(net)
    with pytest.raises(_lib.RvzError):
        rvz.LeafEvaluator(net)
    with pytest.warns(UserWarning, match="ModuleEvaluator"):
        assert isinstance(rvz.network.leaf_evaluator(net), rvz.ModuleEvaluator)
