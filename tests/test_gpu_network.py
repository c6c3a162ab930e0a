"""The leaf evaluator on the GPU: the fused conv epilogue (rvz_nn_bias_act) against PyTorch ops,
and the whole evaluator against the reference-shaped module (fp32 tolerance; bf16 looser)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("relu", [False, True])
def test_bias_act_f32_bit_exact(res, relu):
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
    _lib.check(_lib.load().rvz_nn_bias_act_f32(y.data_ptr(), b.data_ptr(),
                                              r.data_ptr() if res else None, 1000 * 64, 64,
                                              int(relu), _lib.stream_handle()), None, "bias_act")
    assert torch.equal(y, ref)


def test_bias_act_bf16_close():
    from rvz import _lib
    cl = torch.channels_last
    x = torch.randn(512, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    r = torch.randn(512, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    b = torch.randn(64, device="cuda")
    ref = F.relu(x.float() + b.view(1, -1, 1, 1) + r.float()).to(torch.bfloat16)
    y = x.clone(memory_format=cl)
    _lib.check(_lib.load().rvz_nn_bias_act_bf16(y.data_ptr(), b.data_ptr(), r.data_ptr(),
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
    for fused, kern in ((True, "miopen"), (False, "miopen"), (True, "auto")):
        ev = rvz.LeafEvaluator(net, fused_epilogue=fused, kernel=kern)
        l, v = ev(x)
        # fp32 throughout; only the summation order differs (BN folding, NHWC igemm vs NCHW)
        assert (l - lr).abs().max().item() <= 2e-5 * scale
        assert (v - vr).abs().max().item() <= 2e-3   # tanh of large random-init activations
        pr = torch.softmax(lr, 1)
        assert (torch.softmax(l, 1) - pr).abs().max().item() <= 1e-4
    evb = rvz.LeafEvaluator(net, dtype=torch.bfloat16)     # throughput mode, not parity grade
    lb, vb = evb(x)
    # bf16 activations: ~3 significant digits on logits of a deep random-init net
    assert (lb - lr).abs().max().item() <= 0.05 * scale
    assert (lb.argmax(1) == lr.argmax(1)).float().mean().item() > 0.8
    assert (vb - vr).abs().mean().item() < 0.1      # tanh saturates: a few signs flip


def _bn_net(blocks, filters, seed=3):
    import rvz
    torch.manual_seed(seed)
    net = rvz.AlphaZeroNetwork(8, blocks, filters).cuda().eval()
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
    ev = rvz.LeafEvaluator(net)
    assert ev.kernel == "split"
    l, v = ev(x)
    torch.cuda.synchronize()
    assert l.shape == (n, 37)
    scale = lr.abs().max().item()
    assert (l - lr).abs().max().item() <= 2e-5 * scale
    assert (v - vr).abs().max().item() <= 2e-3


@pytest.mark.parametrize("kernel", ["resnet", "split"])
@pytest.mark.parametrize("blocks,filters,n", [(6, 64, 4096), (10, 128, 515), (1, 64, 3), (0, 128, 2)])
def test_resnet_kernel_matches_module(kernel, blocks, filters, n):
    """rvz_resnet_fwd_f32 (f32 MFMA) and rvz_resnet_fwd_split (fp32 split over bf16 MFMA), whole
    forward, vs the nn.Module (fp32): fp32-class arithmetic, different summation order; odd batch
    sizes cover the partial last workgroup."""
    import rvz
    net = _bn_net(blocks, filters)
    x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
    with torch.no_grad():
        lr, vr = net(x)
    ev = rvz.LeafEvaluator(net, kernel=kernel)
    assert ev.use_resnet and ev.kernel == kernel
    l, v = ev(x)
    torch.cuda.synchronize()
    scale = lr.abs().max().item()
    assert (l - lr).abs().max().item() <= 2e-5 * scale
    assert (v - vr).abs().max().item() <= 2e-3


@pytest.mark.parametrize("blocks,filters,n", [(6, 64, 512), (10, 128, 128)])
def test_split_error_is_fp32_class(blocks, filters, n):
    """Error against an fp64 evaluation of the same module: the split kernel's must be of the
    order of the fp32 paths' (f32 MFMA kernel, PyTorch fp32) — not bf16's (~1e-3 relative)."""
    import rvz
    net = _bn_net(blocks, filters, seed=5)
    x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
    with torch.no_grad():
        l64, v64 = net.double().cpu()(x.double().cpu())
        net.float().cuda()
        lm, vm = net(x)
    err = {}
    for kern in ("resnet", "split"):
        l, v = rvz.LeafEvaluator(net, kernel=kern)(x)
        err[kern] = (l.double().cpu() - l64).abs().max().item()
    err["module"] = (lm.double().cpu() - l64).abs().max().item()
    scale = l64.abs().max().item()
    fp32 = max(err["resnet"], err["module"])
    assert err["split"] <= 4 * fp32 + 1e-7 * scale, (err, scale)
    assert err["split"] <= 1e-5 * scale, (err, scale)


@pytest.mark.parametrize("kernel", ["split", "resnet", "miopen"])
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
    ev = rvz.LeafEvaluator(net, kernel=kernel)
    logits, v = ev(torch.from_numpy(x).cuda())
    p = torch.softmax(logits, 1).cpu().numpy()
    dp = np.abs(p - probs).max()
    dv = np.abs(v.cpu().numpy() - value).max()
    assert dp <= 2e-5 and dv <= 5e-4, (dp, dv)
    assert (p.argmax(1) == probs.argmax(1)).mean() > 0.99
