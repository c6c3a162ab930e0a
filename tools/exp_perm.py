#!/usr/bin/env python3
"""Is an h2 evaluation's row independent of its position in the batch? Evaluates x, x.flip(0)
and a random permutation for a few nets; prints the rows that differ (RVZ_LIB selects a
variant library)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402


def bn_net(blocks, filters, seed):
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


out = {"lib": os.environ.get("RVZ_LIB", "in-tree")}
for name, net in (("bn2x64", bn_net(2, 64, 3)), ("plain1x64", None), ("bn2x128", bn_net(2, 128, 3))):
    if net is None:
        torch.manual_seed(72)
        net = rvz.AlphaZeroNetwork(8, 1, 64).cuda().eval()
    ev = rvz.LeafEvaluator(net)
    torch.manual_seed(0)
    x = (torch.rand(64, 3, 8, 8, device="cuda") > 0.6).float()
    l0, v0 = (t.clone() for t in ev(x))
    lf, vf = (t.clone() for t in ev(x.flip(0).contiguous()))
    perm = torch.randperm(64, device="cuda")
    lp, vp = (t.clone() for t in ev(x[perm].contiguous()))
    dflip = ((lf.flip(0) != l0).any(1) | (vf.flip(0) != v0)).nonzero().flatten().tolist()
    dperm = ((lp != l0[perm]).any(1) | (vp != v0[perm])).nonzero().flatten().tolist()
    out[name] = {"flip_rows_differ": dflip, "perm_rows_differ": dperm,
                 "max_abs_diff_flip": (lf.flip(0) - l0).abs().max().item()}
print(json.dumps(out))
