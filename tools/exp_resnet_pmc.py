"""Run only the fused ResNet kernel (C2 shape) a few times, for rocprofv3 --pmc passes."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

blocks, filters = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (6, 64)))
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(8, blocks, filters).cuda().eval()
x = (torch.rand(4096, 3, 8, 8, device="cuda") > 0.6).float()
ev = rvz.LeafEvaluator(net, kernel=sys.argv[3] if len(sys.argv) > 3 else "h2")
for _ in range(6):
    ev(x)
torch.cuda.synchronize()
print("ok")
