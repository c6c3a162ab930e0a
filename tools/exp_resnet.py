"""Time the fused resnet kernels (f32 MFMA, fp32 split over bf16 MFMA) against MIOpen."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools", "alt"))
from alt_eval import AltEvaluator  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from exp_nn import graph_time  # noqa: E402

out = {}
for blocks, filters, n in ((6, 64, 4096), (10, 128, 4096), (0, 64, 4096), (10, 128, 32768)):
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, blocks, filters).cuda().eval()
    x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
    fl = AltEvaluator(net, kernel="miopen").flops_per_row() * n
    for kern in (("miopen", "resnet", "split") if blocks else ("resnet", "split")):
        ev = AltEvaluator(net, kernel=kern)
        ms = graph_time(ev, x)
        out[f"{blocks}x{filters}_{kern}_ms"] = round(ms, 4)
        out[f"{blocks}x{filters}_{kern}_TFs"] = round(fl / ms / 1e9, 1)
print(json.dumps(out))
