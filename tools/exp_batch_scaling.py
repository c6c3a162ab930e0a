"""Trunk kernel time vs leaf-batch size (rounds of resident workgroups): separates the per-board
cost from the fixed ramp / tail cost of a launch. Prints one JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
out = {}
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for n in (1024, 2048, 3072, 4096, 6144, 8192, 16384):
    ev = rvz.LeafEvaluator(net, kernel="h2")
    x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
    ev(x)
    for _ in range(3):
        ev.trunk_only(x)
    ts = []
    for _ in range(5):
        a.record()
        for _ in range(10):
            ev.trunk_only(x)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 10)
    t = sorted(ts)[2]
    out[n] = {"ms": round(t, 4), "us_per_1k_boards": round(t * 1e3 / n * 1024, 2)}
print(json.dumps(out))
