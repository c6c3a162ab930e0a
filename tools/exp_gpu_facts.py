"""GPU fact-finding for design decisions (run on the MI355X box; prints one JSON line).

1. external torch.cuda.Event record nodes inside a captured HIP graph (per-kernel timing of graph
   replays on the launch stream);
2. is the device float64 sqrt correctly rounded (then (float)sqrt((double)n) needs no table)?
3. does the fp32 LeafEvaluator give a row the same bits regardless of its batch position?
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
out = {}

# 2. sqrt
n = torch.arange(0, 2_000_001, dtype=torch.float64, device="cuda")
dev = torch.sqrt(n).float().cpu().numpy()
host = np.sqrt(np.arange(0, 2_000_001, dtype=np.float64)).astype(np.float32)
out["sqrt_f64_then_f32_mismatch"] = int((dev.view(np.int32) != host.view(np.int32)).sum())
dd = torch.sqrt(n).cpu().numpy()
out["sqrt_f64_mismatch"] = int((dd != np.sqrt(np.arange(0, 2_000_001, dtype=np.float64))).sum())

# 1. external events in graph capture
try:
    x = torch.randn(1 << 20, device="cuda")
    s = torch.cuda.Stream()
    evs = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(4)]
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        evs[0].record()
        y = x * 2
        evs[1].record()
        z = y.sin()
        evs[2].record()
        w = z + 1
        evs[3].record()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    out["external_events"] = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(3)]
except Exception as e:  # noqa: BLE001
    out["external_events"] = f"unsupported: {type(e).__name__}: {e}"

# 3. batch-position invariance of the evaluator rows
import rvz  # noqa: E402
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
ev = rvz.LeafEvaluator(net)
xb = (torch.rand(4096, 3, 8, 8, device="cuda") > 0.6).float()
l1, v1 = ev(xb)
perm = torch.randperm(4096, device="cuda")
l2, v2 = ev(xb[perm].contiguous())
out["eval_rows_invariant_to_position"] = bool(torch.equal(l1[perm], l2) and torch.equal(v1[perm], v2))
l3, v3 = ev(xb[:1000].contiguous())
out["eval_rows_invariant_to_batch_size"] = bool(torch.equal(l1[:1000], l3) and torch.equal(v1[:1000], v3))
print(json.dumps(out))
