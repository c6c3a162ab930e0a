"""Do two independent leaf-evaluation chains on two streams overlap on the MI355X (eager and inside
one captured HIP graph)? Times K calls of: one 4096-board evaluator; two 2048-board evaluators on
one stream; the same two on two streams (eager); and both captured in one graph with a fork/join.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402

K = 13
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
ev, ev1, ev2 = (rvz.LeafEvaluator(net) for _ in range(3))
x = (torch.rand(4096, 3, 8, 8, device="cuda") > 0.6).float()
x1, x2 = x[:2048].contiguous(), x[2048:].contiguous()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def one():
    for _ in range(K):
        ev(x)


def two_serial():
    for _ in range(K):
        ev1(x1)
        ev2(x2)


def two_streams():
    main = torch.cuda.current_stream()      # the capture stream inside torch.cuda.graph
    s1.wait_stream(main)
    s2.wait_stream(main)
    with torch.cuda.stream(s1):
        for _ in range(K):
            ev1(x1)
    with torch.cuda.stream(s2):
        for _ in range(K):
            ev2(x2)
    main.wait_stream(s1)
    main.wait_stream(s2)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / K)
    return round(sorted(ts)[len(ts) // 2], 4)


out = {"one_4096": timed(one), "two_serial": timed(two_serial), "two_streams": timed(two_streams)}
for name, fn in (("graph_one", one), ("graph_two_serial", two_serial),
                 ("graph_two_streams", two_streams)):
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    out[name] = timed(g.replay)
l1, _ = ev1(x1)
l, _ = ev(x)
out["rows_equal"] = bool(torch.equal(l[:2048], l1))
print(json.dumps(out))
