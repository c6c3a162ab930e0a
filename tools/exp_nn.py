"""Leaf-evaluator variants on the C2 shape (4,096 x 3 x 8 x 8, 6x64): ms per call.

Variants: memory format (NHWC channels_last vs NCHW), MIOpen find mode (torch.backends.cudnn.benchmark),
bias in the conv vs none (bias/relu/residual then done by other kernels), fp32 vs bf16.
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "alt"))
from alt_eval import AltEvaluator  # noqa: E402


def timeit(fn, x, iters=20):
    for _ in range(3):
        fn(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn(x)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def graph_time(fn, x, iters=20):
    for _ in range(3):
        fn(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn(x)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, 6, 64).cuda().eval()
    x = (torch.rand(4096, 3, 8, 8, device="cuda") > 0.6).float()
    res = {}
    for bench_mode in (False, True):
        torch.backends.cudnn.benchmark = bench_mode
        for dtype in (torch.float32, torch.bfloat16):
            ev = AltEvaluator(net, kernel="miopen", dtype=dtype)
            key = f"nhwc_{'fp32' if dtype == torch.float32 else 'bf16'}_bench{int(bench_mode)}"
            res[key] = round(graph_time(ev, x), 4)
        with torch.no_grad():
            res[f"module_nchw_fp32_bench{int(bench_mode)}"] = round(graph_time(lambda t: net(t), x), 4)

        # conv-only cost of the 12 residual convs (NHWC fp32, no bias)
        w = torch.randn(64, 64, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
        h = torch.randn(4096, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
        res[f"conv3x3_nhwc_fp32_nobias_bench{int(bench_mode)}_ms"] = round(graph_time(lambda t: F.conv2d(t, w, padding=1), h), 4)
        wn, hn = w.contiguous(), h.contiguous()
        res[f"conv3x3_nchw_fp32_nobias_bench{int(bench_mode)}_ms"] = round(graph_time(lambda t: F.conv2d(t, wn, padding=1), hn), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
