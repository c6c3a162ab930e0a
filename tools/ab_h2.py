"""A/B timing of prebuilt variants of the h2 trunk kernel in ONE process (same box, same clock
state), alternating A B A B ... so drift cancels; outputs are checked against the first variant.

    tools/ab_build.sh base "" st0 "-DRVZ_H2_STAGGER=0"
    python tools/ab_h2.py base st0 [blocks filters n]
"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402
from rvz import _lib  # noqa: E402

names = [a for a in sys.argv[1:] if not a.isdigit()]
nums = [int(a) for a in sys.argv[1:] if a.isdigit()]
blocks, filters, n = nums if len(nums) == 3 else (6, 64, 4096)
libs = []
for name in names:
    lib = C.CDLL(os.path.join(ROOT, "tools", "_ab", f"librvz_{name}.so"))
    lib.rvz_resnet_h2_size.restype = C.c_int64
    libs.append((name, lib))
BS = int(os.environ.get("BOARD", 8))
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(BS, blocks, filters).cuda().eval()
ev = rvz.LeafEvaluator(net, kernel="h2")
x = (torch.rand(n, 3, BS, BS, device="cuda") > 0.6).float()
s = C.c_void_p(_lib.stream_handle())
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
bufs = {}
for name, lib in libs:
    blob = torch.empty(lib.rvz_resnet_h2_size(filters, blocks), dtype=torch.int16, device="cuda")
    assert lib.rvz_resnet_h2_weights(P(ev.params), filters, blocks, P(blob), s) == 0
    bufs[name] = (blob, torch.empty(n, BS * BS + 1, device="cuda"), torch.empty(n, device="cuda"),
                  torch.zeros(n * 192 + 4, device="cuda"))


def fwd(name, lib):
    blob, lg, v, wk = bufs[name]
    assert lib.rvz_resnet_fwd_h2(BS, P(x), n, P(ev.params), P(blob), filters, blocks, P(wk), P(lg),
                                 P(v), s) == 0


def trunk(name, lib):
    blob, lg, v, wk = bufs[name]
    assert lib.rvz_resnet_trunk_h2(BS, P(x), n, P(ev.params), P(blob), filters, blocks, P(wk),
                                   s) == 0


for name, lib in libs:
    fwd(name, lib)
torch.cuda.synchronize()
ref = bufs[names[0]]
out = {"shape": [blocks, filters, n]}
for name, lib in libs:
    out[f"{name}_max_dlogit"] = (bufs[name][1] - ref[1]).abs().max().item()
    out[f"{name}_max_dvalue"] = (bufs[name][2] - ref[2]).abs().max().item()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for what, fn in (("trunk", trunk), ("fwd", fwd)):
    times = {name: [] for name in names}
    for rep in range(6):
        for name, lib in libs:
            for _ in range(2):
                fn(name, lib)
            a.record()
            for _ in range(10):
                fn(name, lib)
            b.record()
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(b) / 10)
    for name in names:
        t = sorted(times[name])
        out[f"{name}_{what}_ms_med"] = round(t[len(t) // 2], 4)
print(json.dumps(out))
