"""A/B timing of compile-time variants of the split ResNet kernel in ONE process (same box, same
clock state): each variant is a private build of csrc/rvz_resnet.hip with extra -D flags; the
variants are timed alternately (A B A B ...) so drift cancels.

    RVZ_AB='base:;stem0:-DRVZ_STEM_MFMA=0' python tools/ab_split.py [blocks filters n]
"""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402
from rvz import _lib  # noqa: E402

src = os.path.join(ROOT, "tools", "alt", "rvz_resnet_alt.hip")
variants = []
for item in os.environ.get("RVZ_AB", "base:").split(";"):
    name, flags = item.split(":", 1)
    so = f"/tmp/librvz_ab_{name}.so"
    path = src
    if flags.startswith("@"):          # "@<source file> <flags>": another revision of the source
        path, _, flags = flags[1:].partition(" ")
        path = os.path.join(ROOT, path)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-fPIC", "-ffp-contract=off", "-fno-gpu-flush-denormals-to-zero",
                           "-I", os.path.dirname(src), "-x", "hip", *flags.split(), "-shared",
                           "-o", so, path])
    variants.append((name, C.CDLL(so)))

blocks, filters, n = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (6, 64, 4096)))
torch.manual_seed(0)
net = rvz.AlphaZeroNetwork(8, blocks, filters).cuda().eval()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "alt"))
from alt_eval import AltEvaluator  # noqa: E402
ev = AltEvaluator(net, kernel="split")
x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
lg = torch.empty(n, 65, device="cuda")
v = torch.empty(n, device="cuda")
wk = torch.empty(n * 192, device="cuda")
ref_l, ref_v = ev(x)
ref_l, ref_v = ref_l.clone(), ref_v.clone()
s = _lib.stream_handle()


wsp = {}
for name, lib in variants:   # each variant lays out its own split weights (MFMA shape)
    lib.rvz_resnet_split_size.restype = C.c_int64
    w = torch.empty(lib.rvz_resnet_split_size(filters, blocks), dtype=torch.int16, device="cuda")
    assert lib.rvz_resnet_split_weights(C.c_void_p(ev.params.data_ptr()), filters, blocks,
                                        C.c_void_p(w.data_ptr()), C.c_void_p(s)) == 0
    wsp[name] = w


def run(lib, name):
    rc = lib.rvz_resnet_fwd_split(8, C.c_void_p(x.data_ptr()), n, C.c_void_p(ev.params.data_ptr()),
                                  C.c_void_p(wsp[name].data_ptr()), filters, blocks,
                                  C.c_void_p(wk.data_ptr()), C.c_void_p(lg.data_ptr()),
                                  C.c_void_p(v.data_ptr()), C.c_void_p(s))
    assert rc == 0


res = {name: [] for name, _ in variants}
err = {}
for name, lib in variants:
    run(lib, name)
    torch.cuda.synchronize()
    err[name] = max((lg - ref_l).abs().max().item(), (v - ref_v).abs().max().item())
for rep in range(5):
    for name, lib in variants:
        for _ in range(3):
            run(lib, name)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            run(lib, name)
        b.record()
        torch.cuda.synchronize()
        res[name].append(a.elapsed_time(b) / 20)
print(json.dumps({name: {"ms_min": round(min(t), 4), "ms_med": round(sorted(t)[2], 4),
                         "max_abs_diff_vs_default": err[name]} for name, t in res.items()}))
