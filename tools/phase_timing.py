"""Per-phase cycle split of the fused ResNet trunk kernel (input+stem / trunk / heads).

    KERNEL=h2|split python tools/phase_timing.py

Builds a private copy of librvz with -DRVZ_PHASE_TIMING (s_memtime at phase boundaries, one
record per workgroup), runs one forward at the bench batch and prints mean cycles per phase."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-reversi_amd"))
import rvz  # noqa: E402
from rvz import _lib  # noqa: E402

EXTRA = [f for f in os.environ.get("RVZ_PHASE_FLAGS", "").split() if f]
SO = "/tmp/librvz_phase%s.so" % "".join(EXTRA).replace("-", "_").replace("=", "")
src = os.path.join(ROOT, "alphazero-reversi_amd", "csrc")
if not os.path.exists(SO):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-fPIC", "-ffp-contract=off", "-fno-gpu-flush-denormals-to-zero",
                           "-DRVZ_PHASE_TIMING", *EXTRA, "-shared", "-o", SO,
                           os.path.join(src, "rvz_resnet.hip")])
lib = C.CDLL(SO)
out = {}
for blocks, filters, n in ((6, 64, 4096), (10, 128, 4096)):
    torch.manual_seed(0)
    net = rvz.AlphaZeroNetwork(8, blocks, filters).cuda().eval()
    kern = os.environ.get("KERNEL", "h2")
    ev = rvz.LeafEvaluator(net, kernel=kern)
    fwd = lib.rvz_resnet_fwd_h2 if kern == "h2" else lib.rvz_resnet_fwd_split
    x = (torch.rand(n, 3, 8, 8, device="cuda") > 0.6).float()
    lg = torch.empty(n, 65, device="cuda")
    wk = torch.zeros(n * 192 + 4, device="cuda")
    v = torch.empty(n, device="cuda")
    for _ in range(3):
        rc = fwd(8, C.c_void_p(x.data_ptr()), n, C.c_void_p(ev.params.data_ptr()),
                                      C.c_void_p(ev.wsplit.data_ptr()), filters, blocks,
                                      C.c_void_p(wk.data_ptr()), C.c_void_p(lg.data_ptr()), C.c_void_p(v.data_ptr()),
                                      C.c_void_p(_lib.stream_handle()))
        assert rc == 0
    torch.cuda.synchronize()
    nwg = (n + 1) // 2 if filters == 64 else n
    if kern == "h2":     # persistent: one record per workgroup, phases of its first unit
        nwg = min(nwg, 2 * torch.cuda.get_device_properties(0).multi_processor_count)
    buf = np.zeros((nwg, 8), np.uint64)
    assert lib.rvz_phase_read(buf.ctypes.data_as(C.c_void_p), nwg) == 0
    b = buf.astype(np.int64)
    wv = np.zeros((nwg, 16), np.uint64)
    assert lib.rvz_wave_read(wv.ctypes.data_as(C.c_void_p), nwg) == 0
    wv = wv.astype(np.int64)
    kl = wv[:, :8] - b[:, 1:2]          # per wave: k-loop end of layer 0, from the layer start
    ep = wv[:, 8:] - b[:, 1:2]          # per wave: epilogue end
    out[f"{blocks}x{filters}_waves"] = {"kloop_end": [round(float(v)) for v in kl.mean(0)],
                                        "epi_end": [round(float(v)) for v in ep.mean(0)],
                                        "kloop_end_max_mean": float(kl.max(1).mean())}
    d = np.diff(b[:, :4], axis=1)
    tot = b[:, 3] - b[:, 0]
    key = f"{blocks}x{filters}"
    out[key] = {"stem": float(d[:, 0].mean()), "trunk": float(d[:, 1].mean()),
                "per_layer": float(d[:, 1].mean() / (2 * blocks)), "heads": float(d[:, 2].mean()),
                "wg_total": float(tot.mean()),
                "l0_kloop": float((b[:, 4] - b[:, 1]).mean()),
                "l0_epilogue": float((b[:, 5] - b[:, 4]).mean()),
                "l0_barrier": float((b[:, 6] - b[:, 5]).mean()),
                "n_wg": nwg}
    if hasattr(lib, "rvz_stem_read"):    # builds with the stem stamps (STEM_T)
        st = np.zeros((nwg, 4), np.uint64)
        assert lib.rvz_stem_read(st.ctypes.data_as(C.c_void_p), nwg) == 0
        st = st.astype(np.int64)
        out[key]["stem_split"] = {"loads_zero": float((st[:, 0] - b[:, 0]).mean()),
                                  "sync1": float((st[:, 1] - st[:, 0]).mean()),
                                  "xin_write_sync2": float((st[:, 2] - st[:, 1]).mean()),
                                  "stem_compute": float((st[:, 3] - st[:, 2]).mean()),
                                  "sync3": float((b[:, 1] - st[:, 3]).mean())}
    rt = np.zeros((nwg, 2), np.uint64)
    assert lib.rvz_rt_read(rt.ctypes.data_as(C.c_void_p), nwg) == 0
    rt = rt.astype(np.int64)
    wg_us = (rt[:, 1] - rt[:, 0]) / 100.0                    # 100 MHz
    out[key]["wg_us_mean"] = float(wg_us.mean())
    out[key]["clock_ghz"] = float(tot.mean() / wg_us.mean() / 1e3)
    out[key]["kernel_span_us"] = float((rt[:, 1].max() - rt[:, 0].min()) / 100.0)
    occ = 2 if kern == "h2" else 1
    out[key]["busy_frac"] = float(wg_us.sum() / (256 * occ) / out[key]["kernel_span_us"])
    t0 = rt[:, 0].min()
    st, en = (rt[:, 0] - t0) / 100.0, (rt[:, 1] - t0) / 100.0
    out[key]["start_us_pct"] = [round(float(np.percentile(st, q)), 2) for q in (0, 10, 25, 50, 75, 90, 100)]
    out[key]["end_us_pct"] = [round(float(np.percentile(en, q)), 2) for q in (0, 10, 25, 50, 75, 90, 100)]
    out[key]["wg_us_pct"] = [round(float(np.percentile(wg_us, q)), 2) for q in (0, 10, 50, 90, 100)]
print(json.dumps(out))
