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
SO = os.environ.get("RVZ_PHASE_SO") or \
    "/tmp/librvz_phase%s.so" % "".join(EXTRA).replace("-", "_").replace("=", "")
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
    ev = rvz.LeafEvaluator(net)  # h2 (the split kernel is in tools/alt)
    fwd = lib.rvz_resnet_fwd_h2
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
    # records are per workgroup (blockIdx); with dealt units (RVZ_H2_DYN) the grid has spare
    # workgroups that find no unit and record nothing: keep the workgroups that ran a unit
    ngrid = lib.rvz_resnet_h2_grid(8, filters, n)
    buf = np.zeros((ngrid, 8), np.uint64)
    assert lib.rvz_phase_read(buf.ctypes.data_as(C.c_void_p), ngrid) == 0
    ran = buf[:, 3] != 0
    b = buf.astype(np.int64)[ran]
    wv = np.zeros((ngrid, 16), np.uint64)
    assert lib.rvz_wave_read(wv.ctypes.data_as(C.c_void_p), ngrid) == 0
    wv = wv.astype(np.int64)[ran]
    nwg = int(ran.sum())
    d = np.diff(b[:, :4], axis=1)
    tot = b[:, 3] - b[:, 0]
    key = f"{blocks}x{filters}"
    out[key] = {"stem": float(d[:, 0].mean()), "trunk": float(d[:, 1].mean()),
                "per_layer": float(d[:, 1].mean() / (2 * blocks)), "heads": float(d[:, 2].mean()),
                "wg_total": float(tot.mean()),
                "l0_conv_a": float((b[:, 5] - b[:, 1]).mean()),
                "l0_barrier": float((b[:, 6] - b[:, 5]).mean()),
                "n_wg": nwg}
    if hasattr(lib, "rvz_stem_read"):    # builds with the stem stamps (STEM_T)
        st = np.zeros((ngrid, 8), np.uint64)
        assert lib.rvz_stem_read(st.ctypes.data_as(C.c_void_p), ngrid) == 0
        st = st.astype(np.int64)[ran]
        out[key]["stem_split"] = {"zero_rows_issue_loads": float((st[:, 0] - b[:, 0]).mean()),
                                  "xin_store_wait_loads": float((st[:, 1] - st[:, 0]).mean()),
                                  "sync1": float((st[:, 2] - st[:, 1]).mean()),
                                  "stem_compute": float((st[:, 3] - st[:, 2]).mean()),
                                  "im2col_split": float((st[:, 4] - st[:, 2]).mean()),
                                  "mfma": float((st[:, 5] - st[:, 4]).mean()),
                                  "epilogue": float((st[:, 3] - st[:, 5]).mean()),
                                  "sync2": float((b[:, 1] - st[:, 3]).mean())}
    rt = np.zeros((ngrid, 2), np.uint64)
    assert lib.rvz_rt_read(rt.ctypes.data_as(C.c_void_p), ngrid) == 0
    rt = rt.astype(np.int64)[ran]
    wg_us = (rt[:, 1] - rt[:, 0]) / 100.0                    # 100 MHz
    out[key]["wg_us_mean"] = float(wg_us.mean())
    out[key]["clock_ghz"] = float(tot.mean() / wg_us.mean() / 1e3)
    out[key]["kernel_span_us"] = float((rt[:, 1].max() - rt[:, 0].min()) / 100.0)
    occ = int(os.environ.get("OCC", 2 if kern == "h2" else 1))
    out[key]["busy_frac"] = float(wg_us.sum() / (256 * occ) / out[key]["kernel_span_us"])
    t0 = rt[:, 0].min()
    st, en = (rt[:, 0] - t0) / 100.0, (rt[:, 1] - t0) / 100.0
    out[key]["start_us_pct"] = [round(float(np.percentile(st, q)), 2) for q in (0, 10, 25, 50, 75, 90, 100)]
    out[key]["end_us_pct"] = [round(float(np.percentile(en, q)), 2) for q in (0, 10, 25, 50, 75, 90, 100)]
    out[key]["wg_us_pct"] = [round(float(np.percentile(wg_us, q)), 2) for q in (0, 10, 50, 90, 100)]
    if hasattr(lib, "rvz_hwid_read") and kern == "h2":
        hw = np.zeros((ngrid, 2), np.uint32)
        assert lib.rvz_hwid_read(hw.ctypes.data_as(C.c_void_p), ngrid) == 0
        hw = hw[ran]
        # CU identity: XCC, SE (bits 13-15), SH (12), CU (8-11)
        cu = (hw[:, 1].astype(np.int64) & 0xF) * 4096 + ((hw[:, 0] >> 8) & 0xFF).astype(np.int64)
        by = {}
        for w in range(nwg):
            by.setdefault(int(cu[w]), []).append(w)
        # per CU: workgroups in dispatch order; partner pairs = those resident at the same time
        st0, en0 = rt[:, 0], rt[:, 1]
        dstart, pairs, first_pair = [], 0, []
        for c, ws in by.items():
            ws.sort(key=lambda w: st0[w])
            for i, w in enumerate(ws):
                for v in ws[i + 1:]:
                    if st0[v] < en0[w]:            # overlapping lifetimes: co-resident
                        dstart.append(abs(int(st0[v]) - int(st0[w])) / 100.0)
                        pairs += 1
                        if len(first_pair) < 8:
                            first_pair.append([w, v])
        d = np.array(dstart) if dstart else np.zeros(1)
        xcc = hw[:, 1].astype(np.int64) & 0xF
        out[key]["units_per_xcc"] = [int((xcc == k).sum()) for k in range(8)]
        out[key]["wg_us_per_xcc"] = [round(float(wg_us[xcc == k].mean()), 2) if (xcc == k).any()
                                     else None for k in range(8)]
        out[key]["cus_used"] = len(by)
        out[key]["wg_per_cu"] = [min(len(v) for v in by.values()), max(len(v) for v in by.values())]
        out[key]["coresident_pairs"] = pairs
        out[key]["pair_start_gap_us_pct"] = [round(float(np.percentile(d, q)), 2)
                                             for q in (10, 25, 50, 75, 90)]
        out[key]["example_pairs"] = first_pair
print(json.dumps(out))
