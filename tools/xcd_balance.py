"""Per-XCD balance of the trunk launches from a bench.py --stamps-dump ring (lane 0, timed
region): per launch, the workgroups and evaluated boards each XCD ran and when its last
workgroup ended; summary over launches (means).

    python bench.py --stamps-dump gpurun_out/stamps.npy && python tools/xcd_balance.py gpurun_out/stamps.npy
"""
import json
import sys

import numpy as np

st = np.load(sys.argv[1])                     # [launch, workgroup, 2] int64
start, endw = st[:, :, 0], st[:, :, 1]
end = endw & ((1 << 52) - 1)
xcd = (endw >> 52) & 0xF
boards = (endw >> 56) & 0xFF
ran = end > 0
out = {"launches": int(st.shape[0]), "grid": int(st.shape[1])}
wg, bd, last, busy = [], [], [], []
for k in range(8):
    m = ran & (xcd == k)
    wg.append(float(m.sum(axis=1).mean()))
    bd.append(float(np.where(m, boards, 0).sum(axis=1).mean()))
    t0 = np.where(ran, start, np.iinfo(np.int64).max).min(axis=1)
    le = np.where(m, end, 0).max(axis=1)
    last.append(float(((le - t0) / 100.0).mean()))          # 100 MHz -> us
    busy.append(float((np.where(m, end - start, 0).sum(axis=1) / 100.0).mean()))
span = (np.where(ran, end, 0).max(axis=1) - np.where(ran, start, np.iinfo(np.int64).max).min(axis=1)) / 100.0
out.update({"span_us": float(span.mean()), "workgroups_per_xcd": [round(v, 1) for v in wg],
            "boards_per_xcd": [round(v, 1) for v in bd],
            "last_end_us_per_xcd": [round(v, 1) for v in last],
            "wg_busy_us_per_xcd": [round(v, 1) for v in busy]})
print(json.dumps(out))
