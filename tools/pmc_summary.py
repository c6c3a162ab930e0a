#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc runs into per-kernel HBM traffic per launch (profiles/pmc_traffic.json).

    python tools/pmc_summary.py <fetch_run_dir> <write_run_dir> [out.json]

Each run dir holds one `--pmc FETCH_SIZE` or `--pmc WRITE_SIZE` pass (separate passes: the TCC
block cannot hold both, MI355X_MICROARCH.md §rocprofv3 PMC slots) with --output-format csv.
Correction per MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE counts exactly half the bytes of wide
(16 B/lane) coalesced reads, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (counters are in
KB). Both the raw and the corrected values are written.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# play: the fused self-play launch; its mean is over the last LAST_PLAY dispatches (bench.py's
# --steps-ply launches: the warm-up replays and the timed one; the first eager ply is shorter)
LAST_PLAY = 3
KERNELS = {"play": "k_play<", "step": "k_step<", "act": "k_act<", "expand_backup": "k_expand_backup<",
           "reset": "k_reset<", "nn_trunk": ("k_resnet_h2<", "k_resnet_split<"), "nn_heads": "k_heads_fc(",
           "nn_conv3x3": "igemm_fwd_gtcx35_nhwc_fp32_bx0_ex1_bt128x64x16"}


def load(run_dir, counter):
    files = glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    rows = [r for f in files for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))   # dispatch order
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        for key, pat in KERNELS.items():
            if any(p in r["Kernel_Name"] for p in ((pat,) if isinstance(pat, str) else pat)):
                per[key].append(float(r["Counter_Value"]))
    return per


def main():
    fetch_dir, write_dir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    fetch, write = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    res = {}
    for key in KERNELS:
        if not fetch.get(key) or not write.get(key):
            continue
        fk, wk = fetch[key], write[key]
        if key == "play":
            fk, wk = fk[-LAST_PLAY:], wk[-LAST_PLAY:]
        f = sum(fk) / len(fk)
        w = sum(wk) / len(wk)
        res[key] = {"dispatches": len(fetch[key]), "FETCH_SIZE_KB": round(f, 2),
                    "WRITE_SIZE_KB": round(w, 2),
                    "raw_bytes_per_launch": round((f + w) * 1024),
                    "hbm_bytes_per_launch": round((2 * f + w) * 1024)}
    res["_note"] = ("hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md §HBM "
                    "(FETCH_SIZE counts half of wide coalesced reads on gfx950; Infinity-Cache hits "
                    "are counted as fetches); per-dispatch means over the run")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
