#!/usr/bin/env python3
"""Derived PMC metrics of one kernel from rocprofv3 --pmc run dirs (one counter group per dir):
clock, MFMA pipe busy, L1 / L2 hit rates, L2 requests and fabric bytes per second.

    python tools/pmc_derive.py <kernel substring> [--last N] <run_dir> [<run_dir> ...]

Per run dir the last N matching dispatches (dispatch order) are used (default: all); counters are
averaged per dispatch and divided by the dispatches' mean duration (kernel trace timestamps of
the same rows). Definitions (MI355X_MICROARCH.md):
  clock_GHz      = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / duration
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  l1_hit         = 1 - TCP_TCC_READ_REQ_sum / TCP_TOTAL_CACHE_ACCESSES_sum
  l2_hit         = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  fabric_GBs     = (2 x FETCH_SIZE + WRITE_SIZE) KB / duration (FETCH_SIZE counts half of wide
                   reads on gfx950; Infinity-Cache hits are counted as fetches)
  valu_per_mfma  = SQ_INSTS_VALU / SQ_INSTS_MFMA
Prints one JSON object."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    args = sys.argv[1:]
    pat = args.pop(0)
    last = None
    if args and args[0] == "--last":
        last = int(args[1])
        args = args[2:]
    vals = collections.defaultdict(list)
    durs = []
    for d in args:
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]]
        by_disp = collections.defaultdict(dict)
        for r in rows:
            k = int(r.get("Dispatch_Id", 0) or 0)
            by_disp[k][r["Counter_Name"]] = float(r["Counter_Value"])
            by_disp[k]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        ks = sorted(by_disp)
        if last:
            ks = ks[-last:]
        for k in ks:
            for c, v in by_disp[k].items():
                vals[c].append(v)
    mean = {c: sum(v) / len(v) for c, v in vals.items()}
    dur = mean.get("_dur")
    out = {"kernel": pat, "dispatches_per_dir": last, "mean_duration_ms": round(dur * 1e3, 3)}
    g = mean.get("GRBM_GUI_ACTIVE")
    if g:
        out["clock_GHz"] = round(g / 8 / dur / 1e9, 4)
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
        out["mfma_busy"] = round(mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8), 4)
    if "SQ_INSTS_VALU" in mean and mean.get("SQ_INSTS_MFMA"):
        out["valu_per_mfma"] = round(mean["SQ_INSTS_VALU"] / mean["SQ_INSTS_MFMA"], 3)
        out["lds_per_mfma"] = round(mean.get("SQ_INSTS_LDS", 0) / mean["SQ_INSTS_MFMA"], 3)
    if "SQ_WAVE_CYCLES" in mean:
        w = mean["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in mean:
                out[c.lower() + "_frac"] = round(mean[c] / w, 4)
    if mean.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
        out["l1_hit"] = round(1 - mean["TCP_TCC_READ_REQ_sum"] / mean["TCP_TOTAL_CACHE_ACCESSES_sum"], 4)
        out["l1_to_l2_read_req_per_s"] = round(mean["TCP_TCC_READ_REQ_sum"] / dur / 1e9, 2)
    if "TCC_HIT_sum" in mean:
        h, m = mean["TCC_HIT_sum"], mean["TCC_MISS_sum"]
        out["l2_hit"] = round(h / (h + m), 4)
        out["l2_miss_G_per_s"] = round(m / dur / 1e9, 2)
    if "FETCH_SIZE" in mean:
        out["fetch_GBs_corrected"] = round(2 * mean["FETCH_SIZE"] * 1024 / dur / 1e9, 1)
        out["fetch_bytes_per_dispatch_corrected"] = round(2 * mean["FETCH_SIZE"] * 1024)
    if "WRITE_SIZE" in mean:
        out["write_GBs"] = round(mean["WRITE_SIZE"] * 1024 / dur / 1e9, 1)
        out["write_bytes_per_dispatch"] = round(mean["WRITE_SIZE"] * 1024)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
