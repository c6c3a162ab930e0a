"""Shader clock during each kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace run:
GRBM_GUI_ACTIVE (busy cycles, summed over the 8 XCDs on MI355X) / 8 / the dispatch's duration.

    python tools/pmc_clock.py <run_dir> [kernel substring ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    d, pats = sys.argv[1], sys.argv[2:] or ["k_resnet_h2", "k_step", "k_heads_mfma"]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for r in rows:
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        for p in pats:
            if p in r["Kernel_Name"]:
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                a = agg[p]
                a[0] += float(r["Counter_Value"])
                a[1] += dur
                a[2] += 1
    for p, (cyc, dur, n) in agg.items():
        print(f"{p:16s} {n:5d} dispatches  {cyc / 8 / dur / 1e9:.3f} GHz  "
              f"(GUI_ACTIVE/8 per dispatch {cyc / 8 / n:.0f}, mean {dur / n * 1e6:.1f} us)")


if __name__ == "__main__":
    main()
