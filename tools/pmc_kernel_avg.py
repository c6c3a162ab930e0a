"""Average per-dispatch PMC counters of one kernel over rocprofv3 --pmc run dirs.

    python tools/pmc_kernel_avg.py <kernel substring> <run_dir> [<run_dir> ...]
"""
import collections
import csv
import glob
import os
import sys


def main():
    pat, dirs = sys.argv[1], sys.argv[2:]
    agg = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pat in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{k:32s} {sum(v) / len(v):16.0f}  ({len(v)} dispatches)")


if __name__ == "__main__":
    main()
