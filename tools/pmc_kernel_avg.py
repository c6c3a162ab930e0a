"""Average per-dispatch PMC counters of one kernel over rocprofv3 --pmc run dirs.

    python tools/pmc_kernel_avg.py <kernel substring> [--last N] <run_dir> [<run_dir> ...]

--last N: per run dir, only the last N matching dispatches (in dispatch order) are averaged —
bench.py's k_play dispatches are the phase-stagger launch (shorter, first), the warm-up launches
and the timed one; the last N skip the stagger launch.
"""
import collections
import csv
import glob
import os
import sys


def main():
    args = sys.argv[1:]
    pat = args.pop(0)
    last = None
    if args and args[0] == "--last":
        last = int(args[1])
        args = args[2:]
    agg = collections.defaultdict(list)
    for d in args:
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        per = collections.defaultdict(list)
        for r in rows:
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in per.items():
            agg[k] += v[-last:] if last else v
    for k, v in sorted(agg.items()):
        print(f"{k:32s} {sum(v) / len(v):16.0f}  ({len(v)} dispatches)")


if __name__ == "__main__":
    main()
