"""Reconcile a bench.py line's k_play dispatch accounting with rocprofv3's kernel trace of the same
command: every k_play dispatch in trace order, labelled in the order bench.py made them (the
line's k_play_dispatches.by_label is in dispatch order: stagger, warm-up, timed, then the --evals
modes, per kernel instantiation), with the per-label means from the trace beside the line's own
HIP-event means, and rocprofv3 --stats' per-kernel average beside the line's all-dispatch one.

    python tools/trace_dispatches.py <bench line .json> <rocprofv3 -d dir> [out.md]
"""
import csv
import glob
import json
import os
import sys


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[0])
    d = sys.argv[2]
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = {r["Name"]: r for r in csv.DictReader(open(stats))}
    out = ["# k_play dispatches: bench line vs rocprofv3 (same command)", "",
           f"line: `{os.path.basename(sys.argv[1])}` value {line['value']:.0f} "
           f"{line['unit']}, roofline.avg_ms_per_launch {line['roofline']['avg_ms_per_launch']} "
           "(the timed launch); trace: `" + os.path.relpath(trace) + "`", "",
           "| kernel | label (dispatch order) | n | line HIP events, ms | rocprofv3 trace, ms |",
           "|---|---|---|---|---|"]
    for kern, acc in (line.get("k_play_dispatches") or {}).items():
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
                if kern + "(" in r["Kernel_Name"].replace(">((", ">((").replace(">(", ">(")
                or r["Kernel_Name"].find(kern) >= 0]
        i = 0
        for label, v in acc["by_label"].items():
            seg = durs[i:i + v["n"]]
            i += v["n"]
            tm = sum(seg) / len(seg) if seg else float("nan")
            out.append(f"| `{kern}` | {label} | {v['n']} | {v['avg_ms']:.3f} | {tm:.3f} |")
        srow = next((r for n, r in st.items() if kern in n), None)
        if srow:
            out.append(f"| `{kern}` | **all** (rocprofv3 --stats: {srow['Calls']} calls) | "
                       f"{acc['n']} | {acc['avg_ms']:.3f} | {float(srow['AverageNs']) / 1e6:.3f} |")
        if i != len(durs):
            out.append(f"| `{kern}` | (trace has {len(durs)} dispatches, line {i}) | | | |")
    text = "\n".join(out) + "\n"
    print(text)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text)


if __name__ == "__main__":
    main()
