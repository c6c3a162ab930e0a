"""Per-lane kernel chain of a rocprofv3 --kernel-trace CSV: for each queue, over the dispatches
of the timed region (the longest run of k_step / k_resnet_h2 / k_heads_mfma / k_act dispatches),
the mean duration of each kernel kind and the mean gap from the previous dispatch's end on the same
queue to this one's start; plus how much of the wall time has 0 / 1 / 2+ trunks running.

    python tools/lane_chain.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

KINDS = {"k_step<": "step", "k_resnet_h2<": "trunk", "k_heads_mfma<": "heads", "k_act<": "act",
         "k_env_autoreset": "autoreset"}


def kind(name):
    for p, k in KINDS.items():
        if p in name:
            return k
    return None


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # timed region: from the first trunk dispatch after the last graph capture heuristically =
    # the last 60% of trunk dispatches
    trunks = [r for r in rows if kind(r["Kernel_Name"]) == "trunk"]
    t_lo = int(trunks[int(len(trunks) * 0.4)]["Start_Timestamp"])
    t_hi = int(trunks[-12]["End_Timestamp"])
    per_q = defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t_lo <= s <= t_hi:
            per_q[r["Queue_Id"]].append((s, e, kind(r["Kernel_Name"]) or r["Kernel_Name"][:40]))
    for q, ds in sorted(per_q.items()):
        dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
        prev_end = None
        for s, e, k in ds:
            dur[k] += e - s
            cnt[k] += 1
            if prev_end is not None:
                gap[k] += max(0, s - prev_end)
            prev_end = max(prev_end or 0, e)
        span = ds[-1][1] - ds[0][0]
        print(f"queue {q}: {len(ds)} dispatches over {span / 1e6:.2f} ms")
        for k in sorted(cnt, key=lambda k: -dur[k]):
            print(f"   {k:12s} n={cnt[k]:5d} mean {dur[k] / cnt[k] / 1e3:8.1f} us  "
                  f"gap before {gap[k] / cnt[k] / 1e3:7.1f} us  total {dur[k] / 1e6:7.2f} ms  "
                  f"gaps {gap[k] / 1e6:6.2f} ms")
    # trunk concurrency
    ev = []
    for r in trunks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t_lo <= s <= t_hi:
            ev += [(s, 1), (e, -1)]
    ev.sort()
    acc = defaultdict(int)
    c, last = 0, ev[0][0]
    for t, d in ev:
        acc[min(c, 2)] += t - last
        c += d
        last = t
    tot = sum(acc.values())
    print("trunks running: " + ", ".join(f"{k}: {100 * v / tot:.1f}%" for k, v in sorted(acc.items())))


if __name__ == "__main__":
    main()
