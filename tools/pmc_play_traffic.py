#!/usr/bin/env python3
"""HBM (fabric) bytes and clock of one config's k_play launches from rocprofv3 --pmc passes of a
bench.py run of that config, merged into profiles/pmc_traffic.json (bench.py quotes them as the
config's roofline.traffic).

    python tools/pmc_play_traffic.py --config c3 --games 32768 --plies 20 --last 1 \
        --kernel "k_play<128, 1, 2, 4, 8, 2>" <fetch_dir> <write_dir> [--clock-dir d] \
        [--out profiles/pmc_traffic.json] [--source text]

Key "play" for c2 (the headline), "play_<config>" otherwise. --last: per run dir the last N
dispatches of the instantiation (bench.py's timed launch is the last one of its config).
hbm_bytes = (2 x FETCH_SIZE + WRITE_SIZE) KB x 1024 per MI355X_MICROARCH.md §HBM (FETCH_SIZE
counts half of wide reads on gfx950; Infinity-Cache hits are counted as fetches)."""
import argparse
import csv
import glob
import json
import os


def per_dispatch(d, kernel, counter, last):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f))
                 if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    rows = rows[-last:]
    return ([float(r["Counter_Value"]) for r in rows],
            [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in rows])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--games", type=int, required=True)
    ap.add_argument("--plies", type=int, required=True)
    ap.add_argument("--last", type=int, default=1)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--clock-dir", default=None)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--source", default="")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    a = ap.parse_args()
    f, fd = per_dispatch(a.fetch_dir, a.kernel, "FETCH_SIZE", a.last)
    w, wd = per_dispatch(a.write_dir, a.kernel, "WRITE_SIZE", a.last)
    if not f or not w:
        raise SystemExit(f"no {a.kernel} dispatches with FETCH_SIZE / WRITE_SIZE")
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    ent = {"kernel": a.kernel, "config": a.config, "games": a.games, "plies_per_launch": a.plies,
           "dispatches": len(f), "FETCH_SIZE_KB": round(fk, 2), "WRITE_SIZE_KB": round(wk, 2),
           "raw_bytes_per_launch": round((fk + wk) * 1024),
           "hbm_bytes_per_launch": round((2 * fk + wk) * 1024),
           "ms_per_launch_fetch_pass": round(sum(fd) / len(fd) * 1e3, 3),
           "ms_per_launch_write_pass": round(sum(wd) / len(wd) * 1e3, 3)}
    if a.clock_dir:
        g, gd = per_dispatch(a.clock_dir, a.kernel, "GRBM_GUI_ACTIVE", a.last)
        if g:
            ent["clock_GHz"] = round(sum(g) / len(g) / 8 / (sum(gd) / len(gd)) / 1e9, 4)
            ent["ms_per_launch_clock_pass"] = round(sum(gd) / len(gd) * 1e3, 3)
    ent["source"] = a.source
    key = "play" if a.config == "c2" else f"play_{a.config}"
    d = json.load(open(a.out)) if os.path.exists(a.out) else {}
    d[key] = ent
    json.dump(d, open(a.out, "w"), indent=1)
    print(json.dumps({key: ent}))


if __name__ == "__main__":
    main()
