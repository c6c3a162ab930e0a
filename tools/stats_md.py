"""rocprofv3 --stats kernel CSV -> the markdown summary committed under profiles/.

    python tools/stats_md.py <kernel_stats.csv> <out.md> "<title>" [top=16]"""
import csv
import re
import sys


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    m = re.match(r"([^(]*)", name)
    return (m.group(1) if m else name)[:110]


def main():
    src, dst, title = sys.argv[1:4]
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    rows = sorted(csv.DictReader(open(src)), key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"# {title}", "", "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
    for r in rows[:top]:
        out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{100 * float(r['TotalDurationNs']) / tot:.2f} |")
    open(dst, "w").write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
