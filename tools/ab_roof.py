"""Print the trunk roofline fields of the two gpu_ab_lib.sh bench lines (last base / var run)."""
import json
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for v in ("base", "var"):
    d = json.loads(open(f"{out}/ablib_{v}.json").readline())
    r = d["roofline"]
    print(v, "isolated trunk ms", r["isolated"]["avg_ms_per_launch"], "in-situ ms",
          r["avg_ms_per_launch"], "timed-region frac", r["timed_region_trunk_frac"])
