#!/bin/bash
# Round 6: the per-XCD pass gate at 256 filters — C3's workload with the 10x256 net, gate off vs
# the engine default, alternating (PAIRS pairs). Output: gpurun_out/r06g256/summary.txt.
set -u
OUT=gpurun_out/${OUT:-r06g256}; mkdir -p "$OUT"
for i in $(seq 1 "${PAIRS:-2}"); do
    for g in off default; do
        timeout -k 10 300 python bench.py --config c3 --filters 256 --steps 10 --warmup 3 \
            --no-cpu-baseline --sub-configs none --no-evals-ab --play-gate "$g" \
            > "$OUT/$g.$i.json" 2> "$OUT/$g.$i.err"
        rc=$?; [ $rc -ne 0 ] && { echo "$g $i rc=$rc"; exit $rc; }
        python - "$OUT/$g.$i.json" "$g" "$i" >> "$OUT/summary.txt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"c3-10x256 gate {sys.argv[2]} run {sys.argv[3]}  {d['value']:.1f}  k_play ms "
      f"{r.get('avg_ms_per_launch')}  frac {r.get('frac')}")
PY
        tail -n 1 "$OUT/summary.txt"
    done
done
exit 0
