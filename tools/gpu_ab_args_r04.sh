#!/bin/bash
# Whole-bench A/B of bench.py argument sets on one box, alternating, R rounds:
#   SETS="name1|args1;name2|args2" R=2 bash tools/gpu_ab_args_r04.sh > gpurun_out/ab.txt
set -u
OUT=${OUT:-gpurun_out}; R=${R:-2}
BASE="python bench.py --no-cpu-baseline --sub-configs none --no-evals-ab ${BASE_ARGS:-}"
IFS=';' read -ra S <<< "$SETS"
for r in $(seq 1 $R); do
  for s in "${S[@]}"; do
    name=${s%%|*}; args=${s#*|}
    timeout -k 10 300 $BASE $args > "$OUT/ab_$name.json" 2> "$OUT/ab_$name.err"
    rc=$?; [ $rc -ne 0 ] && { echo "[$name] rc=$rc"; tail -3 "$OUT/ab_$name.err"; exit $rc; }
    python - "$OUT/ab_$name.json" "$name" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[0])
print(f"[{sys.argv[2]}] round {sys.argv[3]}  {d['value']:.0f}  ms/launch {d['roofline']['avg_ms_per_launch']}  rows/ply {d['nn_rows_per_ply']}  table {d.get('table')}", flush=True)
PY
  done
done
