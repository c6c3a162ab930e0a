#!/bin/bash
# Whole-bench A/B of library builds on one box, alternating R rounds:
#   LIBS="name1=path1;name2=path2" ARGS="--config c2" R=3 bash tools/gpu_ab_libs_r04.sh
set -u
OUT=${OUT:-gpurun_out}; R=${R:-3}
BASE="python bench.py --no-cpu-baseline --sub-configs none --no-evals-ab ${ARGS:-}"
IFS=';' read -ra L <<< "$LIBS"
for r in $(seq 1 $R); do
  for l in "${L[@]}"; do
    name=${l%%=*}; path=${l#*=}
    RVZ_LIB=$path timeout -k 10 300 $BASE > "$OUT/abl_$name.json" 2> "$OUT/abl_$name.err"
    rc=$?; [ $rc -ne 0 ] && { echo "[$name] rc=$rc"; tail -3 "$OUT/abl_$name.err"; exit $rc; }
    python - "$OUT/abl_$name.json" "$name" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[0])
print(f"[{sys.argv[2]}] round {sys.argv[3]}  {d['value']:.0f}  ms/launch {d['roofline']['avg_ms_per_launch']}  rows/ply {d['nn_rows_per_ply']}", flush=True)
PY
  done
done
