#!/bin/bash
# Whole-bench A/B of several bench.py argument sets on one library, alternating (drift cancels):
#   ARGSETS="--lanes 2|--lanes 2 --plies-per-graph 2" ROUNDS=2 TAG=x bash tools/gpu_ab_argsets.sh
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-ab}; mkdir -p "$OUT"
ROUNDS=${ROUNDS:-2}
A="--no-cpu-baseline --sub-configs none --no-evals-ab ${ARGS:-}"
IFS='|' read -r -a SETS <<< "$ARGSETS"
for r in $(seq $ROUNDS); do
  for i in "${!SETS[@]}"; do
    timeout -k 10 200 python bench.py $A ${SETS[$i]} > "$OUT/ab_${TAG}_${i}_$r.json" 2> "$OUT/ab_${TAG}_${i}_$r.err"
    rc=$?; [ $rc -ne 0 ] && { echo "set $i rc=$rc"; tail -3 "$OUT/ab_${TAG}_${i}_$r.err"; exit $rc; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print('[${SETS[$i]}] round $r', d['value'], r['avg_ms_per_launch'], r['timed_region_trunk_frac'])" "$OUT/ab_${TAG}_${i}_$r.json" | tee -a "$OUT/ab_$TAG.txt"
  done
done
