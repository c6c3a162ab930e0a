#!/bin/bash
# Lanes A/B on the current headline (--evals lazy): alternating 2 / 3 / 4 lanes, 2 rounds.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r03e}
mkdir -p "$OUT"
A="--no-cpu-baseline --sub-configs none --no-evals-ab ${BENCH_ARGS:-}"
for r in 1 2; do
for L in 2 3 4; do
timeout -k 10 200 python bench.py $A --lanes $L > "$OUT/ab_lanes${L}_${r}_$TAG.json" 2> "$OUT/ab_lanes${L}_${r}_$TAG.err"
rc=$?; [ $rc -ne 0 ] && { echo "lanes $L rc=$rc"; exit $rc; }
python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('lanes',$L,'round',$r,d['value'],d['roofline']['avg_ms_per_launch'],d['roofline']['timed_region_trunk_frac'])" "$OUT/ab_lanes${L}_${r}_$TAG.json" | tee -a "$OUT/ab_lanes_$TAG.txt"
done; done
