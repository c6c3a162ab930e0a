#!/bin/bash
# Lanes A/B (--evals lazy): 4 / 5 / 6 / 8 lanes alternating, 2 rounds; then rocprofv3 kernel stats
# of the 4-lane bench (does the profiled trunk average match the line's in-situ span?).
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r03f}
mkdir -p "$OUT"
A="--no-cpu-baseline --sub-configs none --no-evals-ab ${BENCH_ARGS:-}"
for r in 1 2; do
for L in 4 5 6 8; do
timeout -k 10 200 python bench.py $A --lanes $L > "$OUT/ab_lanes${L}_${r}_$TAG.json" 2> "$OUT/ab_lanes${L}_${r}_$TAG.err"
rc=$?; [ $rc -ne 0 ] && { echo "lanes $L rc=$rc"; exit $rc; }
python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('lanes',$L,'round',$r,d['value'],d['roofline']['avg_ms_per_launch'],d['roofline']['timed_region_trunk_frac'])" "$OUT/ab_lanes${L}_${r}_$TAG.json" | tee -a "$OUT/ab_lanes_$TAG.txt"
done; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_l4_$TAG" -o bench \
    -- python bench.py $A --lanes 4 > "$OUT/bench_prof_l4_$TAG.json" 2> "$OUT/bench_prof_l4_$TAG.err"
rc=$?; echo "prof_rc=$rc"; exit $rc
