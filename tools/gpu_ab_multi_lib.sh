#!/bin/bash
# Whole-bench A/B of several librvz builds on one box, alternating (drift cancels):
#   VARIANTS="base tools/_ab/librvz_b.so tools/_ab/librvz_c.so" ROUNDS=2 ARGS="..." TAG=x \
#     bash tools/gpu_ab_multi_lib.sh     ('base' = the in-tree library)
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-ab}; mkdir -p "$OUT"
ROUNDS=${ROUNDS:-2}
A="--no-cpu-baseline --sub-configs none --no-evals-ab ${ARGS:-}"
for r in $(seq $ROUNDS); do
  for V in $VARIANTS; do
    L=$V; [ "$V" = base ] && L=alphazero-reversi_amd/rvz/librvz.so
    n=$(basename "$L" .so)
    RVZ_LIB=$L timeout -k 10 200 python bench.py $A > "$OUT/ab_${TAG}_${n}_$r.json" 2> "$OUT/ab_${TAG}_${n}_$r.err"
    rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; exit $rc; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print('$n round $r', d['value'], r['avg_ms_per_launch'], r['timed_region_trunk_frac'])" "$OUT/ab_${TAG}_${n}_$r.json" | tee -a "$OUT/ab_$TAG.txt"
  done
done
