#!/bin/bash
# A/B of a variant librvz (RVZ_LIB) against a base build (BASE, default the in-tree one) on the
# default bench, alternating.
#   VARIANT=tools/_ab/librvz_x.so [BASE=tools/_ab/librvz_y.so] [PAIRS=2] ARGS="--no-stamps" \
#     bash tools/gpu_ab_lib.sh
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
PAIRS=${PAIRS:-2}
for V in $(for i in $(seq $PAIRS); do echo base var; done); do
  L=""; [ $V = var ] && L="$VARIANT"
  RVZ_LIB=${L:-${BASE:-alphazero-reversi_amd/rvz/librvz.so}} timeout -k 10 300 python bench.py --no-cpu-baseline ${ARGS:-} > "$OUT/ablib_$V.json" 2> "$OUT/ablib_$V.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/ablib_$V.json')); print('$V', d['value'], d['ms_per_step'])"
done
