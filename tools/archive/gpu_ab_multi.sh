#!/bin/bash
# A/B/C... of variant libraries (tools/_ab/librvz_<name>.so) against the in-tree build on the
# default bench, two alternating passes.   VARIANTS="pd3 apd2" bash tools/gpu_ab_multi.sh
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
for pass in 1 2; do
  for V in base $VARIANTS; do
    L=alphazero-reversi_amd/rvz/librvz.so; [ $V != base ] && L=tools/_ab/librvz_$V.so
    RVZ_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline ${ARGS:-} > "$OUT/abm_$V.json" 2> "$OUT/abm_$V.err" || exit $?
    python -c "import json; d=json.load(open('$OUT/abm_$V.json')); print('$V', d['value'], d['ms_per_step'])"
  done
done
