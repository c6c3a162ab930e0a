#!/bin/bash
# r04o: stagger multiplier A/B (game g at ply (g * K) mod 60): the driver's 20-ply window and the
# 60-ply window, alternating on one box
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
BASE_ARGS="--steps 20 --warmup 5" SETS="m1|--stagger-mult 1;m11|--stagger-mult 11;m7|--stagger-mult 7" R=2 \
  bash tools/gpu_ab_args_r04.sh > "$OUT/r04o_ab_stagger_mult_20.txt" 2>&1
rc=$?; cat "$OUT/r04o_ab_stagger_mult_20.txt"; [ $rc -ne 0 ] && exit $rc
BASE_ARGS="--steps 60 --warmup 3" SETS="m1|--stagger-mult 1;m11|--stagger-mult 11" R=2 \
  bash tools/gpu_ab_args_r04.sh > "$OUT/r04o_ab_stagger_mult_60.txt" 2>&1
rc=$?; cat "$OUT/r04o_ab_stagger_mult_60.txt"; exit $rc
