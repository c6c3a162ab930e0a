#!/bin/bash
# r04o3: --stagger-order blocked (game g of N at ply floor(60 g / N)) vs interleaved (g mod 60),
# the driver's 20-ply window and the 60-ply window, alternating on one box
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
BASE_ARGS="--steps 20 --warmup 5" SETS="inter|--stagger-order interleaved;blocked|--stagger-order blocked" R=3 \
  bash tools/gpu_ab_args_r04.sh > "$OUT/r04o_ab_stagger_order_20.txt" 2>&1
rc=$?; cat "$OUT/r04o_ab_stagger_order_20.txt"; [ $rc -ne 0 ] && exit $rc
BASE_ARGS="--steps 60 --warmup 3" SETS="inter|--stagger-order interleaved;blocked|--stagger-order blocked" R=2 \
  bash tools/gpu_ab_args_r04.sh > "$OUT/r04o_ab_stagger_order_60.txt" 2>&1
rc=$?; cat "$OUT/r04o_ab_stagger_order_60.txt"; exit $rc
