#!/bin/bash
# r04o2: stagger blocks (groups of B consecutive games at the same ply) A/B, 20- and 60-ply windows
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
BASE_ARGS="--steps 20 --warmup 5" SETS="b1|--stagger-block 1;b6|--stagger-block 6;b2|--stagger-block 2" R=2 \
  bash tools/gpu_ab_args_r04.sh > "$OUT/r04o_ab_stagger_block_20.txt" 2>&1
rc=$?; cat "$OUT/r04o_ab_stagger_block_20.txt"; [ $rc -ne 0 ] && exit $rc
BASE_ARGS="--steps 60 --warmup 3" SETS="b1|--stagger-block 1;b6|--stagger-block 6" R=2 \
  bash tools/gpu_ab_args_r04.sh > "$OUT/r04o_ab_stagger_block_60.txt" 2>&1
rc=$?; cat "$OUT/r04o_ab_stagger_block_60.txt"; exit $rc
