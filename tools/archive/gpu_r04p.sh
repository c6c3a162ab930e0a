#!/bin/bash
# r04p: fused-launch group sizes with the blocked stagger (queue: -g), the driver's 20-ply window
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
BASE_ARGS="--steps 20 --warmup 5" SETS="g6|--play-group -6;g5|--play-group -5;g7|--play-group -7;g8|--play-group -8;g4|--play-group -4" R=2 \
  bash tools/gpu_ab_args_r04.sh > "$OUT/r04p_ab_groups_blocked.txt" 2>&1
rc=$?; cat "$OUT/r04p_ab_groups_blocked.txt"; exit $rc
