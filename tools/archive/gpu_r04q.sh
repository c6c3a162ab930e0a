#!/bin/bash
# r04q: per-row efficiency of larger groups in the 60-ply window, where a static owner of a group
# plays every phase of the game once (blocked stagger): queue groups of 6 vs static groups of 8
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
BASE_ARGS="--steps 60 --warmup 3" SETS="q6|--play-group -6;s8|--play-group 8;q8|--play-group -8;s6|--play-group 6" R=2 \
  bash tools/gpu_ab_args_r04.sh > "$OUT/r04q_ab_static_groups_60.txt" 2>&1
rc=$?; cat "$OUT/r04q_ab_static_groups_60.txt"; exit $rc
