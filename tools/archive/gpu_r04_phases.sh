#!/bin/bash
# k_play phase split (instrumented build) with / without the table, then the SQ PMC passes of
# the driver's C2 window (20-ply launches). Each GPU step has its own limit.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r04f}; mkdir -p "$OUT"
for t in 1 0; do
  RVZ_LIB=tools/_ab/librvz_ptime.so TABLE=$t timeout -k 10 200 python tools/exp_play_phases.py \
      > "$OUT/play_phases_${TAG}_table$t.json" 2> "$OUT/play_phases_${TAG}_table$t.err"
  rc=$?; echo "phases table=$t rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cat "$OUT/play_phases_${TAG}_table$t.json"
done
if [ -n "${PMC:-}" ]; then
  OUT=$OUT TAG=$TAG bash tools/gpu_play_pmc.sh
fi
