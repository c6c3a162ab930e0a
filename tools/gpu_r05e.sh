#!/bin/bash
# Round 5: the current library against the one before the activation-range change
# (tools/_ab/librvz_r05pre.so, commit 334c38e) on the fused launches of C2 / C5 / C3 (bench form,
# tools/exp_c3_clock.py), alternating, so box drift cancels.
set -u
OUT=${OUT:-gpurun_out/r05e}; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for rep in 1 2; do
  for CFG in ${CFGS:-c2 c5}; do
    for L in base ${VARIANTS:-tools/_ab/librvz_r05pre.so}; do
      i=$((i+1))
      if [ "$L" = base ]; then unset RVZ_LIB; else export RVZ_LIB=$L; fi
      timeout -k 10 240 python tools/exp_c3_clock.py fused 20 2 $CFG > "$OUT/ab_$i.json" 2> "$OUT/ab_$i.err"
      rc=$?; echo "ab $i $CFG $L rc=$rc"; [ $rc -ne 0 ] && exit $rc
      cat "$OUT/ab_$i.json"
    done
  done
done
exit 0
