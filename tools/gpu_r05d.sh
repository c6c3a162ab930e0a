#!/bin/bash
# Round 5, VERDICT r04 item 1 (Winograd at F = 128): is the fused launch's weight stream the
# bound? A/B of k_play with RVZ_H2_WEXTRA extra weight-fragment loads per k-step (other layers'
# fragments: more L2 / Infinity-Cache bytes per MFMA, as a Winograd layout needs; built from
# tools/patches/wextra.patch into tools/_ab/librvz_wx{4,12}.so) against the in-tree library:
# alternating plain runs (time), then PMC passes per library (clock / MFMA busy, caches, fabric).
set -u
OUT=${OUT:-gpurun_out/r05d}; mkdir -p "$OUT"; export TMPDIR=/tmp
CFG=${CFG:-c3}
LIBS="base tools/_ab/librvz_wx4.so tools/_ab/librvz_wx12.so"
i=0
for rep in 1 2; do
  for L in $LIBS; do
    i=$((i+1))
    if [ "$L" = base ]; then unset RVZ_LIB; else export RVZ_LIB=$L; fi
    timeout -k 10 240 python tools/exp_c3_clock.py fused 20 2 $CFG > "$OUT/plain_${CFG}_$i.json" 2> "$OUT/plain_${CFG}_$i.err"
    rc=$?; echo "plain $i $L rc=$rc"; [ $rc -ne 0 ] && exit $rc
    cat "$OUT/plain_${CFG}_$i.json"
  done
done
unset RVZ_LIB
j=0
for CTRS in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE"; do
  j=$((j+1))
  for L in $LIBS; do
    tag=$(basename $L .so)
    if [ "$L" = base ]; then unset RVZ_LIB; else export RVZ_LIB=$L; fi
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/pmc_${CFG}_${tag}_$j" -o run \
        -- python tools/exp_c3_clock.py fused 20 2 $CFG > "$OUT/pmc_${CFG}_${tag}_$j.log" 2>&1
    rc=$?; echo "pmc $j $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
