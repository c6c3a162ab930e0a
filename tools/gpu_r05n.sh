#!/bin/bash
# Round 5: PMC passes (clock / MFMA busy, caches, fabric fetch) of the C3 bench form
# (tools/exp_c3_clock.py fused 20 2 c3) for the in-tree library and VARIANTS.
set -u
OUT=${OUT:-gpurun_out/r05n}; mkdir -p "$OUT"; export TMPDIR=/tmp
j=0
for CTRS in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE"; do
  j=$((j+1))
  for L in base ${VARIANTS:-}; do
    tag=$(basename $L .so)
    if [ "$L" = base ]; then unset RVZ_LIB; else export RVZ_LIB=$L; fi
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/pmc_${tag}_$j" -o run \
        -- python tools/exp_c3_clock.py fused 20 2 ${CFG:-c3} > "$OUT/pmc_${tag}_$j.log" 2>&1
    rc=$?; echo "pmc $j $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
