#!/bin/bash
# PMC passes on the fused ResNet kernel: clock, MFMA busy, LDS conflicts, waits.
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for CTRS in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
            "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/resnet_pmc_$i" -o run \
      -- python tools/exp_resnet_pmc.py ${SHAPE:-6 64} ${KERNEL:-h2} > "$OUT/resnet_pmc_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
