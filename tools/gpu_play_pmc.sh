#!/bin/bash
# SQ / TCP PMC passes on the fused self-play kernel (k_play) inside bench.py's C2 line: clock,
# MFMA busy, waits, instruction mix, LDS conflicts, L1 -> L2 requests. One counter group per run.
#   TAG=x bash tools/gpu_play_pmc.sh; python tools/pmc_kernel_avg.py k_play gpurun_out/play_pmc_x_*
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-play}; mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS="--no-cpu-baseline --sub-configs none --no-evals-ab --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS:-}"
i=0
for CTRS in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
            "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/play_pmc_${TAG}_$i" -o run \
      -- python bench.py $ARGS > "$OUT/play_pmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python tools/pmc_kernel_avg.py "k_play" --last ${LAST:-3} "$OUT"/play_pmc_${TAG}_* > "$OUT/play_pmc_${TAG}.txt"
cat "$OUT/play_pmc_${TAG}.txt"
