#!/bin/bash
# Round 5, VERDICT r04 item 1: the clock and the caches of C3's 10x128 evaluator, fused (k_play in
# its bench form) vs the trunk alone run back to back for >= 5 s (tools/exp_c3_clock.py).
# One plain run per mode, then PMC passes per mode (one counter group per run, kernel trace only).
set -u
OUT=${OUT:-gpurun_out/r05a}; mkdir -p "$OUT"; export TMPDIR=/tmp
MODES=${MODES:-"fused iso"}
for m in $MODES; do
  timeout -k 10 240 python tools/exp_c3_clock.py $m > "$OUT/plain_$m.json" 2> "$OUT/plain_$m.err"
  rc=$?; echo "plain $m rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cat "$OUT/plain_$m.json"
done
i=0
for CTRS in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  for m in $MODES; do
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/pmc_${m}_$i" -o run \
        -- python tools/exp_c3_clock.py $m > "$OUT/pmc_${m}_$i.log" 2>&1
    rc=$?; echo "pass $i $m rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python tools/pmc_clock.py "$OUT/pmc_fused_1" "k_play" > "$OUT/clock.txt"
python tools/pmc_clock.py "$OUT/pmc_iso_1" "k_resnet_h2" >> "$OUT/clock.txt"
cat "$OUT/clock.txt"
exit 0
