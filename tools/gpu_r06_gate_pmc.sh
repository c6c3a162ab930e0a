#!/bin/bash
# Round 6, VERDICT r05 item 4(b): what the per-XCD pass gate does to C3's caches and clock.
# tools/exp_c3_clock.py fused (k_play in bench's C3 form: stagger, then 2 x 20-ply launches) with
# the gate off and at its default (or GATES="off f,us,late ..."), one plain run each, then one rocprofv3 --pmc pass per counter group
# (kernel trace only). Averages over the last 2 k_play dispatches (the 20-ply launches).
set -u
OUT=${OUT:-gpurun_out/r06pmc}; mkdir -p "$OUT"; export TMPDIR=/tmp
GATES=${GATES:-"off default"}
for g in $GATES; do
  # RVZ_PLAY_GATE="fraction,us,late_us" or "off"; default: the engine's setting (rvz_play_gate)
  if [ "$g" = default ]; then unset RVZ_PLAY_GATE; else export RVZ_PLAY_GATE="$g"; fi
  tag=${g/,/_}
  timeout -k 10 240 python tools/exp_c3_clock.py fused > "$OUT/plain_$tag.json" 2> "$OUT/plain_$tag.err"
  rc=$?; echo "plain $g rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cat "$OUT/plain_$tag.json"
  i=0
  for CTRS in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES" \
              "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY" \
              "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
              "FETCH_SIZE"; do
    i=$((i+1))
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
        -d "$OUT/pmc_${tag}_$i" -o run -- python tools/exp_c3_clock.py fused \
        > "$OUT/pmc_${tag}_$i.log" 2>&1
    rc=$?; echo "pass $i $g rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
  python tools/pmc_clock.py "$OUT/pmc_${tag}_1" "k_play" > "$OUT/clock_$tag.txt"
  python tools/pmc_kernel_avg.py k_play --last 2 "$OUT"/pmc_${tag}_* > "$OUT/avg_$tag.txt"
  cat "$OUT/clock_$tag.txt" "$OUT/avg_$tag.txt"
done
exit 0
