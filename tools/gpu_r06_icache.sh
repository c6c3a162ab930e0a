#!/bin/bash
# Round 6: instruction-cache counters of k_play in bench.py's C2 and C3 forms (one rocprofv3
# --pmc pass per counter group, kernel trace only; averages over the last 2 k_play dispatches).
set -u
OUT=gpurun_out/r06ic; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in ${CONFIGS:-c2 c3}; do
  i=0
  for CTRS in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
              "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
        -d "$OUT/${c}_$i" -o run -- python bench.py --config "$c" --steps 5 --warmup 1 \
        --no-cpu-baseline --sub-configs none --no-evals-ab > "$OUT/${c}_$i.json" 2> "$OUT/${c}_$i.err"
    rc=$?; echo "$c pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
  python tools/pmc_kernel_avg.py k_play --last 2 "$OUT"/${c}_* > "$OUT/avg_$c.txt"
  cat "$OUT/avg_$c.txt"
done
exit 0
