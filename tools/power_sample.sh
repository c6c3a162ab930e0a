#!/bin/bash
# Socket power and clocks while the C2 bench runs a long timed region (informational: is the trunk
# power-limited?). Samples amd-smi every ~0.3 s into $OUT/power_$TAG.jsonl.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-p}; mkdir -p "$OUT"
timeout -k 10 20 amd-smi metric -p -c --json > "$OUT/power_idle_$TAG.json" 2>&1
echo "idle rc=$?"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-1800} > "$OUT/power_bench_$TAG.json" 2> "$OUT/power_bench_$TAG.err" &
BP=$!
: > "$OUT/power_$TAG.jsonl"
while kill -0 $BP 2>/dev/null; do
  { date +%s.%N; timeout -k 5 10 amd-smi metric -p -c --json 2>&1; } | tr '\n' ' ' >> "$OUT/power_$TAG.jsonl"
  echo >> "$OUT/power_$TAG.jsonl"
  sleep 0.2
done
wait $BP; rc=$?
echo "bench rc=$rc"; exit $rc
