#!/bin/bash
# Round 6: a config's k_play PMC passes (CONFIG, default c2 = the headline) on the final code (FETCH_SIZE, WRITE_SIZE,
# GRBM_GUI_ACTIVE: one group per run, kernel trace only) for profiles/pmc_traffic.json "play"
# (merged in the container by tools/pmc_play_traffic.py). Every step under its own limit.
set -u
OUT=${OUT:-gpurun_out/r06pmc2}; mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS="--config ${CONFIG:-c2} --no-cpu-baseline --no-evals-ab --sub-configs none --steps 20 --warmup 5 --instrument-plies 1"
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
      -d "$OUT/pmc_${CONFIG:-c2}_$i" -o run -- python bench.py $ARGS > "$OUT/pmc_${CONFIG:-c2}_$i.json" 2> "$OUT/pmc_${CONFIG:-c2}_$i.err"
  rc=$?; echo "pmc ${CONFIG:-c2} pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
