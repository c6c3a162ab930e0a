#!/bin/bash
# One kernel-iteration round on the MI355X box: evaluator parity tests, a short bench, and (with
# PMC=1) the LDS / MFMA counter passes of the trunk kernel. Each GPU step has its own time limit;
# the script stops at the first failing step.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-it}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_network.py ${TESTS:-} -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/net_$TAG.log" 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -2 "$OUT/net_$TAG.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ "${PMC:-0}" = 1 ]; then
  export TMPDIR=/tmp
  i=0
  for CTRS in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
              "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
        -d "$OUT/pmc_${TAG}_$i" -o run -- python tools/exp_resnet_pmc.py 6 64 h2 \
        > "$OUT/pmc_${TAG}_$i.log" 2>&1
    rc=$?; echo "pmc $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
fi
exit 0
