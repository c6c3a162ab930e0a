#!/bin/bash
# PMC passes for the HBM traffic of the rvz kernels: one counter group per run, kernel trace only.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r01}
mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS="--no-cpu-baseline --instrument-plies 1 --no-evals-ab --sub-configs none ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_$TAG" -o run \
    -- python bench.py $ARGS > "$OUT/pmc_fetch_$TAG.json" 2> "$OUT/pmc_fetch_$TAG.err"
rc=$?; echo "fetch_rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_$TAG" -o run \
    -- python bench.py $ARGS > "$OUT/pmc_write_$TAG.json" 2> "$OUT/pmc_write_$TAG.err"
rc=$?; echo "write_rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/pmc_summary.py "$OUT/pmc_fetch_$TAG" "$OUT/pmc_write_$TAG" "$OUT/pmc_traffic_$TAG.json"
