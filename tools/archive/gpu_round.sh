#!/bin/bash
# One GPU validation round on the MI355X box: parity tests, smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; a crash/timeout (exit > 1) ends the script there.
set -u
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r01}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest_rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke_rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench \
    -- python bench.py --no-cpu-baseline > "$OUT/bench_prof_$TAG.json" 2> "$OUT/bench_prof_$TAG.err"
rc=$?; echo "prof_rc=$rc"; exit $rc
