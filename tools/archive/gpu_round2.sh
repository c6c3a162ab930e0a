#!/bin/bash
# GPU round with the extra configurations: parity tests, smoke, C2 bench + rocprof kernel stats,
# C3 (1 and 2 lanes, 60 plies), C1, C5. Each GPU step has its own time limit; a crash or timeout
# (exit > 1) ends the script there. Outputs under gpurun_out/ with the given TAG.
set -u
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r02}
mkdir -p "$OUT"
step() {   # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -gt 1 ]; then exit $rc; fi
    return 0
}
step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
tail -1 "$OUT/pytest_gpu_$TAG.log"
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
step bench_c2 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
export TMPDIR=/tmp
step prof_c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench \
    -- python bench.py --no-cpu-baseline > "$OUT/bench_prof_$TAG.json" 2> "$OUT/bench_prof_$TAG.err"
if [ -z "${SKIP_EXTRA:-}" ]; then
step bench_c3 400 python bench.py --config c3 --no-cpu-baseline > "$OUT/bench_c3_$TAG.json" 2> "$OUT/bench_c3_$TAG.err"
step bench_c3_l2 400 python bench.py --config c3 --lanes 2 --no-cpu-baseline > "$OUT/bench_c3l2_$TAG.json" 2> "$OUT/bench_c3l2_$TAG.err"
step bench_c1 300 python bench.py --config c1 > "$OUT/bench_c1_$TAG.json" 2> "$OUT/bench_c1_$TAG.err"
step bench_c5 300 python bench.py --config c5 --no-cpu-baseline > "$OUT/bench_c5_$TAG.json" 2> "$OUT/bench_c5_$TAG.err"
fi
echo round-done
