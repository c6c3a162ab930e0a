#!/bin/bash
# Round-3 GPU validation: parity tests, smoke, the default bench line (C2 + C3/C5 sub-objects),
# a 2-rank launcher rehearsal on the one GPU (gloo), and rocprofv3 kernel stats of the C2 bench.
# Every GPU step has its own time limit; a crash/timeout ends the script there.
set -u
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r03}
STEPS=${STEPS:-all}
mkdir -p "$OUT"
if [[ $STEPS == all || $STEPS == *tests* ]]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 "$OUT/pytest_gpu_$TAG.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke_rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench_rc=$rc"; cat "$OUT/bench_$TAG.json" | cut -c1-400; [ $rc -ne 0 ] && exit $rc
fi
if [[ $STEPS == all || $STEPS == *rehearsal* ]]; then
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --games 1024 --no-cpu-baseline > "$OUT/bench_2rank_$TAG.json" 2> "$OUT/bench_2rank_$TAG.err"
rc=$?; echo "rehearsal_rc=$rc"; grep '^{' "$OUT/bench_2rank_$TAG.json" | cut -c1-300; [ $rc -ne 0 ] && exit $rc
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench \
    -- python bench.py --no-cpu-baseline --sub-configs none --no-evals-ab ${BENCH_ARGS:-} > "$OUT/bench_prof_$TAG.json" 2> "$OUT/bench_prof_$TAG.err"
rc=$?; echo "prof_rc=$rc"; exit $rc
fi
