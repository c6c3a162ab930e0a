#!/bin/bash
# Round-4 record: GPU tests, smoke, the driver's exact bench command and the 60-ply window, the
# rocprofv3 kernel trace + stats of the driver's command, the HBM traffic passes, C4 and C1.
# Every GPU step has its own limit; exit > 1 ends the script.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r04g}; mkdir -p "$OUT"; export TMPDIR=/tmp
step() {   # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@"
    local rc=$?
    echo "$name rc=$rc" >&2
    if [ $rc -gt 1 ]; then exit $rc; fi
    return 0
}
if [ -z "${NOTESTS:-}" ]; then
step pytest 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
tail -1 "$OUT/pytest_gpu_$TAG.log" >&2
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
fi
step bench20 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20_$TAG.json" 2> "$OUT/bench20_$TAG.err"
step bench60 600 python3 bench.py > "$OUT/bench60_$TAG.json" 2> "$OUT/bench60_$TAG.err"
step prof20 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20_prof_$TAG.json" 2> "$OUT/bench20_prof_$TAG.err"
if [ -z "${NOTRAFFIC:-}" ]; then
OUT=$OUT TAG=$TAG BENCH_ARGS="--steps 20 --warmup 5" step traffic 400 bash tools/gpu_pmc.sh >&2
fi
if [ -z "${NOC4:-}" ]; then
step c4 600 python3 bench.py --config c4 > "$OUT/bench_c4_$TAG.json" 2> "$OUT/bench_c4_$TAG.err"
step c1 300 python3 bench.py --config c1 > "$OUT/bench_c1_$TAG.json" 2> "$OUT/bench_c1_$TAG.err"
fi
echo record-done >&2
