#!/bin/bash
# Round-6 record: the GPU suite, smoke, the driver's exact bench command, the 60-ply window, and
# the rocprofv3 kernel trace + stats of the driver's command (tools/trace_dispatches.py reconciles
# it with the line afterwards). Every GPU step has its own limit; exit > 1 ends the script.
set -u
OUT=${OUT:-gpurun_out/r06zz}; TAG=${TAG:-r06zz}; mkdir -p "$OUT"; export TMPDIR=/tmp
step() {   # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@"
    local rc=$?
    echo "$name rc=$rc" >&2
    if [ $rc -gt 1 ]; then exit $rc; fi
    return 0
}
if [ -z "${NOTESTS:-}" ]; then
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
tail -1 "$OUT/pytest_gpu_$TAG.log" >&2
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
tail -1 "$OUT/smoke_$TAG.log" >&2
fi
step bench20 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20_$TAG.json" 2> "$OUT/bench20_$TAG.err"
step bench60 400 python3 bench.py > "$OUT/bench60_$TAG.json" 2> "$OUT/bench60_$TAG.err"
step prof20 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20_prof_$TAG.json" 2> "$OUT/bench20_prof_$TAG.err"
echo record-done >&2
