#!/bin/bash
# Round-4 GPU call: the new parity tests first (fused k_play vs the oracle, budgets, C4 shard),
# smoke, the driver's bench command and the 60-step one (phase-neutral window check), the
# cross-game redundancy measurement. Every GPU step has its own limit; exit > 1 ends the script.
set -u
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r04a}
mkdir -p "$OUT"
step() {   # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@"
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -gt 1 ]; then exit $rc; fi
    return 0
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
if [ -n "${TESTS:-}" ]; then
step pytest_new 1200 $PYT $TESTS > "$OUT/pytest_new_$TAG.log" 2>&1
tail -3 "$OUT/pytest_new_$TAG.log"
fi
if [ -n "${SMOKE:-}" ]; then
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
tail -2 "$OUT/smoke_$TAG.log"
fi
if [ -n "${BENCH:-}" ]; then
step bench20 500 python bench.py --steps 20 --warmup 5 > "$OUT/bench20_$TAG.json" 2> "$OUT/bench20_$TAG.err"
step bench60 500 python bench.py --no-evals-ab --sub-configs none --no-cpu-baseline > "$OUT/bench60_$TAG.json" 2> "$OUT/bench60_$TAG.err"
fi
if [ -n "${XGAME:-}" ]; then
step xgame 400 python tools/exp_xgame.py --plies 180 --out "$OUT/xgame_$TAG.json" > "$OUT/xgame_$TAG.log" 2>&1
fi
echo round-done
