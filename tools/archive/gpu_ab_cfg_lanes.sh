#!/bin/bash
# lanes A/B per config (free-running lanes); every GPU step has its own limit.
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > "$OUT/abl_$n.json" 2> "$OUT/abl_$n.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/abl_$n.json')); print('$n', d['value'], d['ms_per_step'])"
}
run c2_l2 --lanes 2
run c2_l4 --lanes 4
run c2_l2b --lanes 2
run c2_l4b --lanes 4
run c5_l1 --config c5 --lanes 1 --steps 30
run c5_l2 --config c5 --lanes 2 --steps 30
run c5_l4 --config c5 --lanes 4 --steps 30
run c3_l1 --config c3 --lanes 1 --steps 8
run c3_l2 --config c3 --lanes 2 --steps 8
