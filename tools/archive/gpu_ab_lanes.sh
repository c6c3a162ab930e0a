#!/bin/bash
# A/B of lanes (and the other configs) on one box; every GPU step has its own time limit.
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
for L in 1 2 4 2 1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --lanes $L > "$OUT/lanes_$L.json" 2> "$OUT/lanes_$L.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/lanes_$L.json')); print('lanes', $L, d['value'], d['ms_per_step'])"
done
for C in c5 c3; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --config $C --steps 20 > "$OUT/cfg_$C.json" 2> "$OUT/cfg_$C.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/cfg_$C.json')); print('$C', d['value'], d['ms_per_step'], d['roofline'].get('live_rows_per_launch_timed'))"
done
