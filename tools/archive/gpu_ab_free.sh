#!/bin/bash
# A/B: 2 lanes joined per ply (one graph) vs free-running lanes (one graph per lane).
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_search.py -x -q -k "lanes" --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pt_free.log" 2>&1 || exit $?
for V in free join free join; do
  F=""; [ $V = join ] && F="--joined-lanes"
  timeout -k 10 300 python bench.py --no-cpu-baseline $F > "$OUT/ab_$V.json" 2> "$OUT/ab_$V.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/ab_$V.json')); print('$V', d['value'], d['ms_per_step'], d['roofline']['avg_ms_per_launch'])"
done
