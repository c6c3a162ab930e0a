#!/bin/bash
# C3 (8x8, 32,768 games, 10x128, 800 sims): the cross-game table's disc limit (--table-discs)
# and slot count, one run each (PASSES to repeat), one box. Output: gpurun_out/r06c3t/.
set -u
out=gpurun_out/r06c3t; mkdir -p "$out"
for i in $(seq 1 "${PASSES:-1}"); do
  for v in ${VARIANTS:-"14:20" "18:21" "22:22"}; do
    d=${v%%:*}; sl=${v##*:}
    timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline \
        --sub-configs none --no-evals-ab --table-discs "$d" --table-slots $((1 << sl)) \
        > "$out/d$d.s$sl.$i.json" 2> "$out/d$d.s$sl.$i.err"
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; exit $rc; }
    python -c "import json; d=json.loads(open('$out/d$d.s$sl.$i.json').read().strip().splitlines()[-1]); t=d.get('table') or {}; print('discs $d slots 2^$sl run $i', round(d['value']), d['nn_rows_per_ply'], t.get('hits_per_ply'))" | tee -a "$out/summary.txt"
  done
done
