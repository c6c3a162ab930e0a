#!/bin/bash
# C5 (6x6, 16,384 games, 400 sims): the cross-game table's disc limit (--table-discs) and slot
# count, alternating on one box. Output: gpurun_out/r06c5/.
set -u
out=gpurun_out/r06c5; mkdir -p "$out"
for i in 1 2; do
  for v in ${VARIANTS:-"14:20" "16:20" "18:20" "20:21" "24:22"}; do
    d=${v%%:*}; sl=${v##*:}
    timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline \
        --sub-configs none --no-evals-ab --table-discs "$d" --table-slots $((1 << sl)) \
        > "$out/d$d.s$sl.$i.json" 2> "$out/d$d.s$sl.$i.err"
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; exit $rc; }
    python -c "import json; d=json.loads(open('$out/d$d.s$sl.$i.json').read().strip().splitlines()[-1]); t=d.get('table') or {}; print('discs $d slots 2^$sl run $i', round(d['value']), d['nn_rows_per_ply'], t.get('hits_per_ply'))"
  done
done
