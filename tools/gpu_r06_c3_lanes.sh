#!/bin/bash
# Round 6: C3 with one vs two game lanes (two concurrent k_play launches of 16,384 games each)
# under the pass gate, alternating on one box. Output: gpurun_out/r06c3l/summary.txt.
set -u
OUT=gpurun_out/r06c3l; mkdir -p "$OUT"
for i in $(seq 1 "${PAIRS:-1}"); do
  for l in 1 2; do
    timeout -k 10 300 python bench.py --config c3 --lanes "$l" --steps 20 --warmup 5 \
        --no-cpu-baseline --sub-configs none --no-evals-ab > "$OUT/l$l.$i.json" 2> "$OUT/l$l.$i.err"
    rc=$?; [ $rc -ne 0 ] && { echo "lanes $l rc=$rc"; exit $rc; }
    python -c "import json; d=json.loads(open('$OUT/l$l.$i.json').read().strip().splitlines()[-1]); print('c3 lanes $l run $i', round(d['value'],1), d['roofline'].get('avg_ms_per_launch'))" | tee -a "$OUT/summary.txt"
  done
done
exit 0
