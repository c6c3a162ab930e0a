#!/bin/bash
# Round 6: the 256-filter trunk's weight prefetch distance (RVZ_H2_PD256 1 = in-tree, 2, 3 =
# tools/_ab/librvz_pd{2,3}.so via RVZ_LIB): pull-style evaluator timing (tools/exp_f256.py) and
# C3's workload with a 10x256 net, fused, alternating. Output: gpurun_out/r06pd/summary.txt.
set -u
OUT=gpurun_out/r06pd; mkdir -p "$OUT"
for i in $(seq 1 "${PAIRS:-1}"); do
  for v in 1 2 3; do
    if [ "$v" = 1 ]; then unset RVZ_LIB; else export RVZ_LIB=$(pwd)/tools/_ab/librvz_pd$v.so; fi
    timeout -k 10 200 python tools/exp_f256.py > "$OUT/exp_pd$v.$i.jsonl" 2> "$OUT/exp_pd$v.$i.err"
    rc=$?; [ $rc -ne 0 ] && { echo "exp pd$v rc=$rc"; exit $rc; }
    grep '"h2"' "$OUT/exp_pd$v.$i.jsonl" | sed "s/^/pd$v run $i /" >> "$OUT/summary.txt"
    timeout -k 10 300 python bench.py --config c3 --filters 256 --steps 10 --warmup 3 \
        --no-cpu-baseline --sub-configs none --no-evals-ab > "$OUT/c3_pd$v.$i.json" 2> "$OUT/c3_pd$v.$i.err"
    rc=$?; [ $rc -ne 0 ] && { echo "c3 pd$v rc=$rc"; exit $rc; }
    python -c "import json; d=json.loads(open('$OUT/c3_pd$v.$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('pd$v run $i c3-10x256', round(d['value'],1), r.get('avg_ms_per_launch'), r.get('frac'), (r.get('isolated') or {}).get('frac'))" | tee -a "$OUT/summary.txt"
  done
done
exit 0
