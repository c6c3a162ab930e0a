#!/bin/bash
# Round 6: C2's task-queue group size (bench.py --play-group -g) re-checked on the final code,
# alternating on one box. Output: gpurun_out/r06c2g/summary.txt.
set -u
OUT=gpurun_out/r06c2g; mkdir -p "$OUT"
for i in $(seq 1 "${PASSES:-2}"); do
  for g in ${GROUPS_C2:--6 -4 -5 -7 -8}; do
    timeout -k 10 200 python bench.py --config c2 --play-group "$g" --steps 20 --warmup 5 \
        --no-cpu-baseline --sub-configs none --no-evals-ab > "$OUT/g$g.$i.json" 2> "$OUT/g$g.$i.err"
    rc=$?; [ $rc -ne 0 ] && { echo "group $g rc=$rc"; exit $rc; }
    python -c "import json; d=json.loads(open('$OUT/g$g.$i.json').read().strip().splitlines()[-1]); print('c2 group $g run $i', round(d['value'],1), d['roofline'].get('avg_ms_per_launch'))" | tee -a "$OUT/summary.txt"
  done
done
exit 0
