#!/bin/bash
# Round 6: pass-gate settings on C3's workload with a 10x256 net (bench.py --play-gate
# fraction,us,late_us), one run each in order, one box. Output: gpurun_out/r06g256s/summary.txt.
set -u
OUT=gpurun_out/r06g256s; mkdir -p "$OUT"
for g in ${GATES:-default 1.0,800,400 0.8,800,400 0.9,400,200 0.6,400,200 default}; do
    tag=${g//,/_}
    timeout -k 10 300 python bench.py --config c3 --filters 256 --steps 10 --warmup 3 \
        --no-cpu-baseline --sub-configs none --no-evals-ab --play-gate "$g" \
        > "$OUT/$tag.json" 2> "$OUT/$tag.err"
    rc=$?; [ $rc -ne 0 ] && { echo "$g rc=$rc"; exit $rc; }
    python -c "import json; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('gate $g', round(d['value'],1), r.get('avg_ms_per_launch'), r.get('frac'))" | tee -a "$OUT/summary.txt"
done
exit 0
