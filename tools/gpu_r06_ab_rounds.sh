#!/bin/bash
# the round-4 and round-5 final trees (tools/_ab/r4, tools/_ab/r5: git archive
# of ce8bfef / d8d05c9 with their own librvz.so, built in this container) and the current tree,
# alternating on ONE box, each running the driver's command (C2 headline + the C3 / C5
# sub-configs in the same line). Output: gpurun_out/r06ab/<tree>.<i>.json and summary.txt.
set -u
out=gpurun_out/r06ab
mkdir -p "$out"
root=$(pwd)
pairs=${PAIRS:-3}
for i in $(seq 1 "$pairs"); do
    for t in r4 r5 r6; do
        if [ "$t" = r6 ]; then d="$root"; else d="$root/tools/_ab/$t"; fi
        (cd "$d" && timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 \
            --no-cpu-baseline) > "$out/$t.$i.json" 2> "$out/$t.$i.err"
        rc=$?
        if [ $rc -ne 0 ]; then echo "$t run $i failed rc=$rc"; exit $rc; fi
        python - "$out/$t.$i.json" "$t" "$i" >> "$out/summary.txt" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("configs") or {}
print(f"{sys.argv[2]} run {sys.argv[3]}  c2 {d['value']:.1f}  c3 "
      f"{(c.get('c3') or {}).get('value')}  c5 {(c.get('c5') or {}).get('value')}  "
      f"k_play ms {d['roofline'].get('avg_ms_per_launch')}")
EOF
        tail -n 1 "$out/summary.txt"
    done
done
