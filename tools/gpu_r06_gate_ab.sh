#!/bin/bash
# the per-XCD pass gate (csrc/rvz_play.hip.h play_gate, RVZ_PLAY_GATE="k,us")
# on C3's fused launch, alternating with the gate off on ONE box. Output:
# gpurun_out/r06gate/<variant>.<i>.json and summary.txt.
set -u
out=gpurun_out/r06gate
mkdir -p "$out"
variants=${VARIANTS:-"off 2,10 4,25 8,50 64,100"}
pairs=${PAIRS:-2}
for i in $(seq 1 "$pairs"); do
    for v in $variants; do
        gate="$v"     # RVZ_PLAY_GATE: "fraction,us,late_us" (round 6 first form: "k,us[,late]"), "off"
        RVZ_PLAY_GATE="$gate" timeout -k 10 240 python bench.py --config c3 --steps 20 \
            --warmup 1 --no-cpu-baseline --sub-configs none > "$out/$v.$i.json" 2> "$out/$v.$i.err"
        rc=$?
        if [ $rc -ne 0 ]; then echo "$v run $i failed rc=$rc"; exit $rc; fi
        python - "$out/$v.$i.json" "$v" "$i" >> "$out/summary.txt" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"gate {sys.argv[2]:>6} run {sys.argv[3]}  c3 {d['value']:.1f}  k_play ms "
      f"{r.get('avg_ms_per_launch')}  frac {r.get('frac')}  rows/ply {d.get('nn_rows_per_ply')}")
EOF
        tail -n 1 "$out/summary.txt"
    done
done
