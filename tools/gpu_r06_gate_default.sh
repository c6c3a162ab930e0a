#!/bin/bash
# The pass gate as the 10x128 default (rvz_play_gate): its tests, then C3's bench form with the
# default against --play-gate off, alternating on one box. Output: gpurun_out/r06gd/.
set -u
out=gpurun_out/r06gd
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread \
    tests/test_gpu_play.py -k "gate or other_geometries" > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$out/pytest.log"; [ $rc -ne 0 ] && exit $rc
for i in $(seq 1 "${PAIRS:-2}"); do
    for v in default off; do
        timeout -k 10 240 python bench.py --config c3 --steps 20 --warmup 1 --no-cpu-baseline \
            --sub-configs none --play-gate "$v" > "$out/$v.$i.json" 2> "$out/$v.$i.err"
        rc=$?; [ $rc -ne 0 ] && { echo "$v $i rc=$rc"; exit $rc; }
        python - "$out/$v.$i.json" "$v" "$i" >> "$out/summary.txt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"gate {sys.argv[2]:>7} run {sys.argv[3]}  c3 {d['value']:.1f}  k_play ms "
      f"{r.get('avg_ms_per_launch')}  frac {r.get('frac')}  useful {r.get('useful_frac')}")
PY
        tail -n 1 "$out/summary.txt"
    done
done
