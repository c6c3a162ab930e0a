#!/bin/bash
# C3 (32,768 games, 10x128): the pull-style preset vs the fused launch (+ table) at a few group
# sizes; 20 timed plies after the stagger and 3 warm-up launches. Outputs one line per variant.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r04d}
C="python bench.py --config c3 --steps 20 --warmup 3 --no-evals-ab --no-cpu-baseline --sub-configs none"
run() { local name=$1; shift
  timeout -k 10 300 $C "$@" > "$OUT/c3ab_${TAG}_$name.json" 2> "$OUT/c3ab_${TAG}_$name.err"
  local rc=$?; echo "$name rc=$rc"; [ $rc -gt 1 ] && exit $rc
  python - "$OUT/c3ab_${TAG}_$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[0])
print(f"[{sys.argv[2]}] {d['value']:.0f} board-steps/s  rows/ply {d['nn_rows_per_ply']}  table {d.get('table')}  roof {d['roofline']['avg_ms_per_launch']} ms frac {d['roofline']['frac']}")
PY
}
[ -z "${NOPULL:-}" ] && run pull
for g in ${GRPS:-0 -2 -8}; do run fused$g --fused --play-group $g; done
echo done
