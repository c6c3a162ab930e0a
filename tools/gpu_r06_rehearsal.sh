#!/bin/bash
# bench.py --gpus 2 / 4 rehearsals (gloo ranks sharing the one card; the
# driver's SCALE runs use nccl = RCCL on 8 GPUs) with the rank-local stagger: every rank's
# nn_rows_per_ply and value should agree. SERIAL=1: --serial-ranks (the ranks take turns on the
# card, so per-rank values compare the shards). Output: gpurun_out/r06reh/bench_<n>rank_gloo*.json.
set -u
out=gpurun_out/r06reh
mkdir -p "$out"
sfx=""; extra=""
if [ "${SERIAL:-0}" = 1 ]; then sfx="_serial"; extra="--serial-ranks"; fi
for n in ${RANKS:-4 2}; do
    games=${GAMES_PER_RANK:-$((2048 / n))}
    f="$out/bench_${n}rank_gloo$sfx"
    timeout -k 10 400 python bench.py --gpus "$n" --dist-backend gloo --games "$games" \
        --steps "${STEPS:-60}" --warmup 5 --no-cpu-baseline $extra > "$f.json" 2> "$f.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$n ranks failed rc=$rc"; exit $rc; fi
    python - "$f.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["ranks"]
print(d["n_gpus"], "ranks: value", d["value"], "spread",
      {k: v["max_over_min"] for k, v in r["spread"].items()})
for p in r["per_rank"]:
    print("  rank", p["rank"], "value", p["value"], "rows/ply", p["nn_rows_per_ply"],
          "table hits/ply", p.get("table_hits_per_ply"), "stagger", p.get("stagger_plies"))
EOF
done
