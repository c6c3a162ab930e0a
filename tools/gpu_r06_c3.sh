#!/bin/bash
# Round 6: C3 with the pass gate on by default — (1) the PMC passes of its bench form (FETCH_SIZE,
# WRITE_SIZE, GRBM_GUI_ACTIVE + MFMA busy, caches) for the stored roofline.traffic
# (tools/pmc_play_traffic.py merges them into profiles/pmc_traffic.json afterwards, in the
# container), (2) C3's queue group size re-checked under the gate, (3) C4 (10x128 self-play +
# DDP training, the gate applies to its fused launch too). Every step under its own limit.
set -u
OUT=${OUT:-gpurun_out/r06c3}; mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS="--config c3 --no-cpu-baseline --no-evals-ab --sub-configs none --steps 20 --warmup 5 --instrument-plies 1"
if [ -z "${NOPMC:-}" ]; then
  i=0
  for CTRS in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
              "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i+1))
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv \
        -d "$OUT/pmc_c3_$i" -o run -- python bench.py $ARGS > "$OUT/pmc_c3_$i.json" 2> "$OUT/pmc_c3_$i.err"
    rc=$?; echo "pmc c3 pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
fi
if [ -z "${NOGROUPS:-}" ]; then
  for g in ${GROUPS_C3:--16 -8 -24 -32 -16}; do
    timeout -k 10 240 python bench.py --config c3 --steps 20 --warmup 1 --no-cpu-baseline \
        --sub-configs none --play-group "$g" > "$OUT/group$g.json" 2> "$OUT/group$g.err"
    rc=$?; [ $rc -ne 0 ] && { echo "group $g rc=$rc"; exit $rc; }
    python -c "import json,sys; d=json.loads(open('$OUT/group$g.json').read().strip().splitlines()[-1]); print('group $g', round(d['value'],1), d['roofline']['avg_ms_per_launch'])"
  done
fi
if [ -z "${NOC4:-}" ]; then
  timeout -k 10 600 python bench.py --config c4 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
  rc=$?; echo "c4 rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python -c "import json; d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1]); print('c4', d['value'], d.get('ms_per_step'))"
fi
exit 0
