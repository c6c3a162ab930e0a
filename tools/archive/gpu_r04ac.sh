#!/bin/bash
# r04ac: the task queue's longest-predicted-first group order (RVZ_PLAY_ORDER=1, k_play_order)
# — fused parity tests with it on, a same-box A/B in the driver's 20-ply window and over 60 plies,
# then the phase split (timing build) of both orders. Libraries built from
# tools/patches/play_order_lpt.patch (tools/ab_lib_build.sh order "" ptimeo -DRVZ_PLAY_TIMING)
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
export RVZ_LIB=$PWD/tools/_ab/librvz_order.so
RVZ_PLAY_ORDER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_play.py tests/test_gpu_play_oracle.py tests/test_gpu_table.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_r04ac.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu_r04ac.log"; [ $rc -ne 0 ] && exit $rc
ab() {   # tag args rounds
  for r in $(seq 1 $3); do
    for o in 0 1; do
      RVZ_PLAY_ORDER=$o timeout -k 10 300 python bench.py --no-cpu-baseline --sub-configs none --no-evals-ab $2 > "$OUT/abo_$o.json" 2> "$OUT/abo_$o.err"
      rc=$?; [ $rc -ne 0 ] && { echo "[order $o] rc=$rc"; tail -3 "$OUT/abo_$o.err"; exit $rc; }
      python - "$OUT/abo_$o.json" "order$o" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[0])
print(f"[{sys.argv[2]}] round {sys.argv[3]}  {d['value']:.0f}  ms/launch {d['roofline']['avg_ms_per_launch']}  rows/ply {d['nn_rows_per_ply']}", flush=True)
PY
    done
  done
}
ab 20 "--steps 20 --warmup 5" 3 > "$OUT/r04ac_ab_order_20.txt" 2>&1; rc=$?; cat "$OUT/r04ac_ab_order_20.txt"; [ $rc -ne 0 ] && exit $rc
ab 60 "--steps 60 --warmup 3" 2 > "$OUT/r04ac_ab_order_60.txt" 2>&1; rc=$?; cat "$OUT/r04ac_ab_order_60.txt"; [ $rc -ne 0 ] && exit $rc
for o in 0 1; do
  RVZ_PLAY_ORDER=$o RVZ_LIB=$PWD/tools/_ab/librvz_ptimeo.so TABLE=1 timeout -k 10 200 python tools/exp_play_phases.py \
      > "$OUT/r04ac_play_phases_order$o.json" 2> "$OUT/r04ac_play_phases_order$o.err"
  rc=$?; echo "phases order=$o rc=$rc"; [ $rc -ne 0 ] && exit $rc
  head -c 1500 "$OUT/r04ac_play_phases_order$o.json"; echo
done
