#!/bin/bash
# r04ab: the FC heads' tiles as independent MFMA chains with their bias / fc2 operands loaded up
# front (RVZ_HEADS_CHAINS 1, the in-tree build) — fused parity tests, a same-box A/B against
# the one-chain heads (tools/_ab/librvz_chains0.so), then the phase split of both (timing builds).
# The knob was not kept (profiles/r04ab_*): rebuilding these libraries needs that patch.
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_play.py tests/test_gpu_play_oracle.py tests/test_gpu_table.py tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_r04ab.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu_r04ab.log"; [ $rc -ne 0 ] && exit $rc
LIBS="c0=tools/_ab/librvz_chains0.so;c1=alphazero-reversi_amd/rvz/librvz.so" ARGS="--steps 20 --warmup 5" R=3 bash tools/gpu_ab_libs_r04.sh > "$OUT/r04ab_ab_heads_chains.txt" 2>&1
rc=$?; cat "$OUT/r04ab_ab_heads_chains.txt"; [ $rc -ne 0 ] && exit $rc
for v in ptime0 ptime; do
  RVZ_LIB=tools/_ab/librvz_$v.so TABLE=1 timeout -k 10 200 python tools/exp_play_phases.py \
      > "$OUT/r04ab_play_phases_$v.json" 2> "$OUT/r04ab_play_phases_$v.err"
  rc=$?; echo "phases $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  head -c 1500 "$OUT/r04ab_play_phases_$v.json"; echo
done
