#!/bin/bash
# r04w: last-ply half tasks (RVZ_PLAY_SPLIT_LAST) — fused parity tests, then a same-box A/B in the
# driver's 20-ply window and the 60-ply window
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_play.py tests/test_gpu_play_oracle.py tests/test_gpu_table.py tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_r04w.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu_r04w.log"; [ $rc -ne 0 ] && exit $rc
LIBS="s0=tools/_ab/librvz_split0.so;s1=alphazero-reversi_amd/rvz/librvz.so" ARGS="--steps 20 --warmup 5" R=3 bash tools/gpu_ab_libs_r04.sh > "$OUT/r04w_ab_split_last_20.txt" 2>&1
rc=$?; cat "$OUT/r04w_ab_split_last_20.txt"; [ $rc -ne 0 ] && exit $rc
LIBS="s0=tools/_ab/librvz_split0.so;s1=alphazero-reversi_amd/rvz/librvz.so" ARGS="--steps 60 --warmup 3" R=2 bash tools/gpu_ab_libs_r04.sh > "$OUT/r04w_ab_split_last_60.txt" 2>&1
rc=$?; cat "$OUT/r04w_ab_split_last_60.txt"; exit $rc
