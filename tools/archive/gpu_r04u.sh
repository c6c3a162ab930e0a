#!/bin/bash
# r04u: packed-fp32 epilogue (RVZ_H2_PK) — the k_play / trunk parity tests, then a same-box A/B
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_play.py tests/test_gpu_play_oracle.py tests/test_gpu_network.py tests/test_gpu_table.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_r04u.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu_r04u.log"; [ $rc -ne 0 ] && exit $rc
LIBS="pk0=tools/_ab/librvz_pk0.so;pk1=alphazero-reversi_amd/rvz/librvz.so" ARGS="--steps 20 --warmup 5" R=3 bash tools/gpu_ab_libs_r04.sh > "$OUT/r04u_ab_pk.txt" 2>&1
rc=$?; cat "$OUT/r04u_ab_pk.txt"; exit $rc
