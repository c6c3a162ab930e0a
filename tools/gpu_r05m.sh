#!/bin/bash
# Round 5: the 10x128 two-board k_play (8-wave workgroups, RVZ_PLAY_C3_BOARDS 2): the tests that
# run k_play at F = 128 (oracle, pull-style equality, C4 records, table), then the C3 bench form
# A/B against the one-board build (tools/_ab/librvz_c3nb1.so), alternating.
set -u
OUT=${OUT:-gpurun_out/r05m}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_play.py tests/test_gpu_play_oracle.py tests/test_gpu_pipeline.py \
    tests/test_gpu_table.py > "$OUT/pytest_c3.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_c3.log"; [ $rc -ne 0 ] && exit $rc
OUT=$OUT CFGS="c3" VARIANTS="tools/_ab/librvz_c3nb1.so" bash tools/gpu_r05e.sh
