#!/bin/bash
# r04n: GPU parity tests on the W128 epilogue build, then a same-box whole-bench A/B against the
# ds_write_b64 epilogue (tools/_ab/librvz_base.so), then the SQ PMC passes of the new build.
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_r04n.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu_r04n.log"; [ $rc -ne 0 ] && exit $rc
LIBS="base=tools/_ab/librvz_base.so;w128=alphazero-reversi_amd/rvz/librvz.so" R=3 bash tools/gpu_ab_libs_r04.sh > "$OUT/r04n_ab_w128.txt" 2>&1
rc=$?; cat "$OUT/r04n_ab_w128.txt"; [ $rc -ne 0 ] && exit $rc
TAG=r04n bash tools/gpu_play_pmc.sh
