#!/bin/bash
# Round 5: the ranged re-run called with by-value arguments: the range tests, then C1 and the
# fused C2 / C5 bench forms against the pre-range library, alternating.
set -u
OUT=${OUT:-gpurun_out/r05r}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_network.py tests/test_gpu_selfplay_parity.py -x -v \
    --timeout 200 --timeout-method thread -m gpu -k "range or large_activation or aggressive" \
    > "$OUT/pytest_range.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest_range.log"; [ $rc -ne 0 ] && exit $rc
OUT=$OUT NOISO=1 bash tools/gpu_r05p.sh || exit $?
OUT=$OUT CFGS="c2 c5" bash tools/gpu_r05e.sh
