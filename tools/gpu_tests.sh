#!/bin/bash
# GPU parity tests only (one process, per-test timeout); log under gpurun_out/.
set -u
OUT=${OUT:-gpurun_out}
TAG=${TAG:-t}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 "$OUT/pytest_gpu_$TAG.log"; exit $rc
