#!/bin/bash
# r04ad: the committed code's GPU tests and smoke (in-tree librvz.so), then the longest-first
# task order experiment (tools/archive/gpu_r04ac.sh, variant libraries)
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_r04ad.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu_r04ad.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_r04ad.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke_r04ad.log"; [ $rc -ne 0 ] && exit $rc
bash tools/archive/gpu_r04ac.sh
