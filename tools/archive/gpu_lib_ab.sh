#!/bin/bash
# bench.py under prebuilt full-library variants (tools/_ab/librvz_full_<name>.so via RVZ_LIB),
# alternating, on one box:   bash tools/gpu_lib_ab.sh "<bench args>" name1 name2 ...
set -u
mkdir -p gpurun_out
ARGS=$1; shift
for rep in 1 2; do
  for V in "$@"; do
    RVZ_LIB=$PWD/tools/_ab/librvz_full_$V.so timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline \
        > gpurun_out/libab_${V}_$rep.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/libab_${V}_$rep.json')); print('$V', d['value'], d['ms_per_step'], d['kernels']['step']['avg_us'])"
  done
done
