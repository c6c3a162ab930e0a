#!/bin/bash
# Build compile-time variants of csrc/rvz_resnet.hip for tools/ab_h2.py, here on the CPU:
#   tools/ab_build.sh name1 "-DFLAG=1" name2 "-DFLAG=2" ...   -> tools/_ab/librvz_<name>.so
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
      -fno-gpu-flush-denormals-to-zero $2 -shared -o "tools/_ab/librvz_$1.so" \
      alphazero-reversi_amd/csrc/rvz_resnet.hip &
  shift 2
done
wait
