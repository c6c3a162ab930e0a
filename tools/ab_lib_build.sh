#!/bin/bash
# Build whole-library variants of librvz.so (engine + evaluator) for tools/gpu_ab_lib.sh /
# tools/gpu_ab_multi_lib.sh, here on the CPU:
#   tools/ab_lib_build.sh name1 "-DFLAG=1" name2 "-DFLAG=2" ...   -> tools/_ab/librvz_<name>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_ab
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
      -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt $2 -shared \
      -o "tools/_ab/librvz_$1.so" alphazero-reversi_amd/csrc/rvz_engine.hip \
      alphazero-reversi_amd/csrc/rvz_resnet.hip -ldl &
  shift 2
done
wait
