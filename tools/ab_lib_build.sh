#!/bin/bash
# Build whole-library variants of librvz.so (engine + evaluator) for tools/gpu_ab_lib.sh /
# tools/gpu_ab_multi_lib.sh, here on the CPU:
#   tools/ab_lib_build.sh name1 "-DFLAG=1" name2 "-DFLAG=2" ...   -> tools/_ab/librvz_<name>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_ab
while [ $# -ge 2 ]; do
  make -s -C alphazero-reversi_amd OUT="$PWD/tools/_ab/librvz_$1.so" BUILD="build/ab_$1" EXTRA="$2" &
  shift 2
done
wait
