#!/bin/bash
# r04aa: FC-head value weights issued before the last pass's head convs (RVZ_PLAY_HEADS_PRE=1,
# tools/_ab/librvz_pre1.so) against the in-tree build in the driver's 20-ply window, then the
# two-rank gloo rehearsal of bench.py on the one GPU
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
LIBS="pre0=alphazero-reversi_amd/rvz/librvz.so;pre1=tools/_ab/librvz_pre1.so" ARGS="--steps 20 --warmup 5" R=3 bash tools/gpu_ab_libs_r04.sh > "$OUT/r04aa_ab_heads_pre.txt" 2>&1
rc=$?; cat "$OUT/r04aa_ab_heads_pre.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --games 1024 --steps 20 --warmup 2 > "$OUT/r04aa_bench_2rank_gloo_1gpu.json" 2> "$OUT/r04aa_bench_2rank.err"
rc=$?; echo "2rank rc=$rc"; cat "$OUT/r04aa_bench_2rank_gloo_1gpu.json"; tail -3 "$OUT/r04aa_bench_2rank.err"; exit $rc
