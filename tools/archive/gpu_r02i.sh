#!/bin/bash
# PMC traffic passes of the current build, C1 line, roctx marker timeline, C4 2-rank rehearsal.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r02i}
mkdir -p "$OUT"; export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -gt 1 ] && exit $rc; return 0; }
OUT=$OUT TAG=$TAG step pmc 700 bash tools/gpu_pmc.sh
step bench_c1 300 python bench.py --config c1 > "$OUT/bench_c1_$TAG.json" 2> "$OUT/bench_c1_$TAG.err"
RVZ_ROCTX=1 step trace 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
    -d "$OUT/trace_$TAG" -o run -- python tools/trace_plies.py 3 > "$OUT/trace_$TAG.log" 2>&1
step c4_2rank 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --config c4 --gpus 2 --dist-backend gloo --games 1024 \
    > "$OUT/bench_c4_2rank_$TAG.json" 2> "$OUT/bench_c4_2rank_$TAG.err"
echo round-done
