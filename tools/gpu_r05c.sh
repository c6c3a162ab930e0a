#!/bin/bash
# Round 5 iteration run: the whole GPU test suite, smoke, the driver's bench command (N = 1,
# with C3 / C5 sub-configs), and a 2-rank gloo rehearsal on one GPU (per-rank report).
set -u
OUT=${OUT:-gpurun_out/r05c}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 600 --timeout-method thread -m gpu \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err"
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
python -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('C2', d['value'], 'C3', d['configs']['c3']['value'], 'C5', d['configs']['c5']['value'])"
if [ -z "${NO2RANK:-}" ]; then
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 2 --dist-backend gloo --games 1024 --steps 20 --warmup 2 \
      --no-evals-ab > "$OUT/bench_2rank_gloo.json" 2> "$OUT/bench_2rank_gloo.err"
  rc=$?; echo "2rank rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
exit 0
