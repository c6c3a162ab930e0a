#!/bin/bash
# Round 5: (1) the new GPU tests (C3 bench form at full size, -16 groups, table capture refusal,
# records need hist), (2) a 2-rank gloo rehearsal on one GPU with the per-rank report, (3) PMC
# passes of the C2 / C3 / C5 bench forms (fabric bytes, clock, MFMA busy, L2) for the
# sub-config rooflines. Every step under its own time limit, chained.
set -u
OUT=${OUT:-gpurun_out/r05b}; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
      tests/test_gpu_play_oracle.py::test_k_play_c3_bench_form_at_full_size \
      "tests/test_gpu_play.py::test_fused_other_geometries" \
      tests/test_gpu_table.py::test_table_blob_switch_is_refused_inside_a_capture \
      tests/test_gpu_table.py::test_play_records_need_hist > "$OUT/pytest_new.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_new.log"; [ $rc -ne 0 ] && exit $rc
fi
if [ -z "${NO2RANK:-}" ]; then
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 2 --dist-backend gloo --games 1024 --steps 20 --warmup 2 \
      --no-evals-ab > "$OUT/bench_2rank_gloo.json" 2> "$OUT/bench_2rank_gloo.err"
  rc=$?; echo "2rank rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
for CFG in ${CFGS:-c2 c3 c5}; do
  ARGS="--config $CFG --no-cpu-baseline --no-evals-ab --sub-configs none --steps 20 --warmup 5 --instrument-plies 1"
  i=0
  for CTRS in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
              "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i+1))
    timeout -k 10 -s KILL 400 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$OUT/pmc_${CFG}_$i" -o run \
        -- python bench.py $ARGS > "$OUT/pmc_${CFG}_$i.json" 2> "$OUT/pmc_${CFG}_$i.err"
    rc=$?; echo "pmc $CFG pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
