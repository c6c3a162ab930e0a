#!/bin/bash
# GPU_MAX_HW_QUEUES=8 (HIP hardware queues per process; the box default is 4) with 2 / 4 / 6
# lanes, then rocprofv3 kernel stats of the 4-lane bench under the same setting.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r03h}
mkdir -p "$OUT"
A="--no-cpu-baseline --sub-configs none --no-evals-ab ${BENCH_ARGS:-}"
export GPU_MAX_HW_QUEUES=${HWQ:-8}
for r in 1 2; do
for L in 2 4 6; do
timeout -k 10 200 python bench.py $A --lanes $L > "$OUT/hwq_lanes${L}_${r}_$TAG.json" 2> "$OUT/hwq_lanes${L}_${r}_$TAG.err"
rc=$?; [ $rc -ne 0 ] && { echo "lanes $L rc=$rc"; exit $rc; }
python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('hwq',$GPU_MAX_HW_QUEUES,'lanes',$L,'round',$r,d['value'],d['roofline']['avg_ms_per_launch'],d['roofline']['timed_region_trunk_frac'])" "$OUT/hwq_lanes${L}_${r}_$TAG.json" | tee -a "$OUT/hwq_$TAG.txt"
done; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_hwq_$TAG" -o bench \
    -- python bench.py $A --lanes 4 > "$OUT/bench_prof_hwq_$TAG.json" 2> "$OUT/bench_prof_hwq_$TAG.err"
rc=$?; echo "prof_rc=$rc"
python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('under rocprof', d['value'],d['roofline']['avg_ms_per_launch'])" "$OUT/bench_prof_hwq_$TAG.json"
exit $rc
