#!/bin/bash
# Same-box A/B of two librvz.so builds under the current Python tree (RVZ_LIB selects the
# library; the C-ABI is unchanged between them): "pre" = tools/_ab/librvz_<PRE>.so, "cur" = the
# in-tree build, alternating, for each config in CONFIGS. Output: gpurun_out/<OUT>/summary.txt.
#   PRE=r06pre CONFIGS="c3 c5" PAIRS=2 bash tools/gpu_r06_ab_lib.sh
set -u
OUT=gpurun_out/${OUT:-r06ablib}
mkdir -p "$OUT"
PRE=${PRE:-r06pre}
pre_lib=$(pwd)/tools/_ab/librvz_$PRE.so
[ -f "$pre_lib" ] || { echo "missing $pre_lib"; exit 2; }
for c in ${CONFIGS:-c3 c5}; do
    for i in $(seq 1 "${PAIRS:-2}"); do
        for t in pre cur; do
            if [ "$t" = pre ]; then export RVZ_LIB="$pre_lib"; else unset RVZ_LIB; fi
            timeout -k 10 300 python bench.py --config "$c" --steps 20 --warmup 5 \
                --no-cpu-baseline --sub-configs none > "$OUT/$c.$t.$i.json" 2> "$OUT/$c.$t.$i.err"
            rc=$?
            if [ $rc -ne 0 ]; then echo "$c $t run $i failed rc=$rc"; exit $rc; fi
            python - "$OUT/$c.$t.$i.json" "$c" "$t" "$i" >> "$OUT/summary.txt" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]} {sys.argv[3]} run {sys.argv[4]}  {d['value']:.1f}  "
      f"k_play ms {d['roofline'].get('avg_ms_per_launch')}")
EOF
            tail -n 1 "$OUT/summary.txt"
        done
    done
done
exit 0
