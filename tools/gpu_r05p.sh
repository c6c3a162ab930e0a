#!/bin/bash
# Round 5: the pull-style trunk (k_resnet_h2, 10x128, 32,768 rows, back to back for 4 s;
# tools/exp_c3_clock.py iso) and C1 (bench.py --config c1), in-tree against the pre-range
# library, alternating.
set -u
OUT=${OUT:-gpurun_out/r05p}; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for rep in 1 2; do
  for L in base ${VARIANTS:-tools/_ab/librvz_r05pre.so}; do
    i=$((i+1))
    if [ "$L" = base ]; then unset RVZ_LIB; else export RVZ_LIB=$L; fi
    [ -n "${NOISO:-}" ] || timeout -k 10 120 python tools/exp_c3_clock.py iso 4 > "$OUT/iso_$i.json" 2> "$OUT/iso_$i.err"
    rc=$?; echo "iso $i $L rc=$rc"; [ $rc -ne 0 ] && exit $rc
    cat "$OUT/iso_$i.json"
    timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > "$OUT/c1_$i.json" 2> "$OUT/c1_$i.err"
    rc=$?; echo "c1 $i $L rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python -c "import json; d=json.load(open('$OUT/c1_$i.json')); print('c1', d['value'])"
  done
done
exit 0
