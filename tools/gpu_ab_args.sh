#!/bin/bash
# A/B of two bench.py argument sets on the same library, alternating (PAIRS pairs).
#   A="--lanes 2" B="--lanes 4" [PAIRS=2] bash tools/gpu_ab_args.sh
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
PAIRS=${PAIRS:-2}
for V in $(for i in $(seq $PAIRS); do echo A B; done); do
  if [ $V = A ]; then X=$A; else X=$B; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline $X > "$OUT/abargs_$V.json" 2> "$OUT/abargs_$V.err" || exit $?
  python -c "import json; d=json.loads(open('$OUT/abargs_$V.json').readline()); print('$V', '$X', d['value'], d['ms_per_step'])"
done
