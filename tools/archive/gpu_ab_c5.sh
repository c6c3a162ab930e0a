set -u
# C5 A/B of (library | bench flags) specs, flags with _ for spaces:
#   SPECS="base| tools/_ab/librvz_x.so|--fused_--play-group_-16" TAG=x bash tools/c5ab_r03zg.sh
OUT=gpurun_out; A="--no-cpu-baseline --sub-configs none --no-evals-ab --config c5"
for r in 1 2; do
for spec in ${SPECS}; do
  L=${spec%%|*}; X=${spec#*|}; X=${X//_/ }; [ "$L" = base ] && L=alphazero-reversi_amd/rvz/librvz.so
  RVZ_LIB=$L timeout -k 10 200 python bench.py $A $X > $OUT/c5ab.json 2> $OUT/c5ab.err || { echo "fail $spec"; tail -3 $OUT/c5ab.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('$OUT/c5ab.json').read().strip().splitlines()[-1]);print('$spec round $r', d['value'], d['roofline'].get('avg_ms_per_launch'))" | tee -a $OUT/ab_${TAG}.txt
done; done
