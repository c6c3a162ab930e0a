#!/bin/bash
# r04z: k_play12 trunk knobs (RVZ_T12_KNOBS 0 / 1 / 2) against k_play with the skip input from
# LDS (same arithmetic), and the default library's k_play, one box
set -u
OUT=${OUT:-gpurun_out}; mkdir -p "$OUT"
for L in k0 k1 k2; do
  RVZ_LIB=tools/_ab/librvz_$L.so GAMES=4096 PLIES=20 timeout -k 10 300 python tools/exp_play12.py > "$OUT/r04z_play12_$L.json" 2> "$OUT/r04z_play12_$L.err" || { echo "$L failed"; tail -3 "$OUT/r04z_play12_$L.err"; exit 1; }
  echo "$L $(tail -1 $OUT/r04z_play12_$L.json)"
done
GAMES=4096 PLIES=20 timeout -k 10 300 python tools/exp_play12.py > "$OUT/r04z_play12_default.json" 2> "$OUT/r04z_play12_default.err"
echo "default $(tail -1 $OUT/r04z_play12_default.json)"
