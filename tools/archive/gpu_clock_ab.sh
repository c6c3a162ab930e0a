#!/bin/bash
# Effective clock of the h2 trunk, default build vs one workgroup per CU (GRBM_GUI_ACTIVE / 8 / duration)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in base occ1; do
  if [ $V = occ1 ]; then export RVZ_LIB=$PWD/tools/_ab/librvz_full_occ1.so; else unset RVZ_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d gpurun_out/clk_$V -o run -- python tools/exp_resnet_pmc.py 6 64 h2 > gpurun_out/clk_$V.log 2>&1 || exit 1
done
echo ok
