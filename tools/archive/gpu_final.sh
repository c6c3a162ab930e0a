#!/bin/bash
# End-of-round GPU record: tests, smoke, C2 bench + rocprof, C3 / C1 / C5 lines, PMC traffic
# passes of the current build. Every GPU step has its own limit; exit > 1 ends the script.
set -u
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r02r}
TAG=$TAG bash tools/archive/gpu_round2.sh; rc=$?; [ $rc -gt 1 ] && exit $rc
OUT=$OUT TAG=$TAG timeout -k 10 700 bash tools/gpu_pmc.sh; rc=$?; echo "pmc rc=$rc"; [ $rc -gt 1 ] && exit $rc
echo final-done
