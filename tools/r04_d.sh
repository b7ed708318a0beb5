#!/bin/bash
# Round 4: fastmath accuracy, the whole -m gpu suite, then phase profile + bench (20 / 200 steps) for the in-tree
# library (fastmath transcendentals) and the device-library variant (nofm).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/fastmath_check.bin > gpurun_out/r4_fastmath.log 2>&1; echo "fastmath rc=$?"; head -6 gpurun_out/r4_fastmath.log; tail -1 gpurun_out/r4_fastmath.log
TAG=d VARIANTS=nofm bash tools/r04_iter.sh
