#!/bin/bash
# Round 4: fastmath accuracy check, then the fused-path tests + phase profile + bench for the in-tree library
# (full symmetric P in LDS) and the packed-P variant.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/fastmath_check.bin > gpurun_out/r4_fastmath.log 2>&1; echo "fastmath rc=$?"; tail -30 gpurun_out/r4_fastmath.log
TAG=c TESTS="fused or closed_loop or per_step or full_step or dropin or hard_states" VARIANTS=nofp bash tools/r04_iter.sh
