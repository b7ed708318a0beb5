#!/bin/bash
# Phase profile of every library build under trajectory_generation_amd/_variants/*/ (experiments).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for d in trajectory_generation_amd/_variants/*/; do
  v=$(basename "$d")
  TRAJMPC_LIB="$PWD/$d/libtrajmpc.so" timeout -k 10 120 python tools/phase_profile.py 0 60 > gpurun_out/vp_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/vp_$v.log; exit 1; }
  echo "== $v"; grep -E "^kernel|condense|stage loop|sincos|P rows" gpurun_out/vp_$v.log
done
