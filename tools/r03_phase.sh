#!/bin/bash
# phase profile (tools/phase_profile.py, per-step kernel with stamps) of library variants
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in $VARIANTS; do
  export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"
  timeout -k 10 120 python tools/phase_profile.py 0 60 > gpurun_out/r3p_$v.log 2>&1 || { tail -5 gpurun_out/r3p_$v.log; exit 1; }
  echo "== $v"; grep -E "^(kernel|inputs|condense|scale|solve|total|iters|solve cycles|solve split|per residual)" gpurun_out/r3p_$v.log
done
