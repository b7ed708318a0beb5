#!/bin/bash
# phase profile (tools/phase_profile.py: 20-step fused launch after 5 warm steps, diagnostics instance) of the
# in-tree library and of the variants named
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = head ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"; fi
  timeout -k 10 120 python tools/phase_profile.py 0 5 20 > gpurun_out/r3p_$v.log 2>&1 || { tail -5 gpurun_out/r3p_$v.log; exit 1; }
  echo "== $v"; grep -E "^(kernel|inputs|condense|scale|solve|total|iters|solve cycles|solve split|per residual|  rollout|  stage loop)" gpurun_out/r3p_$v.log
done
