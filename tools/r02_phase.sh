#!/bin/bash
# Per-phase cycle table of the fused kernel (instances' last item) after 5 warm steps, 20-step launch.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python tools/phase_profile.py 0 5 20 > gpurun_out/phase20.log 2>&1; rc=$?
cat gpurun_out/phase20.log; exit $rc
