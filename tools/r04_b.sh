#!/bin/bash
# Round 4: CU-mask feasibility probe and the heavy-instance chain probe.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/mb_cumask.bin > gpurun_out/r4_cumask.log 2>&1; echo "cumask rc=$?"; cat gpurun_out/r4_cumask.log
timeout -k 10 300 python tools/r04_heavy_probe.py > gpurun_out/r4_heavy_probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/r4_heavy_probe.log | tail -20
