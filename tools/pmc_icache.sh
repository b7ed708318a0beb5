#!/bin/bash
# Instruction-cache counters of the fused solve_kernel at the driver's command (one PMC pass).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU -d gpurun_out/pmc_ic -o run --output-format csv -- python3 bench.py --no-cpu --no-knet --dataset-steps 0 --steps 20 --warmup 5 > gpurun_out/pmc_ic.log 2>&1 &&
python3 tools/pmc_sq.py gpurun_out/pmc_ic > gpurun_out/pmc_ic.json && cat gpurun_out/pmc_ic.json
