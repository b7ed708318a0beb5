#!/bin/bash
# Instruction-cache counters of the fused and the per-step closed-loop kernels (one PMC pass each).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d gpurun_out/pmc_ic -o run --output-format csv -- python3 bench.py --no-cpu --no-knet --steps 20 > gpurun_out/pmc_ic.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d gpurun_out/pmc_ic2 -o run --output-format csv -- python3 bench.py --no-cpu --no-knet --steps 20 --per-step > gpurun_out/pmc_ic2.log 2>&1
