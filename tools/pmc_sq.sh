#!/bin/bash
# SQ counters of the bench launches (solve_kernel utilization): two PMC passes, kernel-trace only.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/pmc_sq1 -o run --output-format csv -- python3 bench.py --no-cpu --no-knet --steps 20 > gpurun_out/pmc_sq1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVES -d gpurun_out/pmc_sq2 -o run --output-format csv -- python3 bench.py --no-cpu --no-knet --steps 20 > gpurun_out/pmc_sq2.log 2>&1
