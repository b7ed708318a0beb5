#!/bin/bash
# SQ counters of the fused solve_kernel at the driver's command: issue / wait / LDS utilization, two PMC
# passes (kernel-trace only), summarized by tools/pmc_sq.py.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --no-cpu --no-knet --dataset-steps 0 --steps 20 --warmup 5"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/pmc_sq1 -o run --output-format csv -- $B > gpurun_out/pmc_sq1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq2 -o run --output-format csv -- $B > gpurun_out/pmc_sq2.log 2>&1 &&
python3 tools/pmc_sq.py gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 > gpurun_out/pmc_sq.json && cat gpurun_out/pmc_sq.json
