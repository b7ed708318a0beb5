#!/bin/bash
# Stall breakdown of the fused 20-step launch (two SQ passes, each with its own limit): where the waves' cycles go
# (active VALU / LDS / any, issue-stalled, parked on waitcnt or barrier) and LDS pressure.  Outputs gpurun_out/r4s_*.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 20 --warmup 5 --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS -d gpurun_out/r4s_a -o run --output-format csv -- $B > gpurun_out/r4s_a.log 2>&1 &&
echo pass a ok &&
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/r4s_b -o run --output-format csv -- $B > gpurun_out/r4s_b.log 2>&1 &&
echo pass b ok
