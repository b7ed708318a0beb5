#!/bin/bash
# f64 instruction mix of the fused MPC launch (issue-side roofline of solve_kernel): one SQ PMC pass,
# kernel-trace only, summarized by tools/pmc_f64.py into gpurun_out/sq_f64_r01.json.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d gpurun_out/pmc_f64 -o run --output-format csv -- python3 bench.py --no-cpu --no-knet --steps 20 > gpurun_out/pmc_f64.log 2>&1 &&
python3 tools/pmc_f64.py gpurun_out/pmc_f64 --batch 4096 --steps-per-launch 20 --out gpurun_out/sq_f64_r01.json
