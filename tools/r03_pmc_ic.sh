#!/bin/bash
# Round 3: instruction-cache and SQ wait counters of the fused solve_kernel at the driver's command (separate passes).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps 20 --warmup 5"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU -d gpurun_out/r3_pmc_ic -o run --output-format csv -- $B > gpurun_out/r3_pmc_ic.log 2>&1 &&
python3 tools/pmc_sq.py gpurun_out/r3_pmc_ic > gpurun_out/r3_pmc_ic.json &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/r3_pmc_sq1 -o run --output-format csv -- $B > gpurun_out/r3_pmc_sq1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/r3_pmc_sq2 -o run --output-format csv -- $B > gpurun_out/r3_pmc_sq2.log 2>&1 &&
python3 tools/pmc_sq.py gpurun_out/r3_pmc_sq1 gpurun_out/r3_pmc_sq2 > gpurun_out/r3_pmc_sq.json &&
python3 -c "
import json
for f in ('gpurun_out/r3_pmc_ic.json','gpurun_out/r3_pmc_sq.json'):
    d=json.load(open(f)); print(f, json.dumps(d.get('per_instance_step'))); print('  split', d.get('wave_cycle_split'), d.get('lds_array_util_per_cu'))
"
