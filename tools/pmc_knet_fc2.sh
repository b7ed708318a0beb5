#!/bin/bash
# PMC passes over FC2 alone (tools/knet_fc2_pmc.py) in each traj_knet_set_fc2_mode mode:
#   gpurun -- 'tools/pmc_knet_fc2.sh TAG'  -> gpurun_out/TAG_fc2_m<mode>_<pass>/
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-f}
O=gpurun_out
mkdir -p $O
for mode in ${MODES:-0 1 2}; do
    n="m$mode"
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/${TAG}_fc2_${n}_a -o run --output-format csv -- \
        python3 tools/knet_fc2_pmc.py $mode > $O/${TAG}_fc2_${n}_a.log 2>&1 || { echo "pass a $n failed"; exit 1; }
    timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $O/${TAG}_fc2_${n}_b -o run --output-format csv -- \
        python3 tools/knet_fc2_pmc.py $mode > $O/${TAG}_fc2_${n}_b.log 2>&1 || { echo "pass b $n failed"; exit 1; }
    echo "ok $n"
done
