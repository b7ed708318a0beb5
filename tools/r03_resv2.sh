#!/bin/bash
# Round 3: the driver's command (--steps 20) and 200 steps, waves per SIMD x SIMD reservation, with the library
# built without the reservation code (noresv) and with it (head).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
run() {   # lib waves resv steps
  local tag=$1_$2_$3_$4
  if [ "$1" = head ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB=$PWD/trajectory_generation_amd/_variants/$1/libtrajmpc.so; fi
  TRAJ_FUSED_WAVES=$2 TRAJ_SIMD_RESERVE=$3 timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 \
    --steps $4 > gpurun_out/r3s_$tag.json 2> gpurun_out/r3s_$tag.err || { tail -5 gpurun_out/r3s_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3s_$tag.json'));print('$tag VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3))"
}
run noresv 2 0 20 && run noresv 3 0 20 && run head 2 0 20 && run head 3 0 20 && run head 2 16 20 && run head 3 16 20 && \
run head 3 64 20 && run noresv 2 0 200 && run noresv 3 0 200 && run head 3 16 200
