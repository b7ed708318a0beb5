#!/bin/bash
# Repeated driver-command benches of the library builds under trajectory_generation_amd/_variants/*/,
# interleaved (round-robin) so that box drift hits every build alike.  Usage: tools/variants_rep.sh [reps]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
R=${1:-5}
for r in $(seq 1 $R); do
  for d in trajectory_generation_amd/_variants/*/; do
    v=$(basename "$d")
    TRAJMPC_LIB="$PWD/$d/libtrajmpc.so" timeout -k 10 200 python bench.py --no-cpu --no-knet --dataset-steps 0 --steps 20 --warmup 5 > gpurun_out/vr.json 2> gpurun_out/vr_$v.err || { echo "$v failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/vr.json'));print('$v', round(d['value']))"
  done
done
