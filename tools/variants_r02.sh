#!/bin/bash
# Bench every library build under trajectory_generation_amd/_variants/*/ at the driver's command
# (20 steps after 5 warmup, twice) and at 200 steps.  Usage: tools/variants_r02.sh [extra bench args]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for d in trajectory_generation_amd/_variants/*/; do
  v=$(basename "$d")
  export TRAJMPC_LIB="$PWD/$d/libtrajmpc.so"
  for s in 20 20 200; do
    timeout -k 10 200 python bench.py --no-cpu --no-knet --dataset-steps 0 --steps $s --warmup 5 "$@" > gpurun_out/vr.json 2> gpurun_out/vr_$v.err || { echo "$v $s failed"; tail -5 gpurun_out/vr_$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/vr.json'));print('$v', $s, 'VALUE', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'iters', round(d['solver_stats']['iters_mean'],2), d['solver_stats']['status_hist'])"
  done
done
