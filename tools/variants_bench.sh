#!/bin/bash
# Fused and per-step bench of every library build under trajectory_generation_amd/_variants/*/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for d in trajectory_generation_amd/_variants/*/; do
  v=$(basename "$d")
  export TRAJMPC_LIB="$PWD/$d/libtrajmpc.so"
  for m in "" "--per-step"; do
    timeout -k 10 200 python bench.py --no-cpu --no-knet --steps 100 $m > gpurun_out/vb.json 2>/dev/null || { echo "$v $m failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/vb.json'));print('$v', '${m:-fused}', 'VALUE', round(d['value']), 'ms/step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['roofline']['kernels_ms'].items()})"
  done
done
