#!/bin/bash
# Compare library builds under trajectory_generation_amd/_variants/*/ (phase profile + bench value).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for d in trajectory_generation_amd/_variants/*/; do
  v=$(basename "$d")
  export TRAJMPC_LIB="$PWD/$d/libtrajmpc.so"
  timeout -k 10 120 python tools/phase_profile.py 0 60 > gpurun_out/v_$v.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu --no-knet --steps 100 > gpurun_out/v_$v.json 2>/dev/null || exit 1
  echo "== $v"; grep -E "per sweep|kernel " gpurun_out/v_$v.log
  python -c "import json;d=json.load(open('gpurun_out/v_$v.json'));print('VALUE',round(d['value']),'solve_ms',round(d['roofline']['kernel_ms'],4))"
done
