#!/bin/bash
# KalmanNet bench leg (tools/knet_bench.py) for every library build under _variants/*/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for d in _variants/*/; do
  v=$(basename "$d")
  export TRAJMPC_LIB="$PWD/$d/libtrajmpc.so"
  timeout -k 10 200 python tools/knet_bench.py > gpurun_out/kv.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/kv.json'));print('$v', round(d['value']), 'us/step', round(1e3*d['ms_per_step'],1), 'fc2 us', round(1e3*d['roofline']['kernel_ms'],1), 'frac', round(d['roofline']['frac'],3))"
done
