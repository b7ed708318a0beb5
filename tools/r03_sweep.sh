#!/bin/bash
# lead / priority sweep of library variants (tools/r03_sweep.py); results in gpurun_out/r3s_<variant>.jsonl
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in $VARIANTS; do
  export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"
  echo "== $v"
  timeout -k 10 300 python tools/r03_sweep.py $SWEEP_ARGS > gpurun_out/r3s_$v.jsonl 2> gpurun_out/r3s_$v.err || { tail -5 gpurun_out/r3s_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/r3s_$v.jsonl'):
    d=json.loads(l); print('  ', d['lead'], 'grid', d['grid'], 'steps', d['steps'], 'M/s', round(d['value']/1e6,3), [round(x/1e6,3) for x in d['values']], 'same', d['bit_identical'])"
done
