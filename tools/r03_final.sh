#!/bin/bash
# Round 3: the whole -m gpu suite, smoke(), then the driver's command (bench.py --gpus 1 --steps 20 --warmup 5).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r03_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r03_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 && cat gpurun_out/r03_smoke.log | tail -1 &&
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err &&
python3 -c "
import json; d=json.load(open('gpurun_out/r03_bench.json'))
print('VALUE', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'frac', d['roofline']['frac'], 'busy', round(d['roofline']['issue']['simd_valu_busy_frac'],3))
print('cold', round(d['cold']['value']), 'knet', round(d['knet']['value']), 'cpu', round(d['cpu_baseline']['value']), 'dataset', round(d['dataset']['traj_steps_per_s']))"
