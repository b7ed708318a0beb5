#!/bin/bash
# Full GPU suite, smoke() and the default bench line (what the driver runs at round end).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/check_tests.log 2>&1; rc=$?
tail -3 gpurun_out/check_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check_smoke.log 2>&1 && tail -1 gpurun_out/check_smoke.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err &&
python -c "import json;d=json.load(open('gpurun_out/check_bench.json'));print('VALUE',round(d['value']),'ms',round(d['ms_per_step'],4),'traffic',d['roofline']['traffic'],'knet',round(d['knet']['value']),d['knet']['mse'],d['knet']['ekf_mse'],'ds',d['dataset']['traj_steps_per_s'])"
