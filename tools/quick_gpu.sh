#!/bin/bash
# Iteration loop on the GPU box: parity tests, phase profile, bench without the CPU/KNet legs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/q_tests.log 2>&1; rc=$?
tail -3 gpurun_out/q_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/phase_profile.py 0 60 > gpurun_out/q_phase.log 2>&1 && cat gpurun_out/q_phase.log &&
timeout -k 10 200 python bench.py --no-cpu --no-knet > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err &&
python -c "import json;d=json.load(open('gpurun_out/q_bench.json'));print('VALUE',round(d['value']),'ms',round(d['ms_per_step'],4),d['roofline']['kernels_ms'],d['solver_stats'])"
