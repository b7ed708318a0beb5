#!/bin/bash
# Round-2 probe: the driver's bench command vs a 200-step launch, and per-instance timelines of both.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --no-knet --steps 20 --warmup 5 > gpurun_out/p_b20.json 2> gpurun_out/p_b20.err &&
timeout -k 10 200 python bench.py --no-cpu --no-knet --steps 200 --warmup 5 > gpurun_out/p_b200.json 2> gpurun_out/p_b200.err &&
timeout -k 10 200 python -c "import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import fused_profile as F; F.main(steps=20)" > gpurun_out/p_fp20.log 2>&1 &&
timeout -k 10 200 python -c "import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import fused_profile as F; F.main(steps=200)" > gpurun_out/p_fp200.log 2>&1
rc=$?
for f in p_b20.json p_b200.json; do python -c "import json;d=json.load(open('gpurun_out/$f'));print('$f',round(d['value']),'ms',round(d['ms_per_step'],4),d['roofline']['kernels_ms'],d['solver_stats'])"; done
cat gpurun_out/p_fp20.log gpurun_out/p_fp200.log
exit $rc
