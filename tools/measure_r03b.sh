#!/bin/bash
# Round-3 headline refresh without the KalmanNet PMC passes (kernel unchanged since traffic_knet_r03.json): kernel-trace
# stats of the driver's command, the solve dispatches, the phase profile and the 20-step item timeline.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3m_kt -o run --output-format csv -- $B > gpurun_out/r3m_kt.log 2>&1 &&
python3 tools/trace_dispatches.py gpurun_out/r3m_kt/run_kernel_trace.csv "solve_kernel<40, true, true" gpurun_out/r03_solve_dispatches.json > /dev/null &&
echo trace ok &&
timeout -k 10 120 python3 tools/phase_profile.py 0 5 20 > gpurun_out/r03_phase20.txt 2>&1 &&
timeout -k 10 120 python3 tools/item_timeline.py 20 5 > gpurun_out/r03_tl20.json 2> gpurun_out/r03_tl20.err &&
echo all ok
