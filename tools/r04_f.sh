#!/bin/bash
# Round 4: the step tests (incl. in-kernel linearization bit-identity) and the drop-in latency probe.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "step or dropin or long_horizon or state_bounds or golden or hard_states" > gpurun_out/r4_f_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_f_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4_f_tests.log | head -30; exit $rc; }
timeout -k 10 200 python tools/r04_dropin_probe.py > gpurun_out/r4_dropin_probe.txt 2>&1; echo "probe rc=$?"; head -60 gpurun_out/r4_dropin_probe.txt
