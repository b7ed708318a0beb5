#!/bin/bash
# KalmanNet GPU tests (fused runner over in_mult 5 / 10 at the 2e-4 bar) and the native loader test.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_knet_gpu.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fused_runner or native_loader or dataset" > gpurun_out/kt.log 2>&1; rc=$?
tail -25 gpurun_out/kt.log; exit $rc
