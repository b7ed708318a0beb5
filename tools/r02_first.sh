#!/bin/bash
# Round-2 first GPU pass: the GPU test suite, then the 20- vs 200-step probe.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r02_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r02_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/r02_probe.sh
