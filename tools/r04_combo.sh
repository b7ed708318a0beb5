#!/bin/bash
# Round-4 combined GPU check: the whole -m gpu suite, the phase profile, the bench at 20 / 200 steps
# (tools/r04_iter.sh with SKIP_TESTS), and the dataset-leg probe.  Each step under its own limit, && chained.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
tag=${TAG:-combo}
timeout -k 10 60 ./tools/microbench/check_ops.bin > gpurun_out/r4_${tag}_check_ops.log 2>&1 || { cat gpurun_out/r4_${tag}_check_ops.log; exit 1; }
cat gpurun_out/r4_${tag}_check_ops.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r4_${tag}_tests.log 2>&1 || { tail -30 gpurun_out/r4_${tag}_tests.log; exit 1; }
tail -2 gpurun_out/r4_${tag}_tests.log
SKIP_TESTS=1 TAG=$tag bash tools/r04_iter.sh || exit 1
if [ "${DSPROBE:-1}" = 1 ]; then
  timeout -k 10 200 python tools/r04_dsprobe.py > gpurun_out/r04_dsprobe.json 2> gpurun_out/r04_dsprobe.err || { tail -5 gpurun_out/r04_dsprobe.err; exit 1; }
  cat gpurun_out/r04_dsprobe.json
fi
