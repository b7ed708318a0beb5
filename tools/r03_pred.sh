#!/bin/bash
# Prediction evaluation (test_prediction.py): GPU tests (+ the KNet suites after the veh_step split), then
# the bench leg alone.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pred; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_knet_predict.py \
  tests/test_knet_gpu.py tests/test_knet_ops.py > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u -c "
import json, torch, bench
r = bench.knet_predict_measure(torch.device('cuda:0'))
print(json.dumps(r))
" > $O/measure.json 2> $O/measure.err
rc=$?; tail -3 $O/tests.log; cat $O/measure.json; echo rc=$rc
[ $rc -eq 0 ] && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 -c "
import json, torch, bench
r = bench.knet_predict_measure(torch.device('cuda:0'), cpu=False)
print(json.dumps(r))
" > $O/prof.log 2>&1
echo prof_rc=$?
