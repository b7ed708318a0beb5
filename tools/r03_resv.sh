#!/bin/bash
# Round 3: fused-run parity/bit-identity tests (N 20/40), config 3 with the capacity-80 instances, then the driver's
# command (--steps 20) for waves per SIMD x SIMD-reservation per mille.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fused or per_step_parity or hard_states" > gpurun_out/r3r_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3r_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3r_tests.log | head -20; exit $rc; }
for wv in 1 2; do
  TRAJ_FUSED_WAVES=$wv timeout -k 10 300 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 \
    --horizon 40 --kind mixed --steps 20 > gpurun_out/r3r_n40_w$wv.json 2> gpurun_out/r3r_n40_w$wv.err || { tail -5 gpurun_out/r3r_n40_w$wv.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3r_n40_w$wv.json'));print('N40 waves $wv VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2), d['solver_stats']['status_hist'])"
done
for cfg in "2 0" "2 16" "3 0" "3 16" "3 32" "3 64"; do
  set -- $cfg
  TRAJ_FUSED_WAVES=$1 TRAJ_SIMD_RESERVE=$2 timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 \
    --steps 20 > gpurun_out/r3r_b_$1_$2.json 2> gpurun_out/r3r_b_$1_$2.err || { tail -5 gpurun_out/r3r_b_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3r_b_$1_$2.json'));print('waves $1 resv $2 VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2))"
done
