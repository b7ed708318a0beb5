cd "$(dirname "$0")" 2>/dev/null; cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_knet_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "config5 or ekf" > gpurun_out/k5_tests.log 2>&1; rc=$?
tail -15 gpurun_out/k5_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_k5.json 2> gpurun_out/bench_k5.err
