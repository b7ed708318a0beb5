cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "hard_states" > gpurun_out/t3.log 2>&1; rc=$?
tail -15 gpurun_out/t3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu --no-knet --dataset-steps 0 --steps 20 --warmup 5 > gpurun_out/t3b.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/t3b.json'));print(d['value'], json.dumps(d['roofline']['issue']))"
