#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fused or closed_loop" > gpurun_out/lead_tests.log 2>&1; rc=$?
tail -3 gpurun_out/lead_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/item_timeline.py 20 5 > gpurun_out/tl20.json 2> gpurun_out/tl20.err && python -c "
import json; d=json.load(open('gpurun_out/tl20.json')); c=d['critical_instance']; print(d['span_us'], d['slot_drain_us'], d['slot_time_split'], c['b'], c['total_iters'], c['chain_work_us'], c['gaps_us'])"
