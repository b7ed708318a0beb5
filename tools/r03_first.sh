#!/bin/bash
# Round 3 (session 2) first GPU call: the -m gpu suite, the driver's bench command, and 20-step item timelines
# of the fused launch at 2 and 3 waves per SIMD.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r3f_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3f_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3f_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3f_bench.json 2> gpurun_out/r3f_bench.err \
  || { tail -20 gpurun_out/r3f_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3f_bench.json'));print('VALUE',round(d['value']),'kernel_ms',d['roofline']['kernel_ms'],'knet',round(d['knet']['value']))"
for w in 2 3; do
  TL_WAVES=$w timeout -k 10 200 python tools/item_timeline.py 20 5 > gpurun_out/r3f_tl_w$w.json 2> gpurun_out/r3f_tl_w$w.err || { tail -5 gpurun_out/r3f_tl_w$w.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r3f_tl_w$w.json'))
c=d['critical_instance']
print('w$w', 'launch_ms', round(d['launch_ms_events'],3), 'slots', d['slots'], 'split', {k:round(v,3) for k,v in d['slot_time_split'].items()}, 'fit', d['work_fit_us'])
print('  drain', {k:round(v) for k,v in d['slot_drain_us'].items()})
print('  crit b', c['b'], 'iters', c['total_iters'], 'chain_work', round(c['chain_work_us']), 'wait', round(c['chain_wait_us']), 'gaps', round(c['gaps_us']))
print('  chain', [(x['iters'], round(x['end']-x['start'])) for x in c['chain']])
print('  busy', d['busy_frac_by_time_bin'])"
done
