#!/bin/bash
# 20-step item timelines of the 2-wave and the 3-wave N = 20 fused instances on one box (TL_WAVES forces the instance).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tlw
for w in 2 3; do
  TL_WAVES=$w timeout -k 10 120 python3 tools/item_timeline.py 20 5 > gpurun_out/tlw/w$w.json 2> gpurun_out/tlw/w$w.err || { tail -3 gpurun_out/tlw/w$w.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/tlw/w$w.json'))
print('w$w', 'ms', round(d['launch_ms_events'],3), 'slots', d['slots'], d['slot_time_split'], 'work/item', round(d['work_fit_us']['per_item'],1), 'per_iter', round(d['work_fit_us']['per_iter'],3))
print('  busy', d['busy_frac_by_time_bin']); print('  wait', d['wait_us']); print('  crit', {k:v for k,v in d['critical_instance'].items() if k!='chain'})
print('  work by step', [round(x) for x in d['item_work_us_by_step']])"
done
