set -o pipefail
for v in head w3t; do
  export TRAJMPC_LIB=$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so
  timeout -k 10 200 python tools/item_timeline.py 20 5 > gpurun_out/r3_tl_$v.json 2> gpurun_out/r3_tl_$v.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/r3_tl_$v.json'))
c=d['critical_instance']
print('$v', 'launch_ms', round(d['launch_ms_events'],3), 'slots', d['slots'], 'split', {k:round(v,3) for k,v in d['slot_time_split'].items()}, 'fit', d['work_fit_us'])
print('  drain', {k:round(v) for k,v in d['slot_drain_us'].items()})
print('  crit b', c['b'], 'iters', c['total_iters'], 'chain_work', round(c['chain_work_us']), 'wait', round(c['chain_wait_us']), 'gaps', round(c['gaps_us']))
print('  chain', [(x['iters'], round(x['end']-x['start'])) for x in c['chain']])
print('  busy', d['busy_frac_by_time_bin'])"
done
