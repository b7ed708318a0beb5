#!/bin/bash
# RCCL on a one-GPU box: the collectives of the multi-GPU path at world size 1 under torch.distributed.run, then
# bench.py under the driver's launcher with a process group forced (TRAJ_BENCH_PG=1): rendezvous, barriers, MAX
# all-reduce of the elapsed time, the dataset leg.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
L="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
timeout -k 10 180 $L --master-port 29517 tools/rccl_probe.py > gpurun_out/r03_rccl_probe.json 2> gpurun_out/r03_rccl_probe.err &&
cat gpurun_out/r03_rccl_probe.json &&
TRAJ_BENCH_PG=1 timeout -k 10 400 $L --master-port 29519 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu \
  > gpurun_out/r03_bench_torchrun_pg.json 2> gpurun_out/r03_bench_torchrun_pg.err &&
python3 -c "
import json; lines=open('gpurun_out/r03_bench_torchrun_pg.json').read().splitlines(); d=json.loads(lines[0])
print('stdout lines', len(lines), '| torchrun+RCCL bench VALUE', round(d['value']), 'n_gpus', d['n_gpus'])
print('dataset', {k: v for k, v in d['dataset'].items() if not isinstance(v, (list, dict))})"
