#!/bin/bash
# Round-2 measurement of the non-headline configs: configs[2] (N=40 mixed refs, 100 fused steps) and
# the configs[3] leg with CSV writing (one GPU's share: 4096 trajectories x 240 steps).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --horizon 40 --kind mixed --steps 100 --warmup 5 --no-cpu --no-knet --dataset-steps 0 > gpurun_out/bench_n40.json 2> gpurun_out/bench_n40.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-knet --dataset-csv gpurun_out/ds > gpurun_out/bench_ds.json 2> gpurun_out/bench_ds.err &&
ls -la gpurun_out/ds && rm -rf gpurun_out/ds
