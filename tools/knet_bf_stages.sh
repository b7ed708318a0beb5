#!/bin/bash
# Stage costs of knet_back_front_kernel: one library per TRAJ_BF_SKIP bit (built here, on the CPU, into
# _variants/), then on the GPU box tools/knet_variants.sh times each.
#   bash tools/knet_bf_stages.sh build      (container)      bash tools/knet_variants.sh   (GPU box)
set -e
cd "$(dirname "$0")/../trajectory_generation_amd/csrc"
B=../_build
for v in 0 1 2 4 8 16 32 64; do
  d=../../_variants/skip$v; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -pragma-unroll-threshold=100000 \
      -DTRAJ_BF_SKIP=$v -c -o $d/knet.o knet.hip &
done
wait
for v in 0 1 2 4 8 16 32 64; do
  d=../../_variants/skip$v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libtrajmpc.so $B/trajmpc.o $d/knet.o $B/mpc_inst_16.o \
      $B/mpc_inst_32.o $B/mpc_inst_40.o $B/mpc_inst_64.o $B/mpc_inst_80.o
  rm -f $d/knet.o
done
