#!/bin/bash
# Driver's command (20 timed steps, MPC only) for library variants under trajectory_generation_amd/_variants/<v>/ and
# the in-tree build, each with the fused instance forced to 2 and to 3 waves per SIMD (TRAJ_FUSED_WAVES), 2 reps.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/wv; mkdir -p $O
for rep in 1 2; do
  for v in head "$@"; do
    for w in 2 3; do
      if [ "$v" = head ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"; fi
      TRAJ_FUSED_WAVES=$w timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps 20 \
        > $O/${v}_w${w}_$rep.json 2> $O/${v}.err || { tail -5 $O/${v}.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${v}_w${w}_$rep.json'));print('$v w$w rep $rep VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3))"
    done
  done
done
