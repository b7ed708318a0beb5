#!/bin/bash
# A/B of kernel variants at the driver's command shape: REPS rounds, each benching the in-tree library and every
# variant in VARIANTS (trajectory_generation_amd/_variants/<v>/libtrajmpc.so) at STEPS (default 20), interleaved.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
tag=${TAG:-ab}
for r in $(seq 1 ${REPS:-3}); do
  for v in base $VARIANTS; do
    if [ "$v" = base ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"; fi
    for s in ${STEPS:-20}; do
      timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps $s > gpurun_out/ab_${tag}_${v}_${s}_${r}.json 2> gpurun_out/ab_${tag}_${v}_${s}_${r}.err || { echo "bench $v $s failed"; tail -5 gpurun_out/ab_${tag}_${v}_${s}_${r}.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab_${tag}_${v}_${s}_${r}.json'));print('$r $v steps=$s VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],4))"
    done
  done
done
