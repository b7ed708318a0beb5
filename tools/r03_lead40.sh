#!/bin/bash
# Config 3 (N = 40 mixed, 20 steps): the fused queue's lead (steps ahead, per mille of heavy instances).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/lead40; mkdir -p $O
for rep in 1 2; do
  for ld in 1,100 2,100 3,100 2,50 4,50 1,200 2,200; do
    TRAJ_QUEUE_LEAD=$ld timeout -k 10 300 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --horizon 40 \
      --kind mixed --steps 20 > $O/l${ld/,/_}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    python -c "import json;d=json.load(open('$O/l${ld/,/_}_$rep.json'));print('lead $ld rep $rep VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3))"
  done
done
