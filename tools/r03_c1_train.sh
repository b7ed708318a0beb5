#!/bin/bash
# config-1 measurement (bench's config1 object) and the trained-KalmanNet MSE recipe on one GPU box
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --no-knet --dataset-steps 0 --no-cold --cpu-traj 256 --cpu-steps 8 \
  > gpurun_out/r3_c1.json 2> gpurun_out/r3_c1.err || { tail -20 gpurun_out/r3_c1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3_c1.json'));print(json.dumps(d['config1'],indent=1))"
timeout -k 10 ${TRAIN_S:-900} python -u tools/knet_train_eval.py --steps ${TRAIN_STEPS:-500} \
  --out gpurun_out/r03_knet_trained_mse.json 2>&1 | tee gpurun_out/r3_train.log
