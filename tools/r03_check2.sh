#!/bin/bash
# GPU suite, then the bench with the config-1 object and the dataset leg writing gathered + per-rank CSVs
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r3c2_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3c2_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3c2_tests.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --steps 20 --no-knet --no-cold --cpu-traj 256 --cpu-steps 8 --dataset-csv /tmp/ds_r3 \
  > gpurun_out/r3c2_bench.json 2> gpurun_out/r3c2_bench.err || { tail -20 gpurun_out/r3c2_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r3c2_bench.json"))
print("value", round(d["value"]), "dataset", json.dumps(d["dataset"]))
for c in d["config1"]["cases"]:
    print(c["case"], {k: round(v["steps_per_s"]) for k, v in c.items() if isinstance(v, dict)},
          "mpc_step_us_median", round(c["dropin"]["mpc_step_us_median"], 1))
PY
