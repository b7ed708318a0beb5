#!/bin/bash
# Round 4: queue-lead sweep at the driver's shape, step-batch in-kernel linearization A/B, 20-step item timeline.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/r04_lead_sweep.py > gpurun_out/r4_lead.json 2> gpurun_out/r4_lead.err; echo "lead rc=$?"; cat gpurun_out/r4_lead.json
timeout -k 10 200 python tools/r04_stepbatch.py > gpurun_out/r4_stepbatch.json 2> gpurun_out/r4_stepbatch.err; echo "stepbatch rc=$?"; cat gpurun_out/r4_stepbatch.json
timeout -k 10 200 python tools/item_timeline.py 20 5 > gpurun_out/r4_tl20.json 2> gpurun_out/r4_tl20.err; echo "tl rc=$?"; python -c "
import json; d=json.load(open('gpurun_out/r4_tl20.json')); print({k: d[k] for k in ('launch_ms_events','span_us','slot_time_split','slot_drain_us','critical_instance')})"
