"""knet_fc2_kernel dispatches of a `rocprofv3 --kernel-trace` run of bench.py: the T graph-replayed launches
of the timed KalmanNet run and the standalone launches bench.py times with HIP events for the roofline.
python tools/knet_fc2_dispatches.py TRACE.csv OUT.json"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "knet_fc2_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
# bench.py order: capture warm-up (2 steps), graph replays (T = 200 each), 1 + 50 standalone launches
standalone = us[-50:]
graph = us[2:-51]
out = {"trace": sys.argv[1], "dispatches": len(us),
       "standalone_launches": {"n": len(standalone), "mean_us": sum(standalone) / len(standalone)},
       "graph_launches": {"n": len(graph), "mean_us": sum(graph) / max(1, len(graph))},
       "all_mean_us": sum(us) / len(us)}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out))
