"""KalmanNet-only measurement (bench.py's knet leg) for profiling: python tools/knet_bench.py [--cpu]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.knet_measure(torch.device("cuda:0"), cpu="--cpu" in sys.argv)))
