#!/bin/bash
# Work-item timeline of config 3 (N = 40, mixed references): is the 20-step launch bound by one
# trajectory's chain of steps?
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tl40; mkdir -p $O
cd $R
TL_N=40 TL_KIND=mixed TL_OUT=$O/tl40_20.json timeout -k 10 300 python -u tools/item_timeline.py 20 5 4096 > $O/tl40.log 2>&1
echo rc=$?
