#!/bin/bash
# KNet row groups: graph vs eager throughput and a kernel trace of groups=2 (do the branches overlap?)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/kgroups; mkdir -p $O
cd $R
timeout -k 10 240 python -u tools/knet_groups.py > $O/graph.txt 2>&1 && \
KEAGER=1 timeout -k 10 240 python -u tools/knet_groups.py > $O/eager.txt 2>&1 && \
KG=2 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_g2 -- python3 tools/knet_groups.py > $O/trace_g2.txt 2>&1 && \
KG=2 KEAGER=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_g2e -- python3 tools/knet_groups.py > $O/trace_g2e.txt 2>&1
echo rc=$?
