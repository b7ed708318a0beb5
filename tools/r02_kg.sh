#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/knet_groups.py > gpurun_out/kg.log 2>&1; rc=$?
cat gpurun_out/kg.log | grep -v amdgpu.ids; exit $rc
