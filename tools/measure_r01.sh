#!/bin/bash
# Round-1 GPU measurement: parity tests, bench line, kernel-trace stats, PMC traffic passes (MPC fused
# launch and the KalmanNet FC2 kernel), the N=40 mixed-reference closed loop (configs[2]) and the
# dataset generation leg (configs[3], one GPU's share).  Every GPU step has its own time limit; steps
# are chained with && (stop at the first failure).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 &&
echo tests ok &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-knet > gpurun_out/prof_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python3 bench.py --no-cpu --no-knet > gpurun_out/prof_write.log 2>&1 &&
python3 tools/pmc_traffic.py --fetch gpurun_out/prof_fetch --write gpurun_out/prof_write --batch 4096 --horizon 20 --fused-steps 200 --out gpurun_out/traffic_r01.json > /dev/null &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/kprof_fetch -o run --output-format csv -- python3 tools/knet_pmc_run.py > gpurun_out/kprof_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/kprof_write -o run --output-format csv -- python3 tools/knet_pmc_run.py > gpurun_out/kprof_write.log 2>&1 &&
python3 tools/pmc_knet_traffic.py --fetch gpurun_out/kprof_fetch --write gpurun_out/kprof_write --batch 1024 --out gpurun_out/traffic_knet_r01.json > /dev/null &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d gpurun_out/pmc_f64 -o run --output-format csv -- python3 bench.py --no-cpu --no-knet --steps 20 > gpurun_out/pmc_f64.log 2>&1 &&
python3 tools/pmc_f64.py gpurun_out/pmc_f64 --batch 4096 --steps-per-launch 20 --out gpurun_out/sq_f64_r01.json > /dev/null &&
echo pmc ok &&
timeout -k 10 300 python bench.py --traffic-json gpurun_out/traffic_r01.json --knet-traffic-json gpurun_out/traffic_knet_r01.json --issue-json gpurun_out/sq_f64_r01.json > gpurun_out/bench.json 2> gpurun_out/bench.err &&
echo bench ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_kt.log 2>&1 &&
python3 tools/trace_dispatches.py gpurun_out/prof_kt/run_kernel_trace.csv "solve_kernel<40, true, true>" gpurun_out/solve_dispatches.json > /dev/null &&
python3 tools/knet_fc2_dispatches.py gpurun_out/prof_kt/run_kernel_trace.csv gpurun_out/knet_fc2_dispatches.json > /dev/null &&
echo trace ok &&
timeout -k 10 300 python bench.py --horizon 40 --kind mixed --steps 100 --no-cpu --no-knet > gpurun_out/bench_n40.json 2> gpurun_out/bench_n40.err &&
timeout -k 10 300 python tools/gen_dataset.py --per-gpu 4096 --steps 240 --out gpurun_out/vehicle_mpc > gpurun_out/dataset.json 2> gpurun_out/dataset.err &&
rm -f gpurun_out/vehicle_mpc_clean.csv gpurun_out/vehicle_mpc_noisy.csv &&
echo all ok
