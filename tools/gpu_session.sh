#!/bin/bash
# The one GPU-session driver (replaces the per-round r0x_*.sh / measure_r0x.sh recipes, which live on in git history).
# Run on the GPU box from the repo root, e.g.
#   gpurun --timeout 1200 -- 'tools/gpu_session.sh tests bench'
# Steps (any order, each under its own time limit, chained: the first failure ends the session):
#   tests       the -m gpu suite (pytest, thread timeouts)                     -> gpurun_out/$TAG_tests.log
#   bench       the driver's command: bench.py --gpus 1 --steps 20 --warmup 5  -> gpurun_out/$TAG_bench.json
#   cfg3        config 3: N = 40, mixed references, 20 steps                  -> gpurun_out/$TAG_n40.json
#   phase       phase profile of the fused 20-step launch (tools/phase_profile.py) -> gpurun_out/$TAG_phase20.txt
#   phase40     the same at N = 40 (config 3)                                  -> gpurun_out/$TAG_phase20_n40.txt
#   timeline    item timeline of the 20-step launch (tools/item_timeline.py)   -> gpurun_out/$TAG_timeline20.json
#   traffic     PMC FETCH_SIZE and WRITE_SIZE passes (separate runs) -> per instance-step HBM bytes
#               (tools/pmc_traffic.py)                                          -> gpurun_out/$TAG_traffic.json
#   traffic40   the same at N = 40 (config 3)                                  -> gpurun_out/$TAG_traffic_n40.json
#   sq          SQ f64 / VALU instruction pass (tools/pmc_f64.py)              -> gpurun_out/$TAG_sq_f64.json
#   sq40        the same at N = 40                                             -> gpurun_out/$TAG_sq_f64_n40.json
#   stall       two SQ passes: wave-cycle split, VALU occupancy (tools/pmc_stall.py) -> gpurun_out/$TAG_stall.json
#   stall40     the same at N = 40 (config 3)                                  -> gpurun_out/$TAG_stall_n40.json
#   trace       rocprofv3 --kernel-trace --stats of the driver's command + the solve dispatches
#               (tools/trace_dispatches.py)                                    -> gpurun_out/$TAG_kt/, $TAG_dispatches.json
#   tiers       horizon tiers: batch (B = 1024) and drop-in per-call times (tools/horizon_tiers.py) -> $TAG_tiers.json
#   ktraffic    PMC FETCH_SIZE / WRITE_SIZE passes over the FC2 launch alone at B = 1024 in the default mode
#               (tools/knet_fc2_pmc.py): its HBM bytes (tools/pmc_knet_traffic.py) -> gpurun_out/$TAG_traffic_knet.json
#   kfc2        PMC passes over FC2 alone in each product mode (tools/pmc_knet_fc2.sh) -> gpurun_out/$TAG_fc2_m*/
#   ab          A/B of library variants (VARIANTS="v1 v2" under _variants/<v>/, built by
#               tools/build_variant.sh) against the in-tree build, REPS rounds of CFGS "steps:waves" configurations
# Environment: TAG (default s5), VARIANTS, REPS, CFGS.  Never kills by pattern; every GPU step has a limit.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-s5}
O=gpurun_out
B20="python3 bench.py --steps 20 --warmup 5"
LEAN="--no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --no-config3 --no-host-io"
N40="--horizon 40 --kind mixed"

pmc_traffic() {   # $1 suffix, $2 extra bench flags, $3 horizon
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/${TAG}_fetch$1 -o run --output-format csv -- $B20 $LEAN $2 \
        > $O/${TAG}_fetch$1.log 2>&1 &&
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/${TAG}_write$1 -o run --output-format csv -- $B20 $LEAN $2 \
        > $O/${TAG}_write$1.log 2>&1 &&
    python3 tools/pmc_traffic.py --fetch $O/${TAG}_fetch$1 --write $O/${TAG}_write$1 --batch 4096 --horizon $3 \
        --fused-steps 20 --out $O/${TAG}_traffic$1.json > /dev/null
}
pmc_sq() {   # $1 suffix, $2 extra bench flags, $3 horizon
    timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
        SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d $O/${TAG}_f64$1 -o run --output-format csv -- \
        $B20 $LEAN $2 > $O/${TAG}_f64$1.log 2>&1 &&
    python3 tools/pmc_f64.py $O/${TAG}_f64$1 --batch 4096 --steps-per-launch 20 --horizon $3 \
        --out $O/${TAG}_sq_f64$1.json > /dev/null
}

pmc_stall() {   # $1 suffix, $2 extra bench flags, $3 horizon: two SQ passes (wave-cycle split, VALU occupancy)
    timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $O/${TAG}_stall_a$1 -o run \
        --output-format csv -- $B20 $LEAN $2 > $O/${TAG}_stall_a$1.log 2>&1 &&
    timeout -s KILL 150 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA \
        SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/${TAG}_stall_b$1 -o run \
        --output-format csv -- $B20 $LEAN $2 > $O/${TAG}_stall_b$1.log 2>&1 &&
    python3 tools/pmc_stall.py $O/${TAG}_stall_a$1 $O/${TAG}_stall_b$1 --horizon $3 --out $O/${TAG}_stall$1.json > /dev/null
}

for step in "$@"; do
    echo "== $step"
    case $step in
    tests)
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
            --timeout-method thread > $O/${TAG}_tests.log 2>&1; rc=$?
        tail -2 $O/${TAG}_tests.log
        [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/${TAG}_tests.log | head -30; exit $rc; } ;;
    bench)
        timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${TAG}_bench.json \
            2> $O/${TAG}_bench.err || { tail -5 $O/${TAG}_bench.err; exit 1; }
        python3 -c "import json;d=json.load(open('$O/${TAG}_bench.json'));print('value',d['value'],'cold',d['cold']['value'],'dataset',d['dataset']['traj_steps_per_s'],'knet',d['knet']['value'])" ;;
    cfg3)
        timeout -k 10 300 python3 bench.py $N40 $LEAN --steps 20 > $O/${TAG}_n40.json 2> $O/${TAG}_n40.err \
            || { tail -5 $O/${TAG}_n40.err; exit 1; }
        python3 -c "import json;d=json.load(open('$O/${TAG}_n40.json'));print('N40 value',d['value'],d['solver_stats'])" ;;
    phase)
        timeout -k 10 150 python3 tools/phase_profile.py 0 5 20 > $O/${TAG}_phase20.txt 2>&1 || exit 1
        grep -E "^(kernel|total|iters)" $O/${TAG}_phase20.txt ;;
    phase40)
        timeout -k 10 300 python3 tools/phase_profile.py 0 5 20 40 mixed > $O/${TAG}_phase20_n40.txt 2>&1 || exit 1
        grep -E "^(kernel|total|iters)" $O/${TAG}_phase20_n40.txt ;;
    timeline)
        timeout -k 10 150 python3 tools/item_timeline.py 20 5 > $O/${TAG}_timeline20.json 2> $O/${TAG}_timeline.err || exit 1 ;;
    traffic) pmc_traffic "" "" 20 && echo ok || exit 1 ;;
    traffic40) pmc_traffic _n40 "$N40" 40 && echo ok || exit 1 ;;
    sq) pmc_sq "" "" 20 && echo ok || exit 1 ;;
    sq40) pmc_sq _n40 "$N40" 40 && echo ok || exit 1 ;;
    stall) pmc_stall "" "" 20 && echo ok || exit 1 ;;
    stall40) pmc_stall _n40 "$N40" 40 && echo ok || exit 1 ;;
    trace)
        timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/${TAG}_kt -o run --output-format csv -- \
            python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${TAG}_kt.log 2>&1 &&
        python3 tools/trace_dispatches.py $O/${TAG}_kt/run_kernel_trace.csv "solve_kernel<40, true, true" \
            $O/${TAG}_dispatches.json > /dev/null && echo ok || exit 1 ;;
    tiers)
        timeout -k 10 600 python3 tools/horizon_tiers.py > $O/${TAG}_tiers.json 2> $O/${TAG}_tiers.err \
            || { tail -5 $O/${TAG}_tiers.err; exit 1; }
        cat $O/${TAG}_tiers.json ;;
    ktraffic)
        timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/${TAG}_kfetch -o run --output-format csv -- \
            python3 tools/knet_fc2_pmc.py 2 > $O/${TAG}_kfetch.log 2>&1 &&
        timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/${TAG}_kwrite -o run --output-format csv -- \
            python3 tools/knet_fc2_pmc.py 2 > $O/${TAG}_kwrite.log 2>&1 &&
        python3 tools/pmc_knet_traffic.py --fetch $O/${TAG}_kfetch --write $O/${TAG}_kwrite --batch 1024 \
            --out $O/${TAG}_traffic_knet.json > /dev/null && echo ok || exit 1 ;;
    kfc2) timeout -k 10 600 tools/pmc_knet_fc2.sh $TAG || exit 1 ;;
    ab)
        for rep in $(seq ${REPS:-3}); do
            for v in base $VARIANTS; do
                if [ "$v" = base ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/_variants/$v/libtrajmpc.so"; fi
                for c in ${CFGS:-20:0 200:0}; do
                    s=${c%%:*}; w=${c##*:}
                    if [ "$w" = 0 ]; then unset TRAJ_FUSED_WAVES; else export TRAJ_FUSED_WAVES=$w; fi
                    timeout -k 10 200 python3 bench.py $LEAN --steps $s $AB_FLAGS > $O/${TAG}_ab.json 2> $O/${TAG}_ab.err \
                        || { echo "bench $v $c failed"; tail -5 $O/${TAG}_ab.err; exit 1; }
                    python3 -c "import json;d=json.load(open('$O/${TAG}_ab.json'));print('rep $rep $v $c value',round(d['value']/1e6,3),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2))"
                done
            done
        done
        unset TRAJMPC_LIB TRAJ_FUSED_WAVES ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
