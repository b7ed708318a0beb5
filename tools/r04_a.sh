cd /root/repo
timeout -k 10 120 ./tools/microbench/mb_f64ops.bin > gpurun_out/r4_mbops.log 2>&1; cat gpurun_out/r4_mbops.log
TAG=a TESTS=fused VARIANTS=bc bash tools/r04_iter.sh
