set -e
timeout -k 10 300 python tools/variants.py run --config C3 --frames 2 prev base > gpurun_out/ab_c3_af.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 1 prev base > gpurun_out/ab_c5_af.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C2 --frames 2 prev base > gpurun_out/ab_c2_af.log 2>&1
timeout -k 10 200 python tools/shard_probe.py --config C3 --worlds 1,8 > gpurun_out/shard_af.log 2>&1
for k in 1 2 3; do timeout -k 10 120 python tools/variants.py child --config C3 --spp 256 --frames 1 --variant base >> gpurun_out/var_af.log 2>&1; done
bash tools/gpu_tests.sh
