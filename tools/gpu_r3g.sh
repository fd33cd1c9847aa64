set -e
bash tools/gpu_tests.sh
timeout -k 10 400 python tools/variants.py run --config C3 --frames 3 nofuse base > gpurun_out/ab_c3_g.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 2 nofuse base > gpurun_out/ab_c5_g.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 256 --frames 2 nofuse base > gpurun_out/ab_c4_g.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C2 --frames 2 nofuse base > gpurun_out/ab_c2_g.log 2>&1
timeout -k 10 300 python tools/shard_probe.py --config C3 --worlds 1,8 --pass-log > gpurun_out/shard_c3_g.log 2>&1
