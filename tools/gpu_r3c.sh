set -e
bash tools/gpu_tests.sh
timeout -k 10 400 python tools/variants.py run --config C4 --spp 256 --frames 3 r3head base r3head base > gpurun_out/ab_c4.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 128 --frames 2 sclk > gpurun_out/sclk_c4.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 2 sclk > gpurun_out/sclk_c5.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C3 --frames 2 sclk > gpurun_out/sclk_c3.log 2>&1
timeout -k 10 300 python tools/first_frame.py --config C4 --frames 2 > gpurun_out/ff_c4.log 2>&1
timeout -k 10 300 python tools/shard_probe.py --config C3 --worlds 1,8 > gpurun_out/shard_c3.log 2>&1
