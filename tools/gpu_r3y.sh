set -e
timeout -k 10 300 python tools/variants.py run --config C4 --spp 128 --frames 2 prev base > gpurun_out/ab_c4_y.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 1 prev base > gpurun_out/ab_c5_y.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C3 --spp 128 --frames 2 prev base > gpurun_out/ab_c3_y.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C2 --spp 64 --frames 2 base prev > gpurun_out/ab_c2_y.log 2>&1
