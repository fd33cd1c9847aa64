set -e
timeout -k 10 300 python tools/variants.py run --config C2 --frames 2 prev base > gpurun_out/ab_c2_ai.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 256 --frames 2 prev base > gpurun_out/ab_c4_ai.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 1 prev base > gpurun_out/ab_c5_ai.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C3 --spp 128 --frames 1 prev base > gpurun_out/ab_c3_ai.log 2>&1
bash tools/gpu_tests.sh
