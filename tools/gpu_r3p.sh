set -e
bash tools/gpu_tests.sh
timeout -k 10 400 python tools/variants.py run --config C3 --frames 3 nostage base > gpurun_out/ab_c3_p.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 2 nostage base > gpurun_out/ab_c5_p.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 256 --frames 2 nostage base > gpurun_out/ab_c4_p.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C2 --frames 2 nostage base > gpurun_out/ab_c2_p.log 2>&1
