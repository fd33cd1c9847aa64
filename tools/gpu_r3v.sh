set -e
timeout -k 10 300 python tools/variants.py run --config C3 --spp 128 --frames 2 base ct075 cl025 cn15 r16 > gpurun_out/ab_c3_v.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 1 base ct075 cl025 > gpurun_out/ab_c5_v.log 2>&1
timeout -k 10 200 python tools/variants.py run --config C5 --spp 32 --frames 1 --leaf-max 3 base > gpurun_out/ab_c5_v3.log 2>&1
timeout -k 10 200 python tools/variants.py run --config C5 --spp 32 --frames 1 --leaf-max 4 base > gpurun_out/ab_c5_v4.log 2>&1
timeout -k 10 200 python tools/variants.py run --config C4 --spp 128 --frames 1 --leaf-max 4 base > gpurun_out/ab_c4_v4.log 2>&1
timeout -k 10 200 python tools/variants.py run --config C4 --spp 128 --frames 1 base ct075 cl025 > gpurun_out/ab_c4_v.log 2>&1
