set -e
timeout -k 10 300 python tools/variants.py run --config C3 --spp 128 --frames 2 base r4 r12 > gpurun_out/ab_c3_z.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 1 base r4 r12 > gpurun_out/ab_c5_z.log 2>&1
