set -e
timeout -k 10 300 python tools/variants.py run --config C3 --spp 128 --frames 2 --no-view-order base > gpurun_out/ab_c3_aa.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C3 --spp 128 --frames 2 base w5r8 w6r8 >> gpurun_out/ab_c3_aa.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 128 --frames 1 --no-view-order base > gpurun_out/ab_c4_aa.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 128 --frames 1 base >> gpurun_out/ab_c4_aa.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 1 --no-view-order base > gpurun_out/ab_c5_aa.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 1 base >> gpurun_out/ab_c5_aa.log 2>&1
