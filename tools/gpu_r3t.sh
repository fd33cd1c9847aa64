set -e
timeout -k 10 300 python tools/variants.py run --config C3 --spp 128 --frames 2 base sah sahdesc sahasc > gpurun_out/ab_c3_t.log 2>&1
timeout -k 10 200 python tools/variants.py run --config C5 --spp 32 --frames 1 base sah > gpurun_out/ab_c5_t.log 2>&1
timeout -k 10 200 python tools/variants.py run --config C4 --spp 128 --frames 1 base sah > gpurun_out/ab_c4_t.log 2>&1
timeout -k 10 200 python tools/variants.py run --config C2 --spp 64 --frames 1 base sah > gpurun_out/ab_c2_t.log 2>&1
