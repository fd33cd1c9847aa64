set -e
timeout -k 10 300 python tools/variants.py run --config C3 --spp 128 --frames 2 base sah sahct2 sahcl1 > gpurun_out/ab_c3_s.log 2>&1
timeout -k 10 200 python tools/variants.py run --config C3 --spp 128 --frames 2 --leaf-max 4 base sah sahct2 >> gpurun_out/ab_c3_s.log 2>&1
