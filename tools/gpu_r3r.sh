set -e
timeout -k 10 500 python tools/variants.py run --config C4 --spp 256 --frames 2 base texnoload texhot nonmap > gpurun_out/ab_c4_r.log 2>&1
