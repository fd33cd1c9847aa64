set -e
timeout -k 10 300 python tools/variants.py run --config C3 --spp 512 --frames 2 prev base > gpurun_out/ab_c3_ac.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --frames 2 prev base > gpurun_out/ab_c4_ac.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C2 --frames 2 prev base > gpurun_out/ab_c2_ac.log 2>&1
rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ac -o run -- python tools/variants.py child --config C3 --frames 2 --variant base > gpurun_out/prof_ac.log 2>&1
