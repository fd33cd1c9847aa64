set -e
bash tools/gpu_tests.sh
timeout -k 10 400 python tools/variants.py run --config C3 --frames 3 nomc base > gpurun_out/ab_c3_i.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 256 --frames 2 nomc base > gpurun_out/ab_c4_i.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 2 nomc base > gpurun_out/ab_c5_i.log 2>&1
timeout -k 10 400 python bench.py --config C4 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c4_i.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 2 --leaf-max 1 base > gpurun_out/c5_leaf.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 2 --leaf-max 2 base >> gpurun_out/c5_leaf.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 256 --frames 2 --leaf-max 2 base > gpurun_out/c4_leaf.log 2>&1
