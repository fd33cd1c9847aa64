set -e
bash tools/gpu_tests.sh
timeout -k 10 400 python tools/variants.py run --config C3 --frames 3 r3head base > gpurun_out/ab_c3_f.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 2 r3head base nosphlpdf > gpurun_out/ab_c5_f.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 256 --frames 2 r3head base > gpurun_out/ab_c4_f.log 2>&1
timeout -k 10 300 python tools/shard_probe.py --config C3 --worlds 1,8 > gpurun_out/shard_c3_f.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C3 --frames 2 --tune slots=134217728 base > gpurun_out/c3_slots_f.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C3 --frames 2 --tune slots=201326592 base >> gpurun_out/c3_slots_f.log 2>&1
timeout -k 10 300 python bench.py --config C4 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/bench_c4_f.log 2>&1
