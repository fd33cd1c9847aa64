set -e
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 2 r3head base rb8 > gpurun_out/ab_c5.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C3 --frames 2 base rb8 > gpurun_out/ab_c3_rb.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C4 --spp 256 --frames 2 --tune slots=80000000 base > gpurun_out/c4_slots.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 128 --frames 1 base > gpurun_out/c5_slots.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 128 --frames 1 --tune slots=64000000 --tune chunk_units=134217728 base >> gpurun_out/c5_slots.log 2>&1
timeout -k 10 300 python tools/shard_probe.py --config C3 --worlds 1,8 --pass-log > gpurun_out/shard_c3_passes.log 2>&1
