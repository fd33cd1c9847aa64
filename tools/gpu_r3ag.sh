set -e
for k in 1 2 3; do
timeout -k 10 120 python tools/variants.py child --config C3 --spp 256 --frames 1 --variant base >> gpurun_out/var_ag.log 2>&1
timeout -k 10 120 python tools/variants.py child --config C3 --spp 256 --frames 1 --variant contig >> gpurun_out/var_ag.log 2>&1
timeout -k 10 120 python tools/variants.py child --config C3 --spp 256 --frames 1 --variant base --tune slots=67108864 >> gpurun_out/var_ag.log 2>&1
done
