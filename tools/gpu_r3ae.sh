set -e
for k in 1 2 3 4 5 6; do timeout -k 10 120 python tools/variants.py child --config C3 --spp 256 --frames 2 --variant base >> gpurun_out/var_ae.log 2>&1; done
