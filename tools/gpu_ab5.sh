# One GPU call: zero-radiance unwinding shortcut (base) against the previous head (C4, C5);
# output grouped by direction octant (oct) and 384-thread shading blocks (t384) on C3.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_materials.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "zero_radiance or c4 or c5 or spectral or pbr or glass or metal or dielectric" > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -2 gpurun_out/t5.log
O=gpurun_out/ab5.log
V="timeout -k 10 300 python tools/variants.py run --frames 1"
$V --config C5 --spp 32 base head base head > $O
$V --config C4 --spp 128 base head base head >> $O
$V --config C3 --spp 128 base oct t384 base oct t384 >> $O
cut -c1-300 $O
