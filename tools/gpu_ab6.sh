# One GPU call: split hit records with (u, v) interleaved for uv scenes (base) against the
# interleaved-only layout (head2) and the pre-zero-shortcut head, C3 / C4 / C5.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_materials.py -x -q --timeout 200 --timeout-method thread -k "kernel_variants or dragon or c3 or c4 or c5 or spectral or pbr or glass or metal or dielectric or zero or trace_closest or sphere" > gpurun_out/t6.log 2>&1 || { tail -30 gpurun_out/t6.log; exit 1; }
tail -2 gpurun_out/t6.log
O=gpurun_out/ab6.log
V="timeout -k 10 300 python tools/variants.py run --frames 1"
$V --config C5 --spp 32 base head2 base head2 > $O
$V --config C4 --spp 128 base head2 base head2 >> $O
$V --config C3 --spp 128 base head2 base head2 >> $O
cut -c1-300 $O
