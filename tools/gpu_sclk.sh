# Shade clocks with the entry-load and texel waits as sections of their own (-DIZPI_SHADE_CLOCKS).
set -e
mkdir -p gpurun_out
O=gpurun_out/sclk.log
timeout -k 10 300 python tools/variants.py run --frames 1 --config C4 --spp 128 base sclk > $O 2>&1
timeout -k 10 300 python tools/variants.py run --frames 1 --config C3 --spp 128 base sclk >> $O 2>&1
timeout -k 10 300 python tools/variants.py run --frames 1 --config C5 --spp 32 base sclk >> $O 2>&1
grep -v amdgpu.ids $O | cut -c1-420
