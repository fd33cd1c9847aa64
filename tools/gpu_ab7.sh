# One GPU call: XCD-segmented dequeue in k_trace2 (base) against one cursor (noseg):
# the parity tests of the trace paths first, then C3 / C4 / C2 / C5 timings and C3 PMC.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "kernel_variants or dragon or c3 or trace_closest" > gpurun_out/t7.log 2>&1 || { tail -30 gpurun_out/t7.log; exit 1; }
tail -2 gpurun_out/t7.log
O=gpurun_out/ab7.log
V="timeout -k 10 300 python tools/variants.py run --frames 1"
$V --config C3 --spp 128 base noseg base noseg > $O
$V --config C4 --spp 128 base noseg base noseg >> $O
$V --config C2 --spp 256 base noseg >> $O
$V --config C5 --spp 32 base noseg >> $O
cut -c1-330 $O
timeout -k 10 400 python tools/pmc_variants.py --config C3 --spp 64 base noseg > gpurun_out/pmc7.log 2>&1
cut -c1-600 gpurun_out/pmc7.log
