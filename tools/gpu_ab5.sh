# One GPU call: the parity suite, then A/B on C3/C4/C5 of this round's shading and state
# changes: head = before the zero-radiance unwinding shortcut, head2 = before the split hit
# records, base = the working tree; oct / t384 = octant-grouped output / 384-thread
# shading blocks on top of base.
set -e
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -2 gpurun_out/t5.log
O=gpurun_out/ab5.log
V="timeout -k 10 300 python tools/variants.py run --frames 1"
$V --config C3 --spp 128 base head2 oct t384 base head2 oct t384 > $O
$V --config C5 --spp 32 base head base head >> $O
$V --config C4 --spp 128 base head base head >> $O
cut -c1-300 $O
