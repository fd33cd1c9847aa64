# k_trace2 launch tuning sweep on the round-3 tree (izpi_render_tuning; every setting is
# bit-identical by construction, the digest column checks it): C3 at 128 spp, C5 at 32 spp.
set -e
mkdir -p gpurun_out
V="timeout -k 10 120 python tools/variants.py run --frames 2"
O=gpurun_out/tune_sweep.log
: > $O
$V --config C3 --spp 128 base >> $O
for t in refill_min=16 refill_min=32 refill_min=40 prim_weight=24 prim_weight=40 prim_weight=48 trace_chunk=256 trace_chunk=1024; do
  $V --config C3 --spp 128 --tune $t base >> $O
done
$V --config C3 --spp 128 base >> $O
$V --config C5 --spp 32 base >> $O
for t in refill_min=16 refill_min=32 prim_weight=24 prim_weight=48; do
  $V --config C5 --spp 32 --tune $t base >> $O
done
$V --config C5 --spp 32 base >> $O
