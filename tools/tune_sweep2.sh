# Second k_trace2 tuning sweep: the small-scene (LDS-resident BVH) configs C2, C4, C5 with
# refill_min / prim_weight combinations, and C3's prim_weight 24 against its default.
set -e
mkdir -p gpurun_out
V="timeout -k 10 120 python tools/variants.py run --frames 2"
O=gpurun_out/tune_sweep2.log
: > $O
for cfg in "C5 --spp 32" "C4 --spp 256" "C2 --spp 128"; do
  $V --config $cfg base >> $O
  $V --config $cfg --tune refill_min=32 base >> $O
  $V --config $cfg --tune prim_weight=24 base >> $O
  $V --config $cfg --tune refill_min=32 --tune prim_weight=24 base >> $O
  $V --config $cfg --tune refill_min=40 --tune prim_weight=24 base >> $O
  $V --config $cfg --tune refill_min=32 --tune prim_weight=16 base >> $O
  $V --config $cfg base >> $O
done
for i in 1 2; do
  $V --config C3 --spp 128 base >> $O
  $V --config C3 --spp 128 --tune prim_weight=24 base >> $O
  $V --config C3 --spp 128 --tune prim_weight=28 base >> $O
done
