set -e
for t in "" "--tune refill_min=16" "--tune refill_min=32" "--tune trace_chunk=256" "--tune trace_chunk=1024" "--tune prim_weight=24" "--tune prim_weight=44"; do
timeout -k 10 120 python tools/variants.py run --config C3 --spp 128 --frames 2 $t base >> gpurun_out/tune_ah.log 2>&1
done
