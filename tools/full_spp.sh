#!/bin/bash
# The non-headline configs at full spp on one GPU, GPU-built tree:
#   bash tools/full_spp.sh TAG
# C2 / C4: full spp, 3 timed frames after a warmup, k_trace2 PMC passes, reference-tree frame
# + image check in the same run. C5 (2048^2 x 4096, ~2 minutes per frame): one timed frame,
# no warmup, no reference tree, no PMC; its roofline comes from a 64-spp run with PMC passes.
set -e
mkdir -p gpurun_out
TAG=${1:-r2c}
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 ${T:-300} python bench.py "$@" --no-cpu-baseline > gpurun_out/full_${TAG}_${name}.log 2>&1
  grep '^{' gpurun_out/full_${TAG}_${name}.log | tail -1 > gpurun_out/full_${TAG}_${name}.json
  python3 -c "import json;d=json.load(open('gpurun_out/full_${TAG}_${name}.json'));x=d['detail'];r=d.get('roofline') or {};print('$name', d['config']['spp'], 'spp', round(d['value'],1), 'Msamples/s', round(d['ms_per_step'],1), 'ms/frame; trace', round(x['rank0_trace_ms_per_step'],1), 'shade', round(x['rank0_shade_ms_per_step'],1), 'frac', r.get('frac'), 'ref', (x.get('reference_tree') or {}).get('value'), (x.get('reference_tree') or {}).get('image_bitwise_equal'))"
}
run C2 --config C2 --spp 256 --steps 3 --warmup 1
run C4 --config C4 --spp 1024 --steps 3 --warmup 1
run C5_64 --config C5 --spp 64 --steps 2 --warmup 1
T=400 run C5 --config C5 --spp 4096 --steps 1 --warmup 0 --no-pmc --no-reference-check
