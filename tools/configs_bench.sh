#!/bin/bash
# The benchmark configs on one GPU: bash tools/configs_bench.sh TAG "C1 16 3" "C2 256 2" ...
# (config, spp, timed frames); GPU-built tree, reference-tree frame + image check in the same
# run unless NO_REF=1. Full JSON lines -> gpurun_out/cfg_TAG_<config>.json, a summary on stdout.
set -e
TAG=$1; shift
mkdir -p gpurun_out
for c in "$@"; do
  set -- $c
  extra=""; [ -n "$NO_REF" ] && extra="--no-reference-check"
  timeout -k 10 ${CFG_TIMEOUT:-400} python bench.py --config $1 --spp $2 --steps $3 --warmup 1 --no-cpu-baseline --no-pmc $extra > gpurun_out/cfg_${TAG}_$1.log 2>&1
  grep '^{' gpurun_out/cfg_${TAG}_$1.log | tail -1 > gpurun_out/cfg_${TAG}_$1.json
  python3 -c "import json;d=json.load(open('gpurun_out/cfg_${TAG}_$1.json'));x=d['detail'];r=x['reference_tree'] or {};print('$1', d['config']['spp'], 'spp', round(d['value'],1), 'Msamples/s', round(d['ms_per_step'],1), 'ms/frame; ref tree', r.get('value'), 'equal', r.get('image_bitwise_equal'), 'trace', round(x['rank0_trace_ms_per_step'],1), 'shade', round(x['rank0_shade_ms_per_step'],1), 'tail', round(x['rank0_tail_ms_per_step'],1), 'hbm', x['hbm_workspace_gb'], 'rays/sample', round(x['rank0_rays_per_step']/d['config']['samples_per_step'],2))"
done
