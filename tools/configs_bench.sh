# Other configs at reduced spp on one GPU (GPU-built tree, reference-tree check in the same run)
set -e
mkdir -p gpurun_out
for c in "C1 16" "C2 64" "C4 64" "C5 32"; do
  set -- $c
  timeout -k 10 400 python bench.py --config $1 --spp $2 --no-cpu-baseline > gpurun_out/cfg_$1.log 2>&1
  grep '^{' gpurun_out/cfg_$1.log | tail -1 | python -c "import json,sys;d=json.load(sys.stdin);x=d['detail'];r=x['reference_tree'];print('$1', d['config']['spp'], 'spp', round(d['value'],1), 'Msamples/s; reference tree', r['value'], 'equal', r['image_bitwise_equal'], 'trace', round(x['rank0_trace_ms_per_step'],1), 'shade', round(x['rank0_shade_ms_per_step'],1))"
done
