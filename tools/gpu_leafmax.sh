# GPU-built BVH: leaf size sweep on C3 (timing only; images checked by the GPU tests)
set -e
mkdir -p gpurun_out
for lm in 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-reference-check --bvh-leaf-max $lm > gpurun_out/lm$lm.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/lm$lm.log').read().strip().splitlines()[-1]);x=d['detail'];print('leaf_max $lm', d['value'], 'trace', round(x['rank0_trace_ms_per_step'],1), 'shade', round(x['rank0_shade_ms_per_step'],1), 'nodes/ray', round(x['rank0_node_visits_per_ray'],2), 'tri/ray', round(x['rank0_tri_tests_per_ray'],2))"
done
