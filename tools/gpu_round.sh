# One GPU call: parity suite, reference-vs-GPU-tree image equality on C1-C5, bench.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 500 python tools/bvh_equality.py --configs C1,C2,C3,C4 > gpurun_out/bvh_eq.log 2>&1
timeout -k 10 300 python tools/bvh_equality.py --configs C5 --spp-cap 32 >> gpurun_out/bvh_eq.log 2>&1
grep '^{' gpurun_out/bvh_eq.log | python -c "import json,sys;[print(d['config'], d['bitwise_equal'], d['differing_pixels'], d['reference_nodes_per_ray'], d['gpu_nodes_per_ray']) for d in map(json.loads, sys.stdin)]"
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
