set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --bvh gpu > gpurun_out/bench_gpubvh.log 2>&1
tail -1 gpurun_out/bench_gpubvh.log
