set -e
bash tools/gpu_tests.sh
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c3_u.log 2>&1
