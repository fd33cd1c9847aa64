set -e
bash tools/gpu_tests.sh
timeout -k 10 400 python bench.py --config C4 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c4_j.log 2>&1
timeout -k 10 600 python bench.py --config C5 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/bench_c5_j.log 2>&1
