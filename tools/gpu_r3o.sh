set -e
(rocminfo | grep -B2 -A3 "GROUP" | head -20) > gpurun_out/rocminfo_lds.txt 2>&1 || true
bash tools/gpu_tests.sh
bash profiles/run_profile.sh r3e
timeout -k 10 400 python bench.py --config C4 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c4_o.log 2>&1
timeout -k 10 600 python bench.py --config C5 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/bench_c5_o.log 2>&1
