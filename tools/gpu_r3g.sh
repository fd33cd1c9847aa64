set -e
bash profiles/run_profile.sh r3g
timeout -k 10 300 python bench.py --config C2 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c2_g.log 2>&1
timeout -k 10 400 python bench.py --config C4 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c4_g.log 2>&1
timeout -k 10 600 python bench.py --config C5 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/bench_c5_g.log 2>&1
