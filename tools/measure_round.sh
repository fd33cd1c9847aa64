#!/bin/bash
# Round measurement on the GPU box, from the repo root:
#   bash tools/measure_round.sh TAG
# the bench workload (C3) with PMC passes + rocprof kernel trace (profiles/run_profile.sh),
# then C2 / C4 / C5 at full spp, each under its own time limit.
set -e
TAG=${1:?tag}
bash profiles/run_profile.sh $TAG
timeout -k 10 300 python bench.py --config C2 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c2_$TAG.log 2>&1
timeout -k 10 400 python bench.py --config C4 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c4_$TAG.log 2>&1
timeout -k 10 600 python bench.py --config C5 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/bench_c5_$TAG.log 2>&1
