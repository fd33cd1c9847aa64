#!/bin/bash
# Round measurement on the GPU box, from the repo root, in two calls:
#   bash tools/measure_round.sh TAG c3     # C3 bench with its PMC passes + rocprof kernel trace (tools/run_profile.sh)
#   bash tools/measure_round.sh TAG other  # C1, C2, C4 at full spp; C2 / C4 / C5 PMC (roofline + wave cycles)
#   bash tools/measure_round.sh TAG c5     # C5 at full spp (one frame, ~100 s)
# each step under its own time limit.
set -e
TAG=${1:?tag}; PART=${2:-c3}
mkdir -p gpurun_out
case $PART in
  c3)
    bash tools/run_profile.sh $TAG ;;
  other)
    timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 --no-pmc --no-cpu-baseline > gpurun_out/bench_c1_$TAG.log 2>&1
    timeout -k 10 300 python bench.py --config C2 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c2_$TAG.log 2>&1
    timeout -k 10 400 python bench.py --config C4 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_c4_$TAG.log 2>&1
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
    timeout -k 10 400 python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline --no-reference-check > gpurun_out/pmc_c2_$TAG.log 2>&1
    timeout -k 10 400 python bench.py --config C4 --spp 128 --steps 2 --warmup 1 --no-cpu-baseline --no-reference-check > gpurun_out/pmc_c4_$TAG.log 2>&1
    timeout -k 10 500 python bench.py --config C5 --spp 64 --steps 1 --warmup 1 --no-cpu-baseline --no-reference-check > gpurun_out/pmc_c5_$TAG.log 2>&1
    for f in gpurun_out/bench_c1_$TAG.log gpurun_out/bench_c2_$TAG.log gpurun_out/bench_c4_$TAG.log gpurun_out/pmc_c2_$TAG.log gpurun_out/pmc_c4_$TAG.log gpurun_out/pmc_c5_$TAG.log; do
      grep '^{' $f | tail -1 | cut -c1-200; done ;;
  c5)
    timeout -k 10 900 python bench.py --config C5 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/bench_c5_$TAG.log 2>&1
    grep '^{' gpurun_out/bench_c5_$TAG.log | tail -1 | cut -c1-300 ;;
esac
