#!/bin/bash
# Profiling recipe for the bench workload (run on the GPU box from the repo root).
#   pass 1: kernel trace + stats (per-kernel durations)      -> gpurun_out/prof_$TAG/trace
#   pass 2: PMC FETCH_SIZE (HBM read bytes, gfx950 reports 1/2 of wide reads)
#   pass 3: PMC WRITE_SIZE
# Counters are collected in their own passes with --kernel-trace only (no sys/runtime trace).
set -e
TAG=${1:-r1}
SPP=${2:-512}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-reference-check --spp $SPP > $OUT/bench_trace.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-reference-check --spp $SPP > $OUT/bench_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-reference-check --spp $SPP > $OUT/bench_write.log 2>&1
find $OUT -name "*.csv" | head -20
