#!/bin/bash
# Profiling recipe for the bench workload (run on the GPU box from the repo root):
#   bash tools/run_profile.sh TAG
# 1. the bench itself (its own PMC passes, CPU baseline, reference-tree check) -> bench.json
# 2. rocprofv3 --kernel-trace --stats over the same timed frames (no PMC children, no
#    CPU baseline: a profiler must not run inside a profiler) -> kernel_stats.csv
set -e
TAG=${1:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 python3 bench.py > $OUT/bench.log 2>&1
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-pmc --no-cpu-baseline --no-reference-check > $OUT/bench_trace.log 2>&1
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
grep '^{' $OUT/bench_trace.log | tail -1 > $OUT/bench_under_rocprof.json
head -5 $OUT/kernel_stats.csv
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'])"
