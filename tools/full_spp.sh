#!/bin/bash
# Full-spp frames of C4 and C5 on one GPU: GPU-built tree.
# C4: 3 timed frames after a warmup, reference-tree frame + image check in the same run.
# C5 (2048^2 x 4096, ~2 minutes per frame): one timed frame, no warmup, no reference tree.
set -e
mkdir -p gpurun_out
TAG=${1:-r2c}
timeout -k 10 300 python bench.py --config C4 --spp 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/full_${TAG}_C4.log 2>&1
grep '^{' gpurun_out/full_${TAG}_C4.log | tail -1 > gpurun_out/full_${TAG}_C4.json
tail -c 600 gpurun_out/full_${TAG}_C4.json; echo
timeout -k 10 400 python bench.py --config C5 --spp 4096 --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --no-reference-check > gpurun_out/full_${TAG}_C5.log 2>&1
grep '^{' gpurun_out/full_${TAG}_C5.log | tail -1 > gpurun_out/full_${TAG}_C5.json
tail -c 600 gpurun_out/full_${TAG}_C5.json; echo
