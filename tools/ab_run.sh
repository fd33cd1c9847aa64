#!/bin/bash
# Run on the GPU box: alternate variants (izpi_amd/_lib/variants/*.so) on one config.
#   VARIANTS="A B" bash tools/ab_run.sh CONFIG SPP ROUNDS
CFG=${1:-C3}; SPP=${2:-256}; R=${3:-2}
cp izpi_amd/_lib/libizpi_gpu.so /tmp/keep.so
for r in $(seq 1 $R); do
  for v in ${VARIANTS:-A B}; do
    cp izpi_amd/_lib/variants/$v.so izpi_amd/_lib/libizpi_gpu.so
    timeout -k 10 300 python tools/tune.py --config $CFG --spp $SPP --rounds 1 2>&1 | grep -E "round|CLOCKS" | sed "s/^/$v /" || exit 1
  done
done
cp /tmp/keep.so izpi_amd/_lib/libizpi_gpu.so
