#!/bin/bash
# Build the library of a git revision as an A/B variant: tools/build_base_variant.sh REV NAME
# -> izpi_amd/_lib/variants/NAME.so (time it against the working tree with tools/vrun.sh)
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}; NAME=${2:-base}
T=$(mktemp -d)
git archive "$REV" izpi_amd/csrc include | tar -x -C "$T"
mkdir -p izpi_amd/_lib/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -shared -I"$T/include" \
  -o izpi_amd/_lib/variants/$NAME.so $T/izpi_amd/csrc/izpi_gpu.hip $T/izpi_amd/csrc/bvh_build.hip \
  $T/izpi_amd/csrc/host_scene.cpp $T/izpi_amd/csrc/scene_io.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$T"
ls -la izpi_amd/_lib/variants/$NAME.so
