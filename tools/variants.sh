#!/bin/bash
# Build experiment variants of libizpi_gpu.so: tools/variants.sh NAME "HIPCC FLAGS" [NAME "FLAGS" ...]
# -> izpi_amd/_lib/variants/NAME.so (load one with IZPI_LIB_PATH=...; tools/vrun.sh times them).
set -e
cd "$(dirname "$0")/.."
mkdir -p izpi_amd/_lib/variants
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -shared"
SRC="izpi_amd/csrc/izpi_gpu.hip izpi_amd/csrc/bvh_build.hip izpi_amd/csrc/host_scene.cpp izpi_amd/csrc/scene_io.cpp"
while [ $# -ge 2 ]; do
  $H $2 -o izpi_amd/_lib/variants/$1.so $SRC -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
  shift 2
done
wait
ls -la izpi_amd/_lib/variants/
