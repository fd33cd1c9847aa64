#!/bin/bash
# Build A/B variants of libizpi_gpu.so into izpi_amd/_lib/variants/:
#   A = HEAD (git stash of the working tree), B = working tree,
#   CLK = working tree with -DIZPI_TRACE_CLOCKS (per-phase cycle counters).
# Extra hipcc flags for B: B_FLAGS="...". Leaves the tree as it was.
set -e
cd "$(dirname "$0")/.."
mkdir -p izpi_amd/_lib/variants
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -shared"
SRC="izpi_amd/csrc/izpi_gpu.hip izpi_amd/csrc/bvh_build.hip izpi_amd/csrc/host_scene.cpp izpi_amd/csrc/scene_io.cpp"
$H $B_FLAGS -o izpi_amd/_lib/variants/B.so $SRC &
if [ -n "$CLK" ]; then $H -DIZPI_TRACE_CLOCKS -o izpi_amd/_lib/variants/CLK.so $SRC & fi
wait
if [ -z "$NO_A" ]; then
  git stash -q
  trap 'git stash pop -q' EXIT
  $H -o izpi_amd/_lib/variants/A.so $SRC
fi
