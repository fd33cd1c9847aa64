// FETCH_SIZE calibration for k_trace2's access shapes (roofline): kernels whose
// memory-side read bytes are known exactly, to be run under `rocprofv3 --pmc FETCH_SIZE`.
//
//   hipcc --offload-arch=gfx950 -O3 -o izpi_amd/_lib/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o run -- izpi_amd/_lib/fetch_calib
//
// Every kernel touches each of its lines exactly once (a bijective line map), from a table
// far larger than the 256 MB Infinity Cache (2 GiB, after a flush of another 2 GiB buffer)
// or from one that fits in it and was read once before (64 MiB, "warm"):
//   stream   : 16 B per lane, consecutive (the guide's calibration shape)
//   node     : one 128-B line per lane, read as eight 16-B loads (an inner BVH4 node)
//   tri80    : one 80-B record per lane at 80-B spacing, five 16-B loads (a GPrim)
//   rec48    : one 48-B record per lane, consecutive lanes consecutive records (a ray refill)
//   half32   : 32 B of a random line per lane (a GLeaf record)
// Each line of the output names the kernel launch order, so the counter CSV's dispatch ids
// map to them.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } \
  } while (0)

// odd multiplier: i -> (i * M) mod 2^k is a bijection on [0, 2^k)
__device__ inline uint64_t perm(uint64_t i, uint64_t mask) { return (i * 0x9E3779B97F4A7C15ull) & mask; }

__global__ void k_stream(const uint4* __restrict__ a, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_node(const uint4* __restrict__ a, uint64_t lines_mask, uint64_t nthreads, uint32_t* out) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  if (t >= nthreads) return;
  const uint4* p = a + perm(t, lines_mask) * 8;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) { const uint4 v = p[k]; acc ^= v.x ^ v.y; }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_tri80(const uint4* __restrict__ a, uint64_t rec_mask, uint64_t nthreads, uint32_t* out) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  if (t >= nthreads) return;
  const uint4* p = a + perm(t, rec_mask) * 5;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 5; k++) { const uint4 v = p[k]; acc ^= v.x ^ v.z; }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_rec48(const uint4* __restrict__ a, uint64_t nthreads, uint32_t* out) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  if (t >= nthreads) return;
  const uint4* p = a + t * 3;
  const uint4 v0 = p[0], v1 = p[1], v2 = p[2];
  const uint32_t acc = v0.x ^ v1.y ^ v2.z;
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_half32(const uint4* __restrict__ a, uint64_t lines_mask, uint64_t nthreads, uint32_t* out) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  if (t >= nthreads) return;
  const uint4* p = a + perm(t, lines_mask) * 8;
  const uint4 v0 = p[0], v1 = p[1];
  const uint32_t acc = v0.x ^ v1.y;
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_touch(uint4* a, uint64_t n16) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
    a[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main() {
  const uint64_t big = 2ull << 30, warm = 64ull << 20;
  uint4 *a, *flush;
  uint32_t* out;
  CK(hipMalloc(&a, big));
  CK(hipMalloc(&flush, big));
  CK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, 0, a, big / 16);
  CK(hipDeviceSynchronize());
  int launch = 0;
  auto flush_all = [&]() { hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, 0, flush, big / 16); launch++; };
  // insts: the wave-level vector-memory load instructions the kernel issues (every lane
  // active; to check which SQ counter counts global_load issue on gfx950)
  auto report = [&](const char* name, const char* table, double bytes, double lines, double insts) {
    printf("{\"launch\": %d, \"kernel\": \"%s\", \"table\": \"%s\", \"useful_bytes\": %.0f, \"line_bytes\": %.0f, "
           "\"load_insts\": %.0f}\n", launch, name, table, bytes, lines * 128, insts);
    launch++;
  };
  for (int pass = 0; pass < 2; pass++) {  // pass 0: cold 2 GiB table, pass 1: 64 MiB table read once before
    const uint64_t tb = pass == 0 ? big : warm;
    const char* tn = pass == 0 ? "cold_2GiB" : "warm_64MiB";
    const uint64_t lines = tb / 128;
    const uint64_t nt = lines / 2;  // half the lines: each once
    const uint64_t grid = (nt + 255) / 256;
    // stream
    if (pass == 0) flush_all(); else { hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, a, tb / 16, out); launch++; }
    hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, a, tb / 16, out);
    report("stream", tn, (double)tb, (double)tb / 128, (double)(tb / 16) / 64);
    // node lines
    if (pass == 0) flush_all(); else { hipLaunchKernelGGL(k_node, dim3(grid), dim3(256), 0, 0, a, lines - 1, nt, out); launch++; }
    hipLaunchKernelGGL(k_node, dim3(grid), dim3(256), 0, 0, a, lines - 1, nt, out);
    report("node128", tn, (double)nt * 128, (double)nt, 8.0 * (double)((nt + 63) / 64));
    // 80-B records: a power-of-two count of them inside the table
    uint64_t recs = 1;
    while (recs * 2 * 80 <= tb) recs *= 2;
    const uint64_t nr = recs / 2, gr = (nr + 255) / 256;
    if (pass == 0) flush_all(); else { hipLaunchKernelGGL(k_tri80, dim3(gr), dim3(256), 0, 0, a, recs - 1, nr, out); launch++; }
    hipLaunchKernelGGL(k_tri80, dim3(gr), dim3(256), 0, 0, a, recs - 1, nr, out);
    double l80 = 0;  // lines each touched record spans (a line shared by two touched records counts twice)
    for (uint64_t t = 0; t < nr; t++) {
      const uint64_t r = (t * 0x9E3779B97F4A7C15ull) & (recs - 1);
      l80 += (double)((80 * r + 79) / 128 - (80 * r) / 128 + 1);
    }
    report("tri80", tn, (double)nr * 80, l80, 5.0 * (double)((nr + 63) / 64));
    // 48-B consecutive records
    const uint64_t n48 = tb / 48 / 2, g48 = (n48 + 255) / 256;
    if (pass == 0) flush_all(); else { hipLaunchKernelGGL(k_rec48, dim3(g48), dim3(256), 0, 0, a, n48, out); launch++; }
    hipLaunchKernelGGL(k_rec48, dim3(g48), dim3(256), 0, 0, a, n48, out);
    report("rec48", tn, (double)n48 * 48, (double)n48 * 48 / 128, 3.0 * (double)((n48 + 63) / 64));
    // 32 B of a random line
    if (pass == 0) flush_all(); else { hipLaunchKernelGGL(k_half32, dim3(grid), dim3(256), 0, 0, a, lines - 1, nt, out); launch++; }
    hipLaunchKernelGGL(k_half32, dim3(grid), dim3(256), 0, 0, a, lines - 1, nt, out);
    report("half32", tn, (double)nt * 32, (double)nt, 2.0 * (double)((nt + 63) / 64));
  }
  CK(hipDeviceSynchronize());
  CK(hipFree(a));
  CK(hipFree(flush));
  CK(hipFree(out));
  return 0;
}
