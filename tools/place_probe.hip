// Placement probe (shading-time modes): does the speed of k_shade's kind of
// access depend on WHICH pages a buffer got? Allocates buffers of a given size several times
// (each new one while the previous ones are still held, so it lands on other pages) and
// times, on each, kernels of one access shape:
//   rec   : 24-B records at random record slots (slot * 192 + level * 24), written then read,
//           as k_shade's unwinding records ([rslot][depth])
//   strm  : 16 B per lane, consecutive (the wavefront state's streams)
//   line  : one 8-B read per random 4-KB page (translation-bound: every access a new page)
// One JSON line per (size, allocation, shape): ms over `reps` launches.
//
//   hipcc --offload-arch=gfx950 -O3 -o izpi_amd/_lib/place_probe tools/place_probe.hip
//   izpi_amd/_lib/place_probe [GB ...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
  } while (0)

__device__ inline uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

// per thread-iteration: write a 24-B record (3 doubles) at a random slot's random level
__global__ void k_rec(double* a, uint64_t slots, uint32_t iters, uint64_t seed) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  for (uint32_t k = 0; k < iters; k++) {
    const uint64_t h = mix(seed ^ (t * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)k << 40));
    const uint64_t slot = h % slots, lvl = (h >> 48) & 7;
    double* r = a + slot * 24 + lvl * 3;
    r[0] = (double)k; r[1] = (double)t; r[2] = 1.0;
  }
}
__global__ void k_recread(const double* a, uint64_t slots, uint32_t iters, uint64_t seed, double* out) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  double acc = 0;
  for (uint32_t k = 0; k < iters; k++) {
    const uint64_t h = mix(seed ^ (t * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)k << 40));
    const uint64_t slot = h % slots;
    const double* r = a + slot * 24;
    acc += r[0] + r[3] + r[6];  // three levels of one slot
  }
  if (acc == 12345.678) out[0] = acc;
}
__global__ void k_strm(uint4* a, uint64_t n16) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    uint4 v = a[i];
    v.x += 1;
    a[i] = v;
  }
}
__global__ void k_page(const double* a, uint64_t pages, uint32_t iters, uint64_t seed, double* out) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  double acc = 0;
  for (uint32_t k = 0; k < iters; k++) {
    const uint64_t h = mix(seed ^ (t * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)k << 40));
    acc += a[(h % pages) * 512];
  }
  if (acc == 12345.678) out[0] = acc;
}

// both at once, as a shading pass does: a streamed 16-B read-modify-write of the state
// buffer s and a random 24-B record write into the record buffer r per thread-iteration
// RW: bytes per record (24: 3 doubles at level * 24; 32: the same 3 doubles at level * 32,
// each record in one aligned 32-B sector; 64: one record per 64-B half line)
// FULL: the record's whole RW / 8 bytes are written (a pad word too), not just its 24 B
template <int RW, bool FULL = false>
__global__ void k_mix(uint4* s, uint64_t n16, double* r, uint64_t slots, uint64_t seed) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint32_t k = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += stride, k++) {
    uint4 v = s[i];
    v.x += 1;
    s[i] = v;
    const uint64_t h = mix(seed ^ (i * 0x9E3779B97F4A7C15ull));
    double* q = r + (h % slots) * (RW) + ((h >> 48) & 7) * (RW / 8);
    q[0] = (double)k; q[1] = (double)v.y; q[2] = 1.0;
    if (FULL)
      for (int w = 3; w < RW / 8; w++) q[w] = 0.0;
  }
}

// `mix` mode: the state buffer and the record buffer re-allocated in turn, each new one
// while the old is held: does the PAIR's placement set the time?
int mix_mode(double state_gb, double rec_gb, int rounds, int rw) {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int blocks = prop.multiProcessorCount * 8;
  const uint64_t sb = (uint64_t)(state_gb * 1e9) & ~((uint64_t)(1 << 21) - 1), rb = (uint64_t)(rec_gb * 1e9) & ~((uint64_t)(1 << 21) - 1);
  void *S = nullptr, *R = nullptr;
  CK(hipMalloc(&S, sb)); CK(hipMalloc(&R, rb));
  CK(hipMemset(S, 0, sb)); CK(hipMemset(R, 0, rb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<void*> old;
  for (int k = 0; k < rounds; k++) {
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
      CK(hipEventRecord(e0));
      // the same number of record slots for every record width (8 levels of rw bytes per slot)
      const uint64_t slots = rb / (8 * 64);
      if (rw == 24) hipLaunchKernelGGL(k_mix<24>, dim3(blocks), dim3(256), 0, 0, (uint4*)S, sb / 16, (double*)R, slots, 11ull + r);
      if (rw == 32) hipLaunchKernelGGL(k_mix<32>, dim3(blocks), dim3(256), 0, 0, (uint4*)S, sb / 16, (double*)R, slots, 11ull + r);
      if (rw == 64) hipLaunchKernelGGL(k_mix<64>, dim3(blocks), dim3(256), 0, 0, (uint4*)S, sb / 16, (double*)R, slots, 11ull + r);
      if (rw == 33) hipLaunchKernelGGL((k_mix<32, true>), dim3(blocks), dim3(256), 0, 0, (uint4*)S, sb / 16, (double*)R, slots, 11ull + r);
      if (rw == 65) hipLaunchKernelGGL((k_mix<64, true>), dim3(blocks), dim3(256), 0, 0, (uint4*)S, sb / 16, (double*)R, slots, 11ull + r);
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("{\"mode\": \"mix\", \"rec_bytes\": %d, \"round\": %d, \"realloc\": \"%s\", \"ms\": %.3f}\n", rw, k, k == 0 ? "none" : (k % 2 ? "rec" : "state"), best);
    fflush(stdout);
    void** which = (k % 2 == 0) ? &R : &S;  // next round: re-allocate one of the two
    const uint64_t bytes = which == &R ? rb : sb;
    void* fresh = nullptr;
    CK(hipMalloc(&fresh, bytes));
    CK(hipMemset(fresh, 0, bytes));
    old.push_back(*which);
    if (old.size() > 2) { CK(hipFree(old.front())); old.erase(old.begin()); }
    *which = fresh;
  }
  return 0;
}

int main(int argc, char** argv) {
  // place_probe mix STATE_GB REC_GB ROUNDS REC_BYTES (24, 32, 64; 33 / 65: 32 / 64 written whole)
  if (argc > 1 && argv[1][0] == 'm')
    return mix_mode(argc > 2 ? atof(argv[2]) : 20.0, argc > 3 ? atof(argv[3]) : 25.0, argc > 4 ? atoi(argv[4]) : 10, argc > 5 ? atoi(argv[5]) : 24);
  std::vector<double> sizes;
  for (int i = 1; i < argc; i++) sizes.push_back(atof(argv[i]));
  if (sizes.empty()) sizes = {25.0, 2.0};
  const int allocs = 4, reps = 3;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int blocks = prop.multiProcessorCount * 8;
  double* out;
  CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (double gb : sizes) {
    const uint64_t bytes = (uint64_t)(gb * 1e9) & ~((uint64_t)(1 << 21) - 1);
    std::vector<void*> held;
    for (int a = 0; a < allocs; a++) {
      void* p = nullptr;
      CK(hipMalloc(&p, bytes));
      held.push_back(p);
      CK(hipMemset(p, 0, bytes));
      const uint64_t slots = bytes / 192, pages = bytes / 4096;
      const uint32_t iters = 64;
      const char* names[] = {"rec_write", "rec_read", "strm", "page"};
      for (int s = 0; s < 4; s++) {
        float best = 1e30f;
        for (int r = 0; r < reps; r++) {
          CK(hipEventRecord(e0));
          if (s == 0) hipLaunchKernelGGL(k_rec, dim3(blocks), dim3(256), 0, 0, (double*)p, slots, iters, 77ull + r);
          if (s == 1) hipLaunchKernelGGL(k_recread, dim3(blocks), dim3(256), 0, 0, (const double*)p, slots, iters, 99ull + r, out);
          if (s == 2) hipLaunchKernelGGL(k_strm, dim3(blocks), dim3(256), 0, 0, (uint4*)p, bytes / 16);
          if (s == 3) hipLaunchKernelGGL(k_page, dim3(blocks), dim3(256), 0, 0, (const double*)p, pages, iters, 55ull + r, out);
          CK(hipGetLastError());
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (ms < best) best = ms;
        }
        const double accesses = (double)blocks * 256 * (s == 2 ? (double)(bytes / 16) / (blocks * 256.0) : iters);
        printf("{\"gb\": %.1f, \"alloc\": %d, \"shape\": \"%s\", \"ms\": %.3f, \"ns_per_access_per_cu\": %.3f}\n", gb, a,
               names[s], best, best * 1e6 / accesses * prop.multiProcessorCount);
        fflush(stdout);
      }
    }
    for (void* p : held) CK(hipFree(p));
  }
  return 0;
}
