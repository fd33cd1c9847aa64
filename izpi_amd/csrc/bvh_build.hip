// bvh_build.hip — GPU BVH4 builder.
//
// The reference builds its BVH4 on the host (hitable/bvh4.go:517-855): a binary tree of
// median splits on a random axis (sort.Slice per node), collapsed to 4-wide nodes by
// collectChildren and flattened with conservative float32 bounds. That topology is
// reproduced bit for bit by host_scene.cpp and stays the default: every parity claim
// rests on it.
//
// This builder is the fast alternative for large meshes. It emits the SAME node format
// (izpi_bvh4_node == BVH4Node: leaf nodes separate, slot 0 = (primStart, count <= 4),
// conservative f32 bounds, empty slots MaxFloat32), so the traversal kernels run on it
// unchanged; only the topology differs (a linear BVH instead of random-axis medians):
//
//   1. per-primitive centroid bounds (two-stage reduction)
//   2. 63-bit Morton codes (21 bits per axis) of the centroids
//   3. rocPRIM radix sort of (code, primitive) pairs
//   4. Karras' binary radix tree over the sorted codes (equal codes split by index):
//      one thread per internal node, no dependency between nodes
//   5. bottom-up f64 box refit (each leaf walks up; the second child to arrive at a
//      node writes its box)
//   6. top-down collapse to BVH4, one level per launch: a frontier node gathers up to
//      four descendants with collectChildren's rule (bvh4.go:796-855; subtrees of <=
//      leaf_max primitives are leaves; the largest-area inner child is expanded first), node indices come from an exclusive scan of the child
//      counts, so the output is deterministic and children follow their parents
//      (breadth-first order: the hot top levels are contiguous)
//
// Images rendered on this tree equal the reference-tree images except where the
// traversal order matters: equal-t hits (the later primitive wins, bvh4.go:123-134) and
// float32 box culling at tMax. The parity tests check the closest-hit distances against
// the reference tree and the images statistically (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/izpi_types.h"
#include "gomath.h"

namespace izpi_bvh {

namespace {

#define BVH_TRY(expr)                                                       \
  do {                                                                      \
    hipError_t e_ = (expr);                                                 \
    if (e_ != hipSuccess) {                                                 \
      err = std::string(#expr) + ": " + hipGetErrorString(e_);              \
      return IZPI_ERR_HIP;                                                  \
    }                                                                       \
  } while (0)

constexpr float kMaxF32 = 3.40282346638528859811704183484516925440e+38f;

// bvh4.go:494-514
__device__ __forceinline__ float cons_min(double v) {
  const float f = (float)v;
  return (double)f > v ? gm::nextafter32(f, -__builtin_inff()) : f;
}
__device__ __forceinline__ float cons_max(double v) {
  const float f = (float)v;
  return (double)f < v ? gm::nextafter32(f, __builtin_inff()) : f;
}

struct Box6 { double v[6]; };  // min xyz, max xyz

__global__ void k_centroid_partial(const Box6* boxes, uint32_t n, double* partial) {
  __shared__ double red[6][256];
  double lo[3] = {__builtin_inf(), __builtin_inf(), __builtin_inf()};
  double hi[3] = {-__builtin_inf(), -__builtin_inf(), -__builtin_inf()};
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const Box6 b = boxes[i];
    for (int k = 0; k < 3; k++) {
      const double c = (b.v[k] + b.v[k + 3]) * 0.5;
      lo[k] = fmin(lo[k], c);
      hi[k] = fmax(hi[k], c);
    }
  }
  for (int k = 0; k < 3; k++) { red[k][threadIdx.x] = lo[k]; red[k + 3][threadIdx.x] = hi[k]; }
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < (unsigned)s)
      for (int k = 0; k < 3; k++) {
        red[k][threadIdx.x] = fmin(red[k][threadIdx.x], red[k][threadIdx.x + s]);
        red[k + 3][threadIdx.x] = fmax(red[k + 3][threadIdx.x], red[k + 3][threadIdx.x + s]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 6) partial[blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void k_centroid_final(const double* partial, uint32_t nblocks, double* bounds) {
  if (threadIdx.x >= 6) return;
  const bool is_min = threadIdx.x < 3;
  double r = is_min ? __builtin_inf() : -__builtin_inf();
  for (uint32_t b = 0; b < nblocks; b++) {
    const double v = partial[b * 6 + threadIdx.x];
    r = is_min ? fmin(r, v) : fmax(r, v);
  }
  bounds[threadIdx.x] = r;
}

__device__ __forceinline__ uint64_t spread21(uint64_t x) {  // 21 bits -> every third bit
  x &= 0x1FFFFFull;
  x = (x | x << 32) & 0x1F00000000FFFFull;
  x = (x | x << 16) & 0x1F0000FF0000FFull;
  x = (x | x << 8) & 0x100F00F00F00F00Full;
  x = (x | x << 4) & 0x10C30C30C30C30C3ull;
  x = (x | x << 2) & 0x1249249249249249ull;
  return x;
}

__global__ void k_morton(const Box6* boxes, uint32_t n, const double* bounds, uint64_t* codes, uint32_t* ids) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const Box6 b = boxes[i];
  uint64_t q[3];
  for (int k = 0; k < 3; k++) {
    const double c = (b.v[k] + b.v[k + 3]) * 0.5;
    const double ext = bounds[k + 3] - bounds[k];
    double t = ext > 0 ? (c - bounds[k]) / ext : 0.0;
    t = fmin(fmax(t * 2097152.0, 0.0), 2097151.0);
    q[k] = (uint64_t)t;
  }
  codes[i] = (spread21(q[0]) << 2) | (spread21(q[1]) << 1) | spread21(q[2]);
  ids[i] = i;
}

// Karras 2012: binary radix tree. Nodes 0..n-2 are internal (0 = root), leaves are
// encoded as n-1+i (sorted position i). Equal codes compare by position.
__device__ __forceinline__ int delta(const uint64_t* k, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  const uint64_t a = k[i], b = k[j];
  if (a == b) return 64 + __clz((uint32_t)(i ^ j));
  return __clzll((long long)(a ^ b));
}

__global__ void k_karras(const uint64_t* k, int n, int32_t* left, int32_t* right, int32_t* first, int32_t* last,
                         int32_t* parent) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n - 1) return;
  const int d = delta(k, n, i, i + 1) - delta(k, n, i, i - 1) >= 0 ? 1 : -1;
  const int dmin = delta(k, n, i, i - d);
  int lmax = 2;
  while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(k, n, i, j);
  int s = 0;
  for (int t = (l + 1) >> 1;; t = (t + 1) >> 1) {
    if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
    if (t == 1) break;
  }
  const int split = i + s * d + min(d, 0);
  const int lo = min(i, j), hi = max(i, j);
  const int L = lo == split ? (n - 1) + split : split;
  const int R = hi == split + 1 ? (n - 1) + split + 1 : split + 1;
  left[i] = L;
  right[i] = R;
  first[i] = lo;
  last[i] = hi;
  parent[L] = i;
  parent[R] = i;
  if (i == 0) parent[0] = -1;
}

// Bottom-up refit of the f64 boxes; leaf boxes are the primitives' boxes.
__global__ void k_refit(const Box6* prim_boxes, const uint32_t* ids, int n, const int32_t* left, const int32_t* right,
                        const int32_t* parent, Box6* nb, uint32_t* flags) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int node = (n - 1) + i;
  nb[node] = prim_boxes[ids[i]];
  if (n == 1) return;
  node = parent[node];
  while (node >= 0) {
    __threadfence();
    if (atomicAdd(&flags[node], 1u) == 0) return;  // first child to arrive: the sibling finishes
    __threadfence();
    // the sibling's box was written by another wave, possibly on another CU: read it
    // past the (non-coherent) L1
    const volatile double* a = nb[left[node]].v;
    const volatile double* b = nb[right[node]].v;
    Box6 r;
    for (int k = 0; k < 3; k++) {
      r.v[k] = fmin(a[k], b[k]);
      r.v[k + 3] = fmax(a[k + 3], b[k + 3]);
    }
    nb[node] = r;
    node = parent[node];
  }
}

struct Tree {
  const int32_t* left;
  const int32_t* right;
  const int32_t* first;
  const int32_t* last;
  const Box6* box;
  int n;
  int leaf_max;
  __device__ int size(int b) const { return b >= n - 1 ? 1 : last[b] - first[b] + 1; }
  __device__ int start(int b) const { return b >= n - 1 ? b - (n - 1) : first[b]; }
  __device__ bool is_leaf(int b) const { return size(b) <= leaf_max; }
};

// collectChildren (bvh4.go:796-855) on the binary tree, leaves = subtrees of <= leaf_max.
// Where the reference expands the first inner child, this expands the one with the
// largest surface area (measured: 7% fewer node visits on C3's mesh).
__device__ int collect(const Tree& t, int b, int* res) {
  int c = 0;
  res[c++] = t.left[b];
  res[c++] = t.right[b];
  bool expanded = true;
  while (expanded && c < 4) {
    expanded = false;
    int pick = -1;
    double best = -1.0;
    for (int i = 0; i < c; i++) {
      if (t.is_leaf(res[i])) continue;
      const double* x = t.box[res[i]].v;
      const double dx = x[3] - x[0], dy = x[4] - x[1], dz = x[5] - x[2];
      const double area = dx * dy + dy * dz + dz * dx;
      if (area > best) { best = area; pick = i; }
    }
    if (pick >= 0) {  // c <= 3 here, so the two children fit
      const int cur = res[pick];
      for (int k = pick; k + 1 < c; k++) res[k] = res[k + 1];
      c--;
      res[c++] = t.left[cur];
      res[c++] = t.right[cur];
      expanded = true;
    }
  }
  return c;
}

// Pass 1 of a level: how many BVH4 nodes each frontier node's children need.
__global__ void k_level_count(const Tree t, const int32_t* frontier, uint32_t nf, uint32_t* counts) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  if (f >= nf) return;
  int res[4];
  counts[f] = (uint32_t)collect(t, frontier[f], res);
}

__device__ void set_slot(izpi_bvh4_node& nd, int s, const Box6& b) {
  nd.min_x[s] = cons_min(b.v[0]); nd.min_y[s] = cons_min(b.v[1]); nd.min_z[s] = cons_min(b.v[2]);
  nd.max_x[s] = cons_max(b.v[3]); nd.max_y[s] = cons_max(b.v[4]); nd.max_z[s] = cons_max(b.v[5]);
}

__device__ izpi_bvh4_node empty_node() {
  izpi_bvh4_node nd;
  for (int s = 0; s < 4; s++) {
    nd.child[s] = -1; nd.prim_count[s] = 0;
    nd.min_x[s] = nd.min_y[s] = nd.min_z[s] = nd.max_x[s] = nd.max_y[s] = nd.max_z[s] = kMaxF32;
  }
  return nd;
}

// Pass 2: write the frontier's BVH4 nodes; children get consecutive indices from the
// scan (base + offset); inner children form the next frontier in the same order.
__global__ void k_level_write(const Tree t, const int32_t* frontier, const uint32_t* fnode, uint32_t nf,
                              const uint32_t* offsets, uint32_t base, izpi_bvh4_node* out, int32_t* next,
                              uint32_t* next_node, uint32_t* next_count) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  if (f >= nf) return;
  int res[4];
  const int c = collect(t, frontier[f], res);
  izpi_bvh4_node nd = empty_node();
  for (int s = 0; s < c; s++) {
    const int b = res[s];
    const uint32_t idx = base + offsets[f] + (uint32_t)s;
    nd.child[s] = (int32_t)idx;
    set_slot(nd, s, t.box[b]);
    if (t.is_leaf(b)) {  // leaf node: slot 0 = (primStart, count), the same box (bvh4.go:736-760)
      izpi_bvh4_node lf = empty_node();
      lf.child[0] = t.start(b);
      lf.prim_count[0] = t.size(b);
      set_slot(lf, 0, t.box[b]);
      out[idx] = lf;
    } else {
      const uint32_t q = atomicAdd(next_count, 1u);
      next[q] = b;
      next_node[q] = idx;
    }
  }
  out[fnode[f]] = nd;
}

__global__ void k_single_leaf(const Tree t, izpi_bvh4_node* out) {
  izpi_bvh4_node lf = empty_node();
  lf.child[0] = 0;
  lf.prim_count[0] = t.n;
  set_slot(lf, 0, t.box[0]);  // binary root: internal node 0, or the lone leaf (n - 1 + 0)
  out[0] = lf;
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t n) { return hipMalloc((void**)&p, std::max<size_t>(1, n) * sizeof(T)); }
};

}  // namespace

// Build a BVH4 over n primitive boxes ([n][6] f64 host array: min xyz, max xyz).
// Outputs the nodes (BVH4Node format, breadth-first, root 0) and the leaf order
// (order[k] = input index of the k-th primitive in leaf order).
int build(hipStream_t st, const double* h_boxes, uint32_t n, uint32_t leaf_max, std::vector<izpi_bvh4_node>& nodes,
          std::vector<uint32_t>& order, float* ms, std::string& err) {
  nodes.clear();
  order.clear();
  if (n == 0) return IZPI_OK;
  if (leaf_max < 1 || leaf_max > 4) { err = "leaf_max must be 1..4 (bvh4.go:638)"; return IZPI_ERR_INVALID; }
  if (n > (1u << 27)) { err = "too many primitives for the leaf-ref encoding"; return IZPI_ERR_UNSUPPORTED; }
  hipEvent_t e0, e1;
  BVH_TRY(hipEventCreate(&e0));
  BVH_TRY(hipEventCreate(&e1));
  DevBuf<Box6> boxes, nb;
  DevBuf<double> partial, bounds;
  DevBuf<uint64_t> codes, codes_s;
  DevBuf<uint32_t> ids, ids_s, flags, counts, offsets, fnode, next_node, next_count;
  DevBuf<int32_t> left, right, first, last, parent, frontier, next;
  DevBuf<izpi_bvh4_node> out;
  DevBuf<uint8_t> temp;
  const int ni = (int)n;
  const uint32_t nint = n > 1 ? n - 1 : 0, ntot = 2 * n - 1;
  BVH_TRY(boxes.alloc(n));
  BVH_TRY(nb.alloc(ntot));
  const uint32_t pblocks = std::min<uint32_t>(1024, (n + 255) / 256);
  BVH_TRY(partial.alloc(pblocks * 6));
  BVH_TRY(bounds.alloc(6));
  BVH_TRY(codes.alloc(n)); BVH_TRY(codes_s.alloc(n));
  BVH_TRY(ids.alloc(n)); BVH_TRY(ids_s.alloc(n));
  BVH_TRY(left.alloc(nint)); BVH_TRY(right.alloc(nint)); BVH_TRY(first.alloc(nint)); BVH_TRY(last.alloc(nint));
  BVH_TRY(parent.alloc(ntot)); BVH_TRY(flags.alloc(nint));
  BVH_TRY(out.alloc(2 * (size_t)n));
  BVH_TRY(frontier.alloc(n)); BVH_TRY(fnode.alloc(n)); BVH_TRY(next.alloc(n)); BVH_TRY(next_node.alloc(n));
  BVH_TRY(counts.alloc(n)); BVH_TRY(offsets.alloc(n + 1)); BVH_TRY(next_count.alloc(1));
  BVH_TRY(hipMemcpyAsync(boxes.p, h_boxes, (size_t)n * sizeof(Box6), hipMemcpyHostToDevice, st));
  BVH_TRY(hipEventRecord(e0, st));
  const dim3 g((n + 255) / 256);
  hipLaunchKernelGGL(k_centroid_partial, dim3(pblocks), dim3(256), 0, st, boxes.p, n, partial.p);
  hipLaunchKernelGGL(k_centroid_final, dim3(1), dim3(64), 0, st, partial.p, pblocks, bounds.p);
  hipLaunchKernelGGL(k_morton, g, dim3(256), 0, st, boxes.p, n, bounds.p, codes.p, ids.p);
  BVH_TRY(hipGetLastError());
  size_t temp_bytes = 0;
  BVH_TRY(rocprim::radix_sort_pairs(nullptr, temp_bytes, codes.p, codes_s.p, ids.p, ids_s.p, (size_t)n, 0, 63, st));
  BVH_TRY(temp.alloc(temp_bytes));
  BVH_TRY(rocprim::radix_sort_pairs(temp.p, temp_bytes, codes.p, codes_s.p, ids.p, ids_s.p, (size_t)n, 0, 63, st));
  Tree t{left.p, right.p, first.p, last.p, nb.p, ni, (int)leaf_max};
  uint32_t total = 0;
  if (n > 1) {
    hipLaunchKernelGGL(k_karras, dim3((nint + 255) / 256), dim3(256), 0, st, codes_s.p, ni, left.p, right.p, first.p,
                       last.p, parent.p);
    BVH_TRY(hipMemsetAsync(flags.p, 0, nint * sizeof(uint32_t), st));
  }
  hipLaunchKernelGGL(k_refit, g, dim3(256), 0, st, boxes.p, ids_s.p, ni, left.p, right.p, parent.p, nb.p, flags.p);
  BVH_TRY(hipGetLastError());
  if (n <= leaf_max) {  // the whole scene is one leaf (bvh4.go:638: len <= 4)
    hipLaunchKernelGGL(k_single_leaf, dim3(1), dim3(1), 0, st, t, out.p);
    total = 1;
  } else {
    // level 0: the binary root becomes BVH4 node 0
    const int32_t root = 0;
    const uint32_t zero = 0;
    BVH_TRY(hipMemcpyAsync(frontier.p, &root, sizeof(root), hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemcpyAsync(fnode.p, &zero, sizeof(zero), hipMemcpyHostToDevice, st));
    uint32_t nf = 1;
    total = 1;
    size_t scan_bytes = 0;
    BVH_TRY(rocprim::exclusive_scan(nullptr, scan_bytes, counts.p, offsets.p, 0u, (size_t)n, rocprim::plus<uint32_t>(), st));
    DevBuf<uint8_t> scan_temp;
    BVH_TRY(scan_temp.alloc(scan_bytes));
    while (nf > 0) {
      hipLaunchKernelGGL(k_level_count, dim3((nf + 255) / 256), dim3(256), 0, st, t, frontier.p, nf, counts.p);
      size_t sb = scan_bytes;
      BVH_TRY(rocprim::exclusive_scan(scan_temp.p, sb, counts.p, offsets.p, 0u, (size_t)nf, rocprim::plus<uint32_t>(), st));
      uint32_t last_count = 0, last_off = 0;
      BVH_TRY(hipMemcpyAsync(&last_count, counts.p + nf - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      BVH_TRY(hipMemcpyAsync(&last_off, offsets.p + nf - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      BVH_TRY(hipMemsetAsync(next_count.p, 0, sizeof(uint32_t), st));
      BVH_TRY(hipStreamSynchronize(st));
      const uint32_t nchild = last_off + last_count;
      hipLaunchKernelGGL(k_level_write, dim3((nf + 255) / 256), dim3(256), 0, st, t, frontier.p, fnode.p, nf, offsets.p,
                         total, out.p, next.p, next_node.p, next_count.p);
      BVH_TRY(hipGetLastError());
      uint32_t nn = 0;
      BVH_TRY(hipMemcpyAsync(&nn, next_count.p, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      BVH_TRY(hipStreamSynchronize(st));
      total += nchild;
      if (nn) {
        // deterministic frontier order: sort the appended entries by their node index
        size_t sb2 = 0;
        BVH_TRY(rocprim::radix_sort_pairs(nullptr, sb2, next_node.p, fnode.p, next.p, frontier.p, (size_t)nn, 0, 32, st));
        if (sb2 > temp_bytes) {
          if (temp.p) (void)hipFree(temp.p);
          temp.p = nullptr;
          BVH_TRY(temp.alloc(sb2));
          temp_bytes = sb2;
        }
        BVH_TRY(rocprim::radix_sort_pairs(temp.p, sb2, next_node.p, fnode.p, next.p, frontier.p, (size_t)nn, 0, 32, st));
      }
      nf = nn;
    }
  }
  BVH_TRY(hipEventRecord(e1, st));
  nodes.resize(total);
  order.resize(n);
  BVH_TRY(hipMemcpyAsync(nodes.data(), out.p, (size_t)total * sizeof(izpi_bvh4_node), hipMemcpyDeviceToHost, st));
  BVH_TRY(hipMemcpyAsync(order.data(), ids_s.p, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  BVH_TRY(hipStreamSynchronize(st));
  if (ms) BVH_TRY(hipEventElapsedTime(ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return IZPI_OK;
}

}  // namespace izpi_bvh
