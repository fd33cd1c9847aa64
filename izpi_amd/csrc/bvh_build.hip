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
//   4. the binary tree, one of two ways:
//      LBVH: Karras' binary radix tree over the sorted codes (equal codes split by
//      index), one thread per internal node, then a bottom-up f64 box refit (each leaf
//      walks up; the second child to arrive at a node writes its box);
//      PLOC (default): Meister & Bittner's locally-ordered clustering on the sorted
//      clusters: nearest neighbour by merged surface area within +-8 positions, mutual
//      pairs merge in place, compaction by scan, repeat; then DFS positions make every
//      subtree a contiguous primitive range (16% fewer node visits than the LBVH on C3)
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

#include "../../include/izpi_gpu.h"
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

constexpr int PLOC_RADIUS = 8;  // PLOC search window (+-positions); 8 and 16 measured equal on C3's mesh

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

// ---- PLOC (Meister & Bittner 2018): parallel locally-ordered clustering. Clusters stay
// in Morton order; each finds the neighbour within +-radius whose merged box has the
// smallest surface area (ties: the lower position), mutual pairs merge in place, the
// array is compacted, until one cluster is left. Ids: leaves 0..n-1 (sorted position),
// internal nodes n.. in creation order (position order within an iteration).
__device__ __forceinline__ Box6 unite(const Box6& a, const Box6& b) {
  Box6 r;
  for (int k = 0; k < 3; k++) {
    r.v[k] = fmin(a.v[k], b.v[k]);
    r.v[k + 3] = fmax(a.v[k + 3], b.v[k + 3]);
  }
  return r;
}
__device__ __forceinline__ double half_area(const Box6& a) {
  const double dx = a.v[3] - a.v[0], dy = a.v[4] - a.v[1], dz = a.v[5] - a.v[2];
  return dx * dy + dy * dz + dz * dx;
}

__global__ void k_ploc_init(const Box6* prim_boxes, const uint32_t* ids_s, uint32_t n, Box6* pbox, uint32_t* psize,
                            int32_t* pparent, int32_t* cl) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  pbox[i] = prim_boxes[ids_s[i]];
  psize[i] = 1;
  pparent[i] = -1;
  cl[i] = (int32_t)i;
}

__global__ void k_ploc_nn(const int32_t* cl, uint32_t m, const Box6* pbox, int radius, int32_t* nn) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (int)m) return;
  const Box6 bi = pbox[cl[i]];
  // ties (equal merged areas, e.g. coincident primitives) go to the nearer position and
  // then to i+1 for even i, i-1 for odd i: equal clusters pair up instead of chaining
  double best = __builtin_inf();
  int bj = -1, bkey = 0;
  const int lo = max(0, i - radius), hi = min((int)m - 1, i + radius);
  for (int j = lo; j <= hi; j++) {
    if (j == i) continue;
    const double a = half_area(unite(bi, pbox[cl[j]]));
    const int key = 2 * abs(j - i) + (((j > i) == ((i & 1) == 0)) ? 0 : 1);
    if (a < best || (a == best && key < bkey)) { best = a; bj = j; bkey = key; }
  }
  nn[i] = bj;
}

__global__ void k_ploc_flags(const int32_t* nn, uint32_t m, uint32_t* mflag, uint32_t* aflag) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (int)m) return;
  const int j = nn[i];
  const bool mutual = j >= 0 && nn[j] == i;
  mflag[i] = mutual && i < j;
  aflag[i] = !(mutual && i > j);
}

__global__ void k_ploc_merge(const int32_t* cl, uint32_t m, const int32_t* nn, const uint32_t* mflag, const uint32_t* mscan,
                             const uint32_t* aflag, const uint32_t* ascan, uint32_t base, int32_t* pl, int32_t* pr,
                             Box6* pbox, uint32_t* psize, int32_t* pparent, int32_t* cl2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (int)m || !aflag[i]) return;
  int32_t c = cl[i];
  if (mflag[i]) {
    const int32_t a = cl[i], b = cl[nn[i]];
    c = (int32_t)(base + mscan[i]);
    pl[c] = a;
    pr[c] = b;
    pbox[c] = unite(pbox[a], pbox[b]);
    psize[c] = psize[a] + psize[b];
    pparent[c] = -1;
    pparent[a] = c;
    pparent[b] = c;
  }
  cl2[ascan[i]] = c;
}

// DFS position of every node: the sizes of the left siblings along its path to the root
__global__ void k_ploc_offsets(uint32_t total, const int32_t* pl, const int32_t* pr, const uint32_t* psize,
                               const int32_t* pparent, uint32_t* off) {
  const uint32_t id = blockIdx.x * 256 + threadIdx.x;
  if (id >= total) return;
  uint32_t o = 0;
  int32_t x = (int32_t)id;
  for (int32_t p = pparent[x]; p >= 0; x = p, p = pparent[x])
    if (pr[p] == x) o += psize[pl[p]];
  off[id] = o;
}

// SAH-optimal collapse (the dynamic programme of Ylitie, Karras & Laine 2017 for 4-wide
// nodes): for every binary node n and i = 1..4, D(n, i) is the least SAH cost of covering
// n's subtree with at most i child slots of the wide node above it. A slot is either a
// leaf (<= leaf_max primitives: a leaf-node visit plus its primitive tests) or a wide node
// (one node visit plus the best split of its two binary children over 4 slots). Costs
// are weighted by surface area; the collapse then follows the recorded decisions instead
// of collectChildren's greedy expansion. dec bits: 0 = the single slot is a leaf, 1-2 =
// the wide node's split (k slots on the left), 3-4 / 5-6 / 7-8 = the split for i = 2 / 3 / 4
// (0: use i - 1 slots).
constexpr double SAH_CN = 1.0;  // visit of a wide node (one node step)
constexpr double SAH_CL = 0.5;  // visit of a leaf node (often skipped by the traversal's leaf shortcut)
constexpr double SAH_CT = 1.0;  // one primitive test
__global__ void k_sah_leaves(uint32_t n, const Box6* pbox, double4* dcost, uint16_t* dec) {
  const uint32_t id = blockIdx.x * 256 + threadIdx.x;
  if (id >= n) return;
  const double c = half_area(pbox[id]) * (SAH_CL + SAH_CT);
  dcost[id] = make_double4(c, c, c, c);
  dec[id] = 1;
}
// Nodes created by one PLOC iteration, ids [b0, b0 + cnt): their children are older.
__global__ void k_sah_level(uint32_t b0, uint32_t cnt, const int32_t* pl, const int32_t* pr, const Box6* pbox,
                            const uint32_t* psize, uint32_t leaf_max, double4* dcost, uint16_t* dec) {
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  if (k >= cnt) return;
  const uint32_t id = b0 + k;
  const double4 l4 = dcost[pl[id]], r4 = dcost[pr[id]];
  const double L[5] = {0, l4.x, l4.y, l4.z, l4.w}, R[5] = {0, r4.x, r4.y, r4.z, r4.w};
  const double area = half_area(pbox[id]);
  double best4 = L[1] + R[3];
  uint32_t k4 = 1;
  for (uint32_t j = 2; j <= 3; j++)
    if (L[j] + R[4 - j] < best4) { best4 = L[j] + R[4 - j]; k4 = j; }
  double d[5];
  d[1] = area * SAH_CN + best4;
  uint32_t bits = k4 << 1;
  if (psize[id] <= leaf_max) {
    const double lc = area * (SAH_CL + SAH_CT * (double)psize[id]);
    if (lc <= d[1]) { d[1] = lc; bits |= 1u; }
  }
  for (uint32_t i = 2; i <= 4; i++) {
    d[i] = d[i - 1];
    uint32_t ki = 0;
    for (uint32_t j = 1; j < i; j++)
      if (L[j] + R[i - j] < d[i]) { d[i] = L[j] + R[i - j]; ki = j; }
    bits |= ki << (1 + 2 * (i - 1));
  }
  dcost[id] = make_double4(d[1], d[2], d[3], d[4]);
  dec[id] = (uint16_t)bits;
}

// To the layout the collapse reads (Karras' numbering): internal node k -> 2n-2-k (the
// root, created last, becomes 0), leaf p -> n-1+DFS position; leaf order from the DFS.
__global__ void k_ploc_to_tree(uint32_t n, const int32_t* pl, const int32_t* pr, const Box6* pbox, const uint32_t* psize,
                               const uint32_t* off, const uint32_t* ids_s, int32_t* left, int32_t* right, int32_t* first,
                               int32_t* last, Box6* nb, uint32_t* order, const uint16_t* dec, uint16_t* dec_t) {
  const uint32_t id = blockIdx.x * 256 + threadIdx.x;
  if (id >= 2 * n - 1) return;
  const int nn1 = (int)n - 1;
  auto map = [&](int32_t x) { return x < (int32_t)n ? nn1 + (int32_t)off[x] : (int32_t)(2 * n - 2) - x; };
  if (dec) dec_t[map((int32_t)id)] = dec[id];
  if (id < n) {
    nb[nn1 + off[id]] = pbox[id];
    order[off[id]] = ids_s[id];
  } else {
    const int32_t t = map((int32_t)id);
    left[t] = map(pl[id]);
    right[t] = map(pr[id]);
    first[t] = (int32_t)off[id];
    last[t] = (int32_t)(off[id] + psize[id] - 1);
    nb[t] = pbox[id];
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
  const uint16_t* dec;  // SAH collapse decisions (k_sah_level), or null: collectChildren's rule
  __device__ int size(int b) const { return b >= n - 1 ? 1 : last[b] - first[b] + 1; }
  __device__ int start(int b) const { return b >= n - 1 ? b - (n - 1) : first[b]; }
  __device__ bool is_leaf(int b) const { return dec ? (dec[b] & 1u) != 0 : size(b) <= leaf_max; }
};

// The wide node b's child slots from the SAH decisions: its split over 4 slots, each side
// expanded by its own recorded split for the slots it gets, in left-to-right order.
__device__ int sah_collect(const Tree& t, int b, int* res) {
  int sn[4], si[4], sp = 0, c = 0;
  const int k4 = (t.dec[b] >> 1) & 3;
  sn[sp] = t.right[b]; si[sp++] = 4 - k4;
  int m = t.left[b], i = k4;
  for (;;) {
    const int ki = (i > 1 && t.size(m) > 1) ? (t.dec[m] >> (1 + 2 * (i - 1))) & 3 : 0;
    if (i > 1 && ki == 0) { i--; continue; }
    if (i <= 1) {
      res[c++] = m;
      if (sp == 0) break;
      sp--; m = sn[sp]; i = si[sp];
      continue;
    }
    sn[sp] = t.right[m]; si[sp++] = i - ki;
    m = t.left[m]; i = ki;
  }
  return c;
}

// collectChildren (bvh4.go:796-855) on the binary tree, leaves = subtrees of <= leaf_max.
// Where the reference expands the first inner child, this expands the one with the
// largest surface area (measured: 7% fewer node visits on C3's mesh).
__device__ int collect(const Tree& t, int b, int* res) {
  if (t.dec) return sah_collect(t, b, res);
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
int build(hipStream_t st, const double* h_boxes, uint32_t n, uint32_t leaf_max, uint32_t method,
          std::vector<izpi_bvh4_node>& nodes, std::vector<uint32_t>& order, float* ms, std::string& err) {
  nodes.clear();
  order.clear();
  if (n == 0) return IZPI_OK;
  if (leaf_max < 1 || leaf_max > 4) { err = "leaf_max must be 1..4 (bvh4.go:638)"; return IZPI_ERR_INVALID; }
  if (n > (1u << 27)) { err = "too many primitives for the leaf-ref encoding"; return IZPI_ERR_UNSUPPORTED; }
  const bool sah = (method & IZPI_BVH_SAH) != 0;
  method &= ~(uint32_t)IZPI_BVH_SAH;
  if (method != IZPI_BVH_LBVH && method != IZPI_BVH_PLOC) { err = "unknown BVH build method"; return IZPI_ERR_INVALID; }
  if (sah && method != IZPI_BVH_PLOC) { err = "the SAH collapse needs the PLOC tree (IZPI_BVH_PLOC)"; return IZPI_ERR_INVALID; }
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
  DevBuf<uint16_t> dec_t;  // SAH collapse decisions in the collapse's numbering (PLOC)
  Tree t{left.p, right.p, first.p, last.p, nb.p, ni, (int)leaf_max, nullptr};
  uint32_t total = 0;
  DevBuf<uint32_t> ord;  // leaf order (PLOC); the sorted ids are the leaf order of the LBVH
  const uint32_t* leaf_order = ids_s.p;
  if (method == IZPI_BVH_LBVH) {
    if (n > 1) {
      hipLaunchKernelGGL(k_karras, dim3((nint + 255) / 256), dim3(256), 0, st, codes_s.p, ni, left.p, right.p, first.p,
                         last.p, parent.p);
      BVH_TRY(hipMemsetAsync(flags.p, 0, nint * sizeof(uint32_t), st));
    }
    hipLaunchKernelGGL(k_refit, g, dim3(256), 0, st, boxes.p, ids_s.p, ni, left.p, right.p, parent.p, nb.p, flags.p);
    BVH_TRY(hipGetLastError());
  } else {
    DevBuf<int32_t> pl, pr, pparent, cl, cl2, nnb;
    DevBuf<Box6> pbox;
    DevBuf<uint32_t> psize, mflag, aflag, mscan, ascan, off;
    BVH_TRY(pl.alloc(ntot)); BVH_TRY(pr.alloc(ntot)); BVH_TRY(pparent.alloc(ntot)); BVH_TRY(pbox.alloc(ntot));
    BVH_TRY(psize.alloc(ntot)); BVH_TRY(off.alloc(ntot)); BVH_TRY(ord.alloc(n));
    BVH_TRY(cl.alloc(n)); BVH_TRY(cl2.alloc(n)); BVH_TRY(nnb.alloc(n));
    BVH_TRY(mflag.alloc(n)); BVH_TRY(aflag.alloc(n)); BVH_TRY(mscan.alloc(n)); BVH_TRY(ascan.alloc(n));
    hipLaunchKernelGGL(k_ploc_init, g, dim3(256), 0, st, boxes.p, ids_s.p, n, pbox.p, psize.p, pparent.p, cl.p);
    size_t sbytes = 0;
    BVH_TRY(rocprim::exclusive_scan(nullptr, sbytes, mflag.p, mscan.p, 0u, (size_t)n, rocprim::plus<uint32_t>(), st));
    DevBuf<uint8_t> stemp;
    BVH_TRY(stemp.alloc(sbytes));
    uint32_t m = n, base = n;
    std::vector<uint32_t> iters;  // ids created per iteration: [iters[k], iters[k + 1])
    iters.push_back(n);
    while (m > 1) {
      const dim3 gm((m + 255) / 256);
      hipLaunchKernelGGL(k_ploc_nn, gm, dim3(256), 0, st, cl.p, m, pbox.p, PLOC_RADIUS, nnb.p);
      hipLaunchKernelGGL(k_ploc_flags, gm, dim3(256), 0, st, nnb.p, m, mflag.p, aflag.p);
      size_t sb = sbytes;
      BVH_TRY(rocprim::exclusive_scan(stemp.p, sb, mflag.p, mscan.p, 0u, (size_t)m, rocprim::plus<uint32_t>(), st));
      sb = sbytes;
      BVH_TRY(rocprim::exclusive_scan(stemp.p, sb, aflag.p, ascan.p, 0u, (size_t)m, rocprim::plus<uint32_t>(), st));
      hipLaunchKernelGGL(k_ploc_merge, gm, dim3(256), 0, st, cl.p, m, nnb.p, mflag.p, mscan.p, aflag.p, ascan.p, base,
                         pl.p, pr.p, pbox.p, psize.p, pparent.p, cl2.p);
      BVH_TRY(hipGetLastError());
      uint32_t tail[4];
      BVH_TRY(hipMemcpyAsync(tail + 0, mflag.p + m - 1, 4, hipMemcpyDeviceToHost, st));
      BVH_TRY(hipMemcpyAsync(tail + 1, mscan.p + m - 1, 4, hipMemcpyDeviceToHost, st));
      BVH_TRY(hipMemcpyAsync(tail + 2, aflag.p + m - 1, 4, hipMemcpyDeviceToHost, st));
      BVH_TRY(hipMemcpyAsync(tail + 3, ascan.p + m - 1, 4, hipMemcpyDeviceToHost, st));
      BVH_TRY(hipStreamSynchronize(st));
      const uint32_t merges = tail[0] + tail[1], alive = tail[2] + tail[3];
      if (merges == 0) { err = "PLOC made no progress"; return IZPI_ERR_INVALID; }  // a global closest pair always exists
      base += merges;
      iters.push_back(base);
      m = alive;
      std::swap(cl.p, cl2.p);
    }
    hipLaunchKernelGGL(k_ploc_offsets, dim3((ntot + 255) / 256), dim3(256), 0, st, ntot, pl.p, pr.p, psize.p, pparent.p,
                       off.p);
    DevBuf<double4> dcost;
    DevBuf<uint16_t> dec;
    if (sah) {
      BVH_TRY(dcost.alloc(ntot)); BVH_TRY(dec.alloc(ntot)); BVH_TRY(dec_t.alloc(ntot));
      hipLaunchKernelGGL(k_sah_leaves, g, dim3(256), 0, st, n, pbox.p, dcost.p, dec.p);
      for (size_t k = 0; k + 1 < iters.size(); k++) {
        const uint32_t cnt = iters[k + 1] - iters[k];
        hipLaunchKernelGGL(k_sah_level, dim3((cnt + 255) / 256), dim3(256), 0, st, iters[k], cnt, pl.p, pr.p, pbox.p,
                           psize.p, leaf_max, dcost.p, dec.p);
      }
      t.dec = dec_t.p;
    }
    hipLaunchKernelGGL(k_ploc_to_tree, dim3((ntot + 255) / 256), dim3(256), 0, st, n, pl.p, pr.p, pbox.p, psize.p, off.p,
                       ids_s.p, left.p, right.p, first.p, last.p, nb.p, ord.p, dec.p, dec_t.p);
    BVH_TRY(hipGetLastError());
    BVH_TRY(hipStreamSynchronize(st));  // the PLOC buffers are freed at the end of this scope
    leaf_order = ord.p;
  }
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
  BVH_TRY(hipMemcpyAsync(order.data(), leaf_order, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  BVH_TRY(hipStreamSynchronize(st));
  if (ms) BVH_TRY(hipEventElapsedTime(ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return IZPI_OK;
}

}  // namespace izpi_bvh
