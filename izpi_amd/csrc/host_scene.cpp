// host_scene.cpp — host-side scene producer: the C++ stand-in for the Go host's
//   transport.ToScene       internal/transport/transport.go:53-92, 551-680
//   camera.New              internal/camera/camera.go:28-58
//   hitable.NewTriangleWithUV  internal/hitable/triangle.go:61-134
//   hitable.NewBVH4         internal/hitable/bvh4.go:517-855 (binary median split on a
//                           random axis with Go's sort.Slice, collapse to 4-wide,
//                           DFS pre-order flatten with conservative f32 bounds)
//   common.Tiles/grid.WalkGrid  common/tiles.go:6-24, grid/grid.go:48-125
// It emits the flattened izpi_scene_desc that izpi_gpu_upload_scene consumes.
//
// Unlike the reference (which copies and re-sorts slices of interface values per
// node) the build works in place on one index array with cached float64 sort keys;
// the resulting node array and primitive order are identical because Go sorts a
// private copy of exactly the same range with the same algorithm (pdqsort_func).
#include <stdint.h>
#include <string.h>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/izpi_host.h"
#include "gomath.h"

namespace {

thread_local std::string g_err;

struct V3 { double x, y, z; };
inline V3 v3(const double* p) { return V3{p[0], p[1], p[2]}; }
inline V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 smul(V3 a, double t) { return V3{a.x * t, a.y * t, a.z * t}; }
inline V3 sdiv(V3 a, double t) { return V3{a.x / t, a.y / t, a.z / t}; }
inline V3 cross(V3 a, V3 b) { return V3{(a.y * b.z) - (a.z * b.y), -((a.x * b.z) - (a.z * b.x)), (a.x * b.y) - (a.y * b.x)}; }
inline double len(V3 a) { return gm::sqrt((a.x * a.x) + (a.y * a.y) + (a.z * a.z)); }
inline V3 unit(V3 a) { double l = len(a); return V3{a.x / l, a.y / l, a.z / l}; }
inline void st(double* p, V3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }

// bvh4.go:494-514
inline float cons_min(double v) { float f = (float)v; return (double)f > v ? gm::nextafter32(f, -__builtin_inff()) : f; }
inline float cons_max(double v) { float f = (float)v; return (double)f < v ? gm::nextafter32(f, __builtin_inff()) : f; }

struct Box { double mn[3], mx[3]; };
inline Box surround(const Box& a, const Box& b) {
  Box r;
  for (int k = 0; k < 3; k++) { r.mn[k] = gm::min(a.mn[k], b.mn[k]); r.mx[k] = gm::max(a.mx[k], b.mx[k]); }
  return r;
}

// fastrandom.LCG (fastrandom.go:41-47) for the split axis (bvh4.go:520,626).
struct Lcg {
  uint64_t s;
  double next() { s = (1664525ull * s + 1013904223ull) % 4294967296ull; return (double)s / 4294967296.0; }
};

// ---- Go sort.Slice (pdqsort_func, sort/zsortfunc.go) over idx[lo:hi) by key -----
struct Sorter {
  int* idx;
  const double* key;  // key[primitive] = box.min[axis]
  bool less(int i, int j) const { return key[idx[i]] < key[idx[j]]; }
  void swap(int i, int j) { int t = idx[i]; idx[i] = idx[j]; idx[j] = t; }

  void insertion(int a, int b) {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && less(j, j - 1); j--) swap(j, j - 1);
  }
  void sift(int lo, int hi, int first) {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && less(first + child, first + child + 1)) child++;
      if (!less(first + root, first + child)) return;
      swap(first + root, first + child);
      root = child;
    }
  }
  void heap(int a, int b) {
    int hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift(i, hi, a);
    for (int i = hi - 1; i >= 0; i--) { swap(a, a + i); sift(0, i, a); }
  }
  static int blen(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }
  void break_patterns(int a, int b) {
    int n = b - a;
    if (n < 8) return;
    uint64_t r = (uint64_t)n;
    uint64_t mod = 1ull << blen((uint64_t)n);
    int idx0 = a + (n / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
      r ^= r << 13; r ^= r >> 7; r ^= r << 17;
      int other = (int)((unsigned)r & (unsigned)(mod - 1));
      if (other >= n) other -= n;
      swap(idx0 - 1 + i, a + other);
    }
  }
  int med(int a, int b, int c, int* sw) {
    if (less(b, a)) { (*sw)++; int t = a; a = b; b = t; }
    if (less(c, b)) { (*sw)++; int t = b; b = c; c = t; }
    if (less(b, a)) { (*sw)++; int t = a; a = b; b = t; }
    return b;
  }
  int pivot(int a, int b, int* hint) {
    int l = b - a, sw = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= 50) { i = med(i - 1, i, i + 1, &sw); j = med(j - 1, j, j + 1, &sw); k = med(k - 1, k, k + 1, &sw); }
      j = med(i, j, k, &sw);
    }
    *hint = sw == 0 ? 1 : (sw == 12 ? 2 : 0);
    return j;
  }
  bool partial_insertion(int base, int a, int b) {
    int i = a + 1;
    for (int step = 0; step < 5; step++) {
      while (i < b && !less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < 50) return false;
      swap(i, i - 1);
      if (i - a >= 2) for (int k = i - 1; k >= base + 1; k--)  // Go: j >= 1 relative to the sorted slice
        { if (!less(k, k - 1)) break; swap(k, k - 1); }
      if (b - i >= 2) for (int k = i + 1; k < b; k++) { if (!less(k, k - 1)) break; swap(k, k - 1); }
    }
    return false;
  }
  int partition_equal(int a, int b, int p) {
    swap(a, p);
    int i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !less(a, i)) i++;
      while (i <= j && less(a, j)) j--;
      if (i > j) break;
      swap(i, j); i++; j--;
    }
    return i;
  }
  int partition(int a, int b, int p, bool* already) {
    swap(a, p);
    int i = a + 1, j = b - 1;
    while (i <= j && less(i, a)) i++;
    while (i <= j && !less(j, a)) j--;
    if (i > j) { swap(j, a); *already = true; return j; }
    swap(i, j); i++; j--;
    for (;;) {
      while (i <= j && less(i, a)) i++;
      while (i <= j && !less(j, a)) j--;
      if (i > j) break;
      swap(i, j); i++; j--;
    }
    swap(j, a);
    *already = false;
    return j;
  }
  // Indices a,b are absolute positions in idx[]; Go's `a > 0` test (zsortfunc.go)
  // refers to the position inside the slice being sorted, so pass `base`.
  void pdq(int base, int a, int b, int limit) {
    bool balanced = true, partitioned = true;
    for (;;) {
      int n = b - a;
      if (n <= 12) { insertion(a, b); return; }
      if (limit == 0) { heap(a, b); return; }
      if (!balanced) { break_patterns(a, b); limit--; }
      int hint;
      int p = pivot(a, b, &hint);
      if (hint == 2) {
        for (int i = a, j = b - 1; i < j; i++, j--) swap(i, j);
        p = (b - 1) - (p - a);
        hint = 1;
      }
      if (balanced && partitioned && hint == 1 && partial_insertion(base, a, b)) return;
      if (a > base && !less(a - 1, p)) { a = partition_equal(a, b, p); continue; }
      bool already;
      int mid = partition(a, b, p, &already);
      partitioned = already;
      int ll = mid - a, rl = b - mid, thr = n / 8;
      if (ll < rl) { balanced = ll >= thr; pdq(base, a, mid, limit); a = mid + 1; }
      else { balanced = rl >= thr; pdq(base, mid + 1, b, limit); b = mid; }
    }
  }
  void sort(int a, int b) { pdq(a, a, b, blen((uint64_t)(b - a))); }
};

// Binary build node (bvh4.go:552-556): leaves hold an index range of `order`.
struct BNode {
  Box box;
  int lo, hi;        // range in order[]
  int left, right;   // child BNode ids (-1 for leaves)
  bool leaf;
};

struct Builder {
  const std::vector<Box>& boxes;
  std::vector<double> key[3];
  std::vector<int> order;
  std::vector<BNode> nodes;
  Lcg rng;
  explicit Builder(const std::vector<Box>& b, uint64_t seed) : boxes(b), rng{seed} {
    for (int k = 0; k < 3; k++) {
      key[k].resize(b.size());
      for (size_t i = 0; i < b.size(); i++) key[k][i] = b[i].mn[k];
    }
    order.resize(b.size());
    for (size_t i = 0; i < b.size(); i++) order[i] = (int)i;
  }
  // buildBinaryBVH (bvh4.go:596-652), recursion order preserved (left then right)
  // so the split-axis LCG draws happen in the reference's order.
  int build(int lo, int hi) {
    int id = (int)nodes.size();
    nodes.push_back(BNode{});
    BNode n;
    n.lo = lo; n.hi = hi; n.left = n.right = -1; n.leaf = false;
    if (hi - lo == 1) {
      n.box = boxes[(size_t)order[(size_t)lo]];
      n.leaf = true;
      nodes[(size_t)id] = n;
      return id;
    }
    Box ob = boxes[(size_t)order[(size_t)lo]];
    for (int i = lo + 1; i < hi; i++) ob = surround(ob, boxes[(size_t)order[(size_t)i]]);
    n.box = ob;
    int axis = (int)(3 * rng.next());
    Sorter s{order.data(), key[axis].data()};
    s.sort(lo, hi);
    if (hi - lo <= 4) {
      n.leaf = true;
      nodes[(size_t)id] = n;
      return id;
    }
    int mid = lo + (hi - lo) / 2;
    nodes[(size_t)id] = n;
    int l = build(lo, mid);
    int r = build(mid, hi);
    nodes[(size_t)id].left = l;
    nodes[(size_t)id].right = r;
    return id;
  }
  // collectChildren (bvh4.go:796-855)
  void collect(int id, int* out, int* count) const {
    const BNode& n = nodes[(size_t)id];
    int res[8]; int c = 0;
    res[c++] = n.left; res[c++] = n.right;
    bool expanded = true;
    while (expanded && c < 4) {
      expanded = false;
      for (int i = 0; i < c; i++) {
        const BNode& cur = nodes[(size_t)res[i]];
        if (cur.leaf) continue;
        if (c - 1 + 2 <= 4) {
          for (int k = i; k + 1 < c; k++) res[k] = res[k + 1];
          c--;
          res[c++] = cur.left; res[c++] = cur.right;
          expanded = true;
          break;
        }
      }
    }
    for (int i = 0; i < c; i++) out[i] = res[i];
    *count = c;
  }
  // flattenBVH4 (bvh4.go:714-792): DFS pre-order.
  int32_t flatten(int id, std::vector<izpi_bvh4_node>& out, std::vector<int>& prim_order) const {
    const BNode& n = nodes[(size_t)id];
    int32_t me = (int32_t)out.size();
    izpi_bvh4_node e;
    for (int i = 0; i < 4; i++) {
      e.child[i] = -1; e.prim_count[i] = 0;
      e.min_x[i] = e.min_y[i] = e.min_z[i] = e.max_x[i] = e.max_y[i] = e.max_z[i] = 3.40282346638528859811704183484516925440e+38f;
    }
    if (n.leaf) {
      e.child[0] = (int32_t)prim_order.size();
      e.prim_count[0] = n.hi - n.lo;
      for (int i = n.lo; i < n.hi; i++) prim_order.push_back(order[(size_t)i]);
      e.min_x[0] = cons_min(n.box.mn[0]); e.min_y[0] = cons_min(n.box.mn[1]); e.min_z[0] = cons_min(n.box.mn[2]);
      e.max_x[0] = cons_max(n.box.mx[0]); e.max_y[0] = cons_max(n.box.mx[1]); e.max_z[0] = cons_max(n.box.mx[2]);
      out.push_back(e);
      return me;
    }
    int ch[4], c;
    collect(id, ch, &c);
    out.push_back(e);
    for (int i = 0; i < c; i++) {
      int32_t ci = flatten(ch[i], out, prim_order);
      const Box& b = nodes[(size_t)ch[i]].box;
      izpi_bvh4_node& p = out[(size_t)me];
      p.child[i] = ci;
      p.min_x[i] = cons_min(b.mn[0]); p.min_y[i] = cons_min(b.mn[1]); p.min_z[i] = cons_min(b.mn[2]);
      p.max_x[i] = cons_max(b.mx[0]); p.max_y[i] = cons_max(b.mx[1]); p.max_z[i] = cons_max(b.mx[2]);
    }
    return me;
  }
};

// Upper bound on the traversal stack (bvh4.go:71-73): along any root-to-leaf path
// a node pushes at most (valid children - 1) entries that stay below its subtree.
uint32_t stack_bound(const std::vector<izpi_bvh4_node>& nodes) {
  if (nodes.empty()) return 0;
  std::vector<uint32_t> best(nodes.size(), 0);
  for (size_t k = nodes.size(); k-- > 0;) {  // children have larger indices (pre-order)
    const izpi_bvh4_node& n = nodes[k];
    if (n.prim_count[0] > 0) { best[k] = 0; continue; }
    uint32_t valid = 0, deepest = 0;
    for (int i = 0; i < 4; i++) {
      if (n.child[i] < 0) continue;
      valid++;
      uint32_t b = best[(size_t)n.child[i]];
      if (b > deepest) deepest = b;
    }
    best[k] = (valid ? valid - 1 : 0) + deepest;
  }
  return best[0];
}

}  // namespace

struct izpi_host_scene {
  izpi_scene_desc desc;
  std::vector<izpi_bvh4_node> nodes;
  std::vector<uint32_t> prim_ref, tri_mat, sph_mat, light_ref;
  std::vector<double> v0, v1, v2, e1, e2, nrm, tan, bitan, uv, area;
  std::vector<double> c0, c1, stime, rad;
  std::vector<double> boxes;  // [prims][6] f64 primitive boxes (transport order), for other BVH builders
  std::vector<izpi_material> mats;
  std::vector<izpi_texture> texs;
  std::vector<double> texels, spd_wl, spd_val;
  uint32_t stack_bound = 0;
  double build_ms = 0;
};

namespace izpi_internal {
void set_host_error(const std::string& s) { g_err = s; }
}

extern "C" {

const char* izpi_host_last_error(void) { return g_err.c_str(); }

int izpi_host_build_scene(const izpi_scene_input* in, izpi_host_scene** out) {
  return izpi_host_build_scene_ex(in, 0, out);
}

int izpi_host_build_scene_ex(const izpi_scene_input* in, uint32_t flags, izpi_host_scene** out) {
  *out = nullptr;
  if (!in) { g_err = "null input"; return IZPI_ERR_INVALID; }
  auto t0 = std::chrono::steady_clock::now();
  izpi_host_scene* s = new izpi_host_scene();
  const uint32_t nt = in->num_tris, ns = in->num_spheres;
  for (uint32_t i = 0; i < nt; i++)
    if (in->tris[i].material >= in->num_materials) { g_err = "triangle material out of range"; delete s; return IZPI_ERR_INVALID; }
  for (uint32_t i = 0; i < ns; i++)
    if (in->spheres[i].material >= in->num_materials) { g_err = "sphere material out of range"; delete s; return IZPI_ERR_INVALID; }
  s->mats.assign(in->materials, in->materials + in->num_materials);
  s->texs.assign(in->textures, in->textures + in->num_textures);
  if (in->num_texels) s->texels.assign(in->texels, in->texels + in->num_texels);
  if (in->num_spd) {
    s->spd_wl.assign(in->spd_wavelengths, in->spd_wavelengths + in->num_spd);
    s->spd_val.assign(in->spd_values, in->spd_values + in->num_spd);
  }
  // --- triangles (NewTriangleWithUV, triangle.go:61-134)
  s->v0.resize(3 * (size_t)nt); s->v1.resize(3 * (size_t)nt); s->v2.resize(3 * (size_t)nt);
  s->e1.resize(3 * (size_t)nt); s->e2.resize(3 * (size_t)nt); s->nrm.resize(3 * (size_t)nt);
  s->tan.resize(3 * (size_t)nt); s->bitan.resize(3 * (size_t)nt); s->uv.resize(6 * (size_t)nt);
  s->area.resize(nt); s->tri_mat.resize(nt);
  std::vector<Box> boxes((size_t)nt + ns);
  for (uint32_t i = 0; i < nt; i++) {
    const izpi_tri_in& t = in->tris[i];
    V3 a = v3(t.v0), b = v3(t.v1), c = v3(t.v2);
    V3 ed1 = sub(b, a), ed2 = sub(c, a);
    V3 n = unit(cross(ed1, ed2));
    double u0 = t.uv[0], vv0 = t.uv[1], u1 = t.uv[2], vv1 = t.uv[3], u2 = t.uv[4], vv2 = t.uv[5];
    double dU1 = u1 - u0, dU2 = u2 - u0, dV1 = vv1 - vv0, dV2 = vv2 - vv0;
    double ar = len(cross(ed1, ed2)) / 2.0;
    double f = 1.0 / (dU1 * dV2 - dU2 * dV1);
    V3 tg = unit(V3{f * (dV2 * ed1.x - dV1 * ed2.x), f * (dV2 * ed1.y - dV1 * ed2.y), f * (dV2 * ed1.z - dV1 * ed2.z)});
    V3 bt = unit(V3{f * (-dU2 * ed1.x + dU1 * ed2.x), f * (-dU2 * ed1.y + dU1 * ed2.y), f * (-dU2 * ed1.z + dU1 * ed2.z)});
    // Min3/Max3 (vec3.go:161-248) then relative epsilon
    double mn[3], mx[3];
    const double* vs[3] = {t.v0, t.v1, t.v2};
    for (int k = 0; k < 3; k++) {
      mn[k] = 1.7976931348623157e308; mx[k] = -1.7976931348623157e308;
      for (int j = 0; j < 3; j++) { if (vs[j][k] < mn[k]) mn[k] = vs[j][k]; if (vs[j][k] > mx[k]) mx[k] = vs[j][k]; }
    }
    double sz[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
    double maxDim = gm::max(sz[0], gm::max(sz[1], sz[2]));
    double eps = gm::max(maxDim * 1e-4, 1e-6);
    Box& bx = boxes[i];
    for (int k = 0; k < 3; k++) { bx.mn[k] = mn[k] - eps; bx.mx[k] = mx[k] + eps; }
    st(&s->v0[3 * i], a); st(&s->v1[3 * i], b); st(&s->v2[3 * i], c);
    st(&s->e1[3 * i], ed1); st(&s->e2[3 * i], ed2); st(&s->nrm[3 * i], n);
    st(&s->tan[3 * i], tg); st(&s->bitan[3 * i], bt);
    memcpy(&s->uv[6 * i], t.uv, 6 * sizeof(double));
    s->area[i] = ar; s->tri_mat[i] = t.material;
  }
  // --- spheres (NewSphere(c, c, 0, 1, r), transport.go:679; BoundingBox sphere.go:485-493)
  s->c0.resize(3 * (size_t)ns); s->c1.resize(3 * (size_t)ns); s->stime.resize(2 * (size_t)ns);
  s->rad.resize(ns); s->sph_mat.resize(ns);
  for (uint32_t i = 0; i < ns; i++) {
    const izpi_sphere_in& sp = in->spheres[i];
    for (int k = 0; k < 3; k++) { s->c0[3 * i + k] = sp.center[k]; s->c1[3 * i + k] = sp.center[k]; }
    s->stime[2 * i] = 0; s->stime[2 * i + 1] = 1;
    s->rad[i] = sp.radius; s->sph_mat[i] = sp.material;
    Box b0, b1;
    for (int k = 0; k < 3; k++) {
      b0.mn[k] = sp.center[k] - sp.radius; b0.mx[k] = sp.center[k] + sp.radius;
      b1.mn[k] = sp.center[k] - sp.radius; b1.mx[k] = sp.center[k] + sp.radius;
    }
    boxes[(size_t)nt + i] = surround(b0, b1);
  }
  // --- lights: every hitable whose material IsEmitter() (transport.go:67-72;
  // DiffuseLight and, quirk A5, Dielectric).
  auto emitter = [&](uint32_t m) {
    uint32_t k = in->materials[m].kind;
    return k == IZPI_MAT_DIFFUSE_LIGHT || k == IZPI_MAT_DIELECTRIC;
  };
  for (uint32_t i = 0; i < nt; i++) if (emitter(in->tris[i].material)) s->light_ref.push_back(IZPI_PRIM_REF(IZPI_PRIM_TRIANGLE, i));
  for (uint32_t i = 0; i < ns; i++) if (emitter(in->spheres[i].material)) s->light_ref.push_back(IZPI_PRIM_REF(IZPI_PRIM_SPHERE, i));
  s->boxes.resize(6 * boxes.size());
  for (size_t i = 0; i < boxes.size(); i++)
    for (int k = 0; k < 3; k++) { s->boxes[6 * i + k] = boxes[i].mn[k]; s->boxes[6 * i + 3 + k] = boxes[i].mx[k]; }
  // --- BVH4 (bvh4.go:517-593)
  if (flags & IZPI_HOST_SKIP_BVH) {  // another builder attaches its tree (izpi_host_scene_set_bvh)
    s->prim_ref.resize((size_t)nt + ns);
    for (uint32_t i = 0; i < nt; i++) s->prim_ref[i] = IZPI_PRIM_REF(IZPI_PRIM_TRIANGLE, i);
    for (uint32_t i = 0; i < ns; i++) s->prim_ref[(size_t)nt + i] = IZPI_PRIM_REF(IZPI_PRIM_SPHERE, i);
  } else if (nt + ns > 0) {
    Builder b(boxes, in->bvh_seed);
    int root = b.build(0, (int)(nt + ns));
    std::vector<int> prim_order;
    prim_order.reserve((size_t)nt + ns);
    s->nodes.reserve((size_t)(nt + ns) / 2 + 8);
    b.flatten(root, s->nodes, prim_order);
    s->prim_ref.resize(prim_order.size());
    for (size_t i = 0; i < prim_order.size(); i++) {
      uint32_t p = (uint32_t)prim_order[i];
      s->prim_ref[i] = p < nt ? IZPI_PRIM_REF(IZPI_PRIM_TRIANGLE, p) : IZPI_PRIM_REF(IZPI_PRIM_SPHERE, p - nt);
    }
    s->stack_bound = stack_bound(s->nodes);
  }
  // --- camera.New (camera.go:28-58) with aspect override (transport.go:522-529)
  izpi_scene_desc& d = s->desc;
  memset(&d, 0, sizeof(d));
  {
    const izpi_camera_in& c = in->camera;
    double aspect = in->aspect_override != 0.0 ? in->aspect_override : c.aspect;
    double lensRadius = c.aperture / 2.0;
    double theta = c.vfov * 3.141592653589793 / 180;
    double halfHeight = gm::tan(theta / 2.0);
    double halfWidth = aspect * halfHeight;
    V3 lf = v3(c.look_from), la = v3(c.look_at), up = v3(c.vup);
    V3 w = unit(sub(lf, la));
    V3 u = unit(cross(up, w));
    V3 v = cross(w, u);
    V3 ll = sub(sub(sub(lf, smul(u, halfWidth * c.focus_dist)), smul(v, halfHeight * c.focus_dist)), smul(w, c.focus_dist));
    st(d.camera.origin, lf);
    st(d.camera.lower_left, ll);
    st(d.camera.horizontal, smul(u, 2.0 * halfWidth * c.focus_dist));
    st(d.camera.vertical, smul(v, 2.0 * halfHeight * c.focus_dist));
    st(d.camera.u, u);
    st(d.camera.v, v);
    d.camera.lens_radius = lensRadius;
    d.camera.time0 = c.time0; d.camera.time1 = c.time1; d.camera.exposure = c.exposure;
  }
  d.abi_version = IZPI_ABI_VERSION;
  d.num_nodes = (uint32_t)s->nodes.size();
  d.num_prims = (uint32_t)s->prim_ref.size();
  d.num_tris = nt; d.num_spheres = ns;
  d.num_lights = (uint32_t)s->light_ref.size();
  d.num_materials = in->num_materials; d.num_textures = in->num_textures;
  d.num_spd = in->num_spd; d.num_texels = in->num_texels;
  d.nodes = s->nodes.data(); d.prim_ref = s->prim_ref.data();
  d.tri_v0 = s->v0.data(); d.tri_v1 = s->v1.data(); d.tri_v2 = s->v2.data();
  d.tri_e1 = s->e1.data(); d.tri_e2 = s->e2.data(); d.tri_normal = s->nrm.data();
  d.tri_tangent = s->tan.data(); d.tri_bitangent = s->bitan.data(); d.tri_uv = s->uv.data();
  d.tri_area = s->area.data(); d.tri_mat = s->tri_mat.data();
  d.sph_center0 = s->c0.data(); d.sph_center1 = s->c1.data(); d.sph_time = s->stime.data();
  d.sph_radius = s->rad.data(); d.sph_mat = s->sph_mat.data();
  d.light_ref = s->light_ref.data();
  d.materials = s->mats.data(); d.textures = s->texs.data();
  d.texels = s->texels.data(); d.spd_wavelengths = s->spd_wl.data(); d.spd_values = s->spd_val.data();
  s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = s;
  return IZPI_OK;
}

const izpi_scene_desc* izpi_host_scene_desc(const izpi_host_scene* s) { return s ? &s->desc : nullptr; }

int izpi_host_scene_prim_boxes(const izpi_host_scene* s, double* boxes) {
  if (!s || !boxes) { g_err = "null argument"; return IZPI_ERR_INVALID; }
  if (!s->boxes.empty()) memcpy(boxes, s->boxes.data(), s->boxes.size() * sizeof(double));
  return IZPI_OK;
}

int izpi_host_scene_set_flags(izpi_host_scene* s, uint32_t flags) {
  if (!s) { g_err = "null argument"; return IZPI_ERR_INVALID; }
  if (flags & ~(uint32_t)IZPI_SCENE_QUANTIZED_BVH) { g_err = "unknown scene flag"; return IZPI_ERR_INVALID; }
  s->desc.flags = flags;
  return IZPI_OK;
}

int izpi_host_scene_set_bvh(izpi_host_scene* s, const izpi_bvh4_node* nodes, uint32_t num_nodes, const uint32_t* order) {
  if (!s || (!nodes && num_nodes) || !order) { g_err = "null argument"; return IZPI_ERR_INVALID; }
  const uint32_t np = s->desc.num_tris + s->desc.num_spheres, nt = s->desc.num_tris;
  if (np > 0 && num_nodes == 0) { g_err = "empty BVH for a non-empty scene"; return IZPI_ERR_INVALID; }
  std::vector<uint8_t> seen(np, 0);
  for (uint32_t k = 0; k < np; k++) {
    if (order[k] >= np || seen[order[k]]) { g_err = "order is not a permutation of the primitives"; return IZPI_ERR_INVALID; }
    seen[order[k]] = 1;
  }
  for (uint32_t k = 0; k < num_nodes; k++) {  // children after parents (stack_bound's single backward pass)
    const izpi_bvh4_node& n = nodes[k];
    if (n.prim_count[0] > 0) {
      if (n.child[0] < 0 || (uint64_t)n.child[0] + (uint64_t)n.prim_count[0] > np) { g_err = "leaf range out of bounds"; return IZPI_ERR_INVALID; }
      continue;
    }
    for (int i = 0; i < 4; i++)
      if (n.child[i] != -1 && (n.child[i] <= (int32_t)k || (uint32_t)n.child[i] >= num_nodes)) {
        g_err = "child index must be in (parent, num_nodes)";
        return IZPI_ERR_INVALID;
      }
  }
  s->nodes.assign(nodes, nodes + num_nodes);
  for (uint32_t k = 0; k < np; k++)
    s->prim_ref[k] = order[k] < nt ? IZPI_PRIM_REF(IZPI_PRIM_TRIANGLE, order[k]) : IZPI_PRIM_REF(IZPI_PRIM_SPHERE, order[k] - nt);
  s->stack_bound = stack_bound(s->nodes);
  s->desc.num_nodes = num_nodes;
  s->desc.nodes = s->nodes.data();
  s->desc.num_prims = np;
  s->desc.prim_ref = s->prim_ref.data();
  return IZPI_OK;
}
uint32_t izpi_host_scene_stack_bound(const izpi_host_scene* s) { return s ? s->stack_bound : 0; }
double izpi_host_scene_build_ms(const izpi_host_scene* s) { return s ? s->build_ms : 0; }
void izpi_host_scene_free(izpi_host_scene* s) { delete s; }

uint32_t izpi_host_tiles(uint32_t width, uint32_t height, uint32_t* tiles, uint32_t max_tiles) {
  static const uint32_t steps[] = {32, 25, 24, 20, 16, 12, 10, 8, 5, 4};
  uint32_t sx = 0, sy = 0;
  for (uint32_t s : steps) if (width % s == 0) { sx = s; break; }
  for (uint32_t s : steps) if (height % s == 0) { sy = s; break; }
  if (!sx || !sy) return 0;
  const int gx = (int)(width / sx), gy = (int)(height / sy);
  const int total = gx * gy;
  // Spiral walk from the centre (grid.go:48-125). The cursor may leave the grid;
  // visited cells are tracked over a padded window.
  const int pad = gx + gy + 2, ww = gx + 2 * pad;
  std::vector<uint8_t> seen((size_t)ww * (size_t)(gy + 2 * pad), 0);
  auto cell = [&](int x, int y) -> uint8_t& { return seen[(size_t)(y + pad) * ww + (size_t)(x + pad)]; };
  int cx = gx / 2, cy = gy / 2, dir = 0, walked = 1;
  uint32_t n = 0;
  auto emit = [&](int x, int y) {
    if (n < max_tiles) {
      tiles[4 * n] = (uint32_t)x * sx; tiles[4 * n + 1] = (uint32_t)y * sy;
      tiles[4 * n + 2] = (uint32_t)x * sx + sx - 1; tiles[4 * n + 3] = (uint32_t)y * sy + sy - 1;
    }
    n++;
  };
  cell(cx, cy) = 1;
  emit(cx, cy);
  static const int dx[4] = {0, 1, 0, -1}, dy[4] = {-1, 0, 1, 0};  // UP, RIGHT, DOWN, LEFT
  while (walked != total) {
    int d = ((dir % 4) + 4) % 4;
    int nx = cx + dx[d], ny = cy + dy[d];
    if (cell(nx, ny)) { dir--; continue; }
    cx = nx; cy = ny; cell(cx, cy) = 1;
    if (cx >= 0 && cx < gx && cy >= 0 && cy < gy) { walked++; emit(cx, cy); }
    dir++;
  }
  return n < max_tiles ? n : max_tiles;
}

uint32_t izpi_host_bvh_leaf_max(const izpi_scene_desc* desc) {
  const uint64_t np = desc ? (uint64_t)desc->num_tris + desc->num_spheres : 0;
  return np > 0 && 4ull * desc->num_spheres >= np ? 2u : 3u;
}

uint32_t izpi_host_share_tiles(const uint32_t* tiles, uint32_t num_tiles, uint32_t share, uint32_t num_shares,
                               uint32_t* out) {
  if (!tiles || !out || num_shares == 0) return 0;
  uint32_t n = 0;
  for (uint32_t t = share; t < num_tiles; t += num_shares, n++)
    for (int k = 0; k < 4; k++) out[4 * n + k] = tiles[4 * (size_t)t + k];
  return n;
}

/* sizeof() of every boundary struct, in the order of IZPI_ABI_STRUCTS (tests compare
 * them with the Python/ctypes and Go-side layouts). */
uint32_t izpi_abi_struct_size(int which) {
  switch (which) {
    case 0: return sizeof(izpi_bvh4_node);
    case 1: return sizeof(izpi_texture);
    case 2: return sizeof(izpi_material);
    case 3: return sizeof(izpi_camera);
    case 4: return sizeof(izpi_scene_desc);
    case 5: return sizeof(izpi_render_req);
    case 6: return sizeof(izpi_render_stats);
    case 7: return sizeof(izpi_hit);
    case 8: return sizeof(izpi_tri_in);
    case 9: return sizeof(izpi_sphere_in);
    case 10: return sizeof(izpi_camera_in);
    case 11: return sizeof(izpi_scene_input);
    case 12: return sizeof(izpi_proto_info);
    case 13: return sizeof(izpi_obj_info);
    case 14: return sizeof(izpi_obj_group);
    case 15: return sizeof(izpi_obj_material);
    case 16: return sizeof(izpi_render_tuning);
  }
  return 0;
}

/* The product's Go-math header compiled for the host (parity hook for tests). */
double izpi_host_gomath(int op, double x, double y) {
  switch (op) {
    case 0: return gm::sin(x);
    case 1: return gm::cos(x);
    case 2: return gm::tan(x);
    case 3: return gm::exp(x);
    case 4: return gm::log(x);
    case 5: return gm::pow(x, y);
    case 6: return gm::atan2(x, y);
    case 7: return gm::asin(x);
    case 8: return gm::sqrt(x);
    case 9: return x / y;
    case 10: return gm::atan(x);
    case 11: case 12: {  // sincos_nonneg: sin, cos parts (x >= 0)
      double sv, cv;
      gm::sincos_nonneg(x, &sv, &cv);
      return op == 11 ? sv : cv;
    }
  }
  return gm::nan();
}

}  // extern "C"
