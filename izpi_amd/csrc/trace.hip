// trace.hip — BVH4.Hit (hitable/bvh4.go:49-164) as the wavefront's traversal kernel k_trace2,
// and the host's choice of its instance (izpi_kern.h).
#include "izpi_kern.h"

// BVH4.Hit, step-scheduled variant. Each lane is in one of two modes: NODE (visit
// the node `cur`: the 4-slot box test of an inner node, or the slot-0 re-test of a
// leaf, A10) or PRIM (test primitive pk of the leaf being scanned, one per step).
// Every loop iteration the wave runs ONE kind of step — the one most of its busy lanes
// want (weighted by the relative cost of a node step and an f64 primitive test) — so
// f32 node code and f64 triangle code no longer serialise inside one iteration. Each
// ray still performs exactly the reference's sequence of node visits and primitive
// tests (bvh4.go:76-160), only interleaved differently with other rays, so results and
// counters are unchanged.
// The traversal stack is a ring of S entries per lane in LDS; when a push finds the
// ring full, the oldest entry is spilled to a per-thread global area (entry e at
// spill[e * stride + gtid], <= 64 entries as bvh4.go:71) and read back on pop. Counters
// are kept per wave in SGPRs (popcounts of ballots).
// TRI: the scene holds no spheres (DevScene::tri_only), so the sphere code is compiled out.
// LB: the whole BVH (inner nodes, leaf records, primitives) is small enough to sit in this
// block's LDS (bvh_lds_fits: at most BVH_LDS_BYTES): every node and primitive load is an
// LDS read instead of an L1/L2 round trip (C2, C4, C5: 10-22 primitives).
// RL: triangle-only scene whose hits need no (u, v) (wp.hit_uv == 0, C3): the lane's f64 ray
// is kept in LDS from its refill on, so a primitive test reads its owner's ray with three
// ds_read_b128 instead of re-reading the 48-B record from global memory, where it has
// usually left the XCD's L2 by then; the (u, v) arrays it does not need make room for it
// (31.8 KB of LDS per block: still 5 blocks per CU).
// Q: the inner nodes are read in their quantised 64-B form (DevScene::innerq, GInnerQ) and
// decoded into the same f32 boxes the 128-B records of a quantised scene hold; the slab test
// and everything after it are unchanged.
constexpr uint32_t BVH_LDS_BYTES = 4096;
template <int S, int WPE, bool DIST, bool TRI, bool LB, bool RL, bool Q>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) k_trace2(const DevScene sc, const WaveParams wp, unsigned long long* counters,
                                                uint32_t* err, int32_t* spill, uint32_t spill_stride, uint32_t prim_w,
                                                uint32_t tchunk, uint32_t refill_min) {
  static_assert((S & (S - 1)) == 0, "ring size must be a power of two");
  static_assert(!LB || DIST, "the LDS-resident BVH instance runs the distributed leaf tests");
  static_assert(!RL || (DIST && (TRI || LB)), "the LDS-resident ray instances: triangle-only global BVH, or the BVH in LDS");
  static_assert(!Q || !LB, "the quantised nodes are read from global memory");
  // (u, v) of the accepted hit: kept in lds_uv until the ray finishes (UVL), stored to the
  // hit record at acceptance (UVS: the BVH-in-LDS ray instance, whose steps issue no global
  // loads for the store to hold up), or not kept (C3's instance: nothing reads it)
  constexpr bool UVL = !RL, UVS = RL && LB, DUV = !RL || LB;
  typedef float v4f __attribute__((ext_vector_type(4)));   // clang vectors: copyable out of an LDS lvalue
  typedef double v2d __attribute__((ext_vector_type(2)));
  typedef const __attribute__((address_space(3))) v4f LF4;
  typedef const __attribute__((address_space(3))) v2d LD2;
  __shared__ float4 bvh_lds[LB ? BVH_LDS_BYTES / 16 : 1];
  // LDS layout: inner nodes (8 float4 each), leaf records by first primitive (2), primitives (5)
  LF4* const l_inner = (LF4*)bvh_lds;
  LF4* const l_leaves = l_inner + (size_t)8 * (LB ? sc.num_inner : 0);
  LD2* const l_prims = (LD2*)(l_leaves + (size_t)2 * (LB ? sc.num_prims : 0));
  if constexpr (LB) {
    const uint32_t ni = 8 * sc.num_inner, nl = 2 * sc.num_prims, np5 = 5 * sc.num_prims;
    for (uint32_t t = threadIdx.x; t < ni + nl + np5; t += 256)
      bvh_lds[t] = t < ni ? reinterpret_cast<const float4*>(sc.inner)[t]
                          : (t < ni + nl ? reinterpret_cast<const float4*>(sc.leaves)[t - ni]
                                         : reinterpret_cast<const float4*>(sc.prims)[t - ni - nl]);
    __syncthreads();
  }
  __shared__ int32_t lds_stack[S * 256];
  // DIST: one wave-wide batch of leaf tests: (primitive << 6 | owner lane), then the
  // test's result flags in the same word; distances and barycentrics
  // (+4: an owner reads its four entries unconditionally, past the wave's last batch entry)
  __shared__ uint32_t dist_owner[DIST ? 260 : 1];
  __shared__ double dist_t[DIST ? 260 : 1], dist_u[DIST && DUV ? 260 : 1], dist_v[DIST && DUV ? 260 : 1];
  // (u, v) of the lane's accepted hit so far: the hit record is stored once, when the ray finishes
  // (a global store per accepted hit would hold up the wave's next load wait, since
  // vmcnt counts stores and loads in one queue)
  __shared__ double2 lds_uv[UVL ? 256 : 1];
  // RL: the lane's ray (o, d) as three double2, written at its refill
  __shared__ double2 ray_lds[RL ? 3 * 256 : 1];
  const uint32_t wbase = threadIdx.x & ~63u;
  int32_t* stk = lds_stack + threadIdx.x;
  int32_t* gsp = spill + blockIdx.x * 256 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n = *wp.in_count;
  if (wp.pool_ctr && blockIdx.x == 0) pool_publish(wp.pool_ctr);
  // the next k_shade appends to out_count from 0 (its old value, an earlier pass's input
  // count, is read by no one any more): no memset launch per pass
  if (wp.out_count && blockIdx.x == 0 && threadIdx.x == 0) *wp.out_count = 0;
  if (wp.out_park && blockIdx.x == 0 && threadIdx.x == 0) *wp.out_park = 0;
  // kind words other than RAY_MAIN exist only with dielectrics (path-length rays), explicit
  // tMin / tMax, or after a shading pass that parked entries on an empty overflow pool (dead
  // entries are recognised by their ray)
  const bool read_kind = wp.read_kind != 0 || (wp.in_park && *wp.in_park != 0);
  // Small queues (the wavefront's tail passes): chunks shrink so the rays spread over
  // more waves, and waves past the last chunk exit at once instead of each paying a
  // dequeue atomic on the one counter word (~88/us chip-wide).
  const uint32_t nwaves = gridDim.x * 4u;
  const uint32_t chunk = min(tchunk, max(16u, (n + nwaves - 1u) / nwaves));
  // each wave's first chunk is its own, without an atomic; the rest is dequeued in chunks
  // (larger static first ranges measured slower: DESIGN 3.6)
  const uint32_t first = chunk;
  if ((uint64_t)(blockIdx.x * 4u + (threadIdx.x >> 6)) * first >= n) return;
  uint64_t c_rays = 0, c_nodes = 0, c_tri = 0, c_sph = 0;  // wave-uniform (SGPR)
  uint64_t c_nstep = 0, c_pstep = 0, c_short = 0;
  bool busy = false, in_prim = false;
  bool exhausted = false;
  uint32_t qi = 0;        // the lane's queue entry (its ray, hit and path state index)
  uint32_t lkind = RAY_MAIN;
  double tmax = 0;
  float ix = 0, iy = 0, iz = 0, ox = 0, oy = 0, oz = 0;
  int32_t cur = -1, pk = 0, pend = 0;
  int sp = 0, low = 0;
  int clean_from = 0;     // stack entries at positions >= clean_from were pushed after the last accepted hit
  int32_t bprim = -1;
  bool fast = false;      // slab4_fast is exact for this ray
#ifdef IZPI_SHADOW
  // measurement: spilled stack entries stored / loaded (wave counts), and a sink for the
  // shadow loads (bit 1: inner nodes, 2: leaf records, 4: primitives)
  uint64_t c_spill_st = 0, c_spill_ld = 0;
  uint32_t sh_acc = 0;
#endif
  // wave-private range [c_pos, c_end) of the input queue; the first one is the wave's own
  uint32_t c_pos = __builtin_amdgcn_readfirstlane((blockIdx.x * 4u + (threadIdx.x >> 6)) * first);  // (uniform: SGPR)
  uint32_t c_end = c_pos + first < n ? c_pos + first : n;
#ifdef IZPI_TRACE_CLOCKS
  uint64_t k_refill = 0, k_node = 0, k_prim = 0, k_adv = 0, k0 = 0, k1 = 0;
#define IZPI_CLK(v) (v) = __builtin_readcyclecounter()
#else
#define IZPI_CLK(v) (void)0
#endif
  for (;;) {
    IZPI_CLK(k0);
    const uint64_t idle = __ballot(!busy);
    if (idle != 0) {
      const uint32_t nidle = (uint32_t)__popcll(idle);
      if (!exhausted && (nidle >= refill_min || idle == ~0ull) && c_pos >= c_end) {
        // the wave's private range of the queue is used up: take the next `chunk`
        // entries with one atomic (a single head word saturates near 88 dequeues/us).
        // Every wave's first chunk is its own (chunk w, set before the loop), without an
        // atomic: a pass of at most nwaves chunks (the tail passes) dequeues without any.
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(wp.trace_next, chunk);
        b = __builtin_amdgcn_readfirstlane(b) + nwaves * first;
        if (b >= n) exhausted = true;
        c_pos = b;
        c_end = b + chunk < n ? b + chunk : n;
      }
      if (!exhausted && (nidle >= refill_min || idle == ~0ull) && c_pos < c_end) {
        const uint32_t take = nidle < c_end - c_pos ? nidle : c_end - c_pos;
        const uint32_t base = c_pos;
        c_pos += take;
        bool main_ray = false;
        const uint32_t rank = (uint32_t)__popcll(idle & ((1ull << lane) - 1));
        const uint32_t my = base + rank;
        if (!busy && rank < take) {
          const uint32_t k = read_kind ? sld(wp.in.kind + my) : (uint32_t)RAY_MAIN;
          // a parked entry is not traced: its hit record (copied by k_shade) stays for the retry
          // (RL: the ray is read once, here, so it is a streamed load; otherwise primitive
          // steps read it again)
          RayOD r;
          if constexpr (RL) {
            r = sld(wp.in.ray + my);
            const double2* rp = reinterpret_cast<const double2*>(&r);
            const double2 r0 = rp[0], r1 = rp[1], r2 = rp[2];
            ray_lds[3 * threadIdx.x] = r0; ray_lds[3 * threadIdx.x + 1] = r1; ray_lds[3 * threadIdx.x + 2] = r2;
          } else {
            r = wp.in.ray[my];
          }
          if (!(k & (RAY_PARKED | RAY_DEAD)) && (uint64_t)__double_as_longlong(r.o[0]) != DEAD_BITS) {
            qi = my;
            lkind = k;
            tmax = ray_tmax(wp.in, my, k);
            main_ray = kind_of(k) == RAY_MAIN;
            ix = (float)(1.0 / r.d[0]); iy = (float)(1.0 / r.d[1]); iz = (float)(1.0 / r.d[2]);
            ox = (float)r.o[0]; oy = (float)r.o[1]; oz = (float)r.o[2];
            fast = sc.nan_free_bounds && ray_fast_ok(ox, oy, oz, ix, iy, iz);
            cur = sc.root;
            sp = 0; low = 0; clean_from = 0;
            in_prim = false;
            bprim = -1;
            busy = cur != -1;
            if (!busy) {
              if ((UVL || UVS) && wp.hit_uv) {  // (t, prim) and (u, v) interleaved: hs == 2
                double2* rec = wp.in.hit + ((size_t)my << 1);
                sst(rec, hit_pack(0.0, -1)); sst(rec + 1, make_double2(0.0, 0.0));
              } else {
                sst(wp.in.hit + my, hit_pack(0.0, -1));
              }
            }
          }
        }
        c_rays += (uint64_t)__popcll(__ballot(main_ray));
        // drain the new rays' loads here: left pending they make the compiler wait for
        // vmcnt(0) at the loop head, i.e. for every hit-record store, on every iteration
        __builtin_amdgcn_s_waitcnt(0x0F70);
      } else if (exhausted && idle == ~0ull) {
        break;
      }
    }
    const uint64_t m_prim = __ballot(busy && in_prim);
    const uint64_t m_node = __ballot(busy && !in_prim);
    if ((m_prim | m_node) == 0) continue;
    const uint32_t n_prim = (uint32_t)__popcll(m_prim), n_node = (uint32_t)__popcll(m_node);
    bool advance = false;   // lane finished its current node / leaf: take next or pop
    bool leaf_next = false; // the step went straight into a leaf whose re-test is known to pass
    int32_t next = -1;
#ifdef IZPI_TRACE_CLOCKS
    IZPI_CLK(k1); k_refill += k1 - k0; k0 = k1;
    const bool clk_prim = n_prim * prim_w >= n_node * 16u;
#endif
    if (n_prim * prim_w >= n_node * 16u) {
      if constexpr (DIST) {
        // ---- distributed primitive step: every pending test of the PRIM lanes' leaves
        // (up to 64) runs on its own lane, then each owner accepts its leaf's results in
        // primitive order against its running tMax (bvh4.go:123-134, triangle.go:219)
        const uint32_t cnt = (busy && in_prim) ? (uint32_t)(pend - pk) : 0u;  // 1..4
        const uint64_t lt = (1ull << lane) - 1;
        const uint32_t base = (uint32_t)__popcll(__ballot(cnt & 1u) & lt) + 2u * (uint32_t)__popcll(__ballot(cnt & 2u) & lt) +
                              4u * (uint32_t)__popcll(__ballot(cnt & 4u) & lt);
        const bool served = cnt > 0 && base + cnt <= 64;
        const uint64_t ms = __ballot(served);
        const int last = 63 - __clzll((long long)ms);
        const uint32_t total = (uint32_t)__shfl((int)(base + cnt), last);
        {  // a leaf has 1..4 primitives (bvh4.go:638): four predicated writes, no loop
          const uint32_t e = ((uint32_t)pk << 6) | lane;
          uint32_t* dq = dist_owner + wbase + base;
          if (served) dq[0] = e;
          if (served && cnt > 1) dq[1] = e + 64u;
          if (served && cnt > 2) dq[2] = e + 128u;
          if (served && cnt > 3) dq[3] = e + 192u;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t ent = lane < total ? dist_owner[wbase + lane] : lane;
        const uint32_t ow = ent & 63u;
        const uint32_t oqi = (uint32_t)__shfl((int)qi, (int)ow);
        const uint32_t okind = (uint32_t)__shfl((int)lkind, (int)ow);
        if (lane < total) {
          const int32_t pi = (int32_t)(ent >> 6);
          double2 r0, r1, r2;
          if constexpr (RL) {
            const uint32_t ro = 3 * (wbase + ow);
            r0 = ray_lds[ro]; r1 = ray_lds[ro + 1]; r2 = ray_lds[ro + 2];
          } else {
            const double2* rp = reinterpret_cast<const double2*>(wp.in.ray + oqi);
            r0 = rp[0]; r1 = rp[1]; r2 = rp[2];
          }
          const double otmin = ray_tmin(wp.in, oqi, okind);
          double2 p0, p1, p2, p3, p4;
          if constexpr (LB) {
            LD2* pp = l_prims + (size_t)5 * pi;
            const v2d a0 = pp[0], a1 = pp[1], a2 = pp[2], a3 = pp[3], a4 = pp[4];
            p0 = make_double2(a0.x, a0.y); p1 = make_double2(a1.x, a1.y); p2 = make_double2(a2.x, a2.y);
            p3 = make_double2(a3.x, a3.y); p4 = make_double2(a4.x, a4.y);
          } else {
            const double2* pp = reinterpret_cast<const double2*>(sc.prims + pi);
            p0 = pp[0]; p1 = pp[1]; p2 = pp[2]; p3 = pp[3]; p4 = pp[4];
#ifdef IZPI_SHADOW
            if (IZPI_SHADOW & 4) {
              const uint4* sq = reinterpret_cast<const uint4*>(sc.sh_prims + pi);
              const uint4 s0 = sq[0], s1 = sq[1], s2 = sq[2], s3 = sq[3], s4 = sq[4];
              sh_acc ^= s0.x ^ s1.y ^ s2.z ^ s3.w ^ s4.x;
            }
#endif
          }
          const double pa[9] = {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y, p4.x};
          double t = 0, u = 0, v = 0;
          const V3 o = mk(r0.x, r0.y, r1.x), d = mk(r1.y, r2.x, r2.y);
          uint32_t flags;
          if (TRI || (uint32_t)__double2loint(p4.y) == IZPI_PRIM_TRIANGLE) {
            flags = tri_intersect_no_tmax(pa, o, d, otmin, t, u, v) ? 1u : 0u;
          } else {
            // sphere: both roots now, their tMin tests as flags; tMax is applied in order
            // by the owner (sphere.go:72-92: root 0 if tMin < t0 < tMax, else root 1)
            // (a scene whose spheres do not move: center(time) == center(time0), no load)
            // (the BVH-in-LDS ray instance runs only on such scenes: make_tracer)
            const double time = (RL && LB) || sc.time_free ? pa[7] : (wp.in.time ? wp.in.time[oqi] : 0.0);
            flags = 2u;
            if (sph_roots(sph_center(pa, time), pa[6], o, d, t, u))
              flags |= 1u | (t > otmin ? 4u : 0u) | (u > otmin ? 8u : 0u);
          }
          dist_t[wbase + lane] = t;
          if constexpr (DUV) { dist_u[wbase + lane] = u; dist_v[wbase + lane] = v; }
          dist_owner[wbase + lane] = flags;
        }
        const uint32_t n_sph_tests = TRI ? 0u : (uint32_t)__popcll(__ballot(lane < total && (dist_owner[wbase + lane] & 2u)));
        __builtin_amdgcn_wave_barrier();
        if (served && (TRI || n_sph_tests == 0)) {
          // triangles only: the leaf's flags and distances come in one LDS round trip, the
          // ordered accept runs in registers, and only the accepted (u, v) is read back
          const uint32_t j0 = wbase + base;
          uint32_t f[4];
          double tt[4];
#pragma unroll
          for (uint32_t i = 0; i < 4; i++) { f[i] = dist_owner[j0 + i]; tt[i] = dist_t[j0 + i]; }
          int32_t acc = -1;
#pragma unroll
          for (uint32_t i = 0; i < 4; i++)  // reject only `t > tMax` (triangle.go:219), in primitive order
            if (i < cnt && (f[i] & 1u) && !(tt[i] > tmax)) { tmax = tt[i]; acc = (int32_t)i; }
          if (acc >= 0) {
            if constexpr (UVL) lds_uv[threadIdx.x] = make_double2(dist_u[j0 + acc], dist_v[j0 + acc]);
            if constexpr (UVS)
              if (wp.hit_uv) sst(wp.in.hit + ((size_t)qi << 1) + 1, make_double2(dist_u[j0 + acc], dist_v[j0 + acc]));
            bprim = pk + acc;
            clean_from = sp;
          }
          pk = pend;
          in_prim = false;
          advance = true;
        } else if (!TRI && served) {
          int32_t acc = -1;
          double acc_u = 0, acc_v = 0;
          for (uint32_t i = 0; i < cnt; i++) {
            const uint32_t j = wbase + base + i;
            const uint32_t f = dist_owner[j];
            if (!(f & 1u)) continue;
            if (!(f & 2u)) {  // triangle: reject only `t > tMax` (triangle.go:219)
              const double t = dist_t[j];
              if (!(t > tmax)) { tmax = t; acc = (int32_t)j; acc_u = dist_u[j]; acc_v = dist_v[j]; bprim = pk + (int32_t)i; }
            } else {  // sphere: strict bounds, root 0 first
              const double ta = dist_t[j], tb = dist_u[j];
              if (ta < tmax && (f & 4u)) { tmax = ta; acc = (int32_t)j; acc_u = 0.0; acc_v = 0.0; bprim = pk + (int32_t)i; }
              else if (tb < tmax && (f & 8u)) { tmax = tb; acc = (int32_t)j; acc_u = 1.0; acc_v = 0.0; bprim = pk + (int32_t)i; }
            }
          }
          if (acc >= 0) {
            if constexpr (UVS) {
              if (wp.hit_uv) sst(wp.in.hit + ((size_t)qi << 1) + 1, make_double2(acc_u, acc_v));
            } else {
              lds_uv[threadIdx.x] = make_double2(acc_u, acc_v);
            }
            clean_from = sp;
          }
          pk = pend;
          in_prim = false;
          advance = true;
        }
        __builtin_amdgcn_wave_barrier();
        c_tri += total - n_sph_tests;
        c_sph += n_sph_tests;
        c_pstep++;
      } else {
      // ---- primitive step: one Hit() per PRIM lane (bvh4.go:123-134)
      bool is_tri = false;
      if (busy && in_prim) {
        // the f64 ray is re-read here (L2) instead of living in 14 VGPRs across node steps
        // (measured: keeping it in LDS instead makes k_shade's later read of the same
        // record miss and costs more than it saves)
        const double2* rp = reinterpret_cast<const double2*>(wp.in.ray + qi);
        const double2 r0 = rp[0], r1 = rp[1], r2 = rp[2];
        const V3 o = mk(r0.x, r0.y, r1.x), d = mk(r1.y, r2.x, r2.y);
        const double tmin = ray_tmin(wp.in, qi, lkind);
        const double2* pp = reinterpret_cast<const double2*>(sc.prims + pk);
        const double2 p0 = pp[0], p1 = pp[1], p2 = pp[2], p3 = pp[3], p4 = pp[4];
        const double pa[9] = {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y, p4.x};
        is_tri = TRI || (uint32_t)__double2loint(p4.y) == IZPI_PRIM_TRIANGLE;
        if (is_tri) {
          double t, u, v;
          if (tri_intersect(pa, o, d, tmin, tmax, t, u, v)) {  // barycentrics wait in LDS (lds_uv)
            tmax = t; bprim = pk; lds_uv[threadIdx.x] = make_double2(u, v); clean_from = sp;
          }
        } else if (!TRI) {
          const double time = wp.in.time ? wp.in.time[qi] : 0.0;  // only spheres read the ray time
          double t; int root;
          if (sph_intersect(pa, o, d, time, tmin, tmax, t, root)) {
            tmax = t; bprim = pk; lds_uv[threadIdx.x] = make_double2((double)root, 0.0); clean_from = sp;
          }
        }
        pk++;
        if (pk == pend) { in_prim = false; advance = true; }
      }
      const uint32_t n_tri = (uint32_t)__popcll(__ballot(is_tri));
      c_tri += n_tri;
      c_sph += n_prim - n_tri;
      c_pstep++;
      }
    } else {
      c_nodes += n_node;
      c_nstep++;
      // ---- node step: visit `cur` (bvh4.go:87-146)
      const bool wave_fast = __ballot(busy && !in_prim && !fast) == 0;
      if (__ballot(busy && !in_prim && sp + 3 - low > S) != 0) {
        // ring too full for this step's three writes: spill the oldest entries (rare)
        if (busy && !in_prim) {
          while (sp + 3 - low > S) {
            gsp[(size_t)low * spill_stride] = stk[(low & (S - 1)) * 256];
            low++;
#ifdef IZPI_SHADOW
            c_spill_st++;
#endif
          }
        }
      }
      if (busy && !in_prim) {
        const float tm = (float)tmax;
        // An inner node (4-slot box test) and a leaf's slot-0 re-test (A10) run as ONE
        // code path: a leaf lane's 32-B GLeaf box lands in slot 0 (selects below), its
        // slots 1-3 are invalid. Mixed waves (nearly every node step) then issue one set
        // of loads and wait once, instead of running the two branches one after the other.
        const bool is_leaf = ref_is_leaf(cur);
        float4 q0, q1, mnz_, mxx_, mxy_, mxz_;
        int4 ch_;
        if constexpr (LB) {
          LF4* lp = is_leaf ? l_leaves + (size_t)2 * leaf_start(cur) : l_inner + (size_t)8 * cur;
          LF4* np = is_leaf ? l_inner : lp;
          const v4f a0 = lp[0], a1 = lp[1], a2 = np[2], a3 = np[3], a4 = np[4], a5 = np[5], c = np[6];
          q0 = make_float4(a0.x, a0.y, a0.z, a0.w); q1 = make_float4(a1.x, a1.y, a1.z, a1.w);
          mnz_ = make_float4(a2.x, a2.y, a2.z, a2.w); mxx_ = make_float4(a3.x, a3.y, a3.z, a3.w);
          mxy_ = make_float4(a4.x, a4.y, a4.z, a4.w); mxz_ = make_float4(a5.x, a5.y, a5.z, a5.w);
          ch_ = make_int4(__float_as_int(c.x), __float_as_int(c.y), __float_as_int(c.z), __float_as_int(c.w));
        } else if constexpr (Q) {
          // GInnerQ = (org, ex), (q mnx, mny, mnz, mxx), (q mxy, mxz, child 0, 1), (child 2, 3, -, -);
          // leaf lanes read their last two loads from the root node (values not used)
          const float4* lp = reinterpret_cast<const float4*>(is_leaf ? (const void*)(sc.leaves + leaf_start(cur))
                                                                     : (const void*)(sc.innerq + cur));
          const float4* np = is_leaf ? reinterpret_cast<const float4*>(sc.innerq) : lp;
          q0 = lp[0]; q1 = lp[1];
          const float4 c2 = np[2], c3 = np[3];
          const uint32_t ex = __float_as_uint(q0.w);
          const float sx = __uint_as_float((ex & 0xFFu) << 23), sy = __uint_as_float(((ex >> 8) & 0xFFu) << 23),
                      sz = __uint_as_float(((ex >> 16) & 0xFFu) << 23);
          // org + q * 2^e: the product is exact, so the fused form rounds once, as qdecode does
          auto dec4 = [](float w, float o, float sc_) {
            const uint32_t b = __float_as_uint(w);
            return make_float4(__builtin_fmaf((float)(b & 0xFFu), sc_, o), __builtin_fmaf((float)((b >> 8) & 0xFFu), sc_, o),
                               __builtin_fmaf((float)((b >> 16) & 0xFFu), sc_, o), __builtin_fmaf((float)(b >> 24), sc_, o));
          };
          // (slot 0 of mnx / mny / ... is replaced by the GLeaf box for leaf lanes below)
          const float4 dmnx = dec4(q1.x, q0.x, sx), dmny = dec4(q1.y, q0.y, sy), dmnz = dec4(q1.z, q0.z, sz);
          const float4 dmxx = dec4(q1.w, q0.x, sx), dmxy = dec4(c2.x, q0.y, sy), dmxz = dec4(c2.y, q0.z, sz);
          // arrange as the 128-B path's registers: q0 / q1 hold the leaf box, the rest slots 1-3
          const float4 l0 = q0, l1 = q1;
          q0 = is_leaf ? l0 : dmnx;
          q1 = is_leaf ? l1 : make_float4(dmny.x, dmny.y, dmny.z, dmny.w);
          mnz_ = dmnz; mxx_ = dmxx; mxy_ = dmxy; mxz_ = dmxz;
          ch_ = make_int4(__float_as_int(c2.z), __float_as_int(c2.w), __float_as_int(c3.x), __float_as_int(c3.y));
        } else {
          const float4* lp = reinterpret_cast<const float4*>(is_leaf ? (const void*)(sc.leaves + leaf_start(cur))
                                                                     : (const void*)(sc.inner + cur));
          // leaf lanes read their last five loads from the root node (a cached valid address;
          // the values are not used)
          const float4* np = is_leaf ? reinterpret_cast<const float4*>(sc.inner) : lp;
          q0 = lp[0]; q1 = lp[1];
          mnz_ = np[2]; mxx_ = np[3]; mxy_ = np[4]; mxz_ = np[5];
          ch_ = *reinterpret_cast<const int4*>(np + 6);
#ifdef IZPI_SHADOW
          if ((IZPI_SHADOW & 1) && !is_leaf) {
            const uint4* sq = reinterpret_cast<const uint4*>(sc.sh_inner + cur);
            const uint4 s0 = sq[0], s1 = sq[1], s2 = sq[2], s3 = sq[3], s4 = sq[4], s5 = sq[5], s6 = sq[6];
            sh_acc ^= s0.x ^ s1.y ^ s2.z ^ s3.w ^ s4.x ^ s5.y ^ s6.z;
          }
          if ((IZPI_SHADOW & 2) && is_leaf) {
            const uint4* sq = reinterpret_cast<const uint4*>(sc.sh_leaves + leaf_start(cur));
            const uint4 s0 = sq[0], s1 = sq[1];
            sh_acc ^= s0.x ^ s1.y;
          }
#endif
        }
        // GLeaf = (mn.x, mn.y, mn.z, mx.x), (mx.y, mx.z, start, count)
        const float4 mnx = q0;
        const float4 mny = make_float4(is_leaf ? q0.y : q1.x, q1.y, q1.z, q1.w);
        const float4 mnz = make_float4(is_leaf ? q0.z : mnz_.x, mnz_.y, mnz_.z, mnz_.w);
        const float4 mxx = make_float4(is_leaf ? q0.w : mxx_.x, mxx_.y, mxx_.z, mxx_.w);
        const float4 mxy = make_float4(is_leaf ? q1.x : mxy_.x, mxy_.y, mxy_.z, mxy_.w);
        const float4 mxz = make_float4(is_leaf ? q1.y : mxz_.x, mxz_.y, mxz_.z, mxz_.w);
        const int4 ch = make_int4(is_leaf ? cur : ch_.x, ch_.y, ch_.z, ch_.w);
        uint32_t hm;
        if (wave_fast) {
          hm = slab4_fast(mnx, mny, mnz, mxx, mxy, mxz, ox, oy, oz, ix, iy, iz, tm);
        } else {
          const float amnx[4] = {mnx.x, mnx.y, mnx.z, mnx.w}, amny[4] = {mny.x, mny.y, mny.z, mny.w},
                      amnz[4] = {mnz.x, mnz.y, mnz.z, mnz.w}, amxx[4] = {mxx.x, mxx.y, mxx.z, mxx.w},
                      amxy[4] = {mxy.x, mxy.y, mxy.z, mxy.w}, amxz[4] = {mxz.x, mxz.y, mxz.z, mxz.w};
          hm = 0;
#pragma unroll
          for (int i = 0; i < 4; i++)
            if (slab(amnx[i], amny[i], amnz[i], amxx[i], amxy[i], amxz[i], ox, oy, oz, ix, iy, iz, tm)) hm |= 1u << i;
        }
        // slots 0..3 with ChildIndex != -1 whose box is hit (bvh4.go:119-146): the first
        // is visited next, the others are pushed in slot order (popped LIFO). Selects
        // instead of branches: each divergent branch costs exec-mask and lane-mask
        // bookkeeping on the scalar unit, which is as busy as the vector unit here.
        const uint32_t valid = is_leaf ? 1u
                                       : ((ch.x != -1 ? 1u : 0u) | (ch.y != -1 ? 2u : 0u) | (ch.z != -1 ? 4u : 0u) |
                                          (ch.w != -1 ? 8u : 0u));
        const uint32_t m = hm & valid;
        const int32_t c01 = (m & 1u) ? ch.x : ch.y, c23 = (m & 4u) ? ch.z : ch.w;
        next = m == 0 ? -1 : ((m & 3u) ? c01 : c23);
        // A passed leaf re-test starts on the leaf's primitives. A leaf visited straight
        // after its parent re-tests the same f32 box with the same tMax (A10): the result
        // is known to be a hit, so its node load is skipped too (the visit is still counted).
        const bool enter = ref_is_leaf(next) && (is_leaf || sc.leaf_shortcut);
        leaf_next = enter && !is_leaf;
        in_prim = enter;
        pk = enter ? leaf_start(next) : pk;
        pend = enter ? leaf_start(next) + leaf_count(next) : pend;
        next = enter ? -1 : next;
        // the other hit children, compacted in slot order, are written unconditionally to
        // ring positions sp..sp+2 (the ring keeps 3 free entries above sp); sp moves by
        // their count
        const uint32_t rest = m & (m - 1u);  // bits 1..3 only
        const int np_ = __builtin_popcount(rest);
        const int32_t e0 = (rest & 2u) ? ch.y : ((rest & 4u) ? ch.z : ch.w);
        const int32_t e1 = ((rest & 6u) == 6u) ? ch.z : ch.w;
        stk[(sp & (S - 1)) * 256] = e0;
        stk[((sp + 1) & (S - 1)) * 256] = e1;
        stk[((sp + 2) & (S - 1)) * 256] = ch.w;
        if (sp + np_ > 64) atomicOr(err, 1u);  // unreachable: the host rejects BVHs deeper than 64 entries
        sp += np_;
        advance = !enter;
      }
    }
#ifdef IZPI_TRACE_CLOCKS
    IZPI_CLK(k1); if (clk_prim) k_prim += k1 - k0; else k_node += k1 - k0; k0 = k1;
#endif
    // ---- advance: next child, else pop (bvh4.go:150-160), else the ray is done
    {
      const bool do_pop = advance && next == -1 && sp > 0;
      const bool do_fin = advance && next == -1 && sp == 0;
      // the LDS read is unconditional (and volatile, so that the compiler keeps it a ds_read:
      // a select of the LDS and spill addresses becomes a flat load, whose wait also
      // drains every store)
      const int spn = sp - 1;
      int32_t top = *(volatile __attribute__((address_space(3))) int32_t*)&lds_stack[threadIdx.x + (spn & (S - 1)) * 256];
      if (__ballot(do_pop && spn < low) != 0) {
        if (do_pop && spn < low) {
          top = gsp[(size_t)spn * spill_stride];
          low = spn;
#ifdef IZPI_SHADOW
          c_spill_ld++;
#endif
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) here, not for every pop
      }
      cur = (advance && next != -1) ? next : (do_pop ? top : cur);
      sp = do_pop ? spn : sp;
      // An entry pushed after the last accepted hit meets the same tMax it was pushed
      // with, so a leaf's re-test against its (identical) box passes: skip the load.
      const bool lf = do_pop && ref_is_leaf(top) && spn >= clean_from && sc.leaf_shortcut;
      in_prim = in_prim || lf;
      leaf_next = leaf_next || lf;
      pk = lf ? leaf_start(top) : pk;
      pend = lf ? leaf_start(top) + leaf_count(top) : pend;
      clean_from = (do_pop && spn < clean_from) ? spn : clean_from;
      if (do_fin) {
        const double2 uv = (UVL && bprim >= 0) ? lds_uv[threadIdx.x] : make_double2(0.0, 0.0);
        if ((UVL || UVS) && wp.hit_uv) {  // (t, prim) and (u, v) in one 32-B record (hs == 2)
          double2* rec = wp.in.hit + ((size_t)qi << 1);
          sst(rec, hit_pack(bprim >= 0 ? tmax : 0.0, bprim));
          if (!UVS || bprim < 0) sst(rec + 1, uv);  // (UVS: an accepted hit's (u, v) is there already)
        } else {  // nothing reads (u, v): 16 B per entry (hs == 1)
          sst(wp.in.hit + qi, hit_pack(bprim >= 0 ? tmax : 0.0, bprim));
        }
        busy = false;
      }
    }
    const uint64_t n_short = (uint64_t)__popcll(__ballot(leaf_next));  // leaf visits taken by a shortcut
    c_nodes += n_short;
    c_short += n_short;
#ifdef IZPI_TRACE_CLOCKS
    IZPI_CLK(k1); k_adv += k1 - k0;
#endif
  }
#ifdef IZPI_TRACE_CLOCKS
  if (lane == 0) {
    atomicAdd(counters + CNT_CLK_REFILL, (unsigned long long)k_refill);
    atomicAdd(counters + CNT_CLK_NODE, (unsigned long long)k_node);
    atomicAdd(counters + CNT_CLK_PRIM, (unsigned long long)k_prim);
    atomicAdd(counters + CNT_CLK_ADV, (unsigned long long)k_adv);
  }
#endif
#ifdef IZPI_SHADOW
  {
    if (c_spill_st) atomicAdd(counters + CNT_CLK_REFILL, (unsigned long long)c_spill_st);
    if (c_spill_ld) atomicAdd(counters + CNT_CLK_NODE, (unsigned long long)c_spill_ld);
    if (sh_acc == 0x9E3779B9u) atomicOr(err, 0u);
  }
#endif
  if (lane == 0) {
    count_add(wp.cpart, counters, CNT_RAYS, c_rays);
    count_add(wp.cpart, counters, CNT_NODES, c_nodes);
    count_add(wp.cpart, counters, CNT_TRI, c_tri);
    count_add(wp.cpart, counters, CNT_SPH, c_sph);
    count_add(wp.cpart, counters, CNT_NSTEP, c_nstep);
    count_add(wp.cpart, counters, CNT_PSTEP, c_pstep);
    count_add(wp.cpart, counters, CNT_SHORT, c_short);
  }
}


// (DIST, TRI, LB, RL, Q) of the compiled instances
#define IZPI_T2_LIST(X)                                                                                           \
  X(true, false, false, false, false) X(true, true, false, false, false) X(false, false, false, false, false)        \
  X(false, true, false, false, false) X(true, false, true, false, false) X(true, true, true, false, false)           \
  X(true, true, false, true, false) X(true, false, true, true, false) X(true, true, true, true, false)               \
  X(true, false, false, false, true) X(true, true, false, false, true) X(true, true, false, true, true)
// The BVH-in-LDS ray instances run an 8-entry stack ring: their trees (at most 4 KB) are
// too shallow to fill it, and the 8 KB it frees hold the rays (still 5 blocks per CU).
constexpr int ring_of(bool lb, bool rl) { return lb && rl ? 8 : TRACE_RING; }

// Pick the k_trace2 instance and its grid (no allocation: the caller grows d_spill to
// t->spill_bytes).
// need_uv: the caller reads the hits' (u, v) (WaveParams::hit_uv).
int make_tracer(izpi_ctx* ctx, const izpi_render_tuning& tu, bool need_uv, Tracer* t) {
  *t = Tracer();
  if (tu.flags & IZPI_TUNE_NO_DIST) t->p2 = false;
  // DIST packs (primitive << 6 | lane) into one LDS word
  if (ctx->num_prims >= (1u << 26)) t->p2 = false;
  t->tri = ctx->sc.tri_only != 0 && !(tu.flags & IZPI_TUNE_GENERAL_TRACE);
  t->lds_bvh = t->p2 && !(tu.flags & IZPI_TUNE_NO_LDS_BVH) &&
               (uint64_t)ctx->sc.num_inner * sizeof(GInner) + (uint64_t)ctx->sc.num_prims * (sizeof(GLeaf) + sizeof(GPrim)) <= BVH_LDS_BYTES;
  if (t->lds_bvh) {
    // With the tree in LDS a step costs little next to a refill's ray loads: refill later
    // and weight primitive steps less (profiles/r3i/tune_sweep2.log, trace per frame
    // against 24 / 32: C5 -10.5%, C4 -6.3%, C2 -5.2%; C3's global-memory instance keeps them)
    t->refill_min = 40;
    t->prim_w = 24;
  }
  t->ray_lds = t->p2 && ((t->tri && !t->lds_bvh && !need_uv) || (t->lds_bvh && (t->tri || ctx->sc.time_free))) &&
               !(tu.flags & IZPI_TUNE_NO_RAY_LDS);
  // a quantised scene's 64-B nodes (the 128-B records hold the same decoded boxes: the
  // other instances traverse the same tree)
  t->qnodes = ctx->sc.quantized && t->p2 && !t->lds_bvh && !(tu.flags & IZPI_TUNE_NO_QNODES);
  if (tu.prim_weight) t->prim_w = tu.prim_weight;
  if (tu.trace_chunk) t->tchunk = tu.trace_chunk;
  if (tu.refill_min) t->refill_min = std::min<uint32_t>(64, tu.refill_min);
  int rc = IZPI_ERR_INVALID;
  ctx->err = "no k_trace2 instance for this scene and tuning";
#define IZPI_T2_OCC(P, T, L, R, Q)                                                               \
  if (t->p2 == P && t->tri == T && t->lds_bvh == L && t->ray_lds == R && t->qnodes == Q) \
    rc = resident_blocks(ctx, k_trace2<ring_of(L, R), TRACE_WPE, P, T, L, R, Q>, &t->blocks);
  IZPI_T2_LIST(IZPI_T2_OCC)
#undef IZPI_T2_OCC
  if (rc) return rc;
  t->spill_bytes = (size_t)t->blocks * 256 * 64 * sizeof(int32_t);
  return IZPI_OK;
}

void launch_trace(izpi_ctx* ctx, const DevScene& sc, const Tracer& t, const WaveParams& wp, hipStream_t st, int32_t* spill) {
  const dim3 g(t.blocks), b(256);
  const uint32_t stride = (uint32_t)t.blocks * 256;
#define IZPI_T2_LAUNCH(P, T, L, R, Q)                                                                          \
  if (t.p2 == P && t.tri == T && t.lds_bvh == L && t.ray_lds == R && t.qnodes == Q) {                          \
    hipLaunchKernelGGL((k_trace2<ring_of(L, R), TRACE_WPE, P, T, L, R, Q>), g, b, 0, st, sc, wp, ctx->d_counters, \
                       misc(ctx, 1), spill, stride, t.prim_w, t.tchunk, t.refill_min);                        \
    return;                                                                                                    \
  }
  IZPI_T2_LIST(IZPI_T2_LAUNCH)
#undef IZPI_T2_LAUNCH
}

