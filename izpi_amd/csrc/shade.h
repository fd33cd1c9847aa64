// shade.h — the sampler, materials and pdfs of one bounce (k_shade), the first fill (k_start),
// the wavefront's tail (k_tail), the ordered per-pixel sums (k_accumulate) and the pass loop
// that drives them with k_trace2 (izpi_kern.h). Compiled by the shade_*.hip translation units,
// one per (sampler, accumulation): each instantiates run_sampler for its pair, so the four
// sets of kernel instances compile in parallel.
#pragma once
#include "izpi_kern.h"

// First fill of the queue (first pass of a chunk): record slot j takes unit j (the host
// starts the unit head at min(slots, units), so no atomic is needed: one counter word
// serialises ~88 atomics/us), then further units from the head while its path needs no
// tracing; the path goes to entry j of `out`.
template <int SAMPLER, bool FWD>
__global__ void __launch_bounds__(256) k_start(const DevScene sc, const ShadeParams sp_in, const WaveParams wp) {
  ShadeParams sp = sp_in;
  sp.staged = 0;  // k_start stages no tables: its path starts read them from global memory
  sp.prims_staged = 0;
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  bool want = j < sp.slots;
  bool push = false;
  bool first = true;
  PathSt P;
  RayRec R;
  P.rslot = j;
  // a wave keeps grabbing while any of its lanes still lacks a traceable path
  for (;;) {
    uint32_t unit;
    if (first) {
      unit = (want && j < sp.total_units) ? j : 0xFFFFFFFFu;
      first = false;
    } else {
      unit = grab_unit(sp, want);
    }
    if (__ballot(want) == 0) break;
    if (want) {
      if (unit == 0xFFFFFFFFu) {
        want = false;
      } else if (start_path<SAMPLER, FWD>(sc, sp, unit, P, R)) {
        want = false;
        push = true;
      }
    }
  }
  // Entry j of the first queue belongs to record slot j (no queue atomic: one per block on
  // one counter word made this kernel 1.9 ms per C3 frame); a slot whose samples all
  // completed without a ray (spectral pdf 0, the units ran out) leaves a dead entry, which
  // the first shading pass drops.
  const uint32_t fill = min(sp.slots, sp.total_units);
  if (j < fill) {
    if (push) store_entry<SAMPLER, FWD>(wp.out, j, P, R);
    else dead_entry(wp.out, j);
  }
  if (j == 0) *wp.out_count = fill;
}

#ifdef IZPI_SHADE_CLOCKS
// Timing builds only: wave cycles per section of shade_item, accumulated in LDS by the
// first active lane of the wave that runs the section (so divergent sections count the
// wave's time once), added to the CNT_SCLK_* counters at the end of the kernel.
enum { SCLK_MAT = 0, SCLK_FIN, SCLK_MIX, SCLK_LPDF, SCLK_ENTRY, SCLK_TEX, SCLK_RB1, SCLK_RATOM, SCLK_RB2, SCLK_N };
IZPI_DEV unsigned long long* sclk_lds() {
  __shared__ unsigned long long c[16][SCLK_N];
  return &c[(threadIdx.x >> 6) & 15][0];
}
IZPI_DEV void sclk_add(int sec, uint64_t dt) {
  const uint64_t act = __ballot(1);
  if ((threadIdx.x & 63) == (uint32_t)(__ffsll((long long)act) - 1)) sclk_lds()[sec] += dt;
}
IZPI_DEV void sclk_flush(unsigned long long* counters) {
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < SCLK_N; k++) atomicAdd(counters + CNT_SCLK_MAT + k, sclk_lds()[k]);
}
IZPI_DEV void sclk_zero() {
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < SCLK_N; k++) sclk_lds()[k] = 0;
  __syncthreads();
}
#define SCLK_T(v) const uint64_t v = __builtin_readcyclecounter()
#define SCLK_ADD(sec, t0) sclk_add(sec, __builtin_readcyclecounter() - (t0))
// wait for every outstanding vector memory access (vmcnt(0); expcnt, lgkmcnt left alone):
// separates a section's memory wait from the work after it
#define SCLK_VMWAIT() __builtin_amdgcn_s_waitcnt(0x0F70)
#else
#define SCLK_VMWAIT() (void)0
#define SCLK_T(v) (void)0
#define SCLK_ADD(sec, t0) (void)0
#endif

// One block-wide reservation phase for a shading iteration (ONE pair of barriers, two
// atomics by one thread): `unit_want` lanes get consecutive work units from the unit
// head (the units past total_units are not granted); lanes with `put` and granted
// `unit_want` lanes get consecutive output entries, `put` lanes first. q_rank: the
// lane's rank among the block's `queue` lanes (deferred unwinding jobs), q_total: their number. A granted lane
// whose new path cannot trace (start_path false) leaves a RAY_DEAD entry behind.
// QSEP: `queue` lanes are a subset of the `unit_want` lanes with a ballot of their own;
// otherwise they are the `unit_want` lanes.
template <bool QSEP>
IZPI_DEV void block_reserve2(const ShadeParams& sp, uint32_t* out_count, bool put, bool unit_want, uint32_t& unit,
                             uint32_t& pos, uint32_t& parity, bool& exhausted, bool queue, uint32_t& q_rank, uint32_t& q_total) {
  __shared__ uint32_t s_p[2][SHADE_WAVES], s_u[2][SHADE_WAVES], s_q[2][SHADE_WAVES];
  __shared__ uint32_t s_pbase[2], s_ubase[2], s_granted[2], s_nput[2], s_nent[2];
  const uint32_t b = parity;
  parity ^= 1u;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1;
  const uint64_t mp = __ballot(put), mu = __ballot(unit_want), mq = QSEP ? __ballot(queue) : 0ull;
  if (lane == 0) { s_p[b][w] = (uint32_t)__popcll(mp); s_u[b][w] = (uint32_t)__popcll(mu); if (QSEP) s_q[b][w] = (uint32_t)__popcll(mq); }
  SCLK_T(rb0);
  __syncthreads();
  SCLK_ADD(SCLK_RB1, rb0);
  SCLK_T(rb1);
  // both atomics in flight together: entries are reserved for every unit_want lane
  // until this block has seen the unit head run out (`exhausted`, thread 0's register);
  // a lane reserved an entry but denied a unit leaves a dead entry (at most one
  // iteration per block, in the frame's last passes)
  uint32_t np = 0, nu = 0, u0 = 0, pb = 0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (uint32_t k = 0; k < SHADE_WAVES; k++) { np += s_p[b][k]; nu += s_u[b][k]; }
    if (exhausted) nu = 0;
    u0 = nu ? atomicAdd(sp.head, nu) : sp.total_units;
    pb = np + nu ? atomicAdd(out_count, np + nu) : 0u;
  }
  if (threadIdx.x == 0) {
    const uint32_t ne = np + nu;
    // (an iteration without finished paths asks for nothing and learns nothing: it must
    // not mark the block exhausted, or the block's later finished paths lose their slots)
    if (nu && u0 + nu >= sp.total_units) exhausted = true;
    s_pbase[b] = pb;
    s_ubase[b] = u0;
    s_granted[b] = u0 >= sp.total_units ? 0u : min(nu, sp.total_units - u0);
    s_nput[b] = np;
    s_nent[b] = ne;
    SCLK_VMWAIT();
    SCLK_ADD(SCLK_RATOM, rb1);
  }
  __syncthreads();
  SCLK_ADD(SCLK_RB2, rb1);
  uint32_t ur = (uint32_t)__popcll(mu & lt), pr = (uint32_t)__popcll(mp & lt);
  for (uint32_t i = 0; i < w; i++) { ur += s_u[b][i]; pr += s_p[b][i]; }
  if constexpr (QSEP) {
    q_rank = (uint32_t)__popcll(mq & lt);
    q_total = 0;
#pragma unroll
    for (uint32_t k = 0; k < SHADE_WAVES; k++) {
      q_rank += k < w ? s_q[b][k] : 0u;
      q_total += s_q[b][k];
    }
  } else {
    q_rank = ur;
    q_total = 0;
#pragma unroll
    for (uint32_t k = 0; k < SHADE_WAVES; k++) q_total += s_u[b][k];
  }
  const bool has_entry = unit_want && s_nput[b] + ur < s_nent[b];
  const bool granted = unit_want && ur < s_granted[b];
  unit = granted ? s_ubase[b] + ur : 0xFFFFFFFFu;
  pos = put ? s_pbase[b] + pr : (has_entry ? s_pbase[b] + s_nput[b] + ur : 0xFFFFFFFFu);
}

// A lane whose path finished got `unit` and entry `pos` (block_reserve2): start the
// unit's path in the finished path's record slot and store it; when its sample completes
// without a ray, take further units one at a time (rare), and leave a dead entry when
// none traces.
template <int SAMPLER, bool FWD>
IZPI_DEV void refill_one(const DevScene& sc, const ShadeParams& sp, const WaveBuf& out, uint32_t unit, uint32_t pos,
                         PathSt& P) {
  RayRec R;
  for (;;) {
    if (start_path<SAMPLER, FWD>(sc, sp, unit, P, R)) {
      store_entry<SAMPLER, FWD>(out, pos, P, R);
      return;
    }
    unit = atomicAdd(sp.head, 1u);
    if (unit >= sp.total_units) {
      dead_entry(out, pos);
      return;
    }
  }
}




// One shading pass of `slot` (its ray was traced): Colour.Sample / SampleSpectral
// one bounce deep (colour.go:33-65, sampler/spectral.go:47-80). Sets `push` when the path
// has a ray to trace next and `done` when its sample finished.
// Entry i of `in`: P is its path state (load_path), with blk set to the path's overflow
// block when it needs one (P.depth >= rec_dense); `kind` its kind word. On return, P and
// R hold the continuing path and its next ray (`push`), or `done` is set and `fblk` is
// the block to free. DEFER: a finished path is not unwound here (`queued`; Colour: only
// one whose unwinding reads records, finish_reads); R.o holds its terminal radiance
// (Spectral: R.o[0]) for the caller's queue (fin_queue), and the caller frees its block
// after the unwinding. (Spectral queues every finished path: the test cost the Spectral
// instances up to 24 more spilled VGPRs, C5 shade 320 -> 352 ms.)
template <int SAMPLER, int MATSET, bool DEFER, bool FWD>
IZPI_DEV void shade_item(const DevScene& sc, const ShadeParams& sp, const WaveBuf& in, uint32_t i, uint32_t kind,
                         const EntryIn& E, PathSt& P, RayRec& R, bool& push, bool& done, uint32_t& fblk, uint32_t& c_lt,
                         uint32_t& c_ls, bool& queued) {
  const bool COLOUR = SAMPLER == IZPI_SAMPLER_COLOUR;
  const bool st = sp.staged != 0;  // the scene's small tables are in this block's LDS
  SCLK_T(sc0);
  SCLK_VMWAIT();
  SCLK_ADD(SCLK_ENTRY, sc0);
  for (int k = 0; k < 3; k++) { R.o[k] = E.ray.o[k]; R.d[k] = E.ray.d[k]; }
  R.kind = kind;
  R.time = E.time;  // NewRay(hr.P, dir, r.Time()): the next ray keeps the time
  HitOut H;
  H.t = E.hit.x; H.prim = (int32_t)__double2loint(E.hit.y); H.pad = 0; H.u = 0; H.v = 0;  // (u, v) read on demand
  Lcg rng;
  rng.s = P.rng;
  const V3 ro = mk(R.o[0], R.o[1], R.o[2]), rd = mk(R.d[0], R.d[1], R.d[2]);
  V3 L = mk(0, 0, 0);
  bool terminal = false;
  bool spec = false, have_pdf = false, zero_spdf = false;
  V3 att = mk(0, 0, 0), next_o = mk(0, 0, 0), next_d = mk(0, 0, 0);
  V3 hit_n = mk(0, 0, 0);
  uint32_t rec_mat = 0;
  Onb cos_onb;
  if (ms_has(MATSET, MS_DIEL) && kind_of(R.kind) == RAY_PATHLEN) {
    // calculatePathLength result (dielectric.go:135-152) -> finish the glass bounce
    const PathCold& pc = in.cold[i];
    const V3 hp = mk(pc.pend[0], pc.pend[1], pc.pend[2]);
    const double len = H.prim >= 0 ? path_length(hp, add(ro, smul(rd, H.t))) : 10.0;  // no exit: dielectric.go:152
    const uint32_t mat_id = R.kind >> KIND_MAT_SHIFT;  // dielectric material stashed by the glass bounce
    const izpi_material gm_ = mat_rec(sc, st, mat_id);
    if (COLOUR) att = mk(gm::exp(-gm_.rgb[0] * len), gm::exp(-gm_.rgb[1] * len), gm::exp(-gm_.rgb[2] * len));
    else att.x = gm_.absorb_tex >= 0 ? gm::exp(-tex_spectral(sc, gm_.absorb_tex, P.lambda, 0.0, 0.0, st) * len) : 1.0;
    spec = true;
    next_o = hp;
    next_d = rd;
  } else if (H.prim < 0) {
    L = COLOUR ? mk(sp.background[0], sp.background[1], sp.background[2])
               : mk(bg_value(sp, P.lambda), 0, 0);
    terminal = true;
  } else {
    const bool pst = sp.prims_staged != 0;
    const GShade gs = gshade_of(sc, pst, H.prim);
    HitRec h;
    hit_record(sc, H, in.huv ? in.huv + (size_t)i * in.hs : nullptr, gs, ro, rd, R.time, (gs_cflags(gs) & 2u) != 0, h, st, ms_has(MATSET, MS_PBR), pst);
    hit_n = h.n;
    rec_mat = h.mat;
    next_o = h.p;
    // the shade record carries the material kind and, for a constant RGB texture, its
    // value: the common Lambert/light hit reads no material or texture record
    const izpi_material m = mat_rec(sc, st, h.mat);
    const bool cconst = COLOUR && (gs_cflags(gs) & 1u) != 0;
    V3 cval = mk(0, 0, 0);
    if (cconst) { const double4 c4 = mat_const_of(sp, h.mat); cval = mk(c4.x, c4.y, c4.z); }
    switch (gs_kind(gs)) {
      case IZPI_MAT_DIFFUSE_LIGHT: {  // no scatter: return emitted (diffuselight.go:49-63)
        if (dot(h.n, rd) < 0.0) {
          if (cconst) L = cval;
          else if (COLOUR) L = tex_rgb(sc, m.albedo_tex, h.u, h.v, st);
          else L.x = tex_spectral(sc, m.spectral_tex, P.lambda, h.u, h.v, st);
        }
        terminal = true;
        break;
      }
      case IZPI_MAT_LAMBERT: {  // lambertian.go:44-70: 2 draws for a ray the sampler discards (A6)
        rng.next();
        rng.next();
        cos_onb.build(h.n);
        if (cconst) att = cval;
        else if (COLOUR) att = tex_rgb(sc, m.albedo_tex, h.u, h.v, st);
        else att.x = tex_spectral(sc, m.spectral_tex, P.lambda, h.u, h.v, st);
        have_pdf = true;
        break;
      }
      case IZPI_MAT_ISOTROPIC: {  // isotropic.go:32-60: a randomInUnitSphere ray the sampler discards,
        // Cosine(N) as the material pdf of the mixture, ScatteringPDF 0; Spectral: the albedo's red
        if constexpr (!ms_has(MATSET, MS_ISO)) { atomicOr(sp.error, 2u); terminal = true; break; }
        (void)random_in_unit_sphere(rng);
        cos_onb.build(h.n);
        const V3 a = tex_rgb(sc, m.albedo_tex, h.u, h.v, st);
        if (COLOUR) att = a; else att.x = a.x;
        have_pdf = true;
        zero_spdf = true;
        break;
      }
      case IZPI_MAT_DIELECTRIC: {  // dielectric.go:156-207
        if constexpr (!ms_has(MATSET, MS_DIEL)) { atomicOr(sp.error, 2u); terminal = true; break; }
        const double ri = COLOUR ? m.ref_idx : tex_spectral(sc, m.spectral_tex, P.lambda, 0.0, 0.0, st);
        bool reflected;
        next_d = dielectric_scatter(rd, h.n, ri, rng, reflected);
        const bool beer_rgb = COLOUR && (m.flags & IZPI_MATF_BEER_LAMBERT) && !(m.rgb[0] == 0 && m.rgb[1] == 0 && m.rgb[2] == 0);
        if (!reflected && (!COLOUR || beer_rgb)) {
          // the extra World.Hit of calculatePathLength: trace it, finish next pass
          P.pend[0] = h.p.x; P.pend[1] = h.p.y; P.pend[2] = h.p.z;
          P.rng = rng.s;
          const V3 po = add(h.p, smul(next_d, 0.001));
          R.o[0] = po.x; R.o[1] = po.y; R.o[2] = po.z;
          R.d[0] = next_d.x; R.d[1] = next_d.y; R.d[2] = next_d.z;
          R.kind = RAY_PATHLEN | (h.mat << KIND_MAT_SHIFT);
          push = true;
          break;
        }
        att = mk(1.0, 1.0, 1.0);
        spec = true;
        break;
      }
      case IZPI_MAT_METAL: {  // metal.go:34-41 (RGB only: SpectralScatter is nonSpectral)
        if constexpr (!ms_has(MATSET, MS_METAL)) { atomicOr(sp.error, 2u); terminal = true; break; }
        if (!COLOUR) { terminal = true; break; }
        V3 reflected = reflect(unit(rd), h.n);
        next_d = add(reflected, smul(random_in_unit_sphere(rng), m.fuzz));
        att = mk(m.rgb[0], m.rgb[1], m.rgb[2]);
        spec = true;
        break;
      }
      case IZPI_MAT_PBR: {  // pbr.go:59-155 / 158-263
        if constexpr (!ms_has(MATSET, MS_PBR)) { atomicOr(sp.error, 2u); terminal = true; break; }
        // the four texture slots (LDS, or one 64-B record); every lookup below is issued
        // before the first of them is used
        SCLK_T(sct);
        const TexSlot s_alb = mat_slot(sc, st, h.mat, 0), s_nrm = mat_slot(sc, st, h.mat, 1),
                      s_rgh = mat_slot(sc, st, h.mat, 2), s_met = mat_slot(sc, st, h.mat, 3);
        // one texel index for the images of the normal map's size (C4: all four)
        const uint32_t w0 = s_nrm.w, h0 = s_nrm.hf & 0x3FFFFFFFu;
        const uint64_t k0 = (s_nrm.hf >> 30) <= TEXF_GRAY ? image_index(w0, h0, h.u, h.v) : 0;
        double alb_s = 0;
        if (COLOUR) att = slot_rgb_k(sc, s_alb, h.u, h.v, st, w0, h0, k0);
        else if (m.spectral_tex >= 0) alb_s = tex_spectral(sc, m.spectral_tex, P.lambda, h.u, h.v, st);
        else { V3 c = slot_rgb_k(sc, s_alb, h.u, h.v, st, w0, h0, k0); alb_s = 0.299 * c.x + 0.587 * c.y + 0.114 * c.z; }
        V3 rough = slot_set(s_rgh) ? slot_rgb_k(sc, s_rgh, h.u, h.v, st, w0, h0, k0) : mk(0.5, 0.5, 0.5);
        V3 metal = slot_set(s_met) ? slot_rgb_k(sc, s_met, h.u, h.v, st, w0, h0, k0) : mk(0.0, 0.0, 0.0);
        const bool has_nmap = slot_set(s_nrm);
        const V3 nuv = has_nmap ? slot_rgb_k(sc, s_nrm, h.u, h.v, st, w0, h0, k0) : mk(0, 0, 0);  // one texel for both uses
        SCLK_VMWAIT();
        SCLK_ADD(SCLK_TEX, sct);
        if (has_nmap && IZPI_PRIM_KIND(gs.ref) == IZPI_PRIM_TRIANGLE) {
          h.n = nmap_tbn(sc, H.prim, h.n, nuv, pst);  // the hit record's normal (triangle.go:250-264)
          hit_n = h.n;
        }
        V3 normal = h.n;
        if (has_nmap) {
          V3 tn = mk(2.0 * nuv.x - 1.0, 2.0 * nuv.y - 1.0, nuv.z);
          V3 nn0 = h.n;
          V3 t = cross(nn0, mk(0, 1, 0));
          if (dot(t, t) < 0.001) t = cross(nn0, mk(1, 0, 0));
          t = sdiv(t, length(t));
          V3 b = cross(nn0, t);
          b = sdiv(b, length(b));
          V3 nn = mk(t.x * tn.x + b.x * tn.y + nn0.x * tn.z, t.y * tn.x + b.y * tn.y + nn0.y * tn.z,
                     t.z * tn.x + b.z * tn.y + nn0.z * tn.z);
          normal = sdiv(nn, length(nn));
        }
        double rv = (rough.x + rough.y + rough.z) / 3.0;
        double mv = (metal.x + metal.y + metal.z) / 3.0;
        cos_onb.build(normal);  // the scatter's ONB and the sampler's Cosine(normal) pdf: one build (onb.go:38-67)
        const Onb& uvw = cos_onb;
        const V3 urd = unit(rd);  // (one evaluation for both uses)
        V3 reflected = reflect(urd, normal);
        double cosTheta = gm::abs(dot(urd, normal));
        double fresnel = 0.04 + (1.0 - 0.04) * gm::pow(1.0 - cosTheta, 5.0);
        fresnel = fresnel + (mv * 0.5);
        double sprob = fresnel * (1.0 - rv);
        if (rng.next() < sprob) {
          double rf = gm::max(0.01, rv * 0.3);
          V3 rdir = random_in_unit_sphere(rng);
          next_d = unit(add(reflected, smul(rdir, rf)));
          spec = true;
        } else {
          next_d = unit(uvw.local(random_cosine_direction(rng)));
          spec = false;
          have_pdf = true;  // the sampler ignores this ray and samples the mixture pdf
        }
        if (!COLOUR) att.x = spec ? alb_s * 1.5 : alb_s;
        break;
      }
      default: {
        atomicOr(sp.error, 2u);
        terminal = true;
      }
    }
  }
  SCLK_ADD(SCLK_MAT, sc0);
  if (!push) {
    if (terminal) {
      SCLK_T(sc1);
      if constexpr (FWD) finish_fwd<SAMPLER>(sp, P, L);
      else if constexpr (DEFER && !COLOUR) { R.o[0] = L.x; R.o[1] = L.y; R.o[2] = L.z; }
      else if (DEFER && finish_reads<SAMPLER, MATSET>(P, L)) { R.o[0] = L.x; R.o[1] = L.y; R.o[2] = L.z; queued = true; }
      else finish<SAMPLER, MATSET>(sp, P, L);
      SCLK_ADD(SCLK_FIN, sc1);
      done = true;
      fblk = P.blk;
    } else {
      SCLK_T(sc2);
      if (have_pdf) {
        // Mixture(Hitable(lights, P), Cosine(N)) (colour.go:48-51, mixture.go:17-33)
        V3 dir;
        if (rng.next() < 0.5) dir = lights_random(sc, st, next_o, rng);
        else dir = cos_onb.local(random_cosine_direction(rng));
        // (evaluated in an order that frees the ONB, normal and attenuation before
        // the light-pdf loop; every value is computed exactly as in the reference)
        const V3 ud = unit(dir);
        const double cosv = dot(ud, cos_onb.w);
        const double cos_pdf = cosv > 0 ? cosv / 3.141592653589793 : 0;
        double sc_cos = dot(hit_n, ud);  // ScatteringPDF with the hit normal
        if (sc_cos < 0) sc_cos = 0;
        const double spdf = zero_spdf ? 0.0 : sc_cos / 3.141592653589793;  // Isotropic.ScatteringPDF is 0
        if constexpr (FWD) {  // T * att now (frees T and att during the light-pdf loop), * (s / p) after it
          P.thr[0] = P.thr[0] * att.x;
          if (COLOUR) { P.thr[1] = P.thr[1] * att.y; P.thr[2] = P.thr[2] * att.z; }
        } else {
          rec_store<SAMPLER, MATSET>(sp, P.rslot, P.blk, P.depth, false, att, spdf, rec_mat);
        }
        SCLK_T(sc3);
        const double pdf_val = 0.5 * lights_pdf(sc, st, next_o, dir, c_lt, c_ls) + 0.5 * cos_pdf;
        SCLK_ADD(SCLK_LPDF, sc3);
        if constexpr (FWD) {
          const double w = spdf / pdf_val;
          P.thr[0] = P.thr[0] * w;
          if (COLOUR) { P.thr[1] = P.thr[1] * w; P.thr[2] = P.thr[2] * w; }
        } else {
          sst(rec_ptr<SAMPLER, MATSET>(sp, P.rslot, P.blk, P.depth) + RecLayout<SAMPLER, MATSET>::P, pdf_val);
          if constexpr (ms_spec(MATSET) || SAMPLER == IZPI_SAMPLER_SPECTRAL) rec_zero_track<SAMPLER>(P.zf, false, att, spdf, pdf_val);
        }
        next_d = dir;
      } else if constexpr (FWD) {
        P.thr[0] = P.thr[0] * att.x;
        if (COLOUR) { P.thr[1] = P.thr[1] * att.y; P.thr[2] = P.thr[2] * att.z; }
      } else {
        rec_store<SAMPLER, MATSET>(sp, P.rslot, P.blk, P.depth, true, att, 0, rec_mat);
        rec_zero_track<SAMPLER>(P.zf, true, att, 0.0, 0.0);
      }
      SCLK_ADD(SCLK_MIX, sc2);
      P.depth++;
      P.rng = rng.s;
      if (P.depth >= sp.max_depth) {
        const V3 Lt = terminal_max_depth(sp, P, COLOUR);
        if constexpr (FWD) finish_fwd<SAMPLER>(sp, P, Lt);
        else if constexpr (DEFER && !COLOUR) { R.o[0] = Lt.x; R.o[1] = Lt.y; R.o[2] = Lt.z; }
        else if (DEFER && finish_reads<SAMPLER, MATSET>(P, Lt)) { R.o[0] = Lt.x; R.o[1] = Lt.y; R.o[2] = Lt.z; queued = true; }
        else finish<SAMPLER, MATSET>(sp, P, Lt);
        done = true;
        fblk = P.blk;
      } else {
        R.o[0] = next_o.x; R.o[1] = next_o.y; R.o[2] = next_o.z;
        R.d[0] = next_d.x; R.d[1] = next_d.y; R.d[2] = next_d.z;
        R.kind = RAY_MAIN;
        push = true;
      }
    }
  }
}

// ---- overflow record blocks
// POOL_SHARDS rings of free block ids. A ring holds its own blocks only: block b belongs
// to ring b >> pool_shift, and a freed block goes back to its ring, so no ring ever holds
// more than its 1 << pool_shift entries. Each ring is a FIFO between an allocation head
// and a free tail (64-bit counters, index = counter & (ring size - 1)). Allocations take
// from the head but only below the PUBLISHED tail, which k_trace2 advances once per pass
// (kernel boundaries order the frees' ring writes before the next pass's reads). A wave
// allocates from its own ring; an allocation that finds no published block there parks
// its slot for one pass (PARK_BIT). Paths that hold a block never wait, so parked slots
// always get one back.
IZPI_DEV unsigned long long* pool_ring_ctr(const ShadeParams& sp, uint32_t r) {
  return sp.pool_ctr + (size_t)r * POOL_CTR_STRIDE;
}
// Wave-aggregated allocation for the lanes with `need`: returns 1 + block, or 0 (`need`
// lanes with 0 are parked).
IZPI_DEV uint32_t pool_alloc(const ShadeParams& sp, bool need) {
  const uint64_t m = __ballot(need);
  if (m == 0) return 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t ring = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (POOL_SHARDS - 1);
  unsigned long long* c = pool_ring_ctr(sp, ring);
  const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1;
  unsigned long long base = 0, pub = 0;
  if (lane == leader) {
    base = atomicAdd(c, (unsigned long long)__popcll(m));
    pub = __atomic_load_n(c + 2, __ATOMIC_RELAXED);
  }
  base = __shfl(base, (int)leader);
  pub = __shfl(pub, (int)leader);
  const unsigned long long idx = base + (unsigned long long)__popcll(m & ((1ull << lane) - 1));
  const uint32_t size_mask = (1u << sp.pool_shift) - 1u;
  return (need && idx < pub) ? sp.pool_ring[((size_t)ring << sp.pool_shift) + (idx & size_mask)] + 1u : 0u;
}
// Return a lane's block (1 + block, 0 = none) to its ring.
IZPI_DEV void pool_free_one(const ShadeParams& sp, uint32_t fblk) {
  const uint32_t b = fblk - 1u, ring = b >> sp.pool_shift, size_mask = (1u << sp.pool_shift) - 1u;
  const unsigned long long pos = atomicAdd(pool_ring_ctr(sp, ring) + 1, 1ull);
  sp.pool_ring[((size_t)ring << sp.pool_shift) + (pos & size_mask)] = b;
}
// Single-lane allocation that tries every ring (k_tail: cannot park), or 0.
IZPI_DEV uint32_t pool_alloc_any(const ShadeParams& sp, uint32_t first) {
  const uint32_t size_mask = (1u << sp.pool_shift) - 1u;
  for (uint32_t k = 0; k < POOL_SHARDS; k++) {
    const uint32_t ring = (first + k) & (POOL_SHARDS - 1);
    unsigned long long* c = pool_ring_ctr(sp, ring);
    if (__atomic_load_n(c, __ATOMIC_RELAXED) >= __atomic_load_n(c + 2, __ATOMIC_RELAXED)) continue;  // exhausted
    const unsigned long long idx = atomicAdd(c, 1ull);
    if (idx < __atomic_load_n(c + 2, __ATOMIC_RELAXED)) return sp.pool_ring[((size_t)ring << sp.pool_shift) + (idx & size_mask)] + 1u;
  }
  return 0u;
}

// Deferred unwinding. A path that ends in a shading pass is unwound (finish) from its
// records, depth - 1 down to 0; done in the finishing lane itself, a wave waits for its
// deepest finishing lane while its other lanes idle (C5: finish took 48% of k_shade's
// wave cycles with a few lanes of a wave finishing per iteration). Instead the finishing
// lane queues a job in its block's queue, and the block unwinds the queued jobs with every
// lane busy once FINQ_FLUSH are queued (and at the end of the launch). The records stay
// put until then: the slot's next path writes its first record in the NEXT pass, after
// its first ray is traced, and the finished path's overflow block is freed by fin_flush.
// A job: unit | rslot << 32, blk | (depth | zf << 16) << 32, then the terminal radiance
// (Colour) or L.x, lambda, lpdf (Spectral), word-major (word k of job j at k * FINQ_CAP + j).
template <int SAMPLER>
IZPI_DEV void fin_queue(unsigned long long* q, uint32_t j, const PathSt& P, const RayRec& R) {
  const bool colour = SAMPLER == IZPI_SAMPLER_COLOUR;
  q[j] = P.unit | (unsigned long long)P.rslot << 32;
  q[FINQ_CAP + j] = P.blk | (unsigned long long)(P.depth | P.zf << 16) << 32;
  q[2 * FINQ_CAP + j] = (unsigned long long)__double_as_longlong(R.o[0]);
  q[3 * FINQ_CAP + j] = (unsigned long long)__double_as_longlong(colour ? R.o[1] : P.lambda);
  q[4 * FINQ_CAP + j] = (unsigned long long)__double_as_longlong(colour ? R.o[2] : P.lpdf);
}
template <int SAMPLER, int MATSET>
IZPI_DEV void fin_flush(const ShadeParams& sp, const unsigned long long* q, uint32_t n) {
  const bool colour = SAMPLER == IZPI_SAMPLER_COLOUR;
  for (uint32_t j = threadIdx.x; j < n; j += SHADE_THREADS) {
    PathSt P;
    const unsigned long long w0 = q[j], w1 = q[FINQ_CAP + j];
    P.unit = (uint32_t)w0; P.rslot = (uint32_t)(w0 >> 32);
    P.blk = (uint32_t)w1; P.depth = (uint32_t)(w1 >> 32) & 0xFFFFu; P.zf = (uint32_t)(w1 >> 48);
    const double a = __longlong_as_double((long long)q[2 * FINQ_CAP + j]);
    const double b = __longlong_as_double((long long)q[3 * FINQ_CAP + j]);
    const double c = __longlong_as_double((long long)q[4 * FINQ_CAP + j]);
    P.lambda = colour ? 0.0 : b; P.lpdf = colour ? 0.0 : c;
    finish<SAMPLER, MATSET>(sp, P, colour ? mk(a, b, c) : mk(a, 0.0, 0.0));
    if (sp.rec_pool && P.blk) pool_free_one(sp, P.blk);
  }
}
// Which k_shade instances defer: 1 = the Spectral ones and the Colour ones with specular
// materials (C5 at 32 spp: shading 377 -> 320 ms; C4, queueing only the unwindings that
// read records: 464.7 -> 453.7 ms), not C1-C3's Lambert-only instances (C3 +3.4% even
// with only the record-reading unwindings queued: they are short, and the queue costs
// stores), 2 = all, 0 = none. Handing each wave's lanes jobs of similar depth (a counting
// sort of a flush's jobs by depth) measured slower: C5 338 ms, C4 +1.4%.

// One shading pass over the slots traced in the previous k_trace.
// k_shade's register budget: 3 waves per SIMD (168 VGPRs). MATSET_BASIC colour at 4 waves spilled
// 47 VGPRs and measured 1% slower; the spectral / MATSET_FULL instances ran C5 7% faster at 3
// waves than at 2 despite ~100 B/lane of spill. The forward instances (153-168 VGPRs, no
// spill) at 4 waves spill 24-71 VGPRs: C2 +1.5%, C3 +0.3%, C4 +2.7%, C5 (256 spp) +23%
// (profiles/r6m).
constexpr int SHADE_WPE = 3;
// Forward mode: a finished path frees its entry and starts nothing; k_refill starts the new
// units after the pass (see there). The recursion's new paths take over the finished
// paths' record slots, here.
template <int SAMPLER, int MATSET, bool FWD>
__global__ void __launch_bounds__(SHADE_THREADS) __attribute__((amdgpu_waves_per_eu(SHADE_WPE)))
k_shade(const DevScene sc, const ShadeParams sp, const WaveParams wp) {
  constexpr bool DREF = FWD;
  shade_stage(sc, sp);
  uint32_t parity = 0;  // block_reserve2 LDS buffer set
  const uint32_t n = *wp.in_count;
  // (forward mode) `in`'s camera entries: their path state is computed, not loaded
  const uint32_t cam_b = FWD && wp.cam ? wp.cam[0] : 0u, cam_u = FWD && wp.cam ? wp.cam[1] : 0u,
                 cam_m = FWD && wp.cam ? wp.cam[2] : 0u;
  // this pass's k_trace2 is done with its dequeue cursor: reset it for the next pass's
  if (blockIdx.x == 0 && threadIdx.x == 0) *wp.trace_next = 0;
  bool exhausted = false;  // (thread 0) this block has seen the unit head run out
  uint32_t c_lt = 0, c_ls = 0, c_park = 0;
  const uint32_t stride = gridDim.x * SHADE_THREADS;
  constexpr bool DEFER = !FWD && (SAMPLER == IZPI_SAMPLER_SPECTRAL || ms_spec(MATSET));
  constexpr bool COLOUR_DEFER = DEFER && SAMPLER == IZPI_SAMPLER_COLOUR;  // a subset of the finished paths is queued
  unsigned long long* fq = sp.finq + (size_t)blockIdx.x * FINQ_WORDS * FINQ_CAP;
  uint32_t fq_n = 0;  // jobs in this block's queue (the same in every thread)
#ifdef IZPI_SHADE_CLOCKS
  uint64_t k_item = 0, k_ref = 0, k_push = 0;
  sclk_zero();
#endif
  // Block-uniform trip count: the unit and queue reservations are block-wide.
  for (uint32_t base = blockIdx.x * SHADE_THREADS; base < n; base += stride) {
    const uint32_t i = base + threadIdx.x;
    const bool valid = i < n;
    bool push = false;      // the path has a ray to trace next (P, R)
    bool done = false;      // its sample finished: start a new unit in its record slot
    bool parked = false;
    uint32_t fblk = 0;
#ifdef IZPI_SHADE_CLOCKS
    uint64_t t0 = __builtin_readcyclecounter();
#endif
    PathSt P;
    RayRec R;
    P.rslot = 0; P.blk = 0; P.depth = 0; P.zf = 0;
    uint32_t kind = RAY_DEAD;
    EntryIn E;
    if (valid) {
      // the kind word, path state, ray and hit record in one round of loads (a dead entry's
      // path and hit are read too, and ignored): waiting for the kind word first, then the
      // path, then the ray put three memory round trips in front of every item
      kind = sld(wp.in.kind + i) & ~(uint32_t)RAY_PARKED;  // a parked entry retries its pass
      if (FWD && i - cam_b < cam_m) camera_path<SAMPLER>(sp, cam_u + (i - cam_b), P);
      else load_path<SAMPLER, FWD>(wp.in, i, P);
      load_entry(wp.in, i, E);
    }
    const bool live = valid && !(kind & RAY_DEAD);
    if (sp.rec_pool) {  // a path at depth >= rec_dense writes its records to an overflow block
      const bool need = live && P.depth >= sp.rec_dense && P.blk == 0;
      const uint32_t b = pool_alloc(sp, need);
      P.blk = need ? b : P.blk;
      parked = need && b == 0;
      c_park += parked ? 1u : 0u;
    }
    bool queued = false;    // (DEFER) its unwinding waits in the block's queue
    if (live && !parked) shade_item<SAMPLER, MATSET, DEFER, FWD>(sc, sp, wp.in, i, kind, E, P, R, push, done, fblk, c_lt, c_ls, queued);
    if (SAMPLER == IZPI_SAMPLER_SPECTRAL) queued = DEFER && done;  // (every finished path)
    // a queued path's overflow block is freed after its unwinding (fin_flush)
    if ((COLOUR_DEFER ? !queued : !DEFER) && sp.rec_pool && fblk) pool_free_one(sp, fblk);
#ifdef IZPI_SHADE_CLOCKS
    uint64_t t1 = __builtin_readcyclecounter();
    k_item += t1 - t0;
    t0 = t1;
#endif
    // one reservation phase: output entries for continuing and parked paths, new units
    // (and their entries) for finished ones
    uint32_t unit, pos, frank, ftotal;
    block_reserve2<COLOUR_DEFER>(sp, wp.out_count, push || parked, done && !DREF, unit, pos, parity, exhausted, queued, frank,
                                 ftotal);
    if (queued) fin_queue<SAMPLER>(fq, fq_n + frank, P, R);  // (before refill_one reuses P)
    fq_n += ftotal;
    if (push) store_entry<SAMPLER, FWD>(wp.out, pos, P, R);
    if (parked) copy_entry(wp.in, i, wp.out, pos);
#ifdef IZPI_SHADE_CLOCKS
    t1 = __builtin_readcyclecounter();
    k_push += t1 - t0;
    t0 = t1;
#endif
    if constexpr (!DREF) {
      if (unit != 0xFFFFFFFFu) refill_one<SAMPLER, FWD>(sc, sp, wp.out, unit, pos, P);
      else if (done && pos != 0xFFFFFFFFu) dead_entry(wp.out, pos);  // entry reserved, the units ran out
    }
#ifdef IZPI_SHADE_CLOCKS
    t1 = __builtin_readcyclecounter();
    k_ref += t1 - t0;
#endif
    if (DEFER && fq_n >= FINQ_FLUSH) {  // (block-uniform; the next iteration's jobs wait for its reservation's barriers)
      __syncthreads();
      fin_flush<SAMPLER, MATSET>(sp, fq, fq_n);
      fq_n = 0;
    }
  }
  if (DEFER && fq_n) {
    __syncthreads();
    fin_flush<SAMPLER, MATSET>(sp, fq, fq_n);
  }
  const uint32_t lane = threadIdx.x & 63;
#ifdef IZPI_SHADE_CLOCKS
  if (lane == 0) {
    atomicAdd(sp.counters + CNT_SCLK_ITEM, (unsigned long long)k_item);
    atomicAdd(sp.counters + CNT_SCLK_REFILL, (unsigned long long)k_ref);
    atomicAdd(sp.counters + CNT_SCLK_PUSH, (unsigned long long)k_push);
  }
  sclk_flush(sp.counters);
#endif
  if (c_park && wp.out_park) *wp.out_park = 1u;  // the next k_trace2 must read kind words
  unsigned long long vals[3] = {c_lt, c_ls, c_park};
  const int idx[3] = {CNT_LTRI, CNT_LSPH, CNT_PARK};
  for (int k = 0; k < 3; k++) {
    unsigned long long s = vals[k];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
    if (lane == 0) count_add(sp.cpart, sp.counters, idx[k], s);
  }
}

// Forward mode's refill (k_shade<..., FWD = true>): after a shading pass, the entries its
// finished paths freed take the next units, as one run of camera rays appended behind the
// continuing paths. k_refill_plan (one thread) reads the pass's continuing entries and the
// unit head and hands out min(free entries, units left); k_refill starts unit head + j in
// entry continuing + j (a start whose sample completes without a ray, spectral pdf 0,
// leaves a dead entry, which the next pass drops). Starting the paths in k_shade, in the
// lanes whose path had finished, ran the start's code on a few lanes of each wave: 1-7%
// slower frames (C3 238.3 vs 236.1 ms, C4 at 256 spp 138.4 vs 131.1 ms, C5 at 256 spp
// 4507 vs 4180 ms; profiles/r6l).
// The new entries start on a multiple of REFILL_ALIGN entries, the gap before them dead:
// an unaligned start split a line of every state array between two k_refill blocks at each
// 256-entry boundary (C3 235.4 -> 233.3 ms per frame aligned, the same at 16 or 64;
// `profiles/r6t/`). Starting 4 or 8 units per thread and iteration with their tile loads
// issued together measured the same as one (`profiles/r6s/`).
constexpr uint32_t REFILL_ALIGN = 64;
// Forward mode's first fill of a chunk: entry j takes unit j, a camera entry (k_refill)
static __global__ void k_plan_first(uint32_t* out_count, uint32_t* plan, uint32_t fill) {
  plan[0] = 0; plan[1] = 0; plan[2] = fill; plan[3] = 0;
  *out_count = fill;
}
static __global__ void k_refill_plan(const ShadeParams sp, uint32_t* out_count, uint32_t* plan) {
  const uint32_t nc = *out_count, h = *sp.head;
  // the new entries start on a REFILL_ALIGN boundary; the gap holds dead entries
  const uint32_t base = min((nc + (REFILL_ALIGN - 1)) / REFILL_ALIGN * REFILL_ALIGN, sp.slots);
  const uint32_t room = sp.slots - base;
  const uint32_t m = h < sp.total_units ? min(room, sp.total_units - h) : 0u;
  plan[0] = m ? base : nc; plan[1] = h; plan[2] = m; plan[3] = nc;
  *out_count = m ? base + m : nc;
  *sp.head = h + m;
}
template <int SAMPLER>
__global__ void __launch_bounds__(256) k_refill(const DevScene sc, const ShadeParams sp_in, const WaveParams wp, const uint32_t* plan) {
  ShadeParams sp = sp_in;
  sp.staged = 0;  // (no tables staged, as k_start)
  sp.prims_staged = 0;
  const uint32_t nc = plan[0], u0 = plan[1], m = plan[2], gap0 = plan[3];
  if (blockIdx.x == 0 && gap0 + threadIdx.x < nc) dead_entry(wp.out, gap0 + threadIdx.x);  // (the gap: < 256 entries)
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < m; j += gridDim.x * 256) {
    PathSt P;
    RayRec R;
    P.rslot = 0;  // (forward mode: no records)
    if (start_path<SAMPLER, true>(sc, sp, u0 + j, P, R)) store_camera_entry(wp.out, nc + j, R);  // (camera_path)
    else dead_entry(wp.out, nc + j);
  }
}

// The wavefront's tail. Once every work unit has started and few paths remain, the
// pass-synchronous loop pays, per pass, the latency of that pass's longest traversal.
// k_tail instead runs each remaining path to its end in one lane: trace, shade, trace...
// (no refill: the unit head is exhausted), so the passes of different paths overlap.
// Same per-ray code paths, results and counters as k_trace + k_shade.
template <int SAMPLER, int MATSET, int STACK, bool FWD>
__global__ void __launch_bounds__(256) k_tail(const DevScene sc, const ShadeParams sp, const WaveParams wp, int32_t* spill) {
  shade_stage(sc, sp);
  __shared__ int32_t lds_stack[std::min(STACK, TAIL_LDS_STACK) * 256];
  int32_t* stk = lds_stack + threadIdx.x;
  const uint32_t gstride = gridDim.x * 256;
  int32_t* gsp = spill + blockIdx.x * 256 + threadIdx.x;
  const uint32_t n = *wp.in_count;
  const uint32_t cam_b = FWD && wp.cam ? wp.cam[0] : 0u, cam_u = FWD && wp.cam ? wp.cam[1] : 0u,
                 cam_m = FWD && wp.cam ? wp.cam[2] : 0u;
  uint32_t c_rays = 0, c_nodes = 0, c_tri = 0, c_sph = 0, c_lt = 0, c_ls = 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    // entry i runs to its end in this lane; its next ray goes back to entry i
    if (wp.in.kind[i] & RAY_DEAD) continue;
    bool traced = (wp.in.kind[i] & RAY_PARKED) != 0;  // a parked entry's ray is already traced
    bool cam = FWD && i - cam_b < cam_m;  // (forward mode) a camera entry's path state is computed once
    for (;;) {
      if (!traced) trace_one<STACK>(sc, wp.in, i, stk, gsp, gstride, c_rays, c_nodes, c_tri, c_sph, sp.error);
      traced = false;
      PathSt P;
      RayRec R;
      if (cam) camera_path<SAMPLER>(sp, cam_u + (i - cam_b), P);
      else load_path<SAMPLER, FWD>(wp.in, i, P);
      cam = false;  // (its next state is stored below)
      const uint32_t kind = wp.in.kind[i] & ~(uint32_t)RAY_PARKED;
      if (sp.rec_pool && P.depth >= sp.rec_dense && P.blk == 0) {
        // The host launches k_tail with at most pool blocks paths, all of the free
        // blocks published, so this cannot fail (guarded anyway: no spin on a bug).
        P.blk = pool_alloc_any(sp, blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
        if (P.blk == 0) { atomicOr(sp.error, 4u); break; }
      }
      bool push = false, done = false;
      uint32_t fblk = 0;
      EntryIn E;
      load_entry(wp.in, i, E);
      bool queued = false;  // (k_tail unwinds in place)
      shade_item<SAMPLER, MATSET, false, FWD>(sc, sp, wp.in, i, kind, E, P, R, push, done, fblk, c_lt, c_ls, queued);
      if (fblk) pool_free_one(sp, fblk);
      if (!push) break;
      store_entry<SAMPLER, FWD>(wp.in, i, P, R);
    }
  }
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long vals[9] = {c_rays, c_nodes, c_tri, c_sph, c_lt, c_ls, c_nodes, c_tri, c_sph};
  const int idx[9] = {CNT_RAYS, CNT_NODES, CNT_TRI, CNT_SPH, CNT_LTRI, CNT_LSPH, CNT_TAIL_NODES, CNT_TAIL_TRI, CNT_TAIL_SPH};
#pragma unroll
  for (int k = 0; k < 9; k++) {
    unsigned long long v = vals[k];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if (lane == 0) count_add(sp.cpart, sp.counters, idx[k], v);
  }
}


// Publish the frees of the last shading pass (k_trace2 does it at its start; k_tail and
// the host's pool checks need it on their own).
static __global__ void k_pool_publish(unsigned long long* ctr) { pool_publish(ctr); }
// Every ring holds all of its blocks at the start of a render.
static __global__ void k_pool_init(uint32_t* ring, uint32_t n, uint32_t per_ring, unsigned long long* ctr) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) ring[i] = i;
  if (i < POOL_SHARDS) {
    unsigned long long* c = ctr + (size_t)i * POOL_CTR_STRIDE;
    c[0] = 0; c[1] = per_ring; c[2] = per_ring;
  }
}

static __global__ void __launch_bounds__(256) k_accumulate(const AccumParams ap) {
  const uint32_t p = blockIdx.x * 256 + threadIdx.x;
  if (p >= ap.num_pixels) return;
  double c0 = ap.running[3 * (size_t)p], c1 = ap.running[3 * (size_t)p + 1], c2 = ap.running[3 * (size_t)p + 2];
  const double* s = ap.samples + (size_t)p * ap.chunk_spp * SMP_D;
  uint32_t k = 0;
  // one sample into the sums (rgb.go:36 col += ..., render/spectral.go:92-96 sum += ...);
  // a raw forward Spectral sample is weighed first
  auto add = [&](double a, double b, double c) {
    if (ap.raw_spectral) {
      double x, y, z;
      spectral_weigh(a, b, c, x, y, z);
      c0 = c0 + x; c1 = c1 + y; c2 = c2 + z;
    } else {
      c0 = c0 + a; c1 = c1 + b; c2 = c2 + c;
    }
  };
  if ( (ap.chunk_spp & 3u) == 0 && blockIdx.x * 256 + 256 <= ap.num_pixels) {
    // Staged through LDS, 4 samples (96 B) of each of the wave's 64 pixels at a time: the
    // wave's lanes load the 64 runs as consecutive 16-B pieces (a load instruction covers
    // ~11 neighbouring runs instead of one piece of 64 runs 12 KB apart), then each lane
    // adds its own pixel's 4 samples from LDS in sample order (rgb.go:36).
    __shared__ double2 st[4][64 * 6];
    double2* w = st[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t p0 = p - lane;  // the wave's first pixel
    const size_t run = (size_t)ap.chunk_spp * 3 / 2;  // double2 per pixel
    const double2* s2 = reinterpret_cast<const double2*>(ap.samples) + (size_t)p0 * run;
    for (; k < ap.chunk_spp; k += 4) {
      double2 v[6];
#pragma unroll
      for (int i = 0; i < 6; i++) {
        const uint32_t q = lane + 64 * i, j = q / 6, c = q % 6;
        v[i] = sld(s2 + (size_t)j * run + (k >> 1) * 3 + c);
      }
#pragma unroll
      for (int i = 0; i < 6; i++) w[lane + 64 * i] = v[i];
      __builtin_amdgcn_wave_barrier();
      const double2 a = w[6 * lane], b = w[6 * lane + 1], c = w[6 * lane + 2];
      const double2 d = w[6 * lane + 3], e = w[6 * lane + 4], f = w[6 * lane + 5];
      __builtin_amdgcn_wave_barrier();
      add(a.x, a.y, b.x);  // sample k
      add(b.y, c.x, c.y);  // sample k + 1
      add(d.x, d.y, e.x);  // sample k + 2
      add(e.y, f.x, f.y);  // sample k + 3
    }
  }
  if ((ap.chunk_spp & 1u) == 0 && k == 0) {
    // two samples (48 B, 16-B aligned for an even chunk_spp) per three 16-B loads: the
    // lanes' runs lie chunk_spp * 24 B apart, so every load instruction touches 64 lines
    // and the instruction count, not the bytes, bounds this loop
    const double2* s2 = reinterpret_cast<const double2*>(s);
    for (; k + 1 < ap.chunk_spp; k += 2) {  // sample order, as rgb.go:36
      const double2 a = s2[3 * (k >> 1)], b = s2[3 * (k >> 1) + 1], c = s2[3 * (k >> 1) + 2];
      add(a.x, a.y, b.x);  // sample k
      add(b.y, c.x, c.y);  // sample k + 1
    }
  }
  for (; k < ap.chunk_spp; k++) add(s[3 * k], s[3 * k + 1], s[3 * k + 2]);  // sample order, as rgb.go:36
  if (!ap.last) {
    ap.running[3 * (size_t)p] = c0; ap.running[3 * (size_t)p + 1] = c1; ap.running[3 * (size_t)p + 2] = c2;
    return;
  }
  double r0, r1, r2;
  if (ap.sampler == IZPI_SAMPLER_COLOUR) {  // vec3.ScalarDiv(col, numSamples)
    r0 = c0 / (double)ap.spp; r1 = c1 / (double)ap.spp; r2 = c2 / (double)ap.spp;
  } else {  // sum * (1/numSamples)
    const double inv = 1.0 / (double)ap.spp;
    r0 = c0 * inv; r1 = c1 * inv; r2 = c2 * inv;
  }
  const uint32_t tile_px = ap.tile_w * ap.tile_h;
  if (ap.out_layout == IZPI_OUT_PACKED) {
    double* o = ap.out + (size_t)p * 4;
    o[0] = r0; o[1] = r1; o[2] = r2; o[3] = 1.0;
    return;
  }
  const uint32_t tile = p / tile_px, in_tile = p % tile_px;
  const uint32_t x = ap.tiles[4 * tile] + in_tile % ap.tile_w;
  const uint32_t y = ap.tiles[4 * tile + 1] + in_tile / ap.tile_w;
  const uint32_t row = ap.height - y;  // canvas.Set(x, ny-y): row ny is dropped (A9)
  if (row < ap.height) {
    double* o = ap.out + ((size_t)row * ap.width + x) * 4;
    o[0] = r0; o[1] = r1; o[2] = r2; o[3] = 1.0;
  }
}


// One chunk loop of the wavefront scheme: k_start fills the slots, then k_trace2 /
// k_shade alternate until no slot has a ray left (the last few paths run to their end
// in k_tail); k_accumulate folds the chunk's per-sample radiance into the pixels in
// sample order.
template <int SAMPLER, int MATSET, bool FWD>
int run_chunks(izpi_ctx* ctx, const izpi_render_req* req, const DevScene& sc, const Tracer& tr, ShadeParams& sp,
               WaveParams& wp, AccumParams& ap, uint32_t num_pixels, uint32_t chunk, uint32_t pool_blocks,
               float* trace_ms, float* shade_ms, float* tail_ms, uint32_t* launches) {
  hipStream_t st = ctx->stream;
  const izpi_render_tuning& tu = tuning_of(req);
  int shade_res = 0;
  const size_t dyn = sc.lds_bytes;  // the staged tables' LDS arena (render_body)
  int rc = resident_blocks(ctx, k_shade<SAMPLER, MATSET, FWD>, &shade_res, (int)SHADE_THREADS, dyn);
  if (rc) return rc;
  // tail kernel: used once every unit has started and at most `tail_max` paths remain
  const bool tail_deep = ctx->stack_needed > 32;
  int tail_res = 0;
  if ((rc = tail_deep ? resident_blocks(ctx, k_tail<SAMPLER, MATSET, 64, FWD>, &tail_res, 256, dyn)
                      : resident_blocks(ctx, k_tail<SAMPLER, MATSET, 32, FWD>, &tail_res, 256, dyn))) return rc;
  if ((uint32_t)std::max({tr.blocks * 4, shade_res * (int)SHADE_WAVES, tail_res * 4}) > ctx->num_cus * CPART_BLOCKS_PER_CU * 4 ||
      (uint32_t)shade_res > ctx->num_cus * CPART_BLOCKS_PER_CU) {
    ctx->err = "grid larger than the counter rows or the unwinding queues";
    return IZPI_ERR_INVALID;
  }
  if (tail_deep && (size_t)tail_res * 256 * (64 - TAIL_LDS_STACK) * sizeof(int32_t) > ctx->spill_cap) {
    ctx->err = "k_tail's stack spill does not fit k_trace2's spill area";
    return IZPI_ERR_INVALID;
  }
  int refill_res = 0;
  if constexpr (FWD)
    if ((rc = resident_blocks(ctx, k_refill<SAMPLER>, &refill_res, 256, 0))) return rc;
  uint64_t tail_max = (uint64_t)tail_res * 256;
  if (tu.tail_paths) tail_max = tu.tail_paths;
  if (tu.flags & IZPI_TUNE_NO_TAIL) tail_max = 0;
  // k_tail's allocations cannot park: every tail path must find a published block
  if (sp.rec_pool) tail_max = std::min<uint64_t>(tail_max, pool_blocks);
  const WaveBuf q[2] = {wp.in, wp.out};  // the two sides of the state; entry counts in d_misc[3..4]
  uint32_t* qn[2] = {misc(ctx, 3), misc(ctx, 4)};
  if (sp.rec_pool)
    hipLaunchKernelGGL(k_pool_init, dim3((pool_blocks + 255) / 256), dim3(256), 0, st, sp.pool_ring, pool_blocks,
                       pool_blocks / POOL_SHARDS, sp.pool_ctr);
  HIP_TRY(hipGetLastError());
  for (uint32_t s0 = 0; s0 < req->spp; s0 += chunk) {
    const uint32_t cs = std::min(chunk, req->spp - s0);
    sp.chunk_spp = cs; sp.s0 = s0; sp.total_units = num_pixels * cs;
    const uint32_t fill = std::min<uint32_t>(sp.slots, sp.total_units);
    HIP_TRY(hipMemsetD32Async(misc(ctx, 0), (int)fill, 1, st));  // unit head: k_start gives slot i unit i
    HIP_TRY(hipMemsetAsync(misc(ctx, 2), 0, 3 * MISC_STRIDE * sizeof(uint32_t), st));  // dequeue cursor, queue counts
    HIP_TRY(hipMemsetAsync(misc(ctx, 6), 0, 2 * MISC_STRIDE * sizeof(uint32_t), st));  // park flags of the two sides
    wp.out = q[0]; wp.out_count = qn[0];
    if constexpr (FWD) {  // camera entries j = unit j (the unit head starts at `fill` above)
      hipLaunchKernelGGL(k_plan_first, dim3(1), dim3(1), 0, st, wp.out_count, misc(ctx, 5), fill);
      hipLaunchKernelGGL(k_refill<SAMPLER>, dim3(refill_res), dim3(256), 0, st, sc, sp, wp, (const uint32_t*)misc(ctx, 5));
    } else {
      hipLaunchKernelGGL((k_start<SAMPLER, FWD>), dim3((fill + 255) / 256), dim3(256), 0, st, sc, sp, wp);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(ctx->h_count, qn[0], sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (tu.flags & IZPI_TUNE_PASS_LOG) fprintf(stderr, "IZPI_T start_synced %.3f\n", diag_clock_ms());
    uint32_t n = ctx->h_count[0];
    int cur = 0;
    // Launch passes in batches without a host round-trip per pass: both kernels read
    // their queue length from device memory and exit at once when it is zero, so the
    // host only polls the queue length once per batch (overshoot costs a few empty
    // launches of ~5 us).
    // Once every unit has started, the queue only shrinks: poll after every pass, so that
    // k_tail takes over as soon as few enough paths remain instead of up to 8 passes later
    // (each of those last passes costs ~0.3-1 ms of mostly idle machine).
    const bool pass_log = (tu.flags & IZPI_TUNE_PASS_LOG) != 0;  // diagnostics: per-pass times on stderr
    int B = pass_log ? 1 : IZPI_PASS_BATCH;  // (the log reads every pass's queue length)
    while (n > 0) {
      for (int b = 0; b < B; b++) {
        wp.in = q[cur]; wp.in_count = qn[cur];
        wp.out = q[1 - cur]; wp.out_count = qn[1 - cur];
        wp.in_park = misc(ctx, 6 + cur); wp.out_park = misc(ctx, 6 + (1 - cur));
        wp.cam = FWD ? misc(ctx, 5) : nullptr;  // (k_refill_plan's plan of the pass before: `in`'s camera entries)
        // (k_trace2 zeroes out_count and out_park, k_shade the dequeue cursor for the next pass)
        HIP_TRY(hipEventRecord(ctx->evb[3 * b], st));
        launch_trace(ctx, sc, tr, wp, st, ctx->d_spill);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ctx->evb[3 * b + 1], st));
        hipLaunchKernelGGL((k_shade<SAMPLER, MATSET, FWD>), dim3(shade_res), dim3(SHADE_THREADS), dyn, st, sc, sp, wp);
        HIP_TRY(hipGetLastError());
        if constexpr (FWD) {
          hipLaunchKernelGGL(k_refill_plan, dim3(1), dim3(1), 0, st, sp, wp.out_count, misc(ctx, 5));
          hipLaunchKernelGGL(k_refill<SAMPLER>, dim3(refill_res), dim3(256), 0, st, sc, sp, wp, (const uint32_t*)misc(ctx, 5));
          HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipEventRecord(ctx->evb[3 * b + 2], st));
        cur = 1 - cur;
      }
      HIP_TRY(hipMemcpyAsync(ctx->h_count, ctx->d_misc, 8 * MISC_STRIDE * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      for (int b = 0; b < B; b++) {
        float t_ms = 0, s_ms = 0;
        HIP_TRY(hipEventElapsedTime(&t_ms, ctx->evb[3 * b], ctx->evb[3 * b + 1]));
        HIP_TRY(hipEventElapsedTime(&s_ms, ctx->evb[3 * b + 1], ctx->evb[3 * b + 2]));
        *trace_ms += t_ms;
        *shade_ms += s_ms;
        if (pass_log) fprintf(stderr, "IZPI_PASS %u trace %.3f shade %.3f\n", *launches, t_ms, s_ms);
        (*launches)++;
      }
      const uint32_t head = ctx->h_count[0];
      n = ctx->h_count[(3 + cur) * MISC_STRIDE];
      {  // units handed out minus the entries still queued: samples finished (a lower bound)
        const uint64_t started = std::min<uint64_t>(head, sp.total_units);
        ctx->prog_done.store((uint64_t)s0 * num_pixels + (started > n ? started - n : 0), std::memory_order_relaxed);
      }
      if (pass_log) fprintf(stderr, "IZPI_BATCH queue %u head %u\n", n, head);
      if (head >= sp.total_units) B = 1;
      // every unit has started: finish the remaining paths in one k_tail launch
      if (n > 0 && n <= tail_max && head >= sp.total_units) {
        wp.in = q[cur]; wp.in_count = qn[cur];
        HIP_TRY(hipEventRecord(ctx->ev2, st));
        if (sp.rec_pool) hipLaunchKernelGGL(k_pool_publish, dim3(1), dim3(256), 0, st, sp.pool_ctr);
        // (the deep instance spills stack entries past 32 into k_trace2's spill area, which
        // holds 64 entries for each of k_trace2's threads, more than k_tail has)
        if (tail_deep) hipLaunchKernelGGL((k_tail<SAMPLER, MATSET, 64, FWD>), dim3(tail_res), dim3(256), dyn, st, sc, sp, wp, ctx->d_spill);
        else hipLaunchKernelGGL((k_tail<SAMPLER, MATSET, 32, FWD>), dim3(tail_res), dim3(256), dyn, st, sc, sp, wp, ctx->d_spill);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ctx->ev3, st));
        HIP_TRY(hipEventSynchronize(ctx->ev3));
        float t_ms = 0;
        HIP_TRY(hipEventElapsedTime(&t_ms, ctx->ev2, ctx->ev3));
        *tail_ms += t_ms;
        n = 0;
      }
    }
    ap.chunk_spp = cs;
    ap.raw_spectral = FWD && SAMPLER == IZPI_SAMPLER_SPECTRAL ? 1u : 0u;
    ap.last = (s0 + cs >= req->spp) ? 1u : 0u;
    ctx->prog_done.store((uint64_t)(s0 + cs) * num_pixels, std::memory_order_relaxed);
    hipLaunchKernelGGL(k_accumulate, dim3((num_pixels + 255) / 256), dim3(256), 0, st, ap);
    HIP_TRY(hipGetLastError());
  }
  return IZPI_OK;
}


// Every chunk of the request through the wavefront passes with the shading instance of the
// scene's smallest material set (izpi_kern.h: run_sampler).
template <int SAMPLER, bool FWD>
int run_sampler(izpi_ctx* ctx, const izpi_render_req* req, const DevScene& sc, const Tracer& tr, ShadeParams& sp,
                WaveParams& wp, AccumParams& ap, uint32_t num_pixels, uint32_t chunk, uint32_t pool_blocks, bool compact,
                float* trace_ms, float* shade_ms, float* tail_ms, uint32_t* launches) {
#define IZPI_RUN(M) run_chunks<SAMPLER, M, FWD>(ctx, req, sc, tr, sp, wp, ap, num_pixels, chunk, pool_blocks, trace_ms, shade_ms, tail_ms, launches)
  const uint32_t ms = ctx->matset;
  const int set = ms == 0 ? MATSET_BASIC : (ms & ~(uint32_t)MATSET_SURF) == 0 ? MATSET_SURF : MATSET_FULL;
  // (the compact records of MATSET_CONST are the recursion's; the forward form has none)
  if constexpr (SAMPLER == IZPI_SAMPLER_COLOUR && !FWD)
    if (compact) return IZPI_RUN(MATSET_CONST);
  return set == MATSET_BASIC ? IZPI_RUN(MATSET_BASIC) : set == MATSET_SURF ? IZPI_RUN(MATSET_SURF) : IZPI_RUN(MATSET_FULL);
#undef IZPI_RUN
}

// Load the kernel code this scene's renders of (SAMPLER, FWD) run, ahead of the first frame:
// the first occupancy query of a kernel loads its code object, ~14 ms that a fresh renderer's
// first frame paid (tools/first_frame_host.py). Called by izpi_gpu_upload_scene.
template <int SAMPLER, bool FWD>
int prepare_sampler(izpi_ctx* ctx, bool compact) {
  const uint32_t ms = ctx->matset;
  const int set = ms == 0 ? MATSET_BASIC : (ms & ~(uint32_t)MATSET_SURF) == 0 ? MATSET_SURF : MATSET_FULL;
  int blocks = 0, rc = IZPI_OK;
  auto query = [&](auto shade, auto tail32, auto tail64) {
    if ((rc = resident_blocks(ctx, shade, &blocks, (int)SHADE_THREADS))) return;
    if ((rc = resident_blocks(ctx, tail32, &blocks))) return;
    rc = resident_blocks(ctx, tail64, &blocks);
  };
#define IZPI_Q(M) query(k_shade<SAMPLER, M, FWD>, k_tail<SAMPLER, M, 32, FWD>, k_tail<SAMPLER, M, 64, FWD>)
  bool done = false;
  if constexpr (SAMPLER == IZPI_SAMPLER_COLOUR && !FWD)
    if (compact) { IZPI_Q(MATSET_CONST); done = true; }
  if (done) {
  } else if (set == MATSET_BASIC) IZPI_Q(MATSET_BASIC);
  else if (set == MATSET_SURF) IZPI_Q(MATSET_SURF);
  else IZPI_Q(MATSET_FULL);
#undef IZPI_Q
  if (rc) return rc;
  if ((rc = resident_blocks(ctx, k_start<SAMPLER, FWD>, &blocks))) return rc;
  if constexpr (FWD)
    if ((rc = resident_blocks(ctx, k_refill<SAMPLER>, &blocks))) return rc;
  return resident_blocks(ctx, k_accumulate, &blocks);
}
