// spt_kernel.hip — MI355X (gfx950) render kernel for the smallpt per-pixel sampling loop,
// and the C ABI of include/spt.h.
//
// Replaces /root/reference/src/smallpt.cpp:528-542 (pixel x sample loop) and :419-480
// (recursive radiance()) with one persistent-lane kernel:
//   * one lane = one pixel-sample path at a time; radiance()'s recursion is an iterative bounce
//     loop in registers (T = throughput, L = radiance so far);
//   * work units = (pixel, chunk of samples); a wave pulls units from a global atomic queue and
//     hands them to its idle lanes with a ballot + mbcnt prefix sum, so lanes whose paths end by
//     Russian roulette / light hits immediately start the next sample (no idle SIMD slots until
//     the queue drains);
//   * the scene (<= 64 primitives) is read with wave-uniform scalar loads in the intersect loop
//     (intersect() :323-335 is a broadcast, never a per-lane HBM read) and staged into LDS for
//     the per-lane (divergent) lookups of the hit primitive;
//   * Philox4x32-10 counter RNG keyed by (seed; pixel, sample, vertex, stream);
//   * per-pixel accumulation in 32.32 fixed point with 64-bit integer atomics: exact, independent
//     of unit size, lane order, queue order and GPU count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/spt.h"
#include "../../include/spt_flops.h"
#include "spt_device.h"

namespace spt {

constexpr int kMaxPrims = 64;
constexpr int kBlock = 256;
constexpr uint32_t kGrab = 64;  // units fetched per queue atomic
constexpr int kStatWords = 32;
constexpr bool kDefaultLdsGeo = false;   // [0,8) path stats, [8,28) region stats (diagnostic build)

// 64-byte device primitive. rect: w1..w5 = k, b1, b2, c1, c2 (in-plane bounds of the two free
// axes in (x,y,z) order); sphere: w1..w4 = px, py, pz, rad^2.
struct alignas(16) DevPrim {
  int kind;
  float w1, w2, w3, w4, w5, pad0, pad1;
  float ex, ey, ez, pmax;
  float cx, cy, cz, pad2;
};
static_assert(sizeof(DevPrim) == 64, "DevPrim layout");

// Intersection geometry, grouped by kind (XY, XZ, YZ rects, then spheres; index order inside a
// group) and read through the constant address space so every load in the intersect loop is a
// wave-uniform s_load (scalar cache broadcast) — never a per-lane memory access.
// rect bounds as |a - ma| <= ha, |b - mb| <= hb (c_rect_mid in the oracle): per axis one
// subtract + one compare, each reading a single SGPR (the VALU constant-bus limit on gfx950).
struct GeoRect { float k, ma, ha, mb, hb; int idx; int pad0, pad1; };   // 32 B
struct GeoSph { float px, py, pz, rad2; int idx; int pad0, pad1, pad2; };  // 32 B
struct SceneGeo {
  int n_xy, n_xz, n_yz, n_sph;
  int pad[4];
  GeoRect rect[kMaxPrims];  // [0,n_xy) XY, [n_xy, n_xy+n_xz) XZ, then YZ
  GeoSph sph[kMaxPrims];
};
#define SPT_CONST __attribute__((address_space(4)))

struct KParams {  // in device memory, read through a laundered constant-space pointer
  const DevPrim* prims;
  const SceneGeo* geo;
  int n_prims;
  float cam[12];  // origin, lower_left_corner, horizontal, vertical
  int width, height, spp;
  uint32_t seed;
  float nee_prob;
  int rr_depth, max_depth, light_id;
  float lx0, ldx, lz0, ldz, ly, larea;
  int light_mode;
  uint32_t ldxi, ldzi;
  int tile_rows, shard_index, shard_count;
  int chunk, n_local_pix;
  uint32_t n_units;
  float inv_spp, inv_w, inv_h;
  // Shadow-ray specialisation: when the light is black (c == 0, HEAD :294) a path that reaches it
  // always ends there (RR with p == 0, :448), so the NEE test only needs "is the nearest hit the
  // light" — an occlusion query without id bookkeeping.
  int light_black, light_kind, light_pos;
  unsigned long long* accum;  // [n_local_pix][3] 32.32 fixed point
  uint32_t* queue;            // [0] = next unit
  unsigned long long* stats;  // [8]
};

// Re-derive a wave-uniform pointer as opaque so uniform loads are re-issued (s_load) where used
// instead of being hoisted into long-lived SGPRs (which spill to VGPR lanes).
template <typename T>
__device__ __forceinline__ const SPT_CONST T* cptr(const T* p) {
  asm volatile("" : "+s"(p));
  return (const SPT_CONST T*)p;
}

// Scene intersection of the counter-mode contract (intersect :323-335 over Rectangle_* :102-112 /
// Sphere :229-239): grouped kind order, strict `<`, id untouched on a miss (oracle c_intersect).
// tmin is carried as key = bits(t) - 1 so "0 < t < tmin" is ONE unsigned compare; the hit is
// tracked as its grouped position (an inline constant when unrolled) and mapped to the primitive
// index through LDS once per ray.
__device__ __forceinline__ uint32_t tkey(float t) { return __float_as_uint(t) - 1u; }

// Scene topology the kernel is specialised for: rect counts per kind (-1 = runtime loop), whether
// spheres exist (runtime loop), and the light's grouped position (-1 = runtime).
// LDSGEO: read the rect records from an LDS copy (broadcast ds_read: VGPR operands, no SALU)
// instead of scalar loads from the constant address space.
template <int NXY_, int NXZ_, int NYZ_, bool SPH_, int LPOS_, bool LDSGEO_ = false>
struct Topo {
  static constexpr int NXY = NXY_, NXZ = NXZ_, NYZ = NYZ_, LPOS = LPOS_;
  static constexpr bool SPH = SPH_, LDSGEO = LDSGEO_;
};
using TopoCornell = Topo<6, 5, 6, false, 8>;     // rect[] of :287-311 (light = XZ #3 -> pos 8)
using TopoCornellLds = Topo<6, 5, 6, false, 8, true>;
using TopoGeneric = Topo<-1, -1, -1, true, -1>;
#define SPT_LDS __attribute__((address_space(3)))

struct Ray6 { float oa, ia, db, ob, dc, oc; };
template <int AXIS>  // plane axis: 2 = z (XY rects), 1 = y (XZ), 0 = x (YZ)
__device__ __forceinline__ Ray6 ray6(f3 o, f3 d, float ix, float iy, float iz) {
  if (AXIS == 2) return Ray6{o.z, iz, d.x, o.x, d.y, o.y};
  if (AXIS == 1) return Ray6{o.y, iy, d.x, o.x, d.z, o.z};
  return Ray6{o.x, ix, d.y, o.y, d.z, o.z};
}

struct RectHit { float tt; bool inb; };
template <class GP>
__device__ __forceinline__ RectHit rect_eval(GP g, const Ray6& r) {
  const float tt = (g->k - r.oa) * r.ia;
  const float a = fmaf(r.db, tt, r.ob), b = fmaf(r.dc, tt, r.oc);
  const bool ia = fabsf(a - g->ma) <= g->ha, ib = fabsf(b - g->mb) <= g->hb;
  return RectHit{tt, (bool)((int)ia & (int)ib)};
}

template <int N, int AXIS, class GP>  // nearest-hit over one kind group
__device__ __forceinline__ void rect_group(GP g, int n_rt, int pos0, const Ray6& r,
                                           uint32_t& tmin_key, int& pos) {
  auto one = [&](GP gj, int q) {
    const RectHit h = rect_eval(gj, r);
    const uint32_t kk = tkey(h.tt);
    const bool acc = h.inb & (kk < tmin_key);
    tmin_key = acc ? kk : tmin_key;
    pos = acc ? q : pos;
  };
  if constexpr (N >= 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) one(g + j, pos0 + j);
  } else {
    for (int j = 0; j < n_rt; ++j) one(g + j, pos0 + j);
  }
}

__device__ __forceinline__ float sphere_t(const SPT_CONST GeoSph& S, f3 o, f3 d) {
  // det = r^2 - |op - b d|^2; nearest root beyond the fp32 epsilon (Sphere::intersect :229-239)
  const f3 op = mk(S.px - o.x, S.py - o.y, S.pz - o.z);
  const float bb = dot3(op, d);
  const f3 q = mk(fmaf(-bb, d.x, op.x), fmaf(-bb, d.y, op.y), fmaf(-bb, d.z, op.z));
  const float det = S.rad2 - dot3(q, q);
  if (!(det >= 0.0f)) return 0.0f;
  const float sd = sqrtf(det);
  const float t1 = bb - sd, t2 = bb + sd;
  return t1 > 2e-3f ? t1 : (t2 > 2e-3f ? t2 : 0.0f);
}

template <class TP>
__device__ __forceinline__ int n_of(int ct, int rt) { return ct >= 0 ? ct : rt; }

template <class TP, class GP>
__device__ __forceinline__ bool intersect_scene(const SPT_CONST SceneGeo* G, GP rect,
                                                const int* pos2idx, f3 o, f3 d, float& t_out,
                                                int& id) {
  const float ix = rcp_nr(d.x), iy = rcp_nr(d.y), iz = rcp_nr(d.z);
  uint32_t tmin_key = tkey(1e20f);
  int pos = -1;
  const int nxy = n_of<TP>(TP::NXY, G->n_xy), nxz = n_of<TP>(TP::NXZ, G->n_xz);
  const int nyz = n_of<TP>(TP::NYZ, G->n_yz);
  rect_group<TP::NXY, 2>(rect, nxy, 0, ray6<2>(o, d, ix, iy, iz), tmin_key, pos);
  rect_group<TP::NXZ, 1>(rect + nxy, nxz, nxy, ray6<1>(o, d, ix, iy, iz), tmin_key, pos);
  rect_group<TP::NYZ, 0>(rect + nxy + nxz, nyz, nxy + nxz, ray6<0>(o, d, ix, iy, iz), tmin_key,
                         pos);
  if constexpr (TP::SPH) {
    const int nsph = G->n_sph, base = nxy + nxz + nyz;
    for (int j = 0; j < nsph; ++j) {
      const uint32_t kk = tkey(sphere_t(G->sph[j], o, d));
      const bool acc = kk < tmin_key;
      tmin_key = acc ? kk : tmin_key;
      pos = acc ? base + j : pos;
    }
  }
  const float tmin = __uint_as_float(tmin_key + 1u);
  t_out = tmin;
  if (pos >= 0) id = pos2idx[pos];
  return tmin < 1e20f;
}

// Occluders of one rect group: prims at grouped positions q accepted with t < tL (q > L) or
// t <= tL (q < L); the light itself (q == L) is skipped.
template <int N, int AXIS, int LPOS, class GP>
__device__ __forceinline__ bool occl_group(GP g, int n_rt, int pos0, int L, const Ray6& r,
                                           uint32_t after, bool occ) {
  if constexpr (N >= 0 && LPOS >= 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int q = pos0 + j;  // compile-time when pos0 is
      if (q == LPOS) continue;
      const RectHit h = rect_eval(g + j, r);
      const uint32_t kk = tkey(h.tt);
      occ |= h.inb & (q < LPOS ? kk <= after : kk < after);
    }
  } else {
    for (int j = 0; j < n_rt; ++j) {
      const int q = pos0 + j;
      if (q == L) continue;
      const RectHit h = rect_eval(g + j, r);
      const uint32_t kk = tkey(h.tt);
      occ |= h.inb & ((kk < after) | ((kk == after) & (q < L)));
    }
  }
  return occ;
}

// NEE shadow test for a black light: identical outcome to intersect_scene() followed by
// `id == light` (:466-467) — the light at grouped position L wins iff it is accepted at t_L, no
// primitive before it in grouped order is accepted with t <= t_L and none after it with t < t_L.
template <class TP, class GP>
__device__ __forceinline__ bool shadow_hits_light(const SPT_CONST KParams* P,
                                                  const SPT_CONST SceneGeo* G, GP rect, f3 o,
                                                  f3 d, float& tL) {
  const float ix = rcp_nr(d.x), iy = rcp_nr(d.y), iz = rcp_nr(d.z);
  const int nxy = n_of<TP>(TP::NXY, G->n_xy), nxz = n_of<TP>(TP::NXZ, G->n_xz);
  const int nyz = n_of<TP>(TP::NYZ, G->n_yz);
  const int nrect = nxy + nxz + nyz;
  const int lk = P->light_kind;
  const int L = TP::LPOS >= 0 ? TP::LPOS : (lk == SPT_SPHERE ? nrect + P->light_pos : P->light_pos);
  bool ok;
  if (TP::LPOS < 0 && lk == SPT_SPHERE) {
    tL = sphere_t(G->sph[L - nrect], o, d);
    ok = tkey(tL) < tkey(1e20f);
  } else {
    Ray6 r;
    if (lk == SPT_RECT_XY) r = ray6<2>(o, d, ix, iy, iz);
    else if (lk == SPT_RECT_XZ) r = ray6<1>(o, d, ix, iy, iz);
    else r = ray6<0>(o, d, ix, iy, iz);
    const RectHit h = rect_eval(rect + L, r);
    tL = h.tt;
    ok = h.inb & (tkey(tL) < tkey(1e20f));
  }
  if (__ballot(ok) == 0) return false;
  const uint32_t after = tkey(tL);
  bool occ = false;
  occ = occl_group<TP::NXY, 2, TP::LPOS>(rect, nxy, 0, L, ray6<2>(o, d, ix, iy, iz), after, occ);
  occ = occl_group<TP::NXZ, 1, TP::LPOS>(rect + nxy, nxz, nxy, L, ray6<1>(o, d, ix, iy, iz),
                                         after, occ);
  occ = occl_group<TP::NYZ, 0, TP::LPOS>(rect + nxy + nxz, nyz, nxy + nxz, L,
                                         ray6<0>(o, d, ix, iy, iz), after, occ);
  if constexpr (TP::SPH) {
    const int nsph = G->n_sph;
    for (int j = 0; j < nsph; ++j) {
      const int q = nrect + j;
      if (q == L) continue;
      const uint32_t kk = tkey(sphere_t(G->sph[j], o, d));
      occ |= (kk < after) | ((kk == after) & (q < L));
    }
  }
  return ok & !occ;
}

// Diagnostic build (-DSPT_REGION_STATS): per code region, wave executions and active lanes,
// counted with wave-uniform SALU ballots and flushed once per wave to stats[8 + 2*region].
#ifdef SPT_REGION_STATS
constexpr int kRegions = 10;
#define SPT_REGION(R) (reg_flags |= 1u << (R))  // per lane; ballot-counted at the loop end
#else
#define SPT_REGION(R) \
  do {                \
  } while (0)
#endif

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <class TP>
__global__ void __launch_bounds__(kBlock) render_kernel(const KParams* __restrict__ Pg) {
  __shared__ DevPrim s_prims[kMaxPrims];
  __shared__ int s_pos2idx[kMaxPrims];  // grouped position -> primitive index
  __shared__ GeoRect s_rect[TP::LDSGEO ? kMaxPrims : 1];
  {
    const SPT_CONST KParams* P = cptr(Pg);
    const SPT_CONST SceneGeo* G = cptr(P->geo);
    const int nrect = G->n_xy + G->n_xz + G->n_yz;
    for (int i = threadIdx.x; i < P->n_prims; i += kBlock) {
      s_prims[i] = P->prims[i];
      s_pos2idx[i] = i < nrect ? G->rect[i].idx : G->sph[i - nrect].idx;
      if (TP::LDSGEO && i < nrect) {
        const SPT_CONST GeoRect& R = G->rect[i];
        s_rect[i].k = R.k; s_rect[i].ma = R.ma; s_rect[i].ha = R.ha;
        s_rect[i].mb = R.mb; s_rect[i].hb = R.hb; s_rect[i].idx = R.idx;
      }
    }
  }
  __syncthreads();
  const SPT_LDS GeoRect* lds_rect = (const SPT_LDS GeoRect*)s_rect;

  const uint32_t lane = __lane_id();
  // ---- per-lane state
  bool has_unit = false, need_cam = true, carried = false, c_hit = false;
  uint32_t lp = 0, s = 0, s_end = 0, pix = 0;
  int px = 0, py = 0, depth = 0, c_id = 0;
  float c_t = 0.0f;
  unsigned long long acc0 = 0, acc1 = 0, acc2 = 0;
  f3 o = mk(0, 0, 0), d = mk(0, 0, 1), T = mk(1, 1, 1), L = mk(0, 0, 0);
  // ---- wave-uniform state
  uint32_t pool_next = 0, pool_end = 0;
  bool exhausted = false;
  // per-lane event counters (VALU adds under the event's own exec mask; reduced once per wave)
  uint32_t n_path = 0, n_shadow = 0, n_vert = 0, n_nee_hit = 0, n_cos = 0, n_miss = 0;
#ifdef SPT_REGION_STATS
  uint32_t reg_exec[kRegions] = {}, reg_lanes[kRegions] = {};
  uint32_t reg_flags = 0;
#endif

  for (;;) {
    const SPT_CONST KParams* P = cptr(Pg);
    // 1) retire finished units: flush the fixed-point sums of their pixel.
    SPT_REGION(0);  // loop iteration
    if (has_unit && need_cam && s >= s_end) {
      SPT_REGION(1);  // unit retire
      unsigned long long* a = P->accum + 3ull * lp;
      if (acc0) atomicAdd(a + 0, acc0);
      if (acc1) atomicAdd(a + 1, acc1);
      if (acc2) atomicAdd(a + 2, acc2);
      acc0 = acc1 = acc2 = 0;
      has_unit = false;
    }
    // 2) refill idle lanes from the wave's pool (ballot + mbcnt prefix sum), pool from the queue.
    bool needs_unit = !has_unit;
    uint64_t need = __ballot(needs_unit);
    while (need != 0 && !exhausted) {
      SPT_REGION(2);  // refill
      const SPT_CONST KParams* Q = cptr(Pg);
      if (pool_next >= pool_end) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(Q->queue, kGrab);
        b = __builtin_amdgcn_readfirstlane(b);
        if (b >= Q->n_units) { exhausted = true; break; }
        pool_next = b;
        pool_end = min(b + kGrab, Q->n_units);
      }
      const uint32_t rank = lane_rank(need);
      const uint32_t avail = pool_end - pool_next;
      if (needs_unit && rank < avail) {
        const uint32_t u = pool_next + rank;
        const uint32_t npix = (uint32_t)Q->n_local_pix, w = (uint32_t)Q->width;
        const uint32_t j = u / npix;  // chunk-major: lanes get adjacent pixels
        lp = u - j * npix;
        s = j * (uint32_t)Q->chunk;
        s_end = min(s + (uint32_t)Q->chunk, (uint32_t)Q->spp);
        const uint32_t lr = lp / w;
        px = (int)(lp - lr * w);
        const uint32_t T_ = (uint32_t)Q->tile_rows;
        const uint32_t tile = lr / T_, within = lr - tile * T_;
        py = (int)((tile * (uint32_t)Q->shard_count + (uint32_t)Q->shard_index) * T_ + within);
        pix = (uint32_t)py * w + (uint32_t)px;
        has_unit = true;
        needs_unit = false;
        need_cam = true;
      }
      pool_next += min((uint32_t)__popcll(need), avail);
      need = __ballot(needs_unit);
    }
    if (__ballot(has_unit) == 0) break;

    if (has_unit) {
      ++n_vert;
      // One Philox call per lane per iteration, for the vertex about to be shaded: top 24 bits of
      // r.x..r.w = light x, light z, scatter xi1, xi2; low bytes = RR draw (r.x, r.y) and NEE-mix
      // draw (r.z, r.w) — at vertex 1 the low bytes are the camera jitter instead.
      const u4 r = philox4x32_10(pix, s, need_cam ? 1u : (uint32_t)depth + 1u, cptr(Pg)->seed);
      // 3) camera ray for lanes starting a sample (:533-536).
      if (need_cam) {
        SPT_REGION(3);  // camera ray
        const SPT_CONST KParams* C = cptr(Pg);
        const float su = (((float)px - 0.5f) + u16(r.x, r.y)) * C->inv_w;
        const float sv = (((float)(C->height - py - 1) - 0.5f) + u16(r.z, r.w)) * C->inv_h;
        o = mk(C->cam[0], C->cam[1], C->cam[2]);
        d = normalize3(mk(fmaf(C->cam[9], sv, fmaf(C->cam[6], su, C->cam[3])) - C->cam[0],
                          fmaf(C->cam[10], sv, fmaf(C->cam[7], su, C->cam[4])) - C->cam[1],
                          fmaf(C->cam[11], sv, fmaf(C->cam[8], su, C->cam[5])) - C->cam[2]));
        T = mk(1, 1, 1);
        L = mk(0, 0, 0);
        depth = 0;
        carried = false;
        need_cam = false;
      }
      // 4) vertex: hittingPoint :371-377 (or the hit carried from a NEE shadow ray).
      int id = 0;
      float t;
      bool hit;
      if (carried) {
        hit = c_hit; t = c_t; id = hit ? c_id : 0;
        carried = false;
      } else {
        SPT_REGION(4);  // path-ray intersect
        const SPT_CONST SceneGeo* G = cptr(P->geo);
        if constexpr (TP::LDSGEO) hit = intersect_scene<TP>(G, lds_rect, s_pos2idx, o, d, t, id);
        else hit = intersect_scene<TP>(G, G->rect, s_pos2idx, o, d, t, id);
        ++n_path;
      }
      const DevPrim& H = s_prims[id];
      const int kind = H.kind;
      f3 x;
      if (!hit) {
        x = mk(0, 0, 0);
        ++n_miss;
      } else {
        float tr = t;  // plane distance as the reference derives it (:103), see DESIGN.md
        if (kind == SPT_RECT_XY) tr = (H.w1 - o.z) / d.z;
        else if (kind == SPT_RECT_XZ) tr = (H.w1 - o.y) / d.y;
        else if (kind == SPT_RECT_YZ) tr = (H.w1 - o.x) / d.x;
        x = mk(o.x + d.x * tr, o.y + d.y * tr, o.z + d.z * tr);
      }
      f3 nl;  // Hitable::normal, oriented against the ray (:123,:166,:209,:251)
      if (kind == SPT_RECT_XY) nl = d.z < 0.0f ? mk(0, 0, 1) : mk(0, 0, -1);
      else if (kind == SPT_RECT_XZ) nl = d.y < 0.0f ? mk(0, 1, 0) : mk(0, -1, 0);
      else if (kind == SPT_RECT_YZ) nl = d.x < 0.0f ? mk(1, 0, 0) : mk(-1, 0, 0);
      else {
        const f3 n = normalize3(mk(x.x - H.w1, x.y - H.w2, x.z - H.w3));
        nl = dot3(n, d) < 0.0f ? n : mk(-n.x, -n.y, -n.z);
      }
      f3 f = mk(H.cx, H.cy, H.cz);
      const f3 e = mk(H.ex, H.ey, H.ez);
      const float p = H.pmax;
      ++depth;
      u4 rl = r;  // RR / NEE-mix draws; at vertex 1 from stream 1 (only configs that need them)
      if (depth == 1) {
        const SPT_CONST KParams* C = cptr(Pg);
        if (C->rr_depth < 1 || (C->nee_prob > 0.0f && C->nee_prob < 1.0f))
          rl = philox4x32_10(pix, s, 1u | 0x80000000u, C->seed);
      }
      // Russian roulette :448-454 (+ optional hard depth cap).
      bool term = false;
      const int max_depth = P->max_depth;
      if (max_depth > 0 && depth >= max_depth) {
        term = true;
      } else if (depth > P->rr_depth || p == 0.0f) {
        if (!(p > 0.0f)) {
          term = true;
        } else {
          bool keep = true;
          if (p < 1.0f) keep = u16(rl.x, rl.y) < p;
          if (keep) {
            const float ip = 1.0f / p;
            f = mk(f.x * ip, f.y * ip, f.z * ip);
          } else {
            term = true;
          }
        }
      }
      if (!term) {
        SPT_REGION(5);  // DIFF shading (continuing vertex)
        // DIFF :457-480.
        const SPT_CONST KParams* C = cptr(Pg);
        bool nee;
        const float q = C->nee_prob;
        if (q >= 1.0f) nee = true;
        else if (q <= 0.0f) nee = false;
        else nee = u16(rl.z, rl.w) < q;
        float w = 1.0f;
        f3 dn;
        bool light_end = false;
        f3 e_light = mk(0, 0, 0);
        bool scatter = true;
        if (nee) {
          // light_sampling :363-369, shadow ray :466, NEE weight :471-472.
          const SPT_CONST KParams* D = cptr(Pg);
          float xl, zl;
          if (D->light_mode == SPT_LIGHT_GLIBC_WRAP) {
            xl = fmaf((float)(int32_t)(((r.x >> 8) << 7) * D->ldxi), 0x1p-31f, D->lx0);
            zl = fmaf((float)(int32_t)(((r.y >> 8) << 7) * D->ldzi), 0x1p-31f, D->lz0);
          } else {
            xl = fmaf(u01(r.x), D->ldx, D->lx0);
            zl = fmaf(u01(r.y), D->ldz, D->lz0);
          }
          const f3 dl = normalize3(mk(xl - x.x, D->ly - x.y, zl - x.z));
          const int light_id = D->light_id;
          float ts;
          bool to_light, sh = true;
          int ids = light_id;
          if (D->light_black) {
            SPT_REGION(6);  // shadow test
            const SPT_CONST SceneGeo* G = cptr(D->geo);
            if constexpr (TP::LDSGEO) to_light = shadow_hits_light<TP>(D, G, lds_rect, x, dl, ts);
            else to_light = shadow_hits_light<TP>(D, G, G->rect, x, dl, ts);
          } else {
            ids = id;
            const SPT_CONST SceneGeo* G = cptr(D->geo);
            if constexpr (TP::LDSGEO) sh = intersect_scene<TP>(G, lds_rect, s_pos2idx, x, dl, ts, ids);
            else sh = intersect_scene<TP>(G, G->rect, s_pos2idx, x, dl, ts, ids);
            to_light = ids == light_id;
          }
          ++n_shadow;
          if (to_light) {
            SPT_REGION(7);  // NEE light hit
            ++n_nee_hit;
            const float pdf = fabsf((cptr(Pg)->larea * dl.y) / (ts * ts));
            const float brdf = fabsf(dot3(dl, nl) * 0.318309886183790672f);
            w = pdf * brdf;
            dn = dl;
            scatter = false;
            if (sh && s_prims[ids].pmax == 0.0f) {
              // The next vertex is the (black) light hit by this very ray: RR with p == 0 ends
              // the path there (:448-453) returning its emission — finish it inline.
              light_end = true;
              e_light = mk(s_prims[ids].ex, s_prims[ids].ey, s_prims[ids].ez);
            } else {
              carried = true; c_hit = sh; c_t = ts; c_id = ids;
            }
          }
        }
        if (scatter) {
          SPT_REGION(8);  // cosine direction
          dn = cosine_dir(nl, r.z, r.w);
          ++n_cos;
        }
        L = mk(fmaf(T.x, e.x, L.x), fmaf(T.y, e.y, L.y), fmaf(T.z, e.z, L.z));
        T = mk((T.x * f.x) * w, (T.y * f.y) * w, (T.z * f.z) * w);
        o = x;
        d = dn;
        if (light_end) {
          ++n_vert;
          L = mk(fmaf(T.x, e_light.x, L.x), fmaf(T.y, e_light.y, L.y), fmaf(T.z, e_light.z, L.z));
          term = true;
        }
      } else {
        L = mk(fmaf(T.x, e.x, L.x), fmaf(T.y, e.y, L.y), fmaf(T.z, e.z, L.z));
      }
      if (term) {
        SPT_REGION(9);  // path end: accumulate
        const float inv_spp = cptr(Pg)->inv_spp;
        acc0 += fix31(L.x, inv_spp);
        acc1 += fix31(L.y, inv_spp);
        acc2 += fix31(L.z, inv_spp);
        ++s;
        need_cam = true;
      }
    }
#ifdef SPT_REGION_STATS
#pragma unroll
    for (int r = 0; r < kRegions; ++r) {
      const uint64_t m = __ballot((reg_flags >> r) & 1u);
      reg_exec[r] += m != 0;
      reg_lanes[r] += (uint32_t)__popcll(m);
    }
    reg_flags = 0;
#endif
  }
  {
    unsigned long long* st = cptr(Pg)->stats;  // wave-reduced by the atomic optimizer
#ifdef SPT_REGION_STATS
    if (lane == 0) {  // wave-uniform values: one lane adds them
      for (int r = 0; r < kRegions; ++r) {
        atomicAdd(st + 8 + 2 * r, (unsigned long long)reg_exec[r]);
        atomicAdd(st + 9 + 2 * r, (unsigned long long)reg_lanes[r]);
      }
    }
#endif
    atomicAdd(st + 1, (unsigned long long)n_path);
    atomicAdd(st + 2, (unsigned long long)n_shadow);
    atomicAdd(st + 3, (unsigned long long)n_vert);
    atomicAdd(st + 4, (unsigned long long)n_shadow);
    atomicAdd(st + 5, (unsigned long long)n_nee_hit);
    atomicAdd(st + 6, (unsigned long long)n_cos);
    atomicAdd(st + 7, (unsigned long long)n_miss);
  }
}

// 1.31 fixed point -> float, clamp :538 (values are >= 0 by construction).
__global__ void __launch_bounds__(kBlock)
finalize_kernel(const unsigned long long* __restrict__ accum, float* __restrict__ rgb, uint32_t n) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) {
    const float v = (float)accum[i] * 0x1p-31f;
    rgb[i] = v > 1.0f ? 1.0f : v;
  }
}

}  // namespace spt

// =====================================================================================
// C ABI
// =====================================================================================
using namespace spt;

static thread_local std::string g_last_error;
static spt_status fail(spt_status s, const std::string& msg) {
  g_last_error = msg;
  return s;
}
#define SPT_HIP(call)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(e_ == hipErrorOutOfMemory ? SPT_ERR_OOM : SPT_ERR_HIP,                 \
                  std::string(#call) + ": " + hipGetErrorString(e_));                    \
  } while (0)

struct spt_context {
  int device = 0;
  int n_cu = 0, blocks_per_cu = 0;      // generic kernel
  int blocks_per_cu_cornell = 0;        // TopoCornell specialisation
  DevPrim* prims = nullptr;
  SceneGeo* geo = nullptr;
  unsigned long long* accum = nullptr;
  size_t accum_cap = 0;  // elements
  uint32_t* queue = nullptr;
  unsigned long long* stats = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool pending = false;
  int n_prims = 0;
  KParams last{};
  // Pinned staging for the async scene upload; reused only after the previous upload completed.
  DevPrim* h_prims = nullptr;
  SceneGeo* h_geo = nullptr;
  KParams* d_kp = nullptr;   // kernel parameters in device memory (read via s_load)
  KParams* h_kp = nullptr;   // pinned staging
  uint64_t samples = 0;      // pixel-samples of the last render (exact, not counted in-kernel)
  double scene_flop = 0;     // FLOP-model cost of one ray against the scene
};

extern "C" int32_t spt_shard_rows(const spt_params* p, int32_t* rows_out, int32_t cap);
int spt_shard_row_count(const spt_params* p);  // spt_host.cpp

static spt_status validate(const spt_prim* prims, int32_t n, const spt_camera* cam,
                           const spt_params* p) {
  if (!prims || !cam || !p) return fail(SPT_ERR_INVALID_ARG, "null argument");
  if (n <= 0 || n > kMaxPrims) return fail(SPT_ERR_INVALID_ARG, "n_prims must be in [1, 64]");
  if (p->width <= 0 || p->height <= 0 || p->spp <= 0)
    return fail(SPT_ERR_INVALID_ARG, "width/height/spp must be positive");
  if ((uint64_t)p->width * (uint64_t)p->height > 0xFFFFFFFFull)
    return fail(SPT_ERR_INVALID_ARG, "image too large for 32-bit pixel counters");
  if (p->shard_count < 1 || p->shard_index < 0 || p->shard_index >= p->shard_count)
    return fail(SPT_ERR_INVALID_ARG, "bad shard_index/shard_count");
  if (p->tile_rows < 0 || p->chunk < 0) return fail(SPT_ERR_INVALID_ARG, "negative tile/chunk");
  if (p->flags != 0) return fail(SPT_ERR_INVALID_ARG, "flags must be 0");
  if (p->light_mode != SPT_LIGHT_GLIBC_WRAP && p->light_mode != SPT_LIGHT_UNIFORM)
    return fail(SPT_ERR_INVALID_ARG, "bad light_mode");
  if (p->light_mode == SPT_LIGHT_GLIBC_WRAP &&
      (p->light_dx != (float)(uint32_t)p->light_dx || p->light_dz != (float)(uint32_t)p->light_dz))
    return fail(SPT_ERR_INVALID_ARG, "GLIBC_WRAP light sampling needs integral light_dx/dz");
  for (int i = 0; i < n; ++i) {
    if (prims[i].kind < SPT_RECT_XY || prims[i].kind > SPT_SPHERE)
      return fail(SPT_ERR_INVALID_ARG, "bad primitive kind");
    if (prims[i].refl != SPT_DIFF)
      return fail(SPT_ERR_UNSUPPORTED, "only DIFF materials are live in the reference (:457)");
  }
  return SPT_OK;
}

static void to_dev(const spt_prim* s, int n, DevPrim* out) {
  for (int i = 0; i < n; ++i) {
    DevPrim P;
    std::memset(&P, 0, sizeof P);
    P.kind = s[i].kind;
    if (s[i].kind == SPT_SPHERE) {
      const float r = (float)s[i].geom[0];
      P.w1 = (float)s[i].geom[1]; P.w2 = (float)s[i].geom[2]; P.w3 = (float)s[i].geom[3];
      P.w4 = r * r;
    } else {
      P.w1 = (float)s[i].geom[4];
      P.w2 = (float)s[i].geom[0]; P.w3 = (float)s[i].geom[1];
      P.w4 = (float)s[i].geom[2]; P.w5 = (float)s[i].geom[3];
    }
    P.ex = (float)s[i].e[0]; P.ey = (float)s[i].e[1]; P.ez = (float)s[i].e[2];
    P.cx = (float)s[i].c[0]; P.cy = (float)s[i].c[1]; P.cz = (float)s[i].c[2];
    P.pmax = P.cx > P.cy && P.cx > P.cz ? P.cx : P.cy > P.cz ? P.cy : P.cz;  // :447
    out[i] = P;
  }
}

// Rect bounds [lo, hi] as |a - mid| <= half (contract; oracle c_rect_mid).
static void rect_mid(double lo, double hi, float* mid, float* half) {
  *mid = (float)((lo + hi) * 0.5);
  *half = hi >= lo ? (float)((hi - lo) * 0.5) : -1.0f;
}

// Grouped geometry; *light_pos = position of prim `light` in rect[] / sph[] (-1 if absent).
static void build_geo(const spt_prim* s, int n, SceneGeo* g, int light, int* light_pos) {
  std::memset(g, 0, sizeof *g);
  *light_pos = -1;
  int r = 0;
  const int kinds[3] = {SPT_RECT_XY, SPT_RECT_XZ, SPT_RECT_YZ};
  int* counts[3] = {&g->n_xy, &g->n_xz, &g->n_yz};
  for (int k = 0; k < 3; ++k) {
    for (int i = 0; i < n; ++i) {
      if (s[i].kind != kinds[k]) continue;
      GeoRect& R = g->rect[r++];
      R.k = (float)s[i].geom[4];
      rect_mid(s[i].geom[0], s[i].geom[1], &R.ma, &R.ha);
      rect_mid(s[i].geom[2], s[i].geom[3], &R.mb, &R.hb);
      R.idx = i;
      if (i == light) *light_pos = r - 1;
      ++*counts[k];
    }
  }
  for (int i = 0; i < n; ++i) {
    if (s[i].kind != SPT_SPHERE) continue;
    GeoSph& S = g->sph[g->n_sph++];
    const float rad = (float)s[i].geom[0];
    S.px = (float)s[i].geom[1]; S.py = (float)s[i].geom[2]; S.pz = (float)s[i].geom[3];
    S.rad2 = rad * rad;
    S.idx = i;
    if (i == light) *light_pos = g->n_sph - 1;
  }
}

static int tile_rows_of(const spt_params* p) { return p->tile_rows > 0 ? p->tile_rows : 8; }

extern "C" spt_status spt_context_create(int32_t device, spt_context** out) {
  if (!out) return fail(SPT_ERR_INVALID_ARG, "null out");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
    return fail(SPT_ERR_NO_DEVICE, "no HIP device");
  if (device < 0 || device >= count) return fail(SPT_ERR_INVALID_ARG, "bad device ordinal");
  SPT_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  SPT_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(SPT_ERR_NO_DEVICE, std::string("built for gfx950, device is ") + prop.gcnArchName);
  spt_context* c = new spt_context();
  c->device = device;
  c->n_cu = prop.multiProcessorCount;
  int bpc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, render_kernel<TopoGeneric>, kBlock, 0) !=
          hipSuccess || bpc <= 0)
    bpc = 4;
  c->blocks_per_cu = bpc;
  bpc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, render_kernel<TopoCornell>, kBlock, 0) !=
          hipSuccess || bpc <= 0)
    bpc = 4;
  c->blocks_per_cu_cornell = bpc;
  hipError_t e = hipMalloc(&c->prims, sizeof(DevPrim) * kMaxPrims);
  if (e == hipSuccess) e = hipMalloc(&c->geo, sizeof(SceneGeo));
  if (e == hipSuccess) e = hipHostMalloc(&c->h_prims, sizeof(DevPrim) * kMaxPrims, hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc(&c->h_geo, sizeof(SceneGeo), hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc(&c->d_kp, sizeof(KParams));
  if (e == hipSuccess) e = hipHostMalloc(&c->h_kp, sizeof(KParams), hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc(&c->queue, sizeof(uint32_t) * 64);
  if (e == hipSuccess) e = hipMalloc(&c->stats, sizeof(unsigned long long) * kStatWords);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e != hipSuccess) {
    spt_context_destroy(c);
    return fail(SPT_ERR_OOM, std::string("context alloc: ") + hipGetErrorString(e));
  }
  *out = c;
  return SPT_OK;
}

extern "C" spt_status spt_context_destroy(spt_context* c) {
  if (!c) return SPT_OK;
  (void)hipSetDevice(c->device);
  if (c->prims) (void)hipFree(c->prims);
  if (c->geo) (void)hipFree(c->geo);
  if (c->h_prims) (void)hipHostFree(c->h_prims);
  if (c->h_geo) (void)hipHostFree(c->h_geo);
  if (c->d_kp) (void)hipFree(c->d_kp);
  if (c->h_kp) (void)hipHostFree(c->h_kp);
  if (c->accum) (void)hipFree(c->accum);
  if (c->queue) (void)hipFree(c->queue);
  if (c->stats) (void)hipFree(c->stats);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  delete c;
  return SPT_OK;
}

extern "C" spt_status spt_context_reserve(spt_context* c, int32_t n_prims, const spt_params* p) {
  if (!c || !p) return fail(SPT_ERR_INVALID_ARG, "null argument");
  (void)n_prims;
  const size_t need = 3ull * (size_t)spt_shard_row_count(p) * (size_t)p->width;
  if (need > c->accum_cap) {
    SPT_HIP(hipSetDevice(c->device));
    if (c->accum) SPT_HIP(hipFree(c->accum));
    c->accum = nullptr;
    c->accum_cap = 0;
    SPT_HIP(hipMalloc(&c->accum, need * sizeof(unsigned long long)));
    c->accum_cap = need;
  }
  return SPT_OK;
}

extern "C" spt_status spt_render_async(spt_context* c, const spt_prim* prims, int32_t n_prims,
                                       const spt_camera* cam, const spt_params* p, float* rgb_dev,
                                       void* stream_v) {
  if (!c || !rgb_dev) return fail(SPT_ERR_INVALID_ARG, "null context/output");
  spt_status st = validate(prims, n_prims, cam, p);
  if (st != SPT_OK) return st;
  st = spt_context_reserve(c, n_prims, p);
  if (st != SPT_OK) return st;
  SPT_HIP(hipSetDevice(c->device));
  hipStream_t stream = (hipStream_t)stream_v;

  KParams K{};
  if (c->pending) SPT_HIP(hipEventSynchronize(c->ev0));  // staging still read by a prior upload
  to_dev(prims, n_prims, c->h_prims);
  int light_pos = -1;
  build_geo(prims, n_prims, c->h_geo, p->light_id, &light_pos);
  SPT_HIP(hipMemcpyAsync(c->prims, c->h_prims, sizeof(DevPrim) * n_prims, hipMemcpyHostToDevice,
                         stream));
  SPT_HIP(hipMemcpyAsync(c->geo, c->h_geo, sizeof(SceneGeo), hipMemcpyHostToDevice, stream));
  K.prims = c->prims;
  K.geo = c->geo;
  K.n_prims = n_prims;
  for (int i = 0; i < 3; ++i) {
    K.cam[i] = (float)cam->origin[i];
    K.cam[3 + i] = (float)cam->lower_left_corner[i];
    K.cam[6 + i] = (float)cam->horizontal[i];
    K.cam[9 + i] = (float)cam->vertical[i];
  }
  K.width = p->width; K.height = p->height; K.spp = p->spp;
  K.seed = p->seed;
  K.nee_prob = p->nee_prob; K.rr_depth = p->rr_depth; K.max_depth = p->max_depth;
  K.light_id = p->light_id;
  K.lx0 = p->light_x0; K.ldx = p->light_dx; K.lz0 = p->light_z0; K.ldz = p->light_dz;
  K.ly = p->light_y; K.larea = p->light_area; K.light_mode = p->light_mode;
  K.ldxi = p->light_mode == SPT_LIGHT_GLIBC_WRAP ? (uint32_t)p->light_dx : 0u;
  K.ldzi = p->light_mode == SPT_LIGHT_GLIBC_WRAP ? (uint32_t)p->light_dz : 0u;
  K.tile_rows = tile_rows_of(p); K.shard_index = p->shard_index; K.shard_count = p->shard_count;
  const int rows = spt_shard_row_count(p);
  K.n_local_pix = rows * p->width;
  // Unit size: enough units for >= 8 per resident lane so the queue drains evenly; never
  // changes results (integer accumulation).
  int chunk = p->chunk;
  if (chunk <= 0) {
    const double lanes = (double)c->n_cu * c->blocks_per_cu * kBlock;
    const double want_units = 8.0 * lanes;
    const double per_pix = std::max(1.0, want_units / std::max(1, K.n_local_pix));
    chunk = (int)std::max(4.0, std::ceil(p->spp / per_pix));
    chunk = std::min(chunk, p->spp);
  }
  K.chunk = chunk;
  const uint64_t n_chunks = ((uint64_t)p->spp + chunk - 1) / chunk;
  const uint64_t n_units = n_chunks * (uint64_t)K.n_local_pix;
  if (n_units >= 0xFFFF0000ull) return fail(SPT_ERR_INVALID_ARG, "too many work units; raise chunk");
  K.n_units = (uint32_t)n_units;
  K.inv_spp = 1.0f / (float)p->spp;
  K.inv_w = 1.0f / (float)p->width;
  K.inv_h = 1.0f / (float)p->height;
  K.accum = c->accum;
  K.queue = c->queue;
  K.stats = c->stats;
  K.light_black = light_pos >= 0 && c->h_prims[p->light_id].pmax == 0.0f ? 1 : 0;
  K.light_kind = light_pos >= 0 ? prims[p->light_id].kind : 0;
  K.light_pos = light_pos;
  c->n_prims = n_prims;
  c->last = K;
  c->samples = (uint64_t)K.n_local_pix * (uint64_t)p->spp;
  c->scene_flop = 0;
  for (int i = 0; i < n_prims; ++i)
    c->scene_flop += prims[i].kind == SPT_SPHERE ? SPT_FLOP_SPHERE : SPT_FLOP_RECT;
  *c->h_kp = K;
  SPT_HIP(hipMemcpyAsync(c->d_kp, c->h_kp, sizeof(KParams), hipMemcpyHostToDevice, stream));

  SPT_HIP(hipMemsetAsync(c->accum, 0, sizeof(unsigned long long) * 3 * (size_t)K.n_local_pix,
                         stream));
  SPT_HIP(hipMemsetAsync(c->queue, 0, sizeof(uint32_t), stream));
  SPT_HIP(hipMemsetAsync(c->stats, 0, sizeof(unsigned long long) * kStatWords, stream));
  // Topology specialisation: the HEAD Cornell box (6 XY, 5 XZ, 6 YZ rects, light at grouped
  // position 8) runs a fully unrolled intersect; anything else the generic loops.
  const SceneGeo& g = *c->h_geo;
  const bool cornell = g.n_xy == 6 && g.n_xz == 5 && g.n_yz == 6 && g.n_sph == 0 && light_pos == 8;
  const int grid = c->n_cu * (cornell ? c->blocks_per_cu_cornell : c->blocks_per_cu);
  SPT_HIP(hipEventRecord(c->ev0, stream));
  static const bool lds_geo = [] {  // SPT_GEO=lds|smem (A/B); default below
    const char* e = std::getenv("SPT_GEO");
    return e ? std::strcmp(e, "lds") == 0 : kDefaultLdsGeo;
  }();
  if (cornell && lds_geo)
    hipLaunchKernelGGL(render_kernel<TopoCornellLds>, dim3(grid), dim3(kBlock), 0, stream,
                       (const KParams*)c->d_kp);
  else if (cornell)
    hipLaunchKernelGGL(render_kernel<TopoCornell>, dim3(grid), dim3(kBlock), 0, stream,
                       (const KParams*)c->d_kp);
  else
    hipLaunchKernelGGL(render_kernel<TopoGeneric>, dim3(grid), dim3(kBlock), 0, stream,
                       (const KParams*)c->d_kp);
  SPT_HIP(hipGetLastError());
  SPT_HIP(hipEventRecord(c->ev1, stream));
  const uint32_t n = 3u * (uint32_t)K.n_local_pix;
  hipLaunchKernelGGL(finalize_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream,
                     (const unsigned long long*)c->accum, rgb_dev, n);
  SPT_HIP(hipGetLastError());
  c->pending = true;
  return SPT_OK;
}

extern "C" spt_status spt_context_stats(spt_context* c, spt_stats* out) {
  if (!c || !out) return fail(SPT_ERR_INVALID_ARG, "null argument");
  SPT_HIP(hipSetDevice(c->device));
  SPT_HIP(hipEventSynchronize(c->ev1));
  unsigned long long h[kStatWords];
  SPT_HIP(hipMemcpy(h, c->stats, sizeof h, hipMemcpyDeviceToHost));
#ifdef SPT_REGION_STATS
  {
    static const char* names[10] = {"iteration", "unit_retire", "refill", "camera", "path_isect",
                                    "diff_shading", "shadow_test", "nee_light_hit", "cosine",
                                    "path_end"};
    std::fprintf(stderr, "SPT_REGION_STATS");
    for (int r = 0; r < 10; ++r)
      std::fprintf(stderr, " %s=%llu/%llu", names[r], h[8 + 2 * r], h[9 + 2 * r]);
    std::fprintf(stderr, "\n");
  }
#endif
  float ms = 0.0f;
  SPT_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  std::memset(out, 0, sizeof *out);
  out->samples = c->samples; out->path_rays = h[1]; out->shadow_rays = h[2]; out->vertices = h[3];
  out->nee_events = h[4]; out->nee_light_hits = h[5]; out->cosine_samples = h[6];
  out->misses = h[7];
  // FLOP model (include/spt_flops.h): scene cost per ray from the primitive mix.
  const double scene = c->scene_flop;
  out->flop = (double)out->samples * SPT_FLOP_SAMPLE +
              (double)(out->path_rays + out->shadow_rays) * scene +
              (double)out->vertices * SPT_FLOP_VERTEX +
              (double)(out->vertices - out->samples) * SPT_FLOP_COMBINE +
              (double)out->cosine_samples * SPT_FLOP_COSINE +
              (double)out->nee_events * SPT_FLOP_NEE + (double)out->nee_light_hits * SPT_FLOP_NEE_HIT;
  out->kernel_ms = ms;
  c->pending = false;
  return SPT_OK;
}

extern "C" spt_status spt_render(const spt_prim* prims, int32_t n_prims, const spt_camera* cam,
                                 const spt_params* p, float* rgb_out, spt_stats* stats) {
  if (!rgb_out) return fail(SPT_ERR_INVALID_ARG, "null rgb_out");
  spt_status st = validate(prims, n_prims, cam, p);
  if (st != SPT_OK) return st;
  spt_context* c = nullptr;
  st = spt_context_create(p->device, &c);
  if (st != SPT_OK) return st;
  const size_t n = 3ull * (size_t)spt_shard_row_count(p) * (size_t)p->width;
  float* dev = nullptr;
  hipError_t e = hipMalloc(&dev, n * sizeof(float));
  if (e != hipSuccess) {
    spt_context_destroy(c);
    return fail(SPT_ERR_OOM, "output alloc");
  }
  st = spt_render_async(c, prims, n_prims, cam, p, dev, nullptr);
  if (st == SPT_OK) {
    spt_stats tmp;
    st = spt_context_stats(c, stats ? stats : &tmp);
  }
  if (st == SPT_OK) {
    e = hipMemcpy(rgb_out, dev, n * sizeof(float), hipMemcpyDeviceToHost);
    if (e != hipSuccess) st = fail(SPT_ERR_HIP, hipGetErrorString(e));
  }
  (void)hipFree(dev);
  spt_context_destroy(c);
  return st;
}

extern "C" int32_t spt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" const char* spt_last_error(void) { return g_last_error.c_str(); }
