// spt_kernel.hip — MI355X (gfx950) render kernel for the smallpt per-pixel sampling loop,
// and the C ABI of include/spt.h.
//
// Replaces /root/reference/src/smallpt.cpp:528-542 (pixel x sample loop) and :419-480
// (recursive radiance()) with one persistent-lane kernel:
//   * one lane = one pixel-sample path at a time; radiance()'s recursion is an iterative bounce
//     loop in registers (T = throughput, L = radiance so far);
//   * work units = (pixel, chunk of samples); a wave pulls units from a global atomic queue and
//     hands them to its idle lanes with a ballot + mbcnt prefix sum, so lanes whose paths end by
//     Russian roulette / light hits immediately start the next sample; once the queue is dry an
//     idle lane takes the upper half of a busy lane's unstarted samples (in-wave stealing);
//   * the scene (<= 64 primitives) never costs a per-lane HBM read in intersect() :323-335: the
//     reference's HEAD scene is compiled into the instruction stream, other scenes' rect tests are
//     staged once per block into LDS (broadcast reads) and their spheres read with wave-uniform
//     scalar loads; the per-lane lookups of the hit primitive (material) come from LDS;
//   * a NEE shadow ray is traced only if the light's own test accepts it; in the reference's room
//     the HEAD NEE kernel resolves most of those at once, where an exact geometric predicate
//     proves that nothing lies between the vertex and the light (early_nee_proven);
//   * Philox4x32-7 counter RNG keyed by (seed; pixel, sample, vertex, stream);
//   * per-pixel accumulation in 1.31 fixed point with 64-bit integer atomics: exact, independent
//     of unit size, lane order, queue order, stealing and GPU count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>

#include "../../include/spt.h"
#include "../../include/spt_flops.h"
#include "spt_device.h"
#include "spt_cornell.h"
#include "spt_diag.h"

#define SPT_STR_(x) #x
#define SPT_XSTR(x) SPT_STR_(x)

namespace spt {

constexpr int kMaxPrims = 64;
constexpr int kBlock = 256;
// Units fetched per queue atomic. Measured (1 GPU): 8/16/32 slower (C2 5.6/5.0/4.7 ms vs 4.6:
// atomics), 128/256 slower for C3 (16.7/17.3 vs 16.0 ms: work hoarded in one wave's pool when the
// queue drains) though faster for C2 (4.45 ms); a guided scheme (static first slice per wave, then
// shares of what is left, 16..256) was 6 % slower on C3-C5.
#ifndef SPT_GRAB
#define SPT_GRAB 64
#endif
constexpr uint32_t kGrab = SPT_GRAB;
// Guided grabs of short launches: left >> (log2(2 x waves) + SPT_GUIDED_EXTRA) units, at least
// SPT_GRAB_MIN. Round 3 (C2, 8 rounds on two boxes): 16 / +0 -> 8 / +1 cut the kernel 1.0-1.6 %;
// 8 / +0, 4 / +0, 16 / +1 and 4 / +2 did not (profiles/r03_ab.txt session 10).
#ifndef SPT_GRAB_MIN
#define SPT_GRAB_MIN 8
#endif
#ifndef SPT_GUIDED_EXTRA
#define SPT_GUIDED_EXTRA 1
#endif
constexpr uint32_t kGrabMin = SPT_GRAB_MIN;  // guided grabs never take fewer (bounds the queue atomics)
// Launches with fewer lane-iterations per resident lane than SPT_SMALL_ITERS deal their units
// almost all at once (SPT_SMALL_UNITS per lane) and balance by stealing (host, spt_render_async).
#ifndef SPT_SMALL_ITERS
#define SPT_SMALL_ITERS 2000.0
#endif
#ifndef SPT_SMALL_UNITS
#define SPT_SMALL_UNITS 1.5
#endif
#ifndef SPT_SMALL_BPC
#define SPT_SMALL_BPC 4  // resident blocks per CU of a short launch (host, spt_render_async)
#endif
// Units per resident lane of a long launch (host, spt_render_async): 8 since round 4 (was 16)
#ifndef SPT_UNITS_PER_LANE
#define SPT_UNITS_PER_LANE 8.0
#endif
// Young blocks of a long launch (host, spt_render_async): the waves of the blocks a CU received
// last (blockIdx >= SPT_YOUNG_RANK x n_cu at 8 blocks per CU) take no new pool once SPT_YOUNG_CUT per
// mille of the units are handed out. The SIMD issues oldest-first, so these waves get the fewest
// slots (C3: the two youngest of a CU's 8 blocks do ~4 % of the work) and the units they hold end
// the launch. Round 5 A/B (profiles/r05_young_cut_ab.json): C3 isolated kernel -1.3 to -1.6 %,
// C4 -0.8 %, values flat; applied to the literal HEAD NEE kernels (and their any-camera forms) and
// the room-literal edited-scene NEE kernels (KV_UPBOX_NEE: -4 %; KV_UPLIGHT_NEE, round 6) only (the
// others lost). It assumes the dispatcher hands
// each CU its blocks in blockIdx order, so blockIdx >= SPT_YOUNG_RANK x n_cu are the blocks a CU
// received last; that holds only with every CU full at 8 blocks, so the host applies it at bpc == 8.
#ifndef SPT_YOUNG_CUT
#define SPT_YOUNG_CUT 300
#endif
#ifndef SPT_YOUNG_RANK
#define SPT_YOUNG_RANK 6
#endif
#ifndef SPT_SCRAMBLE_K
#define SPT_SCRAMBLE_K 8  // pixel-order spreading factor of the work units (1 = off; A/B in DESIGN.md §4)
#endif
// Unit slots: a unit's owner lane stores its three sums to the unit's own slot (plain stores, no
// atomics); only stolen ranges add into the per-pixel accumulator; finalize_slots_kernel sums both
// (rounds 1-2 added every unit's sums atomically)
#ifndef SPT_STEAL_MIN
#define SPT_STEAL_MIN 8  // unstarted samples a donor must hold (in-wave stealing; A/B in DESIGN.md §4)
#endif
#ifndef SPT_STEAL_MIN_SMALL
#define SPT_STEAL_MIN_SMALL 16  // the same for short launches (C2: +2-3 %, profiles/r04_ab.txt s. 9)
#endif
#ifdef SPT_WAVE_TIMES
constexpr int kStatWords = 32 + 3 * 32768;  // diagnostic: per-wave start, end, iterations
#else
constexpr int kStatWords = 32;
#endif
// Lane states of the render loop (render_kernel).
constexpr uint32_t kStIdle = 0;    // no work unit
constexpr uint32_t kStCam = 1;     // next: a camera ray (a new sample; retire the unit at s_end)
constexpr uint32_t kStCos = 2;     // next: the cosine continuation of the last vertex
constexpr uint32_t kStSpec = 3;    // next: a path ray whose direction is already set (SPEC/REFR)
constexpr uint32_t kStPath = 4;    // a path ray is set: trace it, shade its vertex
constexpr uint32_t kStShadow = 5;  // a NEE shadow ray toward the light is set: trace, resolve
constexpr uint32_t kStTerm = 6;    // the path ended at this vertex (within an iteration)
constexpr uint32_t kStEarly = 7;   // a NEE shadow ray proven to reach the light (early_nee_proven)
// Exit condition every wave reaches even if a path never terminated: a C3 wave runs ~4e3
// iterations and a 1-GPU C5 wave ~3e6; stats[0] counts waves that hit the cap.
constexpr uint32_t kMaxWaveIters = 1u << 26;
// stats[]: [0] waves that hit kMaxWaveIters, [1,8) path statistics (spt_stats order), [8] shadow
// rays that passed the light pre-test, [9] sphere vertices, [10] shadow rays of those resolved
// without a trace (early_nee_proven), [12,32) region stats (diagnostic build)
[[maybe_unused]] constexpr int kStatShadowTraced = 8, kStatSphereVertices = 9, kStatShadowProven = 10,
                               kStatRegion = 12;

// 64-byte device primitive. rect: w1..w5 = k, b1, b2, c1, c2 (in-plane bounds of the two free
// axes in (x,y,z) order); sphere: w1..w5 = px, py, pz, rad^2, 1/rad.
struct alignas(16) DevPrim {
  int kind;
  float w1, w2, w3, w4, w5;
  int refl;  // spt_refl
  float ip;  // 1/pmax, correctly rounded on the host (the RR reweighting f * (1/p) of :451)
  float ex, ey, ez, pmax;
  float cx, cy, cz;
  // Russian roulette as integers (host): INT_MIN when pmax == 0 (RR always applies, :448), else
  // ceil(pmax * 2^16) (0 for pmax <= 0, 2^16 for pmax >= 1), so that `u16 * 2^-16 < pmax` (:449,
  // with alive only for pmax > 0) is `(int)u16 < rr_t`: the same decision with no conversion
  int32_t rr_t;
};
static_assert(sizeof(DevPrim) == 64, "DevPrim layout");

// Intersection geometry, grouped by kind (XY, XZ, YZ rects, then spheres; index order inside a
// group) and read through the constant address space so every load in the intersect loop is a
// wave-uniform s_load (scalar cache broadcast) — never a per-lane memory access.
// rect bounds as |a - ma| <= ha, |b - mb| <= hb (c_rect_mid in the oracle): per axis one
// subtract + one compare, each reading a single SGPR (the VALU constant-bus limit on gfx950).
struct GeoRect { float k, ma, ha, mb, hb; int idx; int pad0, pad1; };   // 32 B
struct GeoSph { float px, py, pz, rad2; int idx; int wide, pad1, pad2; };  // 32 B
// fp64 geometry of a wide sphere (radius >= SPT_WIDE_SPHERE_RADIUS: the 1e5 walls of the classic
// smallpt box), tested in double (oracle c_sphere_wide).
struct GeoSphD { double px, py, pz, rad2; };
// A rect test of the contract (oracle c_test): a parallel pair (k0 < k1, shared bounds) or a single
// (k0 == k1, pos0 == pos1); pos* are grouped positions in rect[].
struct GeoTest { float k0, k1, ma, ha, mb, hb; int pos0, pos1; };      // 32 B
struct SceneGeo {
  int n_xy, n_xz, n_yz, n_sph;
  int n_txy, n_txz, n_tyz, n_sph_wide;  // rect tests per kind; wide spheres = the last n_sph_wide
  // contract v5's room (oracle c_find_room): its three pair tests follow the per-kind lists in
  // test[] (XY, XZ, YZ); box = mid, half + 2^-8 for x, y, z
  int has_room, n_box, pad_[2];  // n_box: boxes of contract v6 (their tests follow the room's)
  float pad2_[8];
  GeoRect rect[kMaxPrims];  // [0,n_xy) XY, [n_xy, n_xy+n_xz) XZ, then YZ
  GeoSph sph[kMaxPrims];
  GeoSphD sphd[kMaxPrims];
  GeoTest test[kMaxPrims];  // [0,n_txy) XY, then XZ, then YZ (room tests excluded), then the room
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
  // n / d = (n * m) >> sh for every n < 2^31 (Granlund-Montgomery, host-computed): the refill's
  // divisions by n_local_pix, width and tile_rows without the ~25-instruction integer divide.
  uint32_t m_npix, sh_npix, m_w, sh_w, m_tile, sh_tile;
  // Guided grabs (small launches only, sh_guided < 32): a wave takes min(kGrab, max(units its
  // lanes need, kGrabMin, left >> sh_guided)) units per queue atomic, left = units not yet handed
  // out, so no wave hoards a full pool while the queue runs dry. sh_guided = 32: always kGrab.
  uint32_t sh_guided;
  // young blocks (SPT_YOUNG_CUT): blockIdx >= young_block take no new pool once the queue is at
  // young_cut; young_block = UINT32_MAX: off
  uint32_t young_block, young_cut;
  uint32_t scr_k, scr_q;  // pixel-order spreading of the units: K = 2^scr_k, scr_q = npix / K
  float inv_spp, inv_w, inv_h;
  float fix_scale;  // inv_spp * 2^31 (fix31)
  // camera of contract v5 (jitter_f): Au, Av, Cu = Au 2^-16, Cv = Av 2^-16, L = llc - origin per axis
  float cam_au[3], cam_av[3], cam_cu[3], cam_cv[3], cam_l[3];
  // light sample of contract v5 (oracle c_wrap_sample): GLIBC_WRAP with dx = 2^a odd, 1 <= a <= 24:
  // x0 - 1 + (r >> (7 + a)) 2^(a - 24); else (lattice 0) the rounds-1-4 wrapped multiply
  int lx_lattice, lz_lattice;
  uint32_t lx_shift, lz_shift;
  float lx_scale, lz_scale, lx0m1, lz0m1;
  // Shadow-ray specialisation: when the light is black (c == 0, HEAD :294) a path that reaches it
  // always ends there (RR with p == 0, :448), so the NEE test only needs "is the nearest hit the
  // light" — an occlusion query without id bookkeeping.
  int light_black, light_kind, light_pos;
  int scatter_uniform;  // SPT_FLAG_UNIFORM_SCATTER
  int leak_end;         // contract v6: a leaked path ends at its first miss (host leak_end_of)
  uint32_t steal_min;   // SPT_STEAL_MIN or, for a short launch, SPT_STEAL_MIN_SMALL
  // Sphere NEE kernel: vertices above early_y0 (every sphere's top + 1) in the HEAD room resolve
  // their light-accepted shadow rays early (early_room_proven); +inf when the host cannot prove it
  float early_y0;
  // The uploaded-geometry HEAD-topology NEE kernel's early resolve (early_geo_proven): per box, a
  // vertex at or above eb_top[b] or with sgn * x[axis] <= eb_bnd[b] (axis x, or z where eb_z[b]) has
  // a shadow segment that cannot meet the box; eb_top = +inf and eb_bnd = -inf: no clause (the
  // host could not prove one, or the predicate is off)
  float eb_top[2], eb_sgn[2], eb_bnd[2];
  uint32_t eb_z[2];
  // ... and its room clause (early_geo_setup): the vertex in the room's box below the light plane,
  // per axis (bits(v) - er_lo) <= er_span on the float bits (HEAD: x in [1, 99], y in [0, 81.5),
  // z in [0, 170], the literal early_room_ok); er_lo = 0, er_span = 0 with no clause
  uint32_t er_lo[3], er_span[3];
  uint32_t ul_ybits;  // the room-literal light-uploaded kernel's y bound: bits(y) < bits(y_L)
  int unit_dirs;  // oracle c_unit_dirs: the scene has a sphere or a REFR primitive
  float nee_c;    // light_area / pi rounded once (the free-scale NEE weight, nee_weight)
  unsigned long long* accum;  // [n_local_pix][3] 1.31 fixed point (stolen ranges; every unit without slots)
  unsigned long long* slots;  // [n_units][3] one owner store per unit, unit order (unit slots)
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


// Rect geometry with literal operands: kCornellRects[i] at a compile-time i (spt_cornell.h).
struct CornellRectPtr {
  int i;
  __device__ constexpr CornellRectPtr operator+(int j) const { return CornellRectPtr{i + j}; }
  __device__ constexpr const CRect* operator->() const { return &kCornellRects[i]; }
};

// Scene topology the kernel is specialised for: rect counts per kind (-1 = runtime loop), whether
// spheres exist (runtime loop), the light's grouped position (-1 = runtime), and whether the rect
// bounds are the compile-time HEAD scene (CONSTGEO) or read from the uploaded scene (s_load).
// MAT: SPEC/REFR materials and the uniform-hemisphere flag may occur (generic kernel); the
// specialisations are all-DIFF, cosine-scatter scenes (keeps their cosine block branch-free).
// NT*: rect tests per kind (parallel pairs count once).
template <int NXY_, int NXZ_, int NYZ_, bool SPH_, int LPOS_, bool CONSTGEO_ = false,
          int NTXY_ = -1, int NTXZ_ = -1, int NTYZ_ = -1, bool MAT_ = SPH_, bool WIDE_ = false,
          int NBOX_ = -1, bool UPBOX_ = false, bool UPLIGHT_ = false>
struct Topo {
  static constexpr int NBOX = NBOX_;  // boxes of contract v6 (uploaded geometry; -1 = run time)
  // CONSTGEO with the two boxes uploaded (an edited rect[] whose room and light are HEAD's): the
  // room and light as literals, the boxes' slab tests from LDS, the early resolve's box clauses
  // from KParams (early_geo_proven)
  static constexpr bool UPBOX = UPBOX_;
  // UPBOX with the light uploaded as well (an edited light; the room literal): the light's test from
  // the uploaded scene through scalar loads, its plane's y bound of the early resolve from KParams
  static constexpr bool UPLIGHT = UPLIGHT_;
  static constexpr int NXY = NXY_, NXZ = NXZ_, NYZ = NYZ_, LPOS = LPOS_;
  static constexpr int NTXY = NTXY_, NTXZ = NTXZ_, NTYZ = NTYZ_;
  static constexpr bool SPH = SPH_, CONSTGEO = CONSTGEO_, MAT = MAT_;
  static constexpr bool WIDE = WIDE_;  // fp64 wide spheres may occur (their own kernel: VGPRs)
  // Ray-direction contract (oracle c_unit_dirs): 1 = unit directions (spheres, REFR), 0 = free-scale
  // (rect-only DIFF scenes: path directions normalised with rsq_nr1, the NEE vector not at all),
  // -1 = KParams::unit_dirs at run time (the generic kernels)
  static constexpr int DIRS = MAT_ ? -1 : (SPH_ ? 1 : 0);
};
// rect[] of :287-311 (light = XZ #3 -> pos 8); tests besides the room (contract v5): 2 XY box
// pairs; light + 2 box tops; 2 YZ box pairs
using TopoCornell = Topo<6, 5, 6, false, 8, false, 0, 1, 0, false, false, 2>;
using TopoCornellConst = Topo<kCornellNXY, kCornellNXZ, kCornellNYZ, false, kCornellLightPos, true>;
// the same with the boxes uploaded (a box moved or resized; room, light and topology HEAD's)
using TopoCornellUpBox = Topo<kCornellNXY, kCornellNXZ, kCornellNYZ, false, kCornellLightPos, true, -1, -1,
                              -1, false, false, 2, true>;
// ... and with the light uploaded too (the light moved or resized; the room HEAD's)
using TopoCornellUpLight = Topo<kCornellNXY, kCornellNXZ, kCornellNYZ, false, kCornellLightPos, true, -1, -1,
                                -1, false, false, 2, true, true>;
using TopoGeneric = Topo<-1, -1, -1, true, -1>;
// Any scene with spheres but only DIFF materials and cosine scattering (the C5 32-sphere scene):
// no SPEC/REFR stack and branch words, 8 waves/SIMD instead of the generic kernel's 6.
using TopoSphDiff = Topo<-1, -1, -1, true, -1, false, -1, -1, -1, false>;
// Any other rect-only, all-DIFF, cosine-scatter scene (uploaded geometry, run-time loops): the
// free-scale direction contract at compile time (Topo::DIRS 0), no sphere loop.
using TopoRectDiff = Topo<-1, -1, -1, false, -1>;
// Scenes with wide spheres (radius >= SPT_WIDE_SPHERE_RADIUS, tested in fp64: the classic smallpt
// box): the generic kernel plus the fp64 sphere loop, kept apart because the doubles cost VGPRs.
using TopoGenericWide = Topo<-1, -1, -1, true, -1, false, -1, -1, -1, true, true>;

// Estimator configuration the kernel is specialised for (compile-time where the host can prove
// it, -1 = read from KParams at run time). Only wave-uniform branches and parameter loads go away;
// per lane the arithmetic is the same contract.
//   NEE:   1 = nee_prob >= 1 (HEAD :464), 0 = nee_prob <= 0 (cosine only, :474-477)
//   LMODE: light sampling (SPT_LIGHT_GLIBC_WRAP / SPT_LIGHT_UNIFORM)
//   BLACK: 1 = the light's colour is 0, so a path reaching it ends there (RR with p == 0, :448)
//   MAXD0: 1 = no hard depth cap (max_depth == 0, the reference)
//   NOS1:  1 = no vertex-1 stream-1 draws (rr_depth >= 1 and nee_prob is 0 or 1)
//   CAMAX: 1 = axis-aligned camera (horizontal = (h,0,0), vertical = (0,v,0) up to the sign of
//          zero, origin components nonzero, as the reference's :521 camera): the zero products of
//          the camera's fma chain vanish exactly, so the ray is the same bits with 5 fewer VALU;
//          2 = any camera (Camera :262-275 with any lookat/vup, round 6), its per-pixel P_x, P_y,
//          P_z per work unit and the jitter's Cu, Cv in SGPRs: 6 fmas per camera ray (1: 2,
//          0/-1: 12 and scalar loads); the same bits as the general form (contract v5)
//   LREF:  1 = the reference's light sampling and RR constants (light x0/dx 32/36, z0/dz 63/36,
//          y 81.6, area 1296 :365-367,:471; light id 6 :467; rr_depth 5 :448): literals instead
//          of scalar loads in the loop
//   LEAK:  1 = contract v6's leak-end rule (a leaked path ends at its first miss; the host proves
//          it applies, leak_end_of), 0 = leaked paths go on from the miss vertex as the reference's
//          (SPT_FLAG_REFERENCE_LEAKS, or a scene the rule does not hold for), -1 = KParams::leak_end
template <int NEE_, int LMODE_, int BLACK_, int MAXD0_, int NOS1_, int CAMAX_, int LREF_ = 0,
          int LEAK_ = -1>
struct Cfg {
  static constexpr int NEE = NEE_, LMODE = LMODE_, BLACK = BLACK_, MAXD0 = MAXD0_, NOS1 = NOS1_;
  static constexpr int CAMAX = CAMAX_, LREF = LREF_, LEAK = LEAK_;
};
using CfgRuntime = Cfg<-1, -1, -1, -1, -1, -1>;
// C3/C4: the reference's HEAD estimator; C2: cosine-weighted only (leak-end rule / reference leaks)
using CfgHeadNee = Cfg<1, SPT_LIGHT_GLIBC_WRAP, 1, 1, 1, 1, 1, 1>;
using CfgHeadCos = Cfg<0, SPT_LIGHT_GLIBC_WRAP, 1, 1, 1, 1, 1, 1>;
using CfgHeadNeeRef = Cfg<1, SPT_LIGHT_GLIBC_WRAP, 1, 1, 1, 1, 1, 0>;
// the same estimators with any camera (a tilted lookat)
using CfgHeadNeeCam = Cfg<1, SPT_LIGHT_GLIBC_WRAP, 1, 1, 1, 2, 1, 1>;
using CfgHeadCosCam = Cfg<0, SPT_LIGHT_GLIBC_WRAP, 1, 1, 1, 2, 1, 1>;
using CfgHeadCosRef = Cfg<0, SPT_LIGHT_GLIBC_WRAP, 1, 1, 1, 1, 1, 0>;
// Sphere scenes with the reference's NEE estimator and black light (C5): early NEE resolve
using CfgSphNee = Cfg<1, SPT_LIGHT_GLIBC_WRAP, 1, -1, -1, -1, 1, 1>;
using CfgSphNeeRef = Cfg<1, SPT_LIGHT_GLIBC_WRAP, 1, -1, -1, -1, 1, 0>;
// The LREF constants (the host checks spt_params against them before it picks an LREF kernel).
constexpr int kRefLightId = 6, kRefRrDepth = 5;
constexpr float kRefLx0 = 32.0f, kRefLz0 = 63.0f, kRefLy = 81.6f, kRefLarea = 1296.0f;
constexpr uint32_t kRefLdxi = 36u, kRefLdzi = 36u;
template <class CF> __device__ __forceinline__ int light_id_of(const SPT_CONST KParams* P) {
  if constexpr (CF::LREF == 1) return kRefLightId; else return P->light_id;
}
// The light's id in the kernel's primitive numbering: its grouped position in the HEAD kernels
// (s_prims is loaded in position order there, intersect_scene), its prims[] index elsewhere
template <class TP, class CF> __device__ __forceinline__ int light_slot_of(const SPT_CONST KParams* P) {
  if constexpr (TP::CONSTGEO) return kCornellLightPos; else return light_id_of<CF>(P);
}
template <class CF> __device__ __forceinline__ int rr_depth_of(const SPT_CONST KParams* P) {
  if constexpr (CF::LREF == 1) return kRefRrDepth; else return P->rr_depth;
}
// The ray-direction contract of the launch (oracle c_unit_dirs; Topo::DIRS).
template <class TP>
__device__ __forceinline__ bool unit_dirs_of(const KParams* Pg) {
  if constexpr (TP::DIRS >= 0) {
    (void)Pg;
    return TP::DIRS == 1;
  } else {
    return cptr(Pg)->unit_dirs != 0;
  }
}
template <class TP>
__device__ __forceinline__ auto rects_of(const SPT_CONST SceneGeo* G) {
  if constexpr (TP::CONSTGEO) return CornellRectPtr{0};
  else return G->rect + 0;
}

struct Ray6 { float oa, ia, db, ob, dc, oc; };
template <int AXIS>  // plane axis: 2 = z (XY rects), 1 = y (XZ), 0 = x (YZ)
__device__ __forceinline__ Ray6 ray6(f3 o, f3 d, float ix, float iy, float iz) {
  if (AXIS == 2) return Ray6{o.z, iz, d.x, o.x, d.y, o.y};
  if (AXIS == 1) return Ray6{o.y, iy, d.x, o.x, d.z, o.z};
  return Ray6{o.x, ix, d.y, o.y, d.z, o.z};
}

// ---- Nearest hit, contract v5 (round 4; oracle c_intersect / c_key). A candidate at t on the plane
// or sphere with grouped position pos is ranked by its KEY: the float bits of t with the low 6 bits
// replaced by pos (negatives, inf and NaN rank last; a plane's zero distance is -2^-149, plane_t,
// and a sphere without a root -0); the nearest hit is the smallest key. Per candidate that is one
// v_bitop3 and one v_min_u32 -- where rounds 1-4 compared keys and selected (t, position) through
// lane masks, a v_cmp -> s_and -> two v_cndmask chain per test. With the rest of contract v5 C3
// 13.55 -> 12.75 ms, and the fma'd -2^-149 below (no "minus one" before the key) 12.92 -> 12.42 ms
// on a slower box (A/B, profiles/r04_ab.txt sessions 2-4).
// A parallel pair's candidate is the smaller of its two planes' keys (the smaller positive t: the
// plane the rounds-1-4 pair rule chose); its in-plane test is evaluated at that plane's t. The
// winner's exact t is recomputed by whoever needs it (shading, NEE weight) from its plane or
// sphere: the same bits as in its key.
constexpr uint32_t kKeyNone = __builtin_bit_cast(uint32_t, 1e20f) | 63u;  // tmin = 1e20 (:324)
// A plane's distance (oracle c_plane_t): (k - o_a) * inv_a as one fma with -2^-149 -- the rounded
// product except at an exact rounding tie, and a zero distance (origin on the plane: :106, :328
// reject it) becomes -2^-149 and ranks last like every negative t, so the key needs no "minus one".
constexpr float kNegTiny = -0x1p-149f;
__device__ __forceinline__ float plane_t(float n, float inv) { return fmaf(n, inv, kNegTiny); }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
// c += b for a per-lane event counter as ONE v_addc_co_u32 with b's lane mask as its carry-in
// (LLVM spells c + (b ? 1 : 0) as a v_cndmask and a v_add)
__device__ __forceinline__ void count_if(uint32_t& c, bool b) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(b);
  asm("v_addc_co_u32_e64 %0, vcc, 0, %0, %1" : "+v"(c) : "s"(m) : "vcc");
}
// (bits(t) | 63) ^ (63 - pos) as ONE v_bitop3 (0x36 = (S0 | S2) ^ S1)
template <int POS>
__device__ __forceinline__ uint32_t key_c(float t) {  // compile-time position (inline constant)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, 63 bitop3:0x36" : "=v"(r) : "v"(__float_as_uint(t)), "n"(63 - POS));
  return r;
}
__device__ __forceinline__ uint32_t key_v(float t, uint32_t pos) {  // position in a VGPR
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, 63 bitop3:0x36" : "=v"(r) : "v"(__float_as_uint(t)), "v"(63u - pos));
  return r;
}
__device__ __forceinline__ uint32_t key_s(float t, uint32_t pos) {  // wave-uniform position (SGPR)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, 63 bitop3:0x36" : "=v"(r) : "v"(__float_as_uint(t)), "s"(63u - pos));
  return r;
}

// One rect test (oracle c_intersect): a single (k0 == k1) or a parallel pair. KEYS: the per-plane
// key function for compile-time (CornellTestPtr) or LDS/scalar (GeoTest) geometry.
template <int J> struct CornellTestPtr {
  __device__ constexpr const CTest* operator->() const { return &kCornellTests.t[J]; }
};
template <int J, bool PAIR>
__device__ __forceinline__ void plane_keys(CornellTestPtr<J>, float t0, float t1, uint32_t& kp) {
  if constexpr (PAIR) kp = umin(key_c<kCornellTests.t[J].pos0>(t0), key_c<kCornellTests.t[J].pos1>(t1));
  else kp = key_c<kCornellTests.t[J].pos0>(t0);
}
template <int J, bool PAIR>  // (unused J: a runtime pointer)
__device__ __forceinline__ void plane_keys(const GeoTest* g, float t0, float t1, uint32_t& kp) {
  kp = umin(key_v(t0, (uint32_t)g->pos0), key_v(t1, (uint32_t)g->pos1));
}
template <int J, bool PAIR>
__device__ __forceinline__ void plane_keys(const SPT_CONST GeoTest* g, float t0, float t1, uint32_t& kp) {
  kp = umin(key_v(t0, (uint32_t)g->pos0), key_v(t1, (uint32_t)g->pos1));
}
template <int J, bool PAIR, class GP>
__device__ __forceinline__ void rect_cand(GP g, const Ray6& r, uint32_t& tmin) {
  const float t0 = plane_t(g->k0 - r.oa, r.ia);
  float t1 = t0;
  uint32_t kb = __float_as_uint(t0), kp;
  if constexpr (PAIR) {
    t1 = plane_t(g->k1 - r.oa, r.ia);
    kb = umin(kb, __float_as_uint(t1));
  }
  plane_keys<J, PAIR>(g, t0, t1, kp);
  const float tb = __uint_as_float(kb);  // the chosen plane's t
  // in-plane offsets from the centre, a = d_b * t + (o_b - mid_b): the origin's offset is per ray
  // and shared by every rectangle with that centre (CSE'd across the unrolled tests)
  const float a = fmaf(r.db, tb, r.ob - g->ma), b = fmaf(r.dc, tb, r.oc - g->mb);
  const bool inb = (bool)((int)(fabsf(a) <= g->ha) & (int)(fabsf(b) <= g->hb));
  tmin = umin(tmin, inb ? kp : 0xFFFFFFFFu);
}
template <int J>
__device__ __forceinline__ void cornell_test(const Ray6* rays, uint32_t& tmin) {
  constexpr CTest T = kCornellTests.t[J];
  if constexpr (J != kCornellRoom[0] && J != kCornellRoom[1] && J != kCornellRoom[2] && !cornell_in_box(J))
    rect_cand<J, T.pos0 != T.pos1>(CornellTestPtr<J>{}, rays[T.axis], tmin);
}
// A box of contract v6 (oracle c_find_boxes / c_intersect): an XY pair Z (planes z), a YZ pair X
// (planes x) and an XZ top, standing on the room's floor F (the room's XZ pair, k0). Per axis the two
// planes' keys as signed integers -- for t >= 0 the integer order is the order of t, and every
// negative t is a negative integer -- give the slab interval [min, max]; entry = the largest start,
// exit = the smallest end, crossed iff entry <= exit. The candidate is the entry, or for an origin
// inside the box (negative entry) the exit face, as the per-face tests find it: as unsigned keys
// min(entry, exit). Per box 6 plane keys, 8 integer min/max, one compare: the 4 faces' and the top's
// in-plane compares and lane-mask selects are gone (trace 153 -> 131 VALU per wave-iteration).
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ void box_keys(int kx0, int kx1, int kz0, int kz1, int ky0, int ky1,
                                         uint32_t& tmin) {
  const int en = imax(imax(imin(kx0, kx1), imin(kz0, kz1)), imin(ky0, ky1));
  const int ex = imin(imin(imax(kx0, kx1), imax(kz0, kz1)), imax(ky0, ky1));
  tmin = umin(tmin, en <= ex ? umin((uint32_t)en, (uint32_t)ex) : 0xFFFFFFFFu);
}
// The room of contract v6 as the same slab (from inside: the exit face, the nearest positive wall)
__device__ __forceinline__ void cornell_room(const Ray6* rays, uint32_t& tmin) {
  constexpr CTest Z = kCornellTests.t[kCornellRoom[0]], Y = kCornellTests.t[kCornellRoom[1]];
  constexpr CTest X = kCornellTests.t[kCornellRoom[2]];
  const Ray6 &rz = rays[2], &ry = rays[1], &rx = rays[0];
  box_keys((int)key_c<X.pos0>(plane_t(X.k0 - rx.oa, rx.ia)), (int)key_c<X.pos1>(plane_t(X.k1 - rx.oa, rx.ia)),
           (int)key_c<Z.pos0>(plane_t(Z.k0 - rz.oa, rz.ia)), (int)key_c<Z.pos1>(plane_t(Z.k1 - rz.oa, rz.ia)),
           (int)key_c<Y.pos0>(plane_t(Y.k0 - ry.oa, ry.ia)), (int)key_c<Y.pos1>(plane_t(Y.k1 - ry.oa, ry.ia)),
           tmin);
}
template <int B>
__device__ __forceinline__ void cornell_box(const Ray6* rays, uint32_t& tmin) {
  constexpr CTest Z = kCornellTests.t[kCornellBoxes.t[B][0]], X = kCornellTests.t[kCornellBoxes.t[B][1]];
  constexpr CTest T = kCornellTests.t[kCornellBoxes.t[B][2]], F = kCornellTests.t[kCornellRoom[1]];
  const Ray6 &rz = rays[2], &ry = rays[1], &rx = rays[0];
  box_keys((int)key_c<X.pos0>(plane_t(X.k0 - rx.oa, rx.ia)), (int)key_c<X.pos1>(plane_t(X.k1 - rx.oa, rx.ia)),
           (int)key_c<Z.pos0>(plane_t(Z.k0 - rz.oa, rz.ia)), (int)key_c<Z.pos1>(plane_t(Z.k1 - rz.oa, rz.ia)),
           (int)key_c<F.pos0>(plane_t(F.k0 - ry.oa, ry.ia)), (int)key_c<T.pos0>(plane_t(T.k0 - ry.oa, ry.ia)),
           tmin);
}
template <int... B>
__device__ __forceinline__ void cornell_boxes(std::integer_sequence<int, B...>, const Ray6* rays,
                                              uint32_t& tmin) {
  (cornell_box<B>(rays, tmin), ...);
}
// The same for uploaded geometry: the room (rm[0] its XY pair, rm[1] XZ, rm[2] YZ) and a box (bx[0]
// the XY pair, bx[1] the YZ pair, bx[2] the top; fl the room's XZ pair, its k0 the floor)
template <class GT>
__device__ __forceinline__ void geo_room(GT rm, const Ray6& rz, const Ray6& ry, const Ray6& rx,
                                         uint32_t& tmin) {
  box_keys((int)key_v(plane_t(rm[2].k0 - rx.oa, rx.ia), (uint32_t)rm[2].pos0),
           (int)key_v(plane_t(rm[2].k1 - rx.oa, rx.ia), (uint32_t)rm[2].pos1),
           (int)key_v(plane_t(rm[0].k0 - rz.oa, rz.ia), (uint32_t)rm[0].pos0),
           (int)key_v(plane_t(rm[0].k1 - rz.oa, rz.ia), (uint32_t)rm[0].pos1),
           (int)key_v(plane_t(rm[1].k0 - ry.oa, ry.ia), (uint32_t)rm[1].pos0),
           (int)key_v(plane_t(rm[1].k1 - ry.oa, ry.ia), (uint32_t)rm[1].pos1), tmin);
}
template <class GT>
__device__ __forceinline__ void geo_box(GT bx, GT fl, const Ray6& rz, const Ray6& ry, const Ray6& rx,
                                        uint32_t& tmin) {
  box_keys((int)key_v(plane_t(bx[1].k0 - rx.oa, rx.ia), (uint32_t)bx[1].pos0),
           (int)key_v(plane_t(bx[1].k1 - rx.oa, rx.ia), (uint32_t)bx[1].pos1),
           (int)key_v(plane_t(bx[0].k0 - rz.oa, rz.ia), (uint32_t)bx[0].pos0),
           (int)key_v(plane_t(bx[0].k1 - rz.oa, rz.ia), (uint32_t)bx[0].pos1),
           (int)key_v(plane_t(fl->k0 - ry.oa, ry.ia), (uint32_t)fl->pos0),
           (int)key_v(plane_t(bx[2].k0 - ry.oa, ry.ia), (uint32_t)bx[2].pos0), tmin);
}
template <int... J>
__device__ __forceinline__ void cornell_tests(std::integer_sequence<int, J...>, const Ray6* rays,
                                              uint32_t& tmin) {
  (cornell_test<J>(rays, tmin), ...);
}

template <int N, class GT>  // the tests of one kind group, uploaded geometry (every test as a pair)
__device__ __forceinline__ void test_group(GT g, int n_rt, const Ray6& r, uint32_t& tmin) {
  if constexpr (N >= 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) rect_cand<0, true>(g + j, r, tmin);
  } else {
    for (int j = 0; j < n_rt; ++j) rect_cand<0, true>(g + j, r, tmin);
  }
}

// One rectangle's own test (a single, as inside the trace: contract v5): t, whether its in-plane
// test at t- accepts, and the first in-plane offset there.
struct RectHit { float tt; bool inb; float a; };  // a: first in-plane offset from the centre
template <class GP>
__device__ __forceinline__ RectHit rect_eval(GP g, const Ray6& r) {
  const float tt = plane_t(g->k - r.oa, r.ia);
  const float a = fmaf(r.db, tt, r.ob - g->ma), b = fmaf(r.dc, tt, r.oc - g->mb);
  const bool ia = fabsf(a) <= g->ha, ib = fabsf(b) <= g->hb;
  return RectHit{tt, (bool)((int)ia & (int)ib), a};
}
// The uploaded light of the room-literal UPLIGHT kernels (a single XZ test at the HEAD light's grouped
// position, read from the uploaded scene through scalar loads): rect_cand's arithmetic for a single,
// with the position literal.
template <class GT>
__device__ __forceinline__ void light_cand(const GT& g, const Ray6& r, uint32_t& tmin) {
  const float t0 = plane_t(g.k0 - r.oa, r.ia);
  const float a = fmaf(r.db, t0, r.ob - g.ma), b = fmaf(r.dc, t0, r.oc - g.mb);
  const bool inb = (bool)((int)(fabsf(a) <= g.ha) & (int)(fabsf(b) <= g.hb));
  tmin = umin(tmin, inb ? key_c<kCornellLightPos>(t0) : 0xFFFFFFFFu);
}
// The same light's own test (rect_eval on a GeoTest): t and whether the in-plane test accepts.
template <class GT>
__device__ __forceinline__ RectHit rect_eval_test(const GT& g, const Ray6& r) {
  const float tt = plane_t(g.k0 - r.oa, r.ia);
  const float a = fmaf(r.db, tt, r.ob - g.ma), b = fmaf(r.dc, tt, r.oc - g.mb);
  const bool ia = fabsf(a) <= g.ha, ib = fabsf(b) <= g.hb;
  return RectHit{tt, (bool)((int)ia & (int)ib), a};
}
// A candidate at t with position pos can be the nearest hit at all: its key
// (bits(t) | 63) ^ (63 - pos) ranks below kKeyNone = bits(1e20) | 63, i.e. bits(t) <= kKeyNone for
// pos < 63 (one compare) and bits(t) < kKeyNone & ~63 for pos 63.
__device__ __forceinline__ bool key_valid(float t, uint32_t pos) {
  return pos < 63u ? __float_as_uint(t) <= kKeyNone : __float_as_uint(t) < (kKeyNone & ~63u);
}

template <class SP>
__device__ __forceinline__ float sphere_t(const SP& S, f3 o, f3 d) {
  // Sphere::intersect :229-239 in the reference's own form det = b^2 - op.op + r^2 (:233), as
  // fma(b, b, r^2 - op.op); nearest root beyond the fp32 epsilon. (Round 2: the cancellation-free
  // r^2 - |op - b d|^2 cost 2 more VALU per sphere: C5 at 256 spp 430.4 -> 406.5 ms.)
  const f3 op = mk(S.px - o.x, S.py - o.y, S.pz - o.z);
  const float bb = dot3(op, d);
  const float det = fmaf(bb, bb, S.rad2 - dot3(op, op));
  if (!(det >= 0.0f)) return -0.0f;  // no root: -0 ranks last (contract v5 key)
  // the root as det * rsq_nr2(det) (contract, oracle c_sphere): the IEEE sqrtf sequence costs ~18
  // issue slots, det * rsq_nr(det) 13 (round 2: C5 at 256 spp 452.8 -> 427.3 ms), two Newton steps
  // 10 (round 3: the root within 5e-6 relative, 3e-5 at r = 6, far below the 2e-3 epsilon);
  // det = 0 gives 0
  const float sd = det * rsq_nr2(det);
  const float t1 = bb - sd, t2 = bb + sd;
  return t1 > 2e-3f ? t1 : (t2 > 2e-3f ? t2 : -0.0f);
}

// A wide sphere (the 1e5 walls and the radius-600 light of the classic smallpt box) in fp64: the
// cancellation-free quadratic with explicit fma, IEEE double division and sqrt, the fp32 contract's
// epsilon; t rounded to float (oracle c_sphere_wide). The fp32-normalised direction is not exactly
// unit (|d|^2 = 1 + e, |e| ~ 1e-7), and a radius-1e5 quadratic that assumed |d| = 1 would carry an
// error e * b^2 ~ 1e3 in its discriminant (hit points off the wall by ~0.1: self-hits in rings), so
// the quadratic keeps a = d.d: t = k -+ sqrt(det / a), k = (op.d) / a, det = r^2 - |op - k d|^2.
__device__ __forceinline__ float sphere_t_wide(const SPT_CONST GeoSphD& S, f3 o, f3 d) {
  const double ox = S.px - (double)o.x, oy = S.py - (double)o.y, oz = S.pz - (double)o.z;
  const double dx = d.x, dy = d.y, dz = d.z;
  const double a = fma(dz, dz, fma(dy, dy, dx * dx));
  const double k = fma(oz, dz, fma(oy, dy, ox * dx)) / a;
  const double qx = fma(-k, dx, ox), qy = fma(-k, dy, oy), qz = fma(-k, dz, oz);
  const double det = S.rad2 - fma(qz, qz, fma(qy, qy, qx * qx));
  if (!(det >= 0.0)) return -0.0f;
  const double sd = sqrt(det / a);
  const double t1 = k - sd, t2 = k + sd;
  return (float)(t1 > 2e-3 ? t1 : (t2 > 2e-3 ? t2 : -0.0));
}
__device__ __forceinline__ float sphere_t_any(const SPT_CONST SceneGeo* G, int j, f3 o, f3 d) {
  if (G->sph[j].wide) return sphere_t_wide(G->sphd[j], o, d);  // wave-uniform (scalar load)
  return sphere_t(G->sph[j], o, d);
}

template <class TP>
__device__ __forceinline__ int n_of(int ct, int rt) { return ct >= 0 ? ct : rt; }

// The uploaded scene's rect tests are read from an LDS copy staged once per block (ds_read
// broadcasts into VGPRs) -- the north star's "geometry staged once into LDS". A/B (DESIGN.md
// section 4, round 2 at commit 407a07d): faster than scalar loads through the constant address
// space: generic kernel at C3 27.65 -> 26.26 ms, HEAD-topology kernel 19.1 -> 18.5 ms, C5 at
// 256 spp 460 -> 453.6 ms. Spheres stay on scalar loads (an LDS copy cost C5 1.4 %: four VGPRs per
// unrolled sphere). The HEAD scene itself runs with its bounds as instruction literals (15.5 ms).
// (the fp64 wide-sphere kernel keeps scalar loads: its VGPR budget is the tight one, 78 vs 90)
template <class TP>
__device__ __forceinline__ auto tests_of(const SPT_CONST SceneGeo* G, const GeoTest* lds) {
  constexpr bool kLds = !TP::WIDE;
  if constexpr (TP::CONSTGEO && !TP::UPBOX) {
    (void)G; (void)lds;
    return (const SPT_CONST GeoTest*)nullptr;  // the HEAD tests are literals (kCornellTests)
  } else if constexpr (kLds) {
    (void)G;
    return lds;
  } else {
    (void)lds;
    return G->test + 0;
  }
}
// The scene's room of contract v5 in uploaded geometry: SceneGeo.room_test[] (three GeoTests kept
// out of the per-kind test lists) and the box (host build_geo, oracle c_find_room).
template <class TP, bool COUNT_MISS = false, class GP, class GT, class SP>
__device__ __forceinline__ bool intersect_scene(const SPT_CONST SceneGeo* G, GP rect, GT tests,
                                                SP sphs, const int* pos2idx, f3 o, f3 d, int& id,
                                                float& ia_hit, int& pos_out, uint32_t& n_miss,
                                                f3& inv) {
  const float ix = rcp_nr(d.x), iy = rcp_nr(d.y), iz = rcp_nr(d.z);
  inv = mk(ix, iy, iz);
  uint32_t tmin = kKeyNone;
  if constexpr (TP::CONSTGEO) {
    const Ray6 rays[3] = {ray6<0>(o, d, ix, iy, iz), ray6<1>(o, d, ix, iy, iz),
                          ray6<2>(o, d, ix, iy, iz)};
    cornell_room(rays, tmin);
    if constexpr (TP::UPBOX) {
      // the uploaded HEAD-topology tests (host-checked: n_txy 0, n_txz 1, n_tyz 0): the light, the
      // room's three pairs (its XZ pair's k0 the floor), then the two boxes' three tests each. The
      // room is literal (HEAD's, host-checked), the boxes come from LDS, the light is literal or
      // (UPLIGHT) read through scalar loads from the uploaded scene
      if constexpr (TP::UPLIGHT) light_cand(G->test[0], rays[1], tmin);
      else cornell_tests(std::make_integer_sequence<int, kCornellTests.n>{}, rays, tmin);  // the light
      geo_box(tests + 4, tests + 2, rays[2], rays[1], rays[0], tmin);
      geo_box(tests + 7, tests + 2, rays[2], rays[1], rays[0], tmin);
    } else {
      cornell_tests(std::make_integer_sequence<int, kCornellTests.n>{}, rays, tmin);  // the light
      cornell_boxes(std::make_integer_sequence<int, kCornellBoxes.n>{}, rays, tmin);
    }
  } else {
    const int ntxy = n_of<TP>(TP::NTXY, G->n_txy), ntxz = n_of<TP>(TP::NTXZ, G->n_txz);
    const int ntyz = n_of<TP>(TP::NTYZ, G->n_tyz);
    const Ray6 rz = ray6<2>(o, d, ix, iy, iz), ry = ray6<1>(o, d, ix, iy, iz), rx = ray6<0>(o, d, ix, iy, iz);
    if (G->has_room) {  // wave-uniform; the room tests follow the per-kind lists, then the boxes
      const int nt = ntxy + ntxz + ntyz;
      geo_room(tests + nt, rz, ry, rx, tmin);
      const int nbox = n_of<TP>(TP::NBOX, G->n_box);
      for (int b = 0; b < nbox; ++b) geo_box(tests + nt + 3 + 3 * b, tests + nt + 1, rz, ry, rx, tmin);
    }
    test_group<TP::NTXY>(tests, ntxy, rz, tmin);
    test_group<TP::NTXZ>(tests + ntxy, ntxz, ry, tmin);
    test_group<TP::NTYZ>(tests + ntxy + ntxz, ntyz, rx, tmin);
  }
  (void)rect;
  if constexpr (TP::SPH) {
    const int nsph = G->n_sph, nnar = nsph - G->n_sph_wide, base = G->n_xy + G->n_xz + G->n_yz;
    // unrolled by 4 so the scalar loads of several spheres are issued before one wait; 4, not 8:
    // the 32 SGPRs of 8 spheres pushed the SGPR-capped sphere kernel to 65 VGPRs (7 waves/SIMD);
    // at 4 it has 63 (8 waves): C5 at 256 spp 475 -> 467 ms. By hand, remainder first: the key's
    // inline asm is convergent, and LLVM does not runtime-unroll a loop that holds convergent code.
    auto sph_key = [&](int j) { tmin = umin(tmin, key_s(sphere_t(sphs[j], o, d), (uint32_t)(base + j))); };
    int j = 0;
    for (; j < (nnar & 3); ++j) sph_key(j);
    for (; j < nnar; j += 4) {
      sph_key(j);
      sph_key(j + 1);
      sph_key(j + 2);
      sph_key(j + 3);
    }
    if constexpr (TP::WIDE) {
      for (int j = nnar; j < nsph; ++j)  // wide spheres (fp64)
        tmin = umin(tmin, key_s(sphere_t_wide(G->sphd[j], o, d), (uint32_t)(base + j)));
    }
  }
  const bool hit = tmin < kKeyNone;
  // COUNT_MISS: every lane's miss is a path ray's (a traced shadow ray always meets the light, whose
  // test in the trace is the pre-test's, bit for bit): counted here, where the compare is fresh
  if constexpr (COUNT_MISS) count_if(n_miss, tmin >= kKeyNone);
  int pos = (int)(tmin & 63u);  // (63 on a miss: a valid LDS index, the id is kept)
  // HEAD kernels: a miss reports the position of prim 0, whose id a missed path ray keeps (:373-374),
  // so the shading takes the hit's plane axis from the same two position compares as ia_hit
  if constexpr (TP::CONSTGEO) pos = hit ? pos : kCornellPosOfPrim0;
  // 1/d of the hit rectangle's plane axis (the winner's t and its hit point, see the shading)
  const int nxy = TP::CONSTGEO ? kCornellNXY : n_of<TP>(TP::NXY, G->n_xy);
  const int nxz = TP::CONSTGEO ? kCornellNXZ : n_of<TP>(TP::NXZ, G->n_xz);
  // (the HEAD kernels select it where it is used, from the shading's own plane-axis masks)
  if constexpr (!TP::CONSTGEO) ia_hit = pos < nxy ? iz : (pos < nxy + nxz ? iy : ix);
  // HEAD kernels: the kernel's primitive ids ARE the grouped positions (s_prims is loaded in that
  // order), so no pos -> index lookup; otherwise an unconditional LDS read (no branch)
  int idn;
  if constexpr (TP::CONSTGEO) idn = pos;
  else idn = keep(pos2idx[pos]);
  id = hit ? idn : id;
  pos_out = pos;
  return hit;
}

// The winner's exact t (contract v5: the t its key was made from), for a hit on prims[id] = H at
// grouped position pos: a rectangle's (k - o_a) * inv_a, a sphere's nearest root (sphere_t on the
// same fp32 values as the trace's GeoSph: DevPrim w1..w4 = px, py, pz, r^2), a wide sphere's fp64
// root.
template <class TP>
__device__ __forceinline__ float hit_t(const DevPrim& H, int pos, f3 o, f3 d, float ia,
                                       const SPT_CONST SceneGeo* G) {
  if (H.kind == SPT_RECT_XY) return plane_t(H.w1 - o.z, ia);
  if (H.kind == SPT_RECT_XZ) return plane_t(H.w1 - o.y, ia);
  if (H.kind == SPT_RECT_YZ) return plane_t(H.w1 - o.x, ia);
  if constexpr (TP::WIDE) {
    const int j = pos - (G->n_xy + G->n_xz + G->n_yz);
    if (j >= G->n_sph - G->n_sph_wide) return sphere_t_wide(G->sphd[j], o, d);
  }
  return sphere_t(GeoSph{H.w1, H.w2, H.w3, H.w4, 0, 0, 0, 0}, o, d);
}

// NEE pre-test (light_sampling :363-369 + the shadow ray of :466): is the light itself accepted
// on the ray (x, dl)? Only then can the nearest hit be the light (:467), so only these rays are
// traced against the scene. Bit-identical to the light's own test inside intersect_scene().
template <class TP, class GP>
__device__ __forceinline__ bool light_accepts(const SPT_CONST KParams* P, const SPT_CONST SceneGeo* G,
                                              GP rect, f3 o, f3 d) {
  if constexpr (TP::LPOS >= 0) {
    constexpr int L = TP::LPOS;  // compile-time kind from the grouped position
    static_assert(TP::NXY >= 0 && TP::NXZ >= 0, "LPOS needs static group sizes");
    if constexpr (L < TP::NXY) {
      const RectHit h = rect_eval(rect + L, Ray6{o.z, rcp_nr(d.z), d.x, o.x, d.y, o.y});
      return h.inb & key_valid(h.tt, L);
    } else if constexpr (L < TP::NXY + TP::NXZ) {
      const RectHit h = rect_eval(rect + L, Ray6{o.y, rcp_nr(d.y), d.x, o.x, d.z, o.z});
      return h.inb & key_valid(h.tt, L);
    } else {
      const RectHit h = rect_eval(rect + L, Ray6{o.x, rcp_nr(d.x), d.y, o.y, d.z, o.z});
      return h.inb & key_valid(h.tt, L);
    }
  } else {
    const int lk = P->light_kind, L = P->light_pos;
    if (L < 0) return false;
    const int nrect = G->n_xy + G->n_xz + G->n_yz;
    if (lk == SPT_SPHERE)  // (light_pos: the index in sph[]; its grouped position follows the rects)
      return key_valid(TP::WIDE ? sphere_t_any(G, L, o, d) : sphere_t(G->sph[L], o, d), (uint32_t)(nrect + L));
    Ray6 r;
    if (lk == SPT_RECT_XY) r = Ray6{o.z, rcp_nr(d.z), d.x, o.x, d.y, o.y};
    else if (lk == SPT_RECT_XZ) r = Ray6{o.y, rcp_nr(d.y), d.x, o.x, d.z, o.z};
    else r = Ray6{o.x, rcp_nr(d.x), d.y, o.y, d.z, o.z};
    const RectHit h = rect_eval(rect + L, r);
    return h.inb & key_valid(h.tt, (uint32_t)L);
  }
}

// Early NEE resolve (the HEAD NEE kernel: compile-time HEAD geometry, the reference's light
// constants, black light). A shadow ray (x, dl) whose light test accepts (t_L, crossing
// x_L = 50 + a) cannot meet any primitive before the light when x satisfies the conditions below,
// so intersect() (:323-335, oracle c_intersect) would return the light with t = t_L, bit for bit:
// the lane resolves it in the iteration that sampled it instead of tracing it in the next one.
//   * room: 1 <= x <= 99, 0 <= z <= 170, 0 <= y < 81.5. The room's slab candidate is then its exit
//     wall, never the one the vertex lies on (a vertex rounded outside its wall keeps its self-hit:
//     traced), and that wall lies >= 31 units beyond the light crossing in x (the light spans x
//     32..68), >= 63 in z (z 63..96); the ceiling is 0.1 above the light plane.
//   * short box (x, z in [63, 88], y <= 25): y >= 25 (the ray rises: the slab's y interval ends at
//     t <= 0, so the box's candidate is negative), or x <= 63 and x_L < 63 (x stays below 63 along
//     the segment but at its start; a vertex exactly on the x = 63 face has t = -2^-149 there;
//     x_L < 63 always holds below y = 25, see early_nee_proven).
//   * tall box (x in [12, 42], z in [32, 62], y <= 50): y >= 50, or z >= 62 (z stays at or above 62
//     along the segment -- the light's z >= 63 -- and reaches 62 only at t <= 0: the box's z slab
//     ends behind the origin). Round 4: >= and <= where rounds 2-3 kept a 0.01 margin; a vertex on
//     a box face often lies exactly on its plane: +8.5 % resolved shadow rays, 0 contradictions.
// Faces crossed beyond t_L fail their y bounds (y > 81.5 there) or lose to the light on t. The
// oracle restates the predicate and checks it against its own intersect() (spt_oracle_proof_*,
// tests/test_oracle.py); it covers ~77 % of the shadow rays that reach the light at C3.
__device__ __forceinline__ int early_room_ok(f3 x) {
  return (int)(__float_as_uint(x.x) - __float_as_uint(1.0f) <=
               __float_as_uint(99.0f) - __float_as_uint(1.0f)) &
         (int)(__float_as_uint(x.z) <= __float_as_uint(170.0f)) &
         (int)(__float_as_uint(x.y) < __float_as_uint(81.5f));  // +0 <= v: no sign bit
}
// Sphere scenes in the HEAD room (the sphere NEE kernel, C5): with every sphere's top below
// y0 - 1, a vertex above y0 whose shadow ray goes up (dl.y > 0) cannot meet a sphere for t > 0:
// the real intersections lie at t <= -1, and the fp32 quadratic's rounding (|det| error < 0.02
// for |op| < 200) cannot lift a root above the 2e-3 epsilon. The room as above.
__device__ __forceinline__ bool early_room_proven(f3 x, float y0) {
  return (early_room_ok(x) & (int)(x.y > y0)) != 0;
}
// (Round 4: the short box's "x_L < 63" is implied below y = 25: the reference's wrapped light
// samples lie at x in [31, 33), and the crossing of y = 81.5 lies within 0.1 / (81.6 - y) < 0.0018
// of the way back to the vertex, so x_L < 33.2 there. One compare fewer; the same predicate.)
// The same proof for an edited rect[] of the HEAD topology (the uploaded-geometry kernels; round 6:
// the room and the light may be edited as well): the vertex in the room's box below the light plane
// (early_room_ok_k: the room's exit face lies beyond the light crossing, the host checks the light's
// margins to the walls and the ceiling), each box standing on the floor >= 0.5 below the light
// plane with a clause the host picks from the reference's wrapped light samples (x in [31, 33),
// z in [62, 64), y 81.6; the light plane at most 81.5, so the crossing lies on the segment to the
// sample): a box with x0 >= 33 is clear for a vertex with x <= x0 (the segment to the light stays at
// x <= x0) -- the HEAD short box's clause --, x1 <= 31 for x >= x1, z0 >= 64 for z <= z0, z1 <= 62
// for z >= z1 (the HEAD tall box's); and every box for a vertex at or above its top.
// The oracle restates the choice (c_find_early_clauses) and checks every claim (test_oracle.py).
// The room clause of an edited scene (room and light from KParams, host early_geo_setup): the same
// compares as early_room_ok with the bounds in SGPRs.
__device__ __forceinline__ int early_room_ok_k(f3 x, const SPT_CONST KParams* P) {
  return (int)(__float_as_uint(x.x) - P->er_lo[0] <= P->er_span[0]) &
         (int)(__float_as_uint(x.y) - P->er_lo[1] <= P->er_span[1]) &
         (int)(__float_as_uint(x.z) - P->er_lo[2] <= P->er_span[2]);
}
// ROOM: 0 = the literal HEAD room and light plane (early_room_ok; the boxes-only-uploaded kernels),
// 1 = the literal room with the light plane's bound from KParams (UPLIGHT), 2 = everything from
// KParams (the uploaded-geometry kernels)
template <int ROOM>
__device__ __forceinline__ bool early_geo_proven(f3 x, const SPT_CONST KParams* P) {
  int ok;
  if constexpr (ROOM == 0) {
    ok = early_room_ok(x);
  } else if constexpr (ROOM == 1) {
    ok = (int)(__float_as_uint(x.x) - __float_as_uint(1.0f) <= __float_as_uint(99.0f) - __float_as_uint(1.0f)) &
         (int)(__float_as_uint(x.z) <= __float_as_uint(170.0f)) & (int)(__float_as_uint(x.y) < P->ul_ybits);
  } else {
    ok = early_room_ok_k(x, P);
  }
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const float v = P->eb_z[b] ? x.z : x.x;
    ok &= (int)(x.y >= P->eb_top[b]) | (int)(v * P->eb_sgn[b] <= P->eb_bnd[b]);
  }
  return ok != 0;
}
__device__ __forceinline__ bool early_nee_proven(f3 x) {
  const int room = early_room_ok(x);
  const int short_box = (int)(x.y >= 25.0f) | (int)(x.x <= 63.0f);
  const int tall_box = (int)(x.y >= 50.0f) | (int)(x.z >= 62.0f);
  return (room & short_box & tall_box) != 0;
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

// The hit point's plane distance (n / d_a of :103, n = k - o_a), as one Markstein correction of the
// trace's t = n * rcp_nr(d_a) (oracle c_hit_t): r = n - t*d_a exactly (fma), t + r * rcp. Equal to
// the IEEE quotient in all of 2e8 sampled cases; the contract spells it out so CPU and GPU agree
// by construction.
__device__ __forceinline__ float hit_plane_t(float n, float da, float ia, float t) {
  return fmaf(fmaf(-t, da, n), ia, t);
}
// n / d of the contract where it only weights a sample (the NEE pdf; oracle c_div): n * rcp_nr(d).
__device__ __forceinline__ float div_nr(float n, float d) { return n * rcp_nr(d); }

// PDF_inverse * BRDF of :471-472 for a NEE shadow ray (x, d) whose nearest hit is the light at t
// (oracle c_nee_weight). Unit directions: |area d.y / t^2| |d.nl / pi| as written. Free-scale: d is
// light_vec (:367) itself, not normalised; with dl = d/|d| and the distance t|d| the same quantity
// is (area/pi) |d.y| |d.nl| / (t^2 (d.d)^2): no square root, and the normalize of the shadow
// direction (18 VALU per vertex) is gone.
__device__ __forceinline__ float nee_weight(bool unit, f3 d, f3 nl, float t, float larea, float nee_c) {
  if (unit) {
    const float pdf = fabsf(div_nr(larea * d.y, t * t));            // :471
    const float brdf = fabsf(dot3(d, nl) * 0.318309886183790672f);  // :472
    return pdf * brdf;
  }
  const float num = fabsf(d.y) * fabsf(dot3(d, nl));
  const float vv = dot3(d, d);
  return (num * nee_c) * rcp_nr((t * t) * (vv * vv));
}
constexpr float kRefNeeC = (float)(1296.0 / 3.14159265358979323846);  // kRefLarea / pi

// The camera ray of contract v5 (oracle c_path, :533-536): per component c
//   v_c = fma(Fv, Cv_c, fma(Fu, Cu_c, P_c)),  Fu = 2^23 + ju, Fv = 2^23 + jv,
// with ju, jv the 16-bit jitter draws (the float with bits 0x4B000000 | j is 2^23 + j exactly),
// Cu_c = hor_c (1/w) 2^-16, Cv_c = ver_c (1/h) 2^-16 per launch and the per-pixel
// P_c = fma(Au_c, fx, fma(Av_c, fy, llc_c - origin_c)), Au_c = hor_c (1/w), Av_c = ver_c (1/h),
// fx = (x - 0.5) - 128, fy = (h - y - 1 - 0.5) - 128 (the -128 cancels 2^23 2^-16 in Fu Cu).
// The axis-aligned camera kernels keep P_x, P_y per work unit: one fma per component per ray
// (rounds 1-4: the jitter sum, a scale, an fma and a subtract per component).
__device__ __forceinline__ float jitter_f(uint32_t lo, uint32_t hi) {
  return __uint_as_float(u16i(lo, hi) | 0x4B000000u);
}

__device__ __forceinline__ uint32_t div_magic(uint32_t n, uint32_t m, uint32_t sh) {
  return (uint32_t)(((uint64_t)n * m) >> sh);
}

// A local pixel index (row-tile shard order) -> the Philox pixel key and camera raster terms.
__device__ __forceinline__ void pixel_terms(const SPT_CONST KParams* Q, uint32_t lp, PxKey& pk,
                                            float& fx, float& fy) {
  const uint32_t w = (uint32_t)Q->width;
  const uint32_t lr = div_magic(lp, Q->m_w, Q->sh_w);
  const int px = (int)(lp - lr * w);
  const uint32_t T_ = (uint32_t)Q->tile_rows;
  const uint32_t tile = div_magic(lr, Q->m_tile, Q->sh_tile), within = lr - tile * T_;
  const int py = (int)((tile * (uint32_t)Q->shard_count + (uint32_t)Q->shard_index) * T_ + within);
  pk = philox_pixel_key((uint32_t)py * w + (uint32_t)px, Q->seed);
  // camera raster terms (x - 0.5), (h - y - 1 - 0.5) of :533-534, less 128 (jitter_fma)
  fx = ((float)px - 0.5f) - 128.0f;
  fy = ((float)(Q->height - py - 1) - 0.5f) - 128.0f;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// A unit index -> its (spread) local pixel, as the refill maps it (chunk-major units, pixel order
// spread by scr_k).
__device__ __forceinline__ uint32_t unit_pixel(const SPT_CONST KParams* Q, uint32_t u) {
  const uint32_t r = u - div_magic(u, Q->m_npix, Q->sh_npix) * (uint32_t)Q->n_local_pix;
  return (r & ((1u << Q->scr_k) - 1u)) * Q->scr_q + (r >> Q->scr_k);
}

// One lane = one pixel-sample path at a time, and every iteration traces exactly ONE ray per lane
// with the same nearest-hit loop (intersect :323-335): either the path ray toward the next vertex
// or, after a NEE event whose light sample passes light_accepts(), the shadow ray of :466. The
// wave never runs an occlusion test for lanes that have none (the light pre-test rejects ~75% of
// the NEE samples at HEAD); a lane whose shadow ray is pending simply skips the ray-generation and
// shading blocks of that iteration. Per lane the arithmetic is exactly the counter-mode contract
// (oracle c_path): only the schedule differs.
//   iteration: [refill idle lanes] -> [generate: cosine continuation and camera ray, one Philox
//   call, shared normalize] -> [trace] -> [resolve a shadow ray] -> [shade a vertex: RR, NEE
//   pre-test] -> [path end: accumulate; retire the unit after its last sample].
// The lane state is one VGPR word (kSt*) and the small blocks are branch-free: the loop is bound
// by instruction issue, and LLVM's exec-mask bookkeeping for loop-carried booleans and short
// branches was SALU work on the CU's single scalar unit.
template <class TP, class CF>
// SGPRs capped at 80: with 81-96 SGPRs a CU admits only 7 blocks of 256 threads, not the 8 that the
// compiler's occupancy report and hipOccupancyMaxActiveBlocksPerMultiprocessor() claim (MI355X_MICROARCH
// "256-thread blocks are admitted per CU up to min(API, 8, floor(800 / (ceil(sgpr/16)*16 + 16)))";
// measured here with per-wave start times: the 8th block of every CU started only when the first
// ones retired; C3 16.2 -> 16.0 ms, C2 4.77 -> 4.60 ms). Under the cap the occupancy API is exact.
#ifndef SPT_NUM_SGPR
#define SPT_NUM_SGPR 80
#endif
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_num_sgpr(SPT_NUM_SGPR)))
// The sphere kernels and the estimator-specialised rect kernels allocate for 8 waves/SIMD
// explicitly: the sphere NEE kernel otherwise takes 65 VGPRs (7 waves), the HEAD NEE kernel 65 with
// the round-2 Philox key (philox_pixel_key), the uploaded-geometry HEAD-topology ones 65; with the
// hint all fit 64 with no spills
__attribute__((amdgpu_waves_per_eu((TP::SPH && !TP::MAT && !TP::WIDE) || (!TP::SPH && !TP::MAT && CF::NEE >= 0) ? 8 : 1)))
render_kernel(const KParams* __restrict__ Pg) {
  __shared__ DevPrim s_prims[kMaxPrims];
  __shared__ int s_pos2idx[kMaxPrims];  // grouped position -> primitive index
  __shared__ GeoTest s_test[(TP::CONSTGEO && !TP::UPBOX) || TP::WIDE ? 1 : kMaxPrims];
  // Pending REFR refraction children (:494-495 at depth <= 2), two per lane at most (MAT only):
  // o, d, T, depth, branch.
  struct Node { float o[3], d[3], T[3]; int depth; uint32_t branch; };
  __shared__ Node s_stack[TP::MAT ? kBlock * 2 : 1];
  // Sphere vertices shaded, per wave (SPH only). They are counted inside the divergent shading
  // block, where a wave-uniform register would turn per-lane (a ballot there sees only the active
  // lanes); one LDS add per wave (the atomic optimizer folds the lanes) keeps it out of the VGPRs.
  __shared__ uint32_t s_nsph[TP::SPH ? kBlock / 64 : 1];
  if (TP::SPH && threadIdx.x < kBlock / 64) s_nsph[threadIdx.x] = 0;
  // Shadow rays resolved early, per wave, in the sphere kernels (same reason: no VGPR counter)
  __shared__ uint32_t s_nearly[TP::SPH ? kBlock / 64 : 1];
  if (TP::SPH && threadIdx.x < kBlock / 64) s_nearly[threadIdx.x] = 0;
  {
    const SPT_CONST KParams* P = cptr(Pg);
    const SPT_CONST SceneGeo* G = cptr(P->geo);
    const int nrect = G->n_xy + G->n_xz + G->n_yz;
    for (int i = threadIdx.x; i < P->n_prims; i += kBlock) {
      // HEAD geometry (every primitive a rectangle): s_prims by grouped position (kPosIds)
      s_prims[i] = P->prims[TP::CONSTGEO ? G->rect[i].idx : i];
      s_pos2idx[i] = i < nrect ? G->rect[i].idx : G->sph[i - nrect].idx;
      if ((!TP::CONSTGEO || TP::UPBOX) && !TP::WIDE && i < G->n_txy + G->n_txz + G->n_tyz + 3 * G->has_room + 3 * G->n_box) {
        const SPT_CONST GeoTest& q = G->test[i];
        s_test[i] = GeoTest{q.k0, q.k1, q.ma, q.ha, q.mb, q.hb, q.pos0, q.pos1};
      }
    }
  }
  __syncthreads();

  const uint32_t lane = __lane_id();
  // ---- per-lane state
  // The lane's state is ONE integer in a VGPR (kSt*), not a set of booleans: LLVM keeps loop-carried
  // booleans as 64-bit lane masks and merges each one at every join of the divergent blocks with an
  // s_andn2/s_and/s_or triple, and SALU issue bounds this loop (one scalar unit per CU; a marginal
  // SALU instruction costs ~3x a marginal VALU one here). A VGPR state is
  // written under exec and needs no merge.
  uint32_t ls = kStIdle;
  uint32_t branch = 0;    // path-tree position of a REFR split (counter word 2 bits 24+; MAT only)
  int sp = 0;             // pending refraction children in s_stack (MAT only)
  uint32_t lp = 0, s = 0, s_end = 0;
  PxKey pk = PxKey{0, 0, 0};  // Philox round-1/2 terms of the unit's pixel (philox_pixel_key)
  // dp1: vertices of the current path so far plus one (1 until its first) -- the Philox vertex
  // counter of the ray generated next, with no add per call
  int dp1 = 1, vid = 0;
  // camera raster terms of the unit's pixel, fx = (x - 0.5) - 128, fy = (h - y - 1 - 0.5) - 128;
  // the axis-aligned camera kernels hold P_x, P_y (jitter_f) here instead
  float fx = 0.0f, fy = 0.0f;
  float fz = 0.0f;  // CAMAX 2: P_z (fx, fy hold P_x, P_y)
  unsigned long long acc0 = 0, acc1 = 0, acc2 = 0;
  // o starts at the camera (the first ray of every sample is a camera ray; the path end resets it)
  f3 o = mk(cptr(Pg)->cam[0], cptr(Pg)->cam[1], cptr(Pg)->cam[2]);
  f3 d = mk(0, 0, 1), T = mk(1, 1, 1), L = mk(0, 0, 0), nl = mk(0, 1, 0);
  float w_nee = 0.0f;  // HEAD NEE kernel: the NEE weight of the lane's shadow ray, from its vertex
  u4 r = u4{0, 0, 0, 0};  // Philox words of the vertex the pending path ray leads to
  // ---- wave-uniform state
  // Camera and fixed-point constants of the axis-aligned camera kernels, loaded once and held in
  // SGPRs (each scalar reload in the loop is a wait for the wave).
  struct CamK { float o0, o1, o2, aux, avy, cux, cvy, lx, ly, lz, fs; };
  CamK ck{};
  if constexpr (CF::CAMAX == 1) {
    const SPT_CONST KParams* C = cptr(Pg);
    ck = CamK{C->cam[0], C->cam[1], C->cam[2], C->cam_au[0], C->cam_av[1], C->cam_cu[0],
              C->cam_cv[1], C->cam_l[0], C->cam_l[1], C->cam_l[2], C->fix_scale};
  }
  // CAMAX 2 (any camera): origin, Cu, Cv and the fixed-point scale in SGPRs (Au, Av, L are read at
  // the refill only)
  struct CamG { float o0, o1, o2, cu0, cu1, cu2, cv0, cv1, cv2, fs; };
  CamG cg{};
  if constexpr (CF::CAMAX == 2) {
    const SPT_CONST KParams* C = cptr(Pg);
    cg = CamG{C->cam[0], C->cam[1], C->cam[2], C->cam_cu[0], C->cam_cu[1], C->cam_cu[2],
              C->cam_cv[0], C->cam_cv[1], C->cam_cv[2], C->fix_scale};
  }
  uint32_t pool_next = 0, pool_end = 0, grab_at = 0;  // grab_at: the wave's last queue position
  bool exhausted = false, capped = false;
  // Wave-uniform event counters (SGPRs), fed by ballots at convergent points of the loop: per-lane
  // counters incremented inside the divergent blocks cost ~40 VGPRs of copies.
  // (vertices = path rays + NEE light hits: every path ray shades a vertex, hit or miss, and a
  // shadow ray that reaches the light shades the light's)
  uint32_t n_path = 0, n_cos = 0;
  // Per-lane counts of events that happen inside divergent blocks, incremented in place and
  // summed once at the end (a boolean per event carried to a convergent ballot cost 3 VALU each).
  // NEE events need no counter in the HEAD NEE kernels: with NEE always on and no SPEC/REFR, every
  // non-terminal vertex takes one (nee_events = vertices - samples, added by the host).
  constexpr bool kNeeByIdentity = CF::NEE == 1 && !TP::MAT;
  // Early NEE resolve (early_nee_proven): the HEAD NEE kernel only. The shadow-ray resolve then
  // runs after the shading block, for the rays traced in this iteration and the proven ones.
  constexpr bool kEarlyNee = TP::CONSTGEO && !TP::MAT && !TP::SPH && CF::NEE == 1 &&
                             CF::BLACK == 1 && CF::LREF == 1 && CF::MAXD0 == 1;
  // The sphere NEE kernel (C5): the same early resolve with the sphere-scene predicate.
  constexpr bool kEarlySph = !kEarlyNee && TP::SPH && !TP::MAT && !TP::WIDE && CF::NEE == 1 &&
                             CF::BLACK == 1 && CF::LREF == 1;
  // The uploaded-geometry HEAD-topology NEE kernel (an edited rect[]): early_geo_proven.
  constexpr bool kEarlyGeo = !kEarlyNee && !TP::SPH && !TP::MAT && TP::NBOX == 2 && CF::NEE == 1 &&
                             CF::BLACK == 1 && CF::LREF == 1 && CF::MAXD0 == 1;
  constexpr bool kEarly = kEarlyNee || kEarlySph || kEarlyGeo;
  uint32_t l_early = 0;  // shadow rays resolved early (stats[kStatShadowProven])
  uint32_t l_miss = 0, l_nee = 0, l_hit = 0;
  // Shadow rays traced (NEE samples that passed light_accepts()): per lane in the rect kernels,
  // wave-uniform in the sphere kernels (a ballot of the kStShadow lanes at the convergent point
  // before the trace), whose VGPR budget is the tighter one.
  uint32_t l_shadow = 0;
#ifdef SPT_REGION_STATS
  uint32_t reg_exec[kRegions] = {}, reg_lanes[kRegions] = {};
  uint32_t reg_flags = 0;
#endif

#ifdef SPT_WAVE_TIMES  // diagnostic build: per-wave residency (100 MHz real-time counter)
  const unsigned long long wave_t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t wave_iters = 0;
#endif
  for (uint32_t iter = 0;; ++iter) {
#ifdef SPT_WAVE_TIMES
    wave_iters = iter;
#endif
    const SPT_CONST KParams* P = cptr(Pg);
    SPT_REGION(0);  // loop iteration
    if (__builtin_expect(iter >= kMaxWaveIters, 0)) {  // runaway guard: drop the work, leave
      capped = true;                // through the normal exit (a second loop exit would duplicate
      exhausted = true;             // the loop state)
      ls = kStIdle;
    }
    // 1) (a unit is retired at the end of its last sample, in the path-end block below)
    // 2) refill idle lanes from the wave's pool (ballot + mbcnt prefix sum), pool from the queue.
    //    Everything up to the loop exit test runs only when some lane is idle: most iterations
    //    skip it with one wave-uniform branch (round 4: the loop-head bookkeeping was ~12 SALU per
    //    iteration when no lane needed a unit).
    uint64_t need = __ballot(ls == kStIdle);
    if (need != 0) {
    bool needs_unit = ls == kStIdle;
    while (need != 0 && !exhausted) {
      SPT_REGION(2);
      const SPT_CONST KParams* Q = cptr(Pg);
      if (pool_next >= pool_end) {
        uint32_t want = kGrab;
        if (Q->sh_guided < 32u) {
          const uint32_t left = Q->n_units - min(grab_at, (uint32_t)Q->n_units);
          want = min(kGrab, max(max((uint32_t)__popcll(need), kGrabMin), left >> Q->sh_guided));
        }
        // a young block's wave (SPT_YOUNG_CUT) past the cut takes no new pool: its lanes finish and
        // split what they hold (in-wave stealing) and the wave leaves
        if (blockIdx.x >= Q->young_block) {
          uint32_t q = 0;
          if (lane == 0) q = __hip_atomic_load(Q->queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          q = __builtin_amdgcn_readfirstlane(q);
          if (q >= Q->young_cut) { exhausted = true; break; }
        }
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(Q->queue, want);
        b = __builtin_amdgcn_readfirstlane(b);
        grab_at = b + want;
        if (b >= Q->n_units) { exhausted = true; break; }
        pool_next = b;
        pool_end = min(b + want, Q->n_units);
      }
      const uint32_t rank = lane_rank(need);
      const uint32_t avail = pool_end - pool_next;
      if (needs_unit && rank < avail) {
        const uint32_t u = pool_next + rank;
        const uint32_t npix = (uint32_t)Q->n_local_pix;
        const uint32_t j = div_magic(u, Q->m_npix, Q->sh_npix);  // chunk-major
        lp = u - j * npix;
        // Spread the pixel order (scr_k > 0): unit pixel lp = b * K + a -> a * (npix / K) + b, so a
        // wave's run of consecutive units samples the whole image instead of one row segment, and
        // per-wave work varies less (the image does not change: every pixel-sample is still done
        // once and summed in integers)
        lp = (lp & ((1u << Q->scr_k) - 1u)) * Q->scr_q + (lp >> Q->scr_k);
        s = j * (uint32_t)Q->chunk;
        s_end = min(s + (uint32_t)Q->chunk, (uint32_t)Q->spp);
        pixel_terms(Q, lp, pk, fx, fy);
        if constexpr (CF::CAMAX == 1) {  // the per-pixel P_x, P_y of the camera ray (jitter_f)
          fx = fmaf(ck.aux, fx, ck.lx);
          fy = fmaf(ck.avy, fy, ck.ly);
        } else if constexpr (CF::CAMAX == 2) {  // P_c = fma(Au_c, fx, fma(Av_c, fy, L_c)), c = x, y, z
          const float rx = fx, ry = fy;
          fx = fmaf(Q->cam_au[0], rx, fmaf(Q->cam_av[0], ry, Q->cam_l[0]));
          fy = fmaf(Q->cam_au[1], rx, fmaf(Q->cam_av[1], ry, Q->cam_l[1]));
          fz = fmaf(Q->cam_au[2], rx, fmaf(Q->cam_av[2], ry, Q->cam_l[2]));
        }
        lp = u | 0x80000000u;  // the owner keeps its unit index: the sums go to the unit's slot
        ls = kStCam;
        needs_unit = false;
      }
      pool_next += min((uint32_t)__popcll(need), avail);
      need = __ballot(needs_unit);
    }
    // 2b) the queue is dry: an idle lane takes the upper half of a busy lane's unstarted samples
    //     (same pixel; each flushes its own sums and the accumulation is integer, so the image is
    //     unchanged). A wave's tail is then ~one path instead of ~one unit. Pairs are made by a
    //     scalar loop over the lane masks (readlane + a per-lane select), only in the tail.
    if (exhausted) {
      uint64_t idle = __ballot(ls == kStIdle);
      if (idle != 0) {
        const uint32_t cur = s + (ls == kStCam ? 0u : 1u);  // first unstarted sample
        // donors: lanes with more unstarted samples than the one they start next, and at least
        // steal_min of them (every stolen range flushes its own sums: memory-side atomics)
        const uint32_t smin = cptr(Pg)->steal_min;
        uint64_t dm = __ballot(ls != kStIdle && s_end > cur + (ls == kStCam ? 1u : 0u) &&
                               s_end >= cur + smin);
        while (idle != 0 && dm != 0) {
          const int il = __builtin_ctzll(idle), dl = __builtin_ctzll(dm);
          idle &= idle - 1;
          dm &= dm - 1;
          const uint32_t dcur = (uint32_t)__builtin_amdgcn_readlane((int)cur, dl);
          const uint32_t dend = (uint32_t)__builtin_amdgcn_readlane((int)s_end, dl);
          const uint32_t mid = dcur + (dend - dcur) / 2u;  // donor keeps [.., mid), taker [mid, dend)
          uint32_t d_lp = (uint32_t)__builtin_amdgcn_readlane((int)lp, dl);
          if (d_lp >> 31)  // an owner donor holds its unit index: the taker adds by pixel
            d_lp = unit_pixel(cptr(Pg), d_lp & 0x7FFFFFFFu);
          const uint32_t d_qhi = (uint32_t)__builtin_amdgcn_readlane((int)pk.qhi, dl);
          const uint32_t d_qlo = (uint32_t)__builtin_amdgcn_readlane((int)pk.qlo, dl);
          const uint32_t d_lo = (uint32_t)__builtin_amdgcn_readlane((int)pk.lo, dl);
          const float d_fx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fx), dl));
          const float d_fy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fy), dl));
          float d_fz = 0.0f;
          if constexpr (CF::CAMAX == 2) d_fz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fz), dl));
          const bool tk = lane == (uint32_t)il;  // the taker
          s_end = tk ? dend : (lane == (uint32_t)dl ? mid : s_end);
          s = tk ? mid : s;
          lp = tk ? d_lp : lp;
          pk.qhi = tk ? d_qhi : pk.qhi;
          pk.qlo = tk ? d_qlo : pk.qlo;
          pk.lo = tk ? d_lo : pk.lo;
          fx = tk ? d_fx : fx;
          fy = tk ? d_fy : fy;
          if constexpr (CF::CAMAX == 2) fz = tk ? d_fz : fz;
          ls = tk ? kStCam : ls;
        }
      }
    }
    if (__ballot(ls != kStIdle) == 0) break;
    }
    n_cos += (uint32_t)__popcll(__ballot(ls == kStCos));

    // 3) generate the path ray (kStCam, kStCos, kStSpec): the cosine continuation from the last
    //    vertex (random_scattering :337-347, its xi from that vertex's Philox words) or the camera
    //    ray of a new sample (:533-536, jitter from the low bytes of vertex 1's words), one Philox
    //    call for the vertex the ray leads to, one normalize for both. Both directions are computed
    //    for every generating lane and selected: a wave nearly always holds lanes of both kinds, so
    //    branches would save no VALU and cost their exec-mask SALU.
    if (ls - kStCam < 3u) {
      const bool cam = ls == kStCam;
      if (ls != kStSpec) SPT_REGION(cam ? 3 : 8);
      const bool unit = unit_dirs_of<TP>(Pg);
      f3 v = cosine_vec<!TP::SPH>(nl, r.z, r.w, TP::MAT && cptr(Pg)->scatter_uniform != 0, unit);
      // the vertex this ray leads to: dp1 (1 for a new sample's camera ray)
      const uint32_t ctr2 = (uint32_t)dp1 | (TP::MAT ? branch << 24 : 0u);
      r = philox_px(pk, s, ctr2);
      {
        const SPT_CONST KParams* C = cptr(Pg);
        f3 vc;
        const float Fu = jitter_f(r.x, r.y), Fv = jitter_f(r.z, r.w);
        if constexpr (CF::CAMAX == 1) {
          // the zero terms vanish exactly: fma(F, +-0, y) == y and fma(+-0, f, L) == L for the
          // nonzero y, L the host checks (cam_axis)
          vc = mk(fmaf(Fu, ck.cux, fx), fmaf(Fv, ck.cvy, fy), ck.lz);
        } else if constexpr (CF::CAMAX == 2) {  // the general form with P_c per unit
          vc = mk(fmaf(Fv, cg.cv0, fmaf(Fu, cg.cu0, fx)), fmaf(Fv, cg.cv1, fmaf(Fu, cg.cu1, fy)),
                  fmaf(Fv, cg.cv2, fmaf(Fu, cg.cu2, fz)));
        } else {
          float vv[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const float Pc = fmaf(C->cam_au[c], fx, fmaf(C->cam_av[c], fy, C->cam_l[c]));
            vv[c] = fmaf(Fv, C->cam_cv[c], fmaf(Fu, C->cam_cu[c], Pc));
          }
          vc = mk(vv[0], vv[1], vv[2]);
        }
        v = mk(cam ? vc.x : v.x, cam ? vc.y : v.y, cam ? vc.z : v.z);  // o: set at the path end
      }
      const f3 dn = normalize_dir(v, unit);  // rsq_nr1 in the free-scale contract (v7)
      if constexpr (TP::MAT) {  // a SPEC/REFR direction is set already
        const bool kd = ls == kStSpec;
        d = mk(kd ? d.x : dn.x, kd ? d.y : dn.y, kd ? d.z : dn.z);
      } else {
        d = dn;
      }
      ls = kStPath;
    }

    // Path rays: counted here by the generic kernel only. Without SPEC/REFR every path ray is a
    // sample's camera ray or a cosine continuation, so the others add n_cos + samples at the end.
    if constexpr (TP::MAT) n_path += (uint32_t)__popcll(__ballot(ls == kStPath));
    if constexpr (TP::SPH) l_shadow += (uint32_t)__popcll(__ballot(ls == kStShadow));
    if (ls >= kStPath) {  // kStPath or kStShadow
      // 4) trace the lane's ray (path ray: hittingPoint :371-377; shadow ray: :466).
      SPT_REGION(4);
#ifdef SPT_PROBE_SALU  // diagnostic build SPT_DIAG=3: N extra SALU per wave-iteration (issue cost)
      { uint32_t z_ = iter; asm volatile(".rept " SPT_XSTR(SPT_PROBE_SALU) "\n s_add_u32 %0, %0, 1\n .endr" : "+s"(z_)); }
#endif
#ifdef SPT_PROBE_VALU  // diagnostic build SPT_DIAG=4: N extra VALU per wave-iteration
      { float z_ = o.x; asm volatile(".rept " SPT_XSTR(SPT_PROBE_VALU) "\n v_add_f32 %0, 1.0, %0\n .endr" : "+v"(z_)); }
#endif
      const SPT_CONST SceneGeo* G = TP::CONSTGEO && !TP::UPLIGHT ? nullptr : cptr(P->geo);
      // intersect() leaves id untouched on a miss (:323-335): a shadow ray keeps its vertex's id. The
      // early-resolve HEAD kernel needs no vertex id: its light is black, so no vertex on the light
      // takes a NEE sample, and a missed shadow ray's id (prim 0's) is not the light's either way.
      int id = (!kEarlyNee && ls == kStShadow) ? vid : 0;
      float t = 0.0f, ia_hit = 0.0f;
      int hpos;
      f3 inv;  // 1/d per axis (rcp_nr), the trace's
      // (the early-resolve kernels trace a shadow ray only when the light accepts it: it never misses)
      bool hit = intersect_scene<TP, kEarly>(G, rects_of<TP>(G), tests_of<TP>(G, s_test), G->sph, s_pos2idx,
                                             o, d, id, ia_hit, hpos, l_miss, inv);
      if constexpr (TP::CONSTGEO)
        ia_hit = hpos < kCornellNXY ? inv.z : (hpos < kCornellNXY + kCornellNXZ ? inv.y : inv.x);

      // 5) resolve a shadow ray: the light is reached iff the nearest hit is the light (:467). Then
      //    the light is the next vertex (shaded in the common block below, T = T*f*weight); else the
      //    cosine sample follows (:468-469, T = T*f). The weight is computed for every shadow lane
      //    and applied as T*1 (exact) where the light is not reached: no branch. (The HEAD NEE
      //    kernel resolves in 5') below instead, after the shading block.)
      const bool traced_shadow = ls == kStShadow;
      if (!kEarly && ls == kStShadow) {
        SPT_REGION(6);
        const SPT_CONST KParams* D = cptr(Pg);
        const bool lh = id == light_slot_of<TP, CF>(D);
        if (lh) SPT_REGION(7);
        count_if(l_hit, lh);
        if constexpr (!TP::SPH) ++l_shadow;
        const float larea = CF::LREF == 1 ? kRefLarea : D->larea;
        const float nee_c = CF::LREF == 1 ? kRefNeeC : D->nee_c;
        t = hit_t<TP>(s_prims[id], hpos, o, d, ia_hit, G);  // the light's t (the winner's)
        const float w = lh ? nee_weight(unit_dirs_of<TP>(Pg), d, nl, t, larea, nee_c) : 1.0f;
        T = mk(T.x * w, T.y * w, T.z * w);  // T holds T*f of the shading vertex
        // A black light (HEAD :294) ends the path there by RR with p == 0 (:448-453) without a
        // random draw; anything else is shaded with that vertex's own Philox words.
        if (CF::BLACK != 1 && lh && !(hit && s_prims[id].pmax == 0.0f))
          r = philox_px(pk, s, (uint32_t)dp1 | (TP::MAT ? branch << 24 : 0u));
        ls = lh ? kStPath : kStCos;
      }

      // 6) shade a vertex (:422, :444-480).
      if (ls == kStPath) {
        SPT_REGION(5);
        const DevPrim& H = s_prims[id];
        const int kind = H.kind;
        f3 x;
        f3 gn = mk(0, 0, 0);
        bool ax_xy = false, ax_xz = false;  // the normal's axis (rect-only kernels)
        if constexpr (!TP::SPH) {
          // Rect-only scenes, branch-free: the plane axis of the hit kind selects (o_a, d_a); the
          // hit point re-derives t = (k - o_a) / d_a as the reference does (:103) and
          // the normal is the axis, oriented against the ray (:123,:166,:209).
          bool kxy, kxz;
          if constexpr (TP::CONSTGEO) {  // the axis from the position (intersect_scene)
            kxy = hpos < kCornellNXY;
            kxz = !kxy && hpos < kCornellNXY + kCornellNXZ;
          } else {
            kxy = kind == SPT_RECT_XY;
            kxz = kind == SPT_RECT_XZ;
          }
          ax_xy = kxy;
          ax_xz = kxz;
          const bool kyz = !kxy && !kxz;
          const float oa = kxy ? o.z : (kxz ? o.y : o.x);
          const float da = kxy ? d.z : (kxz ? d.y : d.x);
          const float n_ = H.w1 - oa;
          float ia = ia_hit;
          if constexpr (TP::CONSTGEO) ia = kxy ? inv.z : (kxz ? inv.y : inv.x);  // (= ia_hit)
          const float tr = hit_plane_t(n_, da, ia, plane_t(n_, ia));  // the winner's t, corrected
          x = mk(keep(o.x + d.x * tr), keep(o.y + d.y * tr), keep(o.z + d.z * tr));
          // a miss vertex is the origin (:373-374); a leaked path ending at its miss (the LEAK == 1
          // kernels, see below) never reads it
          if constexpr (CF::LEAK != 1) x = hit ? x : mk(0, 0, 0);
          if constexpr (!kEarly) l_miss += hit ? 0u : 1u;
          const float sg = da < 0.0f ? 1.0f : -1.0f;
          nl = mk(kyz ? sg : 0.0f, kxz ? sg : 0.0f, kxy ? sg : 0.0f);
          if (TP::MAT) gn = mk(kyz ? 1.0f : 0.0f, kxz ? 1.0f : 0.0f, kxy ? 1.0f : 0.0f);
        } else {
        if (!hit) {
          x = mk(0, 0, 0);
          if constexpr (!kEarly) ++l_miss;
        } else {
          // plane distance as the reference derives it (:103); spheres: the root
          float tr = hit_t<TP>(H, hpos, o, d, ia_hit, G);
          if (kind == SPT_RECT_XY) tr = hit_plane_t(H.w1 - o.z, d.z, ia_hit, tr);
          else if (kind == SPT_RECT_XZ) tr = hit_plane_t(H.w1 - o.y, d.y, ia_hit, tr);
          else if (kind == SPT_RECT_YZ) tr = hit_plane_t(H.w1 - o.x, d.x, ia_hit, tr);
          x = mk(o.x + d.x * tr, o.y + d.y * tr, o.z + d.z * tr);
        }
        // Hitable::normal, oriented against the ray (:123,:166,:209,:251); gn = the unoriented
        // (geometric) normal `n` of the SPEC/REFR code :482-491 (MAT only)
        if (kind == SPT_RECT_XY) {
          nl = d.z < 0.0f ? mk(0, 0, 1) : mk(0, 0, -1);
          if (TP::MAT) gn = mk(0, 0, 1);
        } else if (kind == SPT_RECT_XZ) {
          nl = d.y < 0.0f ? mk(0, 1, 0) : mk(0, -1, 0);
          if (TP::MAT) gn = mk(0, 1, 0);
        } else if (kind == SPT_RECT_YZ) {
          nl = d.x < 0.0f ? mk(1, 0, 0) : mk(-1, 0, 0);
          if (TP::MAT) gn = mk(1, 0, 0);
        } else {
          // Sphere::normal :248 as (x - p) * (1/r): x lies on the sphere to ~1e-7, so this is the
          // unit normal without the normalize's rsq (contract, oracle c_path; C5 -0.7 %)
          const f3 n = mk((x.x - H.w1) * H.w5, (x.y - H.w2) * H.w5, (x.z - H.w3) * H.w5);
          nl = dot3(n, d) < 0.0f ? n : mk(-n.x, -n.y, -n.z);
          if (TP::MAT) gn = n;
          atomicAdd(&s_nsph[threadIdx.x / 64], 1u);  // the lanes shading a sphere vertex
        }
        }
        f3 f = mk(H.cx, H.cy, H.cz);
        const f3 e = mk(H.ex, H.ey, H.ez);
        const int rr_t = H.rr_t;
        const int depth = dp1++;  // this vertex's depth (1 = the first)
        u4 rl = r;  // RR / NEE-mix draws; at vertex 1 from stream 1 (only configs that need them)
        if (CF::NOS1 != 1 && depth == 1) {
          const SPT_CONST KParams* C = cptr(Pg);
          if (C->rr_depth < 1 || (C->nee_prob > 0.0f && C->nee_prob < 1.0f))
            rl = philox_px(pk, s, 1u | 0x80000000u);
        }
        // Russian roulette :448-454 (+ optional hard depth cap), branch-free: f is scaled by the
        // host-rounded 1/p wherever RR applies (f * 1 elsewhere, exact); f is unused on a path that
        // ends here.
        const int max_depth = CF::MAXD0 == 1 ? 0 : P->max_depth;
        const bool capd = (max_depth > 0) & (depth >= max_depth);
        const bool rr = (depth > rr_depth_of<CF>(P)) | (rr_t < 0);   // p == 0
        const bool alive = (int)u16i(rl.x, rl.y) < rr_t;              // (p > 0) & (p >= 1 | u16 < p)
        // contract v6: a leaked path ends at its first miss (host leak_end_of, oracle
        // c_find_leak_end); the host launches the LEAK == 1 kernels only where that rule holds
        const bool leak = CF::LEAK == 1 || (CF::LEAK < 0 && P->leak_end != 0);
        const bool term = capd | (rr & !alive) | (!hit & leak);
        const float ip = keep(H.ip);  // == 1.0f / p, read unconditionally (no branch)
        const float fsc = rr ? ip : 1.0f;
        f = mk(f.x * fsc, f.y * fsc, f.z * fsc);
        L = mk(fmaf(T.x, e.x, L.x), fmaf(T.y, e.y, L.y), fmaf(T.z, e.z, L.z));
        // Every vertex lane takes T*f and moves its origin to x. A lane whose path ends here
        // restarts at the camera (or pops a REFR child), which resets both; doing it
        // unconditionally saves the register copies of a conditional update.
        T = mk(T.x * f.x, T.y * f.y, T.z * f.z);
        o = x;
        if constexpr (!kEarlyNee) vid = id;
        uint32_t nxt = kStCos;  // the state after this vertex unless the path ends here
        if (TP::MAT && !term && H.refl != SPT_DIFF) {
          // SPEC :481-482 and REFR :484-495 (smallpt's commented-out code; oracle c_path): no NEE.
          // reflRay direction r.d - n*2*n.dot(r.d), not renormalised.
          const f3 Tf = T;
          const float k2 = 2.0f * dot3(gn, d);
          const f3 refl = mk(d.x - gn.x * k2, d.y - gn.y * k2, d.z - gn.z * k2);
          bool use_refl = true;
          if (H.refl == SPT_REFR) {
            const bool into = dot3(gn, nl) > 0.0f;                 // :485
            const float nnt = into ? 1.0f / 1.5f : 1.5f / 1.0f;    // nc = 1, nt = 1.5 :486
            const float ddn = dot3(d, nl);
            const float cos2t = 1.0f - nnt * nnt * (1.0f - ddn * ddn);
            if (!(cos2t < 0.0f)) {                                 // else total internal reflection
              const float kk = (into ? 1.0f : -1.0f) * (ddn * nnt + sqrtf(cos2t));
              const f3 tdir = normalize3(mk(d.x * nnt - gn.x * kk, d.y * nnt - gn.y * kk,
                                            d.z * nnt - gn.z * kk));  // :489
              const float a = 1.5f - 1.0f, b = 1.5f + 1.0f, R0 = a * a / (b * b);
              const float c = 1.0f - (into ? -ddn : dot3(tdir, gn));
              const float Re = R0 + (1.0f - R0) * c * c * c * c * c, Tr = 1.0f - Re;
              const float Pp = 0.25f + 0.5f * Re, RP = Re / Pp, TP_ = Tr / (1.0f - Pp);  // :491
              if (depth > 2) {  // Russian roulette between the two :492-493
                if (u16(rl.z, rl.w) < Pp) {
                  T = mk(Tf.x * RP, Tf.y * RP, Tf.z * RP);
                } else {
                  T = mk(Tf.x * TP_, Tf.y * TP_, Tf.z * TP_);
                  d = tdir;
                  use_refl = false;
                }
              } else {  // both :494-495: reflection now, the refraction child later (same L)
                Node& N = s_stack[threadIdx.x * 2 + sp];
                N.o[0] = x.x; N.o[1] = x.y; N.o[2] = x.z;
                N.d[0] = tdir.x; N.d[1] = tdir.y; N.d[2] = tdir.z;
                N.T[0] = Tf.x * Tr; N.T[1] = Tf.y * Tr; N.T[2] = Tf.z * Tr;
                N.depth = depth;
                N.branch = branch | (1u << (depth - 1));
                ++sp;
                T = mk(Tf.x * Re, Tf.y * Re, Tf.z * Re);
              }
            }
          }
          if (use_refl) d = refl;
          nxt = kStSpec;
        } else {
          // DIFF :457-480. T is T*f now; the NEE weight (if the light is reached) multiplies it
          // when the shadow ray resolves, so T = (T*f)*w exactly as the contract rounds it.
          // Computed for every vertex lane (a lane whose path ends here discards it): no branch.
          const SPT_CONST KParams* D = cptr(Pg);
          bool nee;
          if constexpr (CF::NEE == 1) {
            nee = true;
          } else if constexpr (CF::NEE == 0) {
            nee = false;
          } else {
            const float q = D->nee_prob;
            if (q >= 1.0f) nee = true;
            else if (q <= 0.0f) nee = false;
            else nee = u16(rl.z, rl.w) < q;
          }
          if (nee) {
            // light_sampling :363-369 and the shadow-ray direction :466.
            float xl, zl;
            const int lmode = CF::LMODE >= 0 ? CF::LMODE : D->light_mode;
            if (lmode == SPT_LIGHT_GLIBC_WRAP) {
              const uint32_t ldxi = CF::LREF == 1 ? kRefLdxi : D->ldxi;
              const uint32_t ldzi = CF::LREF == 1 ? kRefLdzi : D->ldzi;
              const float lx0 = CF::LREF == 1 ? kRefLx0 : D->lx0, lz0 = CF::LREF == 1 ? kRefLz0 : D->lz0;
              if constexpr (CF::LREF == 1) {
                // dx = dz = 36 = 4 * 9: the lattice x0 - 1 + m 2^-22, m = r >> 9 (oracle
                // c_wrap_sample) as fma(2^23 + m, 2^-22, x0 - 3) -- the float with bits
                // 0x4B000000 | m is 2^23 + m, so the sum is the same real, rounded once: one or and
                // one fma (rounds 1-4: shift, 24-bit multiply, conversion, fma)
                static_assert(kRefLdxi == 36u && kRefLdzi == 36u, "LREF light lattice");
                xl = fmaf(__uint_as_float(0x4B000000u | (r.x >> 9)), 0x1p-22f, lx0 - 3.0f);
                zl = fmaf(__uint_as_float(0x4B000000u | (r.y >> 9)), 0x1p-22f, lz0 - 3.0f);
              } else {
                xl = D->lx_lattice ? fmaf((float)(r.x >> D->lx_shift), D->lx_scale, D->lx0m1)
                                   : fmaf((float)(int32_t)(((r.x >> 8) << 7) * ldxi), 0x1p-31f, lx0);
                zl = D->lz_lattice ? fmaf((float)(r.y >> D->lz_shift), D->lz_scale, D->lz0m1)
                                   : fmaf((float)(int32_t)(((r.y >> 8) << 7) * ldzi), 0x1p-31f, lz0);
              }
            } else {
              xl = fmaf(u01(r.x), D->ldx, D->lx0);
              zl = fmaf(u01(r.y), D->ldz, D->lz0);
            }
            const float ly = CF::LREF == 1 ? kRefLy : D->ly;
            // light_vec (:367); normalised only in the unit-direction contract (nee_weight)
            const f3 vl = mk(xl - x.x, ly - x.y, zl - x.z);
            const f3 dl = unit_dirs_of<TP>(Pg) ? normalize3(vl) : vl;
            if constexpr (!kNeeByIdentity) l_nee += term ? 0u : 1u;
            const SPT_CONST SceneGeo* G2 = TP::CONSTGEO ? nullptr : cptr(D->geo);
            // a miss keeps id (:466-467), so a vertex ON the light always traces its shadow ray
            bool la, early = false;
            if constexpr (kEarlyNee) {  // the light's own test (light_accepts), keeping t and a
              const Ray6 rl6{x.y, rcp_nr(dl.y), dl.x, x.x, dl.z, x.z};
              RectHit h;
              if constexpr (TP::UPLIGHT) h = rect_eval_test(cptr(D->geo)->test[0], rl6);  // the uploaded light
              else h = rect_eval(CornellRectPtr{kCornellLightPos}, rl6);
              la = h.inb & key_valid(h.tt, kCornellLightPos);
              if constexpr (TP::UPLIGHT) early = la & early_geo_proven<1>(x, D);
              else if constexpr (TP::UPBOX) early = la & early_geo_proven<0>(x, D);
              else early = la & early_nee_proven(x);
              // The weight of :471-472 now, for a proven lane and a traced one alike: nee_weight's
              // arithmetic with |dl . nl| = |dl_a| on the normal's axis a (the dot's zero terms are
              // exact) and t = the light's own t, the bits the trace returns for it. The resolve
              // then needs neither the light's t nor the weight (round 4: -5 VALU per iteration).
              const float adot = fabsf(ax_xy ? dl.z : (ax_xz ? dl.y : dl.x));
              const float num = fabsf(dl.y) * adot;
              const float vv = dot3(dl, dl);
              w_nee = (num * kRefNeeC) * rcp_nr((h.tt * h.tt) * (vv * vv));
            } else if constexpr (kEarlySph || kEarlyGeo) {  // the uploaded light rect (XZ, host-checked)
              const RectHit h = rect_eval(G2->rect + D->light_pos,
                                          Ray6{x.y, rcp_nr(dl.y), dl.x, x.x, dl.z, x.z});
              la = h.inb & key_valid(h.tt, (uint32_t)D->light_pos);
              if constexpr (kEarlySph) early = la & early_room_proven(x, D->early_y0);
              else early = la & early_geo_proven<2>(x, D);
              t = early ? h.tt : t;
            } else {
              la = light_accepts<TP>(D, G2, rects_of<TP>(G2), x, dl);
            }
            const bool cand = (id == light_slot_of<TP, CF>(D)) | la;
            d = dl;  // a rejected lane generates its cosine direction next iteration anyway
            nxt = early ? kStEarly : (cand ? kStShadow : kStCos);
          }
        }
        ls = term ? kStTerm : nxt;
      }
      // 5') the HEAD NEE kernel resolves shadow rays here, after the shading block: the ones traced
      //    in this iteration and the ones early_nee_proven() has just resolved (t = the light's t,
      //    the same bits the trace returns). Same arithmetic as 5); the light is black, so a ray
      //    that reaches it shades the light vertex as L += (T*w)*e and ends the path (RR with
      //    p == 0, :448), which is all the common vertex block would do there.
      if constexpr (kEarly) {
        if (traced_shadow || ls == kStEarly) {
          SPT_REGION(6);
          const bool ea = ls == kStEarly;
          // a traced shadow ray that reached the light; never a proven lane (its path ray hit what
          // it shaded, not the black light, which would have ended the path)
          const bool th = id == light_slot_of<TP, CF>(cptr(Pg));
          const bool lh = ea | th;
          if (lh) SPT_REGION(7);
          count_if(l_hit, th);  // (+ the proven ones, l_early / s_nearly, at the end)
          if constexpr (TP::SPH) {  // (sphere kernels ballot-count the traced ones)
            if (ea) atomicAdd(&s_nearly[threadIdx.x / 64], 1u);
          } else {
            l_early += ea ? 1u : 0u;
            ++l_shadow;
          }
          float wl;
          if constexpr (kEarlyNee) {
            wl = w_nee;  // (from the vertex, above)
          } else {
            // the light's t: the pre-test's for a proven lane, else the traced light hit's own
            // (k_L - o.y) / d.y as the trace ranked it (the light is an XZ rect)
            const float kl = s_prims[light_slot_of<TP, CF>(cptr(Pg))].w1;
            const float tl = ea ? t : plane_t(kl - o.y, ia_hit);
            // (computed for every resolving lane: a branch around it cost exec-mask SALU)
            wl = keep(nee_weight(unit_dirs_of<TP>(Pg), d, nl, tl, kRefLarea, kRefNeeC));
          }
          // the black light ends a path that reaches it, so only the light vertex's L needs T*w
          // (a lane whose shadow ray is blocked keeps T: the cosine sample follows). A blocked
          // lane adds (T*0)*e = +0 instead of selecting: L + 0 is L bit for bit, T being finite
          // and >= 0 on a path that has not reached the light (one select, not three)
          const float wh = lh ? wl : 0.0f;
          const f3 Tw = mk(T.x * wh, T.y * wh, T.z * wh);
          const DevPrim& H = s_prims[light_slot_of<TP, CF>(cptr(Pg))];
          L = mk(fmaf(Tw.x, H.ex, L.x), fmaf(Tw.y, H.ey, L.y), fmaf(Tw.z, H.ez, L.z));
          ls = lh ? kStTerm : kStCos;
        }
      }
      // 7) path end: accumulate this sample (:536-538) and start the next one.
      if (ls == kStTerm) {
        if (TP::MAT && sp > 0) {  // the pending refraction child of a REFR split
          --sp;
          const Node& N = s_stack[threadIdx.x * 2 + sp];
          o = mk(N.o[0], N.o[1], N.o[2]);
          d = mk(N.d[0], N.d[1], N.d[2]);
          T = mk(N.T[0], N.T[1], N.T[2]);
          dp1 = N.depth + 1;
          branch = N.branch;
          ls = kStSpec;
        } else {
          SPT_REGION(9);
          const float scale = CF::CAMAX == 1 ? ck.fs : (CF::CAMAX == 2 ? cg.fs : cptr(Pg)->fix_scale);
          acc0 += fix31(L.x, scale);
          acc1 += fix31(L.y, scale);
          acc2 += fix31(L.z, scale);
          ++s;
          L = mk(0, 0, 0);
          T = mk(1, 1, 1);
          dp1 = 1;
          {
            const SPT_CONST KParams* C = cptr(Pg);
            o = CF::CAMAX == 1   ? mk(ck.o0, ck.o1, ck.o2)
                : CF::CAMAX == 2 ? mk(cg.o0, cg.o1, cg.o2)
                                 : mk(C->cam[0], C->cam[1], C->cam[2]);
          }
          if (TP::MAT) branch = 0;
          ls = kStCam;
          if (s >= s_end) {  // the unit's last sample: flush its pixel's fixed-point sums
            SPT_REGION(1);
            if (lp >> 31) {  // the unit's owner: its slot, written exactly once (zeros included)
              unsigned long long* a = cptr(Pg)->slots + 3ull * (lp & 0x7FFFFFFFu);
              a[0] = acc0;
              a[1] = acc1;
              a[2] = acc2;
            } else {  // a stolen range: add into its pixel's accumulator
              unsigned long long* a = cptr(Pg)->accum + 3ull * lp;
              if (acc0) atomicAdd(a + 0, acc0);
              if (acc1) atomicAdd(a + 1, acc1);
              if (acc2) atomicAdd(a + 2, acc2);
            }
            acc0 = acc1 = acc2 = 0;
            ls = kStIdle;
          }
        }
      }
    }
#ifdef SPT_REGION_STATS
#pragma unroll
    for (int k = 0; k < kRegions; ++k) {
      const uint64_t m = __ballot((reg_flags >> k) & 1u);
      reg_exec[k] += m != 0;
      reg_lanes[k] += (uint32_t)__popcll(m);
    }
    reg_flags = 0;
#endif
  }
  {
    unsigned long long* st = cptr(Pg)->stats;  // wave-reduced by the atomic optimizer
#ifdef SPT_WAVE_TIMES
    if (lane == 0) {  // [12] sum of durations, [13] sum of squares, [14] min start, [15] max end,
                      // [16] sum of iterations, [17] max iterations (stats words 12+ are free here)
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), dt = t1 - wave_t0;
      atomicAdd(st + 12, dt);
      atomicAdd(st + 13, dt * dt);
      atomicMin(st + 14, wave_t0);
      atomicMax(st + 15, t1);
      atomicAdd(st + 16, (unsigned long long)wave_iters);
      atomicMax(st + 17, (unsigned long long)wave_iters);
      atomicAdd(st + 18, wave_t0 >> 4);  // sums of start / end times (/16: no overflow)
      atomicAdd(st + 19, t1 >> 4);
      atomicAdd(st + 20, (unsigned long long)__smid());
      const uint32_t wid = blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
      if (wid < 32768) {
        st[32 + 3 * wid] = wave_t0;
        st[33 + 3 * wid] = t1;
        st[34 + 3 * wid] = ((unsigned long long)__smid() << 32) | wave_iters;
      }
    }
#endif
#ifdef SPT_REGION_STATS
    if (lane == 0) {  // wave-uniform values: one lane adds them
      for (int k = 0; k < kRegions; ++k) {
        atomicAdd(st + kStatRegion + 2 * k, (unsigned long long)reg_exec[k]);
        atomicAdd(st + kStatRegion + 1 + 2 * k, (unsigned long long)reg_lanes[k]);
      }
    }
#endif
    if (lane == 0) {  // wave-uniform counters: one lane adds them
      if (capped) atomicAdd(st + 0, 1ull);  // the host reports an error
      const unsigned long long np = TP::MAT ? n_path : n_cos;  // (+ samples below, !MAT)
      atomicAdd(st + 1, np);
      atomicAdd(st + 3, np);  // + the light hits, added per lane below
      atomicAdd(st + 6, (unsigned long long)n_cos);
    }
    if (!TP::MAT && blockIdx.x == 0 && threadIdx.x == 0) {  // one camera ray per sample
      const SPT_CONST KParams* C = cptr(Pg);
      const unsigned long long samples = (unsigned long long)C->n_local_pix * (unsigned long long)C->spp;
      atomicAdd(st + 1, samples);
      atomicAdd(st + 3, samples);
    }
    {  // per-lane event counts (the atomic optimizer reduces each over the wave)
      if constexpr (!kNeeByIdentity) {
        atomicAdd(st + 2, (unsigned long long)l_nee);
        atomicAdd(st + 4, (unsigned long long)l_nee);
      }
      if constexpr (kEarlyNee || kEarlyGeo) l_hit += l_early;  // proven shadow rays reach the light
      atomicAdd(st + 3, (unsigned long long)l_hit);
      atomicAdd(st + 5, (unsigned long long)l_hit);
      atomicAdd(st + 7, (unsigned long long)l_miss);
      if constexpr (TP::SPH) {
        if (lane == 0) atomicAdd(st + kStatShadowTraced, (unsigned long long)l_shadow);
      } else {
        atomicAdd(st + kStatShadowTraced, (unsigned long long)l_shadow);
      }
      if constexpr (TP::SPH)
        if (lane == 0) atomicAdd(st + kStatSphereVertices, (unsigned long long)s_nsph[threadIdx.x / 64]);
      if constexpr (kEarlyNee || kEarlyGeo) atomicAdd(st + kStatShadowProven, (unsigned long long)l_early);
      if constexpr (kEarlySph) {
        if (lane == 0) {
          const unsigned long long ne = s_nearly[threadIdx.x / 64];
          atomicAdd(st + kStatShadowProven, ne);
          atomicAdd(st + kStatShadowTraced, ne);
          atomicAdd(st + 3, ne);  // proven shadow rays reach the light (vertices, light hits)
          atomicAdd(st + 5, ne);
        }
      }
    }
  }
}
// 1.31 fixed point -> float, clamp :538 (values are >= 0 by construction). Thread t takes
// unit-order pixel t (coalesced slot reads, chunk j's slot at j * npix + t), adds the pixel's
// stolen-range sums and writes its spread pixel p = (t mod K) * (npix / K) + t / K. Integer sums:
// the order of the adds cannot matter.
__global__ void __launch_bounds__(kBlock)
finalize_slots_kernel(const unsigned long long* __restrict__ accum,
                      const unsigned long long* __restrict__ slots, float* __restrict__ rgb,
                      uint32_t npix, uint32_t n_chunks, uint32_t scr_k, uint32_t scr_q,
                      const unsigned long long* __restrict__ stats) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= npix) return;
  const uint32_t p = (t & ((1u << scr_k) - 1u)) * scr_q + (t >> scr_k);
  if (stats[0] != 0) {  // the launch hit its iteration cap: the slots of the units it dropped hold an
    rgb[3ull * p] = rgb[3ull * p + 1] = rgb[3ull * p + 2] = __builtin_nanf("");  // earlier launch's
    return;                                                                  // sums; no image at all
  }
  unsigned long long v0 = accum[3ull * p], v1 = accum[3ull * p + 1], v2 = accum[3ull * p + 2];
  for (uint32_t j = 0; j < n_chunks; ++j) {
    const unsigned long long* q = slots + 3ull * ((size_t)j * npix + t);
    v0 += q[0];
    v1 += q[1];
    v2 += q[2];
  }
  const float f0 = (float)v0 * 0x1p-31f, f1 = (float)v1 * 0x1p-31f, f2 = (float)v2 * 0x1p-31f;
  rgb[3ull * p] = f0 > 1.0f ? 1.0f : f0;
  rgb[3ull * p + 1] = f1 > 1.0f ? 1.0f : f1;
  rgb[3ull * p + 2] = f2 > 1.0f ? 1.0f : f2;
}

}  // namespace spt

// =====================================================================================
// C ABI
// =====================================================================================
using namespace spt;

static thread_local std::string g_last_error;
void spt_set_last_error(const std::string& msg) { g_last_error = msg; }
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

// Kernel variants, from the most general to the most specialised (SPT_FLAG_KERNEL_LEVEL caps the
// level).
using RenderFn = void (*)(const KParams*);
enum { KV_GENERIC, KV_CORNELL, KV_CONST, KV_CONST_NEE, KV_CONST_COS, KV_SPHDIFF, KV_WIDE,
       KV_SPHDIFF_NEE, KV_RECTDIFF, KV_CONST_NEE_REF, KV_CONST_COS_REF, KV_SPHDIFF_NEE_REF,
       KV_CORNELL_NEE, KV_CORNELL_COS, KV_RECTDIFF_NEE, KV_RECTDIFF_COS, KV_UPBOX_NEE, KV_UPBOX_COS,
       KV_CONST_NEE_CAM, KV_CONST_COS_CAM, KV_UPBOX_NEE_CAM, KV_UPBOX_COS_CAM, KV_UPLIGHT_NEE,
       KV_UPLIGHT_COS, KV_UPLIGHT_NEE_CAM, KV_UPLIGHT_COS_CAM, KV_COUNT };
static const RenderFn kRenderKernels[KV_COUNT] = {
    render_kernel<TopoGeneric, CfgRuntime>, render_kernel<TopoCornell, CfgRuntime>,
    render_kernel<TopoCornellConst, CfgRuntime>, render_kernel<TopoCornellConst, CfgHeadNee>,
    render_kernel<TopoCornellConst, CfgHeadCos>, render_kernel<TopoSphDiff, CfgRuntime>,
    render_kernel<TopoGenericWide, CfgRuntime>, render_kernel<TopoSphDiff, CfgSphNee>,
    render_kernel<TopoRectDiff, CfgRuntime>, render_kernel<TopoCornellConst, CfgHeadNeeRef>,
    render_kernel<TopoCornellConst, CfgHeadCosRef>, render_kernel<TopoSphDiff, CfgSphNeeRef>,
    render_kernel<TopoCornell, CfgHeadNee>, render_kernel<TopoCornell, CfgHeadCos>,
    render_kernel<TopoRectDiff, CfgHeadNee>, render_kernel<TopoRectDiff, CfgHeadCos>,
    render_kernel<TopoCornellUpBox, CfgHeadNee>, render_kernel<TopoCornellUpBox, CfgHeadCos>,
    render_kernel<TopoCornellConst, CfgHeadNeeCam>, render_kernel<TopoCornellConst, CfgHeadCosCam>,
    render_kernel<TopoCornellUpBox, CfgHeadNeeCam>, render_kernel<TopoCornellUpBox, CfgHeadCosCam>,
    render_kernel<TopoCornellUpLight, CfgHeadNee>, render_kernel<TopoCornellUpLight, CfgHeadCos>,
    render_kernel<TopoCornellUpLight, CfgHeadNeeCam>, render_kernel<TopoCornellUpLight, CfgHeadCosCam>};

struct spt_context {
  int device = 0;
  int n_cu = 0, blocks_per_cu = 0;      // generic kernel
  int bpc[KV_COUNT] = {};               // resident blocks per CU of each variant
  DevPrim* prims = nullptr;
  SceneGeo* geo = nullptr;
  unsigned long long* accum = nullptr;
  size_t accum_cap = 0;  // elements
  unsigned long long* slots = nullptr;  // [n_units][3] unit slots, grown on demand
  size_t slots_cap = 0;                 // elements
  uint32_t* queue = nullptr;
  unsigned long long* stats = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // the launch's statistics words, copied to pinned host memory on the launch's stream after the
  // finalize (ev2 marks the copy): spt_context_stats() waits for that launch only, never for work
  // queued behind it on the stream
  unsigned long long* h_stats = nullptr;
  hipEvent_t ev2 = nullptr;
  bool pending = false;
  bool launched = false;  // a render has been enqueued (spt_context_stats has events to read)
  int n_prims = 0;
  KParams last{};
  // Pinned staging for the async scene upload; reused only after the previous upload completed.
  DevPrim* h_prims = nullptr;
  SceneGeo* h_geo = nullptr;
  KParams* d_kp = nullptr;   // kernel parameters in device memory (read via s_load)
  KParams* h_kp = nullptr;   // pinned staging
  uint64_t samples = 0;      // pixel-samples of the last render (exact, not counted in-kernel)
  bool nee_by_identity = false;  // the last kernel derives nee_events from vertices - samples
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
  if (p->flags & ~(SPT_FLAG_UNIFORM_SCATTER | SPT_FLAG_REFERENCE_LEAKS | SPT_FLAG_KERNEL_LEVEL_MASK))
    return fail(SPT_ERR_INVALID_ARG, "unknown flags");
  if (((p->flags & SPT_FLAG_KERNEL_LEVEL_MASK) >> 8) > SPT_KERNEL_LEVEL_CONST)
    return fail(SPT_ERR_INVALID_ARG, "bad kernel level");
  if (p->light_mode != SPT_LIGHT_GLIBC_WRAP && p->light_mode != SPT_LIGHT_UNIFORM)
    return fail(SPT_ERR_INVALID_ARG, "bad light_mode");
  if (p->light_mode == SPT_LIGHT_GLIBC_WRAP &&
      (p->light_dx != (float)(uint32_t)p->light_dx || p->light_dz != (float)(uint32_t)p->light_dz))
    return fail(SPT_ERR_INVALID_ARG, "GLIBC_WRAP light sampling needs integral light_dx/dz");
  for (int i = 0; i < n; ++i) {
    if (prims[i].kind < SPT_RECT_XY || prims[i].kind > SPT_SPHERE)
      return fail(SPT_ERR_INVALID_ARG, "bad primitive kind");
    // Sphere::normal (:248) is (x - p).norm(); the contract's (x - p) * (1/r) equals it only for
    // r > 0 (a negative radius would flip the geometric normal of the REFR test :485)
    if (prims[i].kind == SPT_SPHERE && !(prims[i].geom[0] > 0.0 && std::isfinite(prims[i].geom[0])))
      return fail(SPT_ERR_INVALID_ARG, "sphere radius must be positive and finite");
    if (prims[i].refl < SPT_DIFF || prims[i].refl > SPT_REFR)
      return fail(SPT_ERR_INVALID_ARG, "bad material");
  }
  // NEE (:464-472) weights shadow rays that reach prims[light_id] as light hits: that primitive
  // must exist and emit, or the image is silently wrong (e.g. the classic sphere box with the HEAD
  // light id 6, a ball).
  if (p->nee_prob > 0.0f) {
    if (p->light_id < 0 || p->light_id >= n)
      return fail(SPT_ERR_INVALID_ARG, "nee_prob > 0 needs light_id in [0, n_prims)");
    const double* e = prims[p->light_id].e;
    if (!(e[0] != 0.0 || e[1] != 0.0 || e[2] != 0.0))
      return fail(SPT_ERR_INVALID_ARG, "nee_prob > 0 but prims[light_id] emits nothing");
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
      P.w5 = 1.0f / r;  // the normal as (x - p) * (1/r) (contract, oracle c_path)
    } else {
      P.w1 = plane_k(s[i].geom[4]);  // contract plane coordinate (spt_cornell.h)
      P.w2 = (float)s[i].geom[0]; P.w3 = (float)s[i].geom[1];
      P.w4 = (float)s[i].geom[2]; P.w5 = (float)s[i].geom[3];
    }
    P.ex = (float)s[i].e[0]; P.ey = (float)s[i].e[1]; P.ez = (float)s[i].e[2];
    P.cx = (float)s[i].c[0]; P.cy = (float)s[i].c[1]; P.cz = (float)s[i].c[2];
    P.pmax = P.cx > P.cy && P.cx > P.cz ? P.cx : P.cy > P.cz ? P.cy : P.cz;  // :447
    P.ip = 1.0f / P.pmax;  // IEEE single division, as the device's 1.0f / p
    // u * 2^-16 < p (u < 2^16 an integer, p * 2^16 exact) <=> u < ceil(p * 2^16): the RR draw as
    // one integer compare instead of a conversion, a scale and a float compare (same decision)
    P.rr_t = P.pmax == 0.0f ? INT32_MIN
             : !(P.pmax > 0.0f) ? 0
             : P.pmax >= 1.0f   ? 65536
                                : (int32_t)std::ceil((double)P.pmax * 65536.0);
    P.refl = s[i].refl;
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
      R.k = plane_k(s[i].geom[4]);
      rect_mid(s[i].geom[0], s[i].geom[1], &R.ma, &R.ha);
      rect_mid(s[i].geom[2], s[i].geom[3], &R.mb, &R.hb);
      R.idx = i;
      if (i == light) *light_pos = r - 1;
      ++*counts[k];
    }
  }
  // Rect tests (oracle c_build_tests): inside each kind group, in order, a rectangle pairs with the
  // first later unpaired one of bit-identical bounds on a different plane; the light never pairs.
  {
    bool used[kMaxPrims] = {};
    const int grp[4] = {0, g->n_xy, g->n_xy + g->n_xz, g->n_xy + g->n_xz + g->n_yz};
    int* tcounts[3] = {&g->n_txy, &g->n_txz, &g->n_tyz};
    int nt = 0;
    auto bits = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; };
    for (int k = 0; k < 3; ++k) {
      for (int i = grp[k]; i < grp[k + 1]; ++i) {
        if (used[i]) continue;
        used[i] = true;
        const GeoRect& A = g->rect[i];
        GeoTest& T = g->test[nt++];
        T = GeoTest{A.k, A.k, A.ma, A.ha, A.mb, A.hb, i, i};
        ++*tcounts[k];
        if (i == *light_pos) continue;
        for (int j = i + 1; j < grp[k + 1]; ++j) {
          const GeoRect& B = g->rect[j];
          if (used[j] || j == *light_pos || bits(A.ma) != bits(B.ma) || bits(A.ha) != bits(B.ha) ||
              bits(A.mb) != bits(B.mb) || bits(A.hb) != bits(B.hb) || bits(A.k) == bits(B.k) ||
              !(A.k == A.k) || !(B.k == B.k))
            continue;
          used[j] = true;
          if (A.k < B.k) { T.k1 = B.k; T.pos1 = j; }
          else { T.k0 = B.k; T.pos0 = j; T.k1 = A.k; T.pos1 = i; }
          break;
        }
      }
    }
  }
  // Contract v5's room (oracle c_find_room): the first XY, XZ, YZ pair tests (test order) whose
  // planes are exactly -- in the caller's doubles -- the other pairs' in-plane bounds (each pair's
  // bounds read from its k0 member). Its tests move behind the per-kind lists (the nearest hit is a
  // minimum of keys, so test order cannot matter).
  {
    const int nt = g->n_txy + g->n_txz + g->n_tyz;
    auto member = [&](int pos) -> const spt_prim& { return s[g->rect[pos].idx]; };
    auto same_range = [](double k1, double k2, double b1, double b2) {
      return std::min(k1, k2) == b1 && std::max(k1, k2) == b2;
    };
    int room[3] = {-1, -1, -1};
    for (int a = 0; a < g->n_txy && room[0] < 0; ++a) {
      const GeoTest& A = g->test[a];
      if (A.pos0 == A.pos1) continue;
      for (int b = g->n_txy; b < g->n_txy + g->n_txz && room[0] < 0; ++b) {
        const GeoTest& B = g->test[b];
        if (B.pos0 == B.pos1) continue;
        for (int c = g->n_txy + g->n_txz; c < nt; ++c) {
          const GeoTest& D = g->test[c];
          if (D.pos0 == D.pos1) continue;
          const double* ga = member(A.pos0).geom, *gb = member(B.pos0).geom, *gd = member(D.pos0).geom;
          const double zA = ga[4], zB = member(A.pos1).geom[4], yA = gb[4], yB = member(B.pos1).geom[4];
          const double xA = gd[4], xB = member(D.pos1).geom[4];
          if (!same_range(xA, xB, ga[0], ga[1]) || !same_range(xA, xB, gb[0], gb[1]) ||
              !same_range(yA, yB, ga[2], ga[3]) || !same_range(yA, yB, gd[0], gd[1]) ||
              !same_range(zA, zB, gb[2], gb[3]) || !same_range(zA, zB, gd[2], gd[3]))
            continue;
          room[0] = a; room[1] = b; room[2] = c;
          break;
        }
      }
    }
    g->has_room = room[0] >= 0;
    if (g->has_room) {
      const GeoTest A = g->test[room[0]], B = g->test[room[1]], D = g->test[room[2]];
      GeoTest rest[kMaxPrims];
      int n = 0;
      for (int i = 0; i < nt; ++i)
        if (i != room[0] && i != room[1] && i != room[2]) rest[n++] = g->test[i];
      for (int i = 0; i < n; ++i) g->test[i] = rest[i];
      g->test[n] = A; g->test[n + 1] = B; g->test[n + 2] = D;
      --g->n_txy; --g->n_txz; --g->n_tyz;
    }
  }
  // Contract v6's boxes (oracle c_find_boxes): an XY pair, a YZ pair and an XZ top (not the light)
  // closing a box on the room's floor, inside the floor's bounds, in the caller's doubles; searched
  // in test order. Their tests move behind the room's, three per box (XY pair, YZ pair, top).
  if (g->has_room) {
    const int nt = g->n_txy + g->n_txz + g->n_tyz;
    auto member = [&](int pos) -> const spt_prim& { return s[g->rect[pos].idx]; };
    auto same_range = [](double k1, double k2, double b1, double b2) {
      return std::min(k1, k2) == b1 && std::max(k1, k2) == b2;
    };
    const GeoTest& F = g->test[nt + 1];
    const double floor_k = std::min(member(F.pos0).geom[4], member(F.pos1).geom[4]);
    const double* gf = member(F.pos0).geom;
    bool used[kMaxPrims] = {};
    int box[kMaxPrims / 5][3], nb = 0;
    for (int a = 0; a < g->n_txy && nb < kMaxPrims / 5; ++a) {  // (5 rects a box: <= 12 of them)
      const GeoTest& A = g->test[a];
      if (A.pos0 == A.pos1 || used[a]) continue;
      for (int b = g->n_txy + g->n_txz; b < nt && !used[a]; ++b) {
        const GeoTest& D = g->test[b];
        if (D.pos0 == D.pos1 || used[b]) continue;
        for (int c = g->n_txy; c < g->n_txy + g->n_txz; ++c) {
          const GeoTest& T = g->test[c];
          if (T.pos0 != T.pos1 || T.pos0 == *light_pos || used[c]) continue;
          const double *ga = member(A.pos0).geom, *gd = member(D.pos0).geom, *gt = member(T.pos0).geom;
          const double xA = gd[4], xB = member(D.pos1).geom[4], zA = ga[4], zB = member(A.pos1).geom[4];
          if (!same_range(xA, xB, ga[0], ga[1]) || !same_range(xA, xB, gt[0], gt[1]) ||
              !same_range(zA, zB, gd[2], gd[3]) || !same_range(zA, zB, gt[2], gt[3]) ||
              !same_range(floor_k, gt[4], ga[2], ga[3]) || !same_range(floor_k, gt[4], gd[0], gd[1]) ||
              !(gt[4] > floor_k))
            continue;
          if (!(gf[0] <= ga[0] && ga[1] <= gf[1] && gf[2] <= gd[2] && gd[3] <= gf[3])) continue;
          used[a] = used[b] = used[c] = true;
          box[nb][0] = a; box[nb][1] = b; box[nb][2] = c;
          ++nb;
          break;
        }
      }
    }
    if (nb > 0) {
      GeoTest rest[kMaxPrims];
      int n = 0, kind_n[3] = {0, 0, 0};
      for (int i = 0; i < nt; ++i) {
        if (used[i]) continue;
        rest[n++] = g->test[i];
        ++kind_n[i < g->n_txy ? 0 : (i < g->n_txy + g->n_txz ? 1 : 2)];
      }
      for (int r = 0; r < 3; ++r) rest[n + r] = g->test[nt + r];  // the room
      for (int b = 0; b < nb; ++b)
        for (int r = 0; r < 3; ++r) rest[n + 3 + 3 * b + r] = g->test[box[b][r]];
      for (int i = 0; i < n + 3 + 3 * nb; ++i) g->test[i] = rest[i];
      g->n_txy = kind_n[0]; g->n_txz = kind_n[1]; g->n_tyz = kind_n[2];
      g->n_box = nb;
    }
  }
  // Spheres in index order, the narrow (fp32) ones first, then the wide (fp64) ones (oracle
  // c_intersect): the kernel's fp32 loop carries no per-sphere precision test.
  for (int pass = 0; pass < 2; ++pass)
  for (int i = 0; i < n; ++i) {
    if (s[i].kind != SPT_SPHERE) continue;
    if ((s[i].geom[0] >= SPT_WIDE_SPHERE_RADIUS) != (pass == 1)) continue;
    g->n_sph_wide += pass;
    GeoSph& S = g->sph[g->n_sph++];
    const float rad = (float)s[i].geom[0];
    S.px = (float)s[i].geom[1]; S.py = (float)s[i].geom[2]; S.pz = (float)s[i].geom[3];
    S.rad2 = rad * rad;
    S.idx = i;
    S.wide = s[i].geom[0] >= SPT_WIDE_SPHERE_RADIUS ? 1 : 0;
    GeoSphD& D = g->sphd[g->n_sph - 1];
    D.px = s[i].geom[1]; D.py = s[i].geom[2]; D.pz = s[i].geom[3];
    D.rad2 = s[i].geom[0] * s[i].geom[0];
    if (i == light) *light_pos = g->n_sph - 1;
  }
}

// Contract v6 (oracle c_find_leak_end): a leaked path ends at its first miss when the scene has a
// room, the miss vertex (the origin, :373-374) lies strictly outside the room's box, prim 0 does
// not emit and every emitter lies strictly inside the box -- compared on the caller's doubles.
static int leak_end_of(const spt_prim* s, int n, const SceneGeo& g) {
  if (!g.has_room) return 0;
  const int nt = g.n_txy + g.n_txz + g.n_tyz;
  double lo[3], hi[3];
  for (int a = 0; a < 3; ++a) {  // room tests: XY pair (planes z), XZ (y), YZ (x)
    const GeoTest& T = g.test[nt + a];
    const double k0 = s[g.rect[T.pos0].idx].geom[4], k1 = s[g.rect[T.pos1].idx].geom[4];
    const int ax = a == 0 ? 2 : (a == 1 ? 1 : 0);
    lo[ax] = std::min(k0, k1);
    hi[ax] = std::max(k0, k1);
  }
  if (!(0.0 < lo[0] || 0.0 > hi[0] || 0.0 < lo[1] || 0.0 > hi[1] || 0.0 < lo[2] || 0.0 > hi[2])) return 0;
  if (s[0].e[0] != 0.0 || s[0].e[1] != 0.0 || s[0].e[2] != 0.0) return 0;
  for (int i = 0; i < n; ++i) {
    const double* gm = s[i].geom;
    if (s[i].e[0] == 0.0 && s[i].e[1] == 0.0 && s[i].e[2] == 0.0) continue;
    if (s[i].kind == SPT_SPHERE) {
      for (int a = 0; a < 3; ++a)
        if (!(gm[1 + a] - gm[0] > lo[a] && gm[1 + a] + gm[0] < hi[a])) return 0;
      continue;
    }
    const int pa = s[i].kind == SPT_RECT_XY ? 2 : (s[i].kind == SPT_RECT_XZ ? 1 : 0);
    const int ua = s[i].kind == SPT_RECT_YZ ? 1 : 0, va = s[i].kind == SPT_RECT_XY ? 1 : 2;
    if (!(gm[4] > lo[pa] && gm[4] < hi[pa] && gm[0] >= lo[ua] && gm[1] <= hi[ua] && gm[2] >= lo[va] &&
          gm[3] <= hi[va]))
      return 0;
  }
  return 1;
}

static int tile_rows_of(const spt_params* p) { return p->tile_rows > 0 ? p->tile_rows : 8; }

// Multiply-shift reciprocal of d for 31-bit numerators: l = ceil(log2 d), m = floor(2^(31+l)/d) + 1
// (< 2^32), n / d = (n * m) >> (31 + l) exactly for all n < 2^31 (Granlund & Montgomery 1994).
static void magic31(uint32_t d, uint32_t* m, uint32_t* sh) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  *m = (uint32_t)(((unsigned __int128)1 << (31 + l)) / d + 1);
  *sh = 31 + l;
}

// Does the uploaded scene's grouped geometry equal the compile-time HEAD scene bit for bit?
static bool cornell_const_match(const SceneGeo& g, int light_pos) {
  if (g.n_xy != kCornellNXY || g.n_xz != kCornellNXZ || g.n_yz != kCornellNYZ || g.n_sph != 0 ||
      light_pos != kCornellLightPos || !g.has_room)
    return false;
  {  // the same room (tests behind the per-kind lists) and box as the compile-time kCornellRoom
    const int nt = g.n_txy + g.n_txz + g.n_tyz;
    for (int r = 0; r < 3; ++r) {
      const CTest& C = kCornellTests.t[kCornellRoom[r]];
      if (g.test[nt + r].pos0 != C.pos0 || g.test[nt + r].pos1 != C.pos1) return false;
    }
    if (g.n_box != kCornellBoxes.n) return false;  // and the same boxes (their tests behind the room's)
    for (int b = 0; b < kCornellBoxes.n; ++b)
      for (int r = 0; r < 3; ++r) {
        const CTest& C = kCornellTests.t[kCornellBoxes.t[b][r]];
        const GeoTest& T = g.test[nt + 3 + 3 * b + r];
        if (T.pos0 != C.pos0 || T.pos1 != C.pos1) return false;
      }
  }
  for (int i = 0; i < kCornellNXY + kCornellNXZ + kCornellNYZ; ++i) {
    const GeoRect& R = g.rect[i];
    const CRect& C = kCornellRects[i];
    const float a[5] = {R.k, R.ma, R.ha, R.mb, R.hb}, b[5] = {C.k, C.ma, C.ha, C.mb, C.hb};
    if (std::memcmp(a, b, sizeof a) != 0 || R.idx != C.idx) return false;
  }
  return true;
}

// The room of a HEAD-topology scene is the reference's (:288-293): its three pair tests at HEAD's
// grouped positions with HEAD's fp32 geometry (materials may differ). The boxes-only-uploaded
// kernels (TopoCornellUpBox) take the room as literals and everything else from LDS.
static bool cornell_room_match(const SceneGeo& g) {
  if (g.n_xy != kCornellNXY || g.n_xz != kCornellNXZ || g.n_yz != kCornellNYZ || g.n_sph != 0 ||
      !g.has_room || g.n_txy != 0 || g.n_txz != 1 || g.n_tyz != 0 || g.n_box != 2)
    return false;
  const int nt = g.n_txy + g.n_txz + g.n_tyz;
  for (int r = 0; r < 3; ++r) {
    const CTest& C = kCornellTests.t[kCornellRoom[r]];
    if (g.test[nt + r].pos0 != C.pos0 || g.test[nt + r].pos1 != C.pos1) return false;
    for (const int pos : {C.pos0, C.pos1}) {
      const GeoRect& R = g.rect[pos];
      const CRect& H = kCornellRects[pos];
      const float a[5] = {R.k, R.ma, R.ha, R.mb, R.hb}, b[5] = {H.k, H.ma, H.ha, H.mb, H.hb};
      if (std::memcmp(a, b, sizeof a) != 0 || R.idx != H.idx) return false;
    }
  }
  return true;
}

// The light of a HEAD-room scene is the reference's (:294, fp32 geometry at grouped position 8): the
// boxes-only-uploaded kernels keep it literal, the UPLIGHT ones read it from the uploaded scene.
static bool cornell_light_match(const SceneGeo& g, int light_pos) {
  if (light_pos != kCornellLightPos) return false;
  const GeoRect& R = g.rect[light_pos];
  const CRect& H = kCornellRects[light_pos];
  const float a[5] = {R.k, R.ma, R.ha, R.mb, R.hb}, b[5] = {H.k, H.ma, H.ha, H.mb, H.hb};
  return std::memcmp(a, b, sizeof a) == 0 && R.idx == H.idx;
}

// The early resolve's clauses for a HEAD-topology scene with the reference's estimator (oracle
// c_find_early_clauses, which the proof tests check claim by claim): the room's box with y below
// the light plane (early_room_ok_k), the light's rectangle >= 1 inside the side walls and >= 1 above
// the floor, its plane <= 81.5 (0.1 below the reference's sample plane :367) and >= 0.05 below the
// ceiling, the room < 1000 across with X0, Y0, Z0 >= 0; per box a top >= 0.5 below the light plane
// and the clause its position allows against the reference's wrapped samples (x in [31, 33), z in
// [62, 64)). on = false, or a condition failing: no clause (+inf / -inf, nothing resolved early).
static void early_geo_setup(const SceneGeo& g, int light_pos, bool on, KParams* K) {
  for (int b = 0; b < 2; ++b) {
    K->eb_top[b] = INFINITY; K->eb_sgn[b] = 1.0f; K->eb_bnd[b] = -INFINITY; K->eb_z[b] = 0;
  }
  for (int a = 0; a < 3; ++a) K->er_lo[a] = K->er_span[a] = 0;
  bool ok = on && g.has_room && g.n_box == 2 && light_pos >= 0 && light_pos < g.n_xy + g.n_xz + g.n_yz &&
            light_pos >= g.n_xy && light_pos < g.n_xy + g.n_xz;  // an XZ light
  if (!ok) return;
  const int nt = g.n_txy + g.n_txz + g.n_tyz;
  float lo[3], hi[3];
  for (int a = 0; a < 3; ++a) {  // room tests: XY pair (planes z), XZ (y), YZ (x)
    const GeoTest& R = g.test[nt + a];
    const int ax = a == 0 ? 2 : (a == 1 ? 1 : 0);
    lo[ax] = std::min(R.k0, R.k1);
    hi[ax] = std::max(R.k0, R.k1);
    ok = ok && lo[ax] >= 0.0f && hi[ax] - lo[ax] <= 1000.0f;
  }
  const GeoRect& L = g.rect[light_pos];
  const float yl = L.k;
  ok = ok && L.ha >= 0.0f && L.hb >= 0.0f && L.ma - L.ha >= lo[0] + 1.0f && L.ma + L.ha <= hi[0] - 1.0f &&
       L.mb - L.hb >= lo[2] + 1.0f && L.mb + L.hb <= hi[2] - 1.0f && yl >= lo[1] + 1.0f && yl <= 81.5f &&
       hi[1] >= yl + 0.05f;
  for (int b = 0; ok && b < 2; ++b) {
    const GeoTest &XY = g.test[nt + 3 + 3 * b], &YZ = g.test[nt + 4 + 3 * b], &T = g.test[nt + 5 + 3 * b];
    const float z0 = std::min(XY.k0, XY.k1), z1 = std::max(XY.k0, XY.k1);
    const float x0 = std::min(YZ.k0, YZ.k1), x1 = std::max(YZ.k0, YZ.k1);
    // the box top at least 0.5 below the light plane (a top just under the plane left
    // the box's y-slab exit within rounding of the light crossing)
    if (!(T.k0 <= yl - 0.5f)) { ok = false; break; }
    K->eb_top[b] = T.k0;
    if (x0 >= 33.0f) { K->eb_sgn[b] = 1.0f; K->eb_bnd[b] = x0; K->eb_z[b] = 0; }
    else if (x1 <= 31.0f) { K->eb_sgn[b] = -1.0f; K->eb_bnd[b] = -x1; K->eb_z[b] = 0; }
    else if (z0 >= 64.0f) { K->eb_sgn[b] = 1.0f; K->eb_bnd[b] = z0; K->eb_z[b] = 1; }
    else if (z1 <= 62.0f) { K->eb_sgn[b] = -1.0f; K->eb_bnd[b] = -z1; K->eb_z[b] = 1; }
  }
  if (!ok) {
    for (int b = 0; b < 2; ++b) { K->eb_top[b] = INFINITY; K->eb_sgn[b] = 1.0f; K->eb_bnd[b] = -INFINITY; }
    return;
  }
  for (int a = 0; a < 3; ++a) {
    const float top = a == 1 ? std::nextafter(yl, 0.0f) : hi[a];  // y < y_L
    uint32_t blo, btop;
    std::memcpy(&blo, &lo[a], 4);
    std::memcpy(&btop, &top, 4);
    K->er_lo[a] = blo;
    K->er_span[a] = btop - blo;
  }
}

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
  for (int v = 0; v < KV_COUNT; ++v) {
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, kRenderKernels[v], kBlock, 0) !=
            hipSuccess || bpc <= 0)
      bpc = 4;
    c->bpc[v] = bpc;
  }
  c->blocks_per_cu = c->bpc[KV_GENERIC];

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
  if (e == hipSuccess) e = hipEventCreate(&c->ev2);
  if (e == hipSuccess) e = hipHostMalloc(&c->h_stats, sizeof(unsigned long long) * kStatWords, hipHostMallocDefault);
  if (e == hipSuccess) std::memset(c->h_stats, 0, sizeof(unsigned long long) * kStatWords);  // stats before any launch: zeros
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
  if (c->slots) (void)hipFree(c->slots);
  if (c->queue) (void)hipFree(c->queue);
  if (c->stats) (void)hipFree(c->stats);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev2) (void)hipEventDestroy(c->ev2);
  if (c->h_stats) (void)hipHostFree(c->h_stats);
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
  if (rows == 0) {  // a shard that owns no rows (more shards than row tiles): nothing to render
    c->samples = 0;
    c->nee_by_identity = false;
    c->scene_flop = 0;
    SPT_HIP(hipMemsetAsync(c->stats, 0, sizeof(unsigned long long) * kStatWords, stream));
    SPT_HIP(hipEventRecord(c->ev0, stream));
    SPT_HIP(hipEventRecord(c->ev1, stream));
    SPT_HIP(hipMemcpyAsync(c->h_stats, c->stats, sizeof(unsigned long long) * kStatWords,
                           hipMemcpyDeviceToHost, stream));
    SPT_HIP(hipEventRecord(c->ev2, stream));
    c->pending = true;
    c->launched = true;
    return SPT_OK;
  }
  K.n_local_pix = rows * p->width;
  K.light_black = light_pos >= 0 && c->h_prims[p->light_id].pmax == 0.0f ? 1 : 0;
  // Topology specialisation: the HEAD Cornell box (6 XY, 5 XZ, 6 YZ rects, light at grouped
  // position 8) runs a fully unrolled intersect; anything else the generic loops.
  const SceneGeo& g = *c->h_geo;
  bool all_diff = true;
  for (int i = 0; i < n_prims; ++i) all_diff = all_diff && prims[i].refl == SPT_DIFF;
  // The HEAD-topology kernels are all-DIFF, cosine-scatter specialisations; anything else (SPEC/
  // REFR, the uniform hemisphere) runs the generic kernel.
  // spt_params.flags SPT_FLAG_KERNEL_LEVEL (A/B and tests; never changes results): cap the
  // specialisation level. 0 = auto (the most specialised kernel the host can prove).
  const uint32_t klevel = (p->flags & SPT_FLAG_KERNEL_LEVEL_MASK) >> 8;
  const int kcap = klevel == SPT_KERNEL_LEVEL_GENERIC   ? 0
                   : klevel == SPT_KERNEL_LEVEL_CORNELL ? 1
                   : klevel == SPT_KERNEL_LEVEL_CONST   ? 2
                                                        : 3;
  const bool cornell = kcap >= 1 && all_diff && !(p->flags & SPT_FLAG_UNIFORM_SCATTER) &&
                       g.n_xy == 6 && g.n_xz == 5 && g.n_yz == 6 && g.n_sph == 0 && light_pos == 8 &&
                       g.n_txy == 0 && g.n_txz == 1 && g.n_tyz == 0 && g.has_room && g.n_box == 2;
  const bool cconst = cornell && kcap >= 2 && cornell_const_match(g, light_pos);
  // Estimator specialisations of the HEAD-geometry kernel (Cfg): the reference's own settings.
  // axis-aligned camera (Cfg CAMAX): horizontal.y/z and vertical.x/z zero, origin nonzero
  // (the contract-v5 terms L = llc - origin and Au_x, Av_y nonzero: the zero products then vanish
  // exactly, see the kernel's camera ray)
  bool cam_axis = K.cam[7] == 0.0f && K.cam[8] == 0.0f && K.cam[9] == 0.0f && K.cam[11] == 0.0f;
  for (int c = 0; c < 3; ++c) cam_axis = cam_axis && (K.cam[3 + c] - K.cam[c]) != 0.0f;
  cam_axis = cam_axis && K.cam[6] * (1.0f / (float)p->width) != 0.0f &&
             K.cam[10] * (1.0f / (float)p->height) != 0.0f;
  for (int i = 0; i < 12; ++i) cam_axis = cam_axis && std::isfinite(K.cam[i]);
  const bool lref = p->rr_depth == kRefRrDepth && p->light_id == kRefLightId &&
                    p->light_x0 == kRefLx0 && p->light_dx == 36.0f && p->light_z0 == kRefLz0 &&
                    p->light_dz == 36.0f && p->light_y == kRefLy && p->light_area == kRefLarea;
  K.leak_end = (p->flags & SPT_FLAG_REFERENCE_LEAKS) ? 0 : leak_end_of(prims, n_prims, g);
  // (each estimator kernel in two forms: the leak-end rule, or leaked paths as the reference's)
  const bool ref_est = K.light_black && p->max_depth == 0 && p->rr_depth >= 1 && cam_axis && lref;
  const bool head_est = cconst && kcap >= 3 && ref_est;
  // any other camera (finite): the literal kernels' CAMAX 2 forms (round 6; leak-end rule only)
  bool cam_fin = true;
  for (int i = 0; i < 12; ++i) cam_fin = cam_fin && std::isfinite(K.cam[i]);
  const bool ref_est_cam = K.light_black && p->max_depth == 0 && p->rr_depth >= 1 && cam_fin && lref &&
                           !cam_axis && K.leak_end;
  const bool head_est_cam = cconst && kcap >= 3 && ref_est_cam;
  const bool upbox_cam = cornell && !cconst && kcap >= 3 && ref_est_cam && cornell_room_match(g);
  const bool wrap_nee = p->nee_prob >= 1.0f && p->light_mode == SPT_LIGHT_GLIBC_WRAP;
  // the HEAD topology with uploaded geometry (an edited rect[]: a box moved, a wall resized) and
  // the reference's estimator: geometry from LDS, the estimator's branches compile-time
  const bool cornell_est = cornell && !cconst && kcap >= 2 && ref_est && K.leak_end;
  int kv = g.n_sph_wide > 0 ? KV_WIDE : KV_GENERIC;  // (only the wide kernel has the fp64 loop)
  if (head_est && p->nee_prob >= 1.0f && p->light_mode == SPT_LIGHT_GLIBC_WRAP)
    kv = K.leak_end ? KV_CONST_NEE : KV_CONST_NEE_REF;
  else if (head_est && p->nee_prob <= 0.0f) kv = K.leak_end ? KV_CONST_COS : KV_CONST_COS_REF;
  else if (head_est_cam && wrap_nee) kv = KV_CONST_NEE_CAM;
  else if (head_est_cam && p->nee_prob <= 0.0f) kv = KV_CONST_COS_CAM;
  else if (cconst) kv = KV_CONST;
  else if (upbox_cam && wrap_nee) kv = KV_UPBOX_NEE_CAM;
  else if (upbox_cam && p->nee_prob <= 0.0f) kv = KV_UPBOX_COS_CAM;
  else if (cornell_est && p->nee_prob >= 1.0f && p->light_mode == SPT_LIGHT_GLIBC_WRAP) kv = KV_CORNELL_NEE;
  else if (cornell_est && p->nee_prob <= 0.0f) kv = KV_CORNELL_COS;
  else if (cornell) kv = KV_CORNELL;
  else if (kv == KV_GENERIC && kcap >= 1 && all_diff && !(p->flags & SPT_FLAG_UNIFORM_SCATTER))
    kv = g.n_sph == 0
             // any other rect-only DIFF scene: run-time loops over the uploaded tests; with the
             // reference's estimator its branches compile-time as well
             ? (kcap >= 2 && ref_est && K.leak_end && p->nee_prob >= 1.0f &&
                        p->light_mode == SPT_LIGHT_GLIBC_WRAP
                    ? KV_RECTDIFF_NEE
                    : kcap >= 2 && ref_est && K.leak_end && p->nee_prob <= 0.0f ? KV_RECTDIFF_COS
                                                                                 : KV_RECTDIFF)
         : kcap >= 3 && K.light_black && lref && p->nee_prob >= 1.0f &&
                 p->light_mode == SPT_LIGHT_GLIBC_WRAP && light_pos >= 0 &&
                 prims[p->light_id].kind == SPT_RECT_XZ
             ? (K.leak_end ? KV_SPHDIFF_NEE : KV_SPHDIFF_NEE_REF)
             : KV_SPHDIFF;
  // the room HEAD's: the room literal, the boxes uploaded, the light literal when it is HEAD's too
  const bool light_head = cornell_light_match(g, light_pos);
  if (kv == KV_CORNELL_COS && kcap >= 3 && cornell_room_match(g)) kv = light_head ? KV_UPBOX_COS : KV_UPLIGHT_COS;
  if (kv == KV_UPBOX_NEE_CAM && !light_head) kv = KV_UPLIGHT_NEE_CAM;
  if (kv == KV_UPBOX_COS_CAM && !light_head) kv = KV_UPLIGHT_COS_CAM;
  // The sphere NEE kernel's early resolve needs the HEAD room (rect[] :287-294, light at index 6)
  // as prims 0..6, nothing else but narrow spheres, and a threshold above every sphere's top
  // (early_room_proven); otherwise it stays off (+inf) and every shadow ray is traced.
  K.early_y0 = INFINITY;
  if ((kv == KV_SPHDIFF_NEE || kv == KV_SPHDIFF_NEE_REF) && n_prims > 7 && g.n_sph_wide == 0) {
    spt_prim head[17];
    int32_t nh = 0;
    bool ok = spt_scene_cornell(head, 17, &nh) == SPT_OK;
    for (int i = 0; ok && i < 7; ++i) ok = std::memcmp(&prims[i], &head[i], sizeof(spt_prim)) == 0;
    double top = -INFINITY;
    for (int i = 7; ok && i < n_prims; ++i) {
      const double* g = prims[i].geom;
      ok = prims[i].kind == SPT_SPHERE && std::isfinite(g[0]) && std::isfinite(g[1]) &&
           std::isfinite(g[2]) && std::isfinite(g[3]);
      top = std::max(top, g[2] + std::fabs(g[0]));
      // the fp32 rounding argument of early_room_proven holds for |op| < 200 (and r < 200): every
      // sphere centre within 190 of every room corner, so no vertex in the room is farther away
      for (int c = 0; ok && c < 8; ++c) {
        const double cx = (c & 1) ? 99.0 : 1.0, cy = (c & 2) ? 81.6 : 0.0, cz = (c & 4) ? 170.0 : 0.0;
        ok = std::sqrt((g[1] - cx) * (g[1] - cx) + (g[2] - cy) * (g[2] - cy) +
                       (g[3] - cz) * (g[3] - cz)) < 190.0 && std::fabs(g[0]) < 190.0;
      }
    }
    if (ok && top + 1.0 < 81.0) {
      float y0 = (float)(top + 1.0);
      if ((double)y0 < top + 1.0) y0 = std::nextafter(y0, INFINITY);
      K.early_y0 = y0;
    }
  }
  // The uploaded-geometry HEAD-topology NEE kernel's early resolve (early_geo_proven): the room,
  // the light and two boxes with the margins early_geo_setup checks, the clauses it picks (oracle
  // c_find_early_clauses). Anything else: no clause, nothing resolved early.
  early_geo_setup(g, light_pos, kv == KV_CORNELL_NEE || kv == KV_UPBOX_NEE_CAM || kv == KV_UPLIGHT_NEE_CAM, &K);
  {
    const float yl = light_pos >= 0 ? g.rect[light_pos].k : 0.0f;
    std::memcpy(&K.ul_ybits, &yl, 4);
  }
  // the room HEAD's: at the auto level the kernel with the room literal (the light, the boxes and
  // the estimator's constants uploaded / literal); the const level keeps the uploaded-geometry one
  if (kv == KV_CORNELL_NEE && kcap >= 3 && cornell_room_match(g)) kv = light_head ? KV_UPBOX_NEE : KV_UPLIGHT_NEE;
  // Unit size: SPT_UNITS_PER_LANE (8) units per resident lane (C3: 96 samples); never changes
  // results (integer accumulation). Round 1 chose 16 (25.0 ms vs 26.0 ms at 8 units/lane, before
  // in-wave stealing); re-measured in round 4 with stealing, unit slots and two frames in flight
  // (profiles/r04_ab.txt session 6, 3 rounds): bench value 35.7 / 36.1 / 36.3 / 36.4 / 36.5
  // Gsamples/s at 48 / 64 / 80 / 96 / 112 samples per unit, isolated kernel 11.67 / 11.60 / 11.60 /
  // 11.68 / 11.70 ms -- fewer refills and retires, and the next frame fills the longer tail.
  int chunk = p->chunk;
  const double rays_per_sample = p->nee_prob > 0.0f ? 5.3 : 8.9;  // HEAD: NEE / cosine only
  const double lane_iters = (double)K.n_local_pix * p->spp * rays_per_sample /
                            ((double)c->n_cu * c->bpc[kv] * kBlock);
  const bool small_launch = lane_iters < SPT_SMALL_ITERS;
  // A short launch takes at most SPT_SMALL_BPC blocks per CU (half the chip's wave slots): its tail
  // is most of it, and the frame behind it (frames in flight) then runs beside it on the other half
  // instead of only in its tail. C2, round 5 (profiles/r05_blocks_per_cu_ab.json, 4 rounds): bench
  // value 17.9-18.8 -> 21.4-22.1 Gsamples/s, isolated kernel 2.88-2.95 -> 2.84-2.88 ms. Long launches
  // keep every slot (C3 at 4 blocks: isolated +8 %, value within 1 %).
  const int bpc = small_launch ? std::min(c->bpc[kv], SPT_SMALL_BPC) : c->bpc[kv];
  const double lanes = (double)c->n_cu * bpc * kBlock;  // resident lanes of THIS launch
  if (chunk <= 0) {
    if (small_launch) {
      // A short launch (C2: ~860 lane-iterations per lane): deal ~SPT_SMALL_UNITS units per lane
      // and let the in-wave stealing and guided grabs balance the rest (C2: chunk 23 -> 64,
      // 4.6 -> 4.0 ms; measured, scripts/ab_r02e.sh).
      const double units_per_pix = std::max(1.0, std::ceil(SPT_SMALL_UNITS * lanes / std::max(1, K.n_local_pix)));
      chunk = (int)std::ceil(p->spp / units_per_pix);
    } else {
      // SPT_UNITS_PER_LANE units per resident lane (above)...
      const double per_pix = std::max(1.0, SPT_UNITS_PER_LANE * lanes / std::max(1, K.n_local_pix));
      chunk = (int)std::max(4.0, std::ceil(p->spp / per_pix));
    }
    // ...but a unit should last >= ~200 lane-iterations: every unit costs a refill (~35 VALU +
    // ~40 SALU for the whole wave) and a retire (C2: 6 -> 23 samples per unit, 4.73 -> ~4.6 ms).
    chunk = std::max(chunk, (int)std::ceil(200.0 / rays_per_sample));
    chunk = std::min(chunk, p->spp);
  }
  {
    const uint32_t waves = (uint32_t)(c->n_cu * bpc * (kBlock / 64));
    uint32_t sh = 1;  // 2^sh >= 2 x waves
    while ((1u << sh) < 2u * waves && sh < 31) ++sh;
    sh = std::min(31u, sh + (uint32_t)SPT_GUIDED_EXTRA);
    K.sh_guided = small_launch ? sh : 32u;  // guided grabs cost C3 ~1 % (A/B), help C2
  }
  K.chunk = chunk;
  K.young_block = 0xFFFFFFFFu;
  K.young_cut = 0xFFFFFFFFu;
  K.steal_min = small_launch ? SPT_STEAL_MIN_SMALL : SPT_STEAL_MIN;
  const uint64_t n_chunks = ((uint64_t)p->spp + chunk - 1) / chunk;
  const uint64_t n_units = n_chunks * (uint64_t)K.n_local_pix;
  if (n_units >= 0x80000000ull) return fail(SPT_ERR_INVALID_ARG, "too many work units; raise chunk");
  K.n_units = (uint32_t)n_units;
  // the literal HEAD NEE kernels (and the boxes-only-uploaded one: edited scene -4 %) at 8 blocks
  // per CU only (the measured shape): the sphere kernel (C5) lost 3.6 %, the uploaded-geometry
  // kernels 0.5-2.4 % of kernel time or ~1.5 % of pipelined value (profiles/r05_young_cut_ab.json)
  if (!small_launch && bpc == 8 &&
      (kv == KV_CONST_NEE || kv == KV_CONST_NEE_REF || kv == KV_UPBOX_NEE || kv == KV_CONST_NEE_CAM ||
       kv == KV_UPBOX_NEE_CAM || kv == KV_UPLIGHT_NEE || kv == KV_UPLIGHT_NEE_CAM) &&
      SPT_YOUNG_CUT > 0) {
    K.young_block = (uint32_t)(SPT_YOUNG_RANK * c->n_cu);
    K.young_cut = (uint32_t)(n_units * (uint64_t)SPT_YOUNG_CUT / 1000u);
  }
  magic31((uint32_t)K.n_local_pix, &K.m_npix, &K.sh_npix);
  // pixel-order spreading: the largest K = 2^k <= SPT_SCRAMBLE_K dividing n_local_pix
  K.scr_k = 0;
  while ((1 << (K.scr_k + 1)) <= SPT_SCRAMBLE_K && K.n_local_pix % (1 << (K.scr_k + 1)) == 0) ++K.scr_k;
  K.scr_q = (uint32_t)K.n_local_pix >> K.scr_k;
  magic31((uint32_t)p->width, &K.m_w, &K.sh_w);
  magic31((uint32_t)K.tile_rows, &K.m_tile, &K.sh_tile);
  K.inv_spp = 1.0f / (float)p->spp;
  K.fix_scale = K.inv_spp * 2147483648.0f;
  K.inv_w = 1.0f / (float)p->width;
  K.inv_h = 1.0f / (float)p->height;
  for (int c = 0; c < 3; ++c) {  // camera of contract v5 (oracle c_path)
    K.cam_au[c] = K.cam[6 + c] * K.inv_w;
    K.cam_av[c] = K.cam[9 + c] * K.inv_h;
    K.cam_cu[c] = K.cam_au[c] * 0x1p-16f;
    K.cam_cv[c] = K.cam_av[c] * 0x1p-16f;
    K.cam_l[c] = K.cam[3 + c] - K.cam[c];
  }
  {  // light sample lattice of contract v5 (oracle c_wrap_sample)
    auto lattice = [](uint32_t dx, float x0, int* on, uint32_t* shift, float* scale, float* x0m1) {
      int a = 0;
      while (a < 32 && dx != 0 && !((dx >> a) & 1u)) ++a;
      *on = dx != 0 && a >= 1 && a <= 24;
      *shift = *on ? 7u + (uint32_t)a : 0u;
      *scale = std::ldexp(1.0f, a - 24);
      *x0m1 = x0 - 1.0f;
    };
    lattice(K.ldxi, K.lx0, &K.lx_lattice, &K.lx_shift, &K.lx_scale, &K.lx0m1);
    lattice(K.ldzi, K.lz0, &K.lz_lattice, &K.lz_shift, &K.lz_scale, &K.lz0m1);
  }
  K.accum = c->accum;
  if (3ull * n_units > c->slots_cap) {  // one owner store per unit (24 B): C3 208 MB, C4/C5 ~400 MB
    if (c->slots) SPT_HIP(hipFree(c->slots));
    c->slots = nullptr;
    c->slots_cap = 0;
    SPT_HIP(hipMalloc(&c->slots, 3ull * n_units * sizeof(unsigned long long)));
    c->slots_cap = 3ull * n_units;
  }
  K.slots = c->slots;
  K.queue = c->queue;
  K.stats = c->stats;
  K.light_kind = light_pos >= 0 ? prims[p->light_id].kind : 0;
  K.light_pos = light_pos;
  K.scatter_uniform = (p->flags & SPT_FLAG_UNIFORM_SCATTER) ? 1 : 0;
  // Ray-direction contract (oracle c_unit_dirs): unit directions iff a sphere or a REFR primitive
  K.unit_dirs = 0;
  for (int i = 0; i < n_prims; ++i)
    if (prims[i].kind == SPT_SPHERE || prims[i].refl == SPT_REFR) K.unit_dirs = 1;
  K.nee_c = (float)((double)p->light_area / 3.14159265358979323846);
  c->n_prims = n_prims;
  c->last = K;
  c->samples = (uint64_t)K.n_local_pix * (uint64_t)p->spp;
  c->scene_flop = 0;
  for (int i = 0; i < n_prims; ++i)
    c->scene_flop += prims[i].kind == SPT_SPHERE ? SPT_FLOP_SPHERE : SPT_FLOP_RECT;

  SPT_HIP(hipMemsetAsync(c->accum, 0, sizeof(unsigned long long) * 3 * (size_t)K.n_local_pix,
                         stream));
  SPT_HIP(hipMemsetAsync(c->queue, 0, sizeof(uint32_t), stream));
  SPT_HIP(hipMemsetAsync(c->stats, 0, sizeof(unsigned long long) * kStatWords, stream));
#ifdef SPT_WAVE_TIMES
  SPT_HIP(hipMemsetAsync(c->stats + 14, 0xFF, sizeof(unsigned long long), stream));
#endif
  c->nee_by_identity = kv == KV_CONST_NEE_CAM || kv == KV_UPBOX_NEE_CAM || kv == KV_UPLIGHT_NEE ||
                       kv == KV_UPLIGHT_NEE_CAM ||
                       kv == KV_CONST_NEE || kv == KV_SPHDIFF_NEE || kv == KV_CONST_NEE_REF ||
                       kv == KV_SPHDIFF_NEE_REF || kv == KV_CORNELL_NEE || kv == KV_RECTDIFF_NEE ||
                       kv == KV_UPBOX_NEE;
  const int grid = c->n_cu * bpc;
  *c->h_kp = K;
  SPT_HIP(hipMemcpyAsync(c->d_kp, c->h_kp, sizeof(KParams), hipMemcpyHostToDevice, stream));
  SPT_HIP(hipEventRecord(c->ev0, stream));
  hipLaunchKernelGGL(kRenderKernels[kv], dim3(grid), dim3(kBlock), 0, stream,
                     (const KParams*)c->d_kp);
  SPT_HIP(hipGetLastError());
  SPT_HIP(hipEventRecord(c->ev1, stream));
  const uint32_t np = (uint32_t)K.n_local_pix;
  hipLaunchKernelGGL(finalize_slots_kernel, dim3((np + kBlock - 1) / kBlock), dim3(kBlock), 0, stream,
                     (const unsigned long long*)c->accum, (const unsigned long long*)c->slots,
                     rgb_dev, np, (uint32_t)n_chunks, K.scr_k, K.scr_q,
                     (const unsigned long long*)c->stats);
  SPT_HIP(hipGetLastError());
  SPT_HIP(hipMemcpyAsync(c->h_stats, c->stats, sizeof(unsigned long long) * kStatWords,
                         hipMemcpyDeviceToHost, stream));
  SPT_HIP(hipEventRecord(c->ev2, stream));
  c->pending = true;
  c->launched = true;
  return SPT_OK;
}

extern "C" spt_status spt_context_stats(spt_context* c, spt_stats* out) {
  if (!c || !out) return fail(SPT_ERR_INVALID_ARG, "null argument");
  if (!c->launched) return fail(SPT_ERR_INVALID_ARG, "no render has been enqueued on this context");
  SPT_HIP(hipSetDevice(c->device));
  SPT_HIP(hipEventSynchronize(c->ev2));
  const unsigned long long* h = c->h_stats;
#ifdef SPT_WAVE_TIMES
  std::fprintf(stderr, "SPT_WAVE_TIMES sum=%llu sumsq=%llu first=%llu last=%llu iters=%llu maxiters=%llu "
               "sumstart16=%llu sumend16=%llu smid=%llu\n",
               h[12], h[13], h[14], h[15], h[16], h[17], h[18], h[19], h[20]);
  if (const char* path = std::getenv("SPT_WAVE_DUMP")) {  // diagnostic build only
    if (FILE* f = std::fopen(path, "wb")) {
      std::fwrite(h + 32, sizeof(unsigned long long), 3 * 32768, f);
      std::fclose(f);
    }
  }
#endif
#ifdef SPT_REGION_STATS
  {
    static const char* names[10] = {"iteration", "unit_retire", "refill", "camera", "path_isect",
                                    "diff_shading", "shadow_test", "nee_light_hit", "cosine",
                                    "path_end"};
    std::fprintf(stderr, "SPT_REGION_STATS");
    for (int r = 0; r < 10; ++r)
      std::fprintf(stderr, " %s=%llu/%llu", names[r], h[kStatRegion + 2 * r],
                   h[kStatRegion + 1 + 2 * r]);
    std::fprintf(stderr, "\n");
  }
#endif
  if (h[0] != 0) {
    c->pending = false;
    return fail(SPT_ERR_HIP, "render kernel hit its iteration cap in " + std::to_string(h[0]) +
                                 " waves (a path did not terminate); the image is incomplete");
  }
  float ms = 0.0f;
  SPT_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  std::memset(out, 0, sizeof *out);
  out->samples = c->samples; out->path_rays = h[1]; out->shadow_rays = h[2]; out->vertices = h[3];
  out->nee_events = h[4]; out->nee_light_hits = h[5]; out->cosine_samples = h[6];
  out->misses = h[7];
  out->shadow_traced = h[kStatShadowTraced];
  out->sphere_vertices = h[kStatSphereVertices];
  out->shadow_proven = h[kStatShadowProven];
  if (c->nee_by_identity) {  // HEAD NEE kernels: one NEE event per non-terminal vertex
    out->nee_events = out->vertices - out->samples;
    out->shadow_rays = out->nee_events;
  }
  // FLOP model (include/spt_flops.h): scene cost per ray from the primitive mix. `flop` charges
  // a full scene test for every shadow ray of the reference (:466); `flop_executed` only for the
  // shadow rays the kernel traced (the others are rejected exactly by the light pre-test or
  // resolved by early_nee_proven()).
  const double scene = c->scene_flop;
  const double common = (double)out->samples * SPT_FLOP_SAMPLE +
                        (double)out->path_rays * scene + (double)out->vertices * SPT_FLOP_VERTEX +
                        (double)out->sphere_vertices * SPT_FLOP_SPHERE_NORMAL +
                        (double)(out->vertices - out->samples) * SPT_FLOP_COMBINE +
                        (double)out->cosine_samples * SPT_FLOP_COSINE +
                        (double)out->nee_events * SPT_FLOP_NEE +
                        (double)out->nee_light_hits * SPT_FLOP_NEE_HIT;
  out->flop = common + (double)out->shadow_rays * scene;
  out->flop_executed = common + (double)(out->shadow_traced - out->shadow_proven) * scene;
  out->kernel_ms = ms;
  c->pending = false;
  return SPT_OK;
}

// The one-shot drop-in (spt_render) keeps one context and one device output buffer per device for
// the life of the process (or until spt_shutdown), so a caller that renders repeatedly -- the
// reference's main() replaced by smallpt_amd, or a Python loop over spt.render -- pays context
// creation, the unit-slot allocation (~200 MB at C3) and the cold first launch once, not per call.
// Calls on one device are serialised by that device's mutex; different devices run concurrently.
namespace {
constexpr int kMaxDropInDevices = 64;
struct DropIn {
  std::mutex mu;
  spt_context* ctx = nullptr;
  float* out = nullptr;  // device output, grown on demand
  size_t out_cap = 0;    // floats
};
DropIn g_dropin[kMaxDropInDevices];
}  // namespace

extern "C" spt_status spt_render(const spt_prim* prims, int32_t n_prims, const spt_camera* cam,
                                 const spt_params* p, float* rgb_out, spt_stats* stats) {
  if (!rgb_out) return fail(SPT_ERR_INVALID_ARG, "null rgb_out");
  spt_status st = validate(prims, n_prims, cam, p);
  if (st != SPT_OK) return st;
  if (p->device < 0 || p->device >= kMaxDropInDevices) return fail(SPT_ERR_INVALID_ARG, "bad device ordinal");
  const size_t n = 3ull * (size_t)spt_shard_row_count(p) * (size_t)p->width;
  if (n == 0) {  // this shard owns no rows: nothing to render, no context or device memory
    if (stats) std::memset(stats, 0, sizeof *stats);
    return SPT_OK;
  }
  DropIn& D = g_dropin[p->device];
  std::lock_guard<std::mutex> lock(D.mu);
  if (!D.ctx) {
    st = spt_context_create(p->device, &D.ctx);
    if (st != SPT_OK) {
      D.ctx = nullptr;
      return st;
    }
  }
  SPT_HIP(hipSetDevice(p->device));
  if (n > D.out_cap) {
    if (D.out) SPT_HIP(hipFree(D.out));
    D.out = nullptr;
    D.out_cap = 0;
    SPT_HIP(hipMalloc(&D.out, n * sizeof(float)));
    D.out_cap = n;
  }
  st = spt_render_async(D.ctx, prims, n_prims, cam, p, D.out, nullptr);
  if (st == SPT_OK) {
    spt_stats tmp;
    st = spt_context_stats(D.ctx, stats ? stats : &tmp);
  }
  if (st == SPT_OK) SPT_HIP(hipMemcpy(rgb_out, D.out, n * sizeof(float), hipMemcpyDeviceToHost));
  return st;
}

extern "C" spt_status spt_shutdown(void) {
  for (DropIn& D : g_dropin) {
    std::lock_guard<std::mutex> lock(D.mu);
    if (D.ctx) {
      const int dev = D.ctx->device;
      spt_context_destroy(D.ctx);
      D.ctx = nullptr;
      if (D.out) {
        (void)hipSetDevice(dev);
        (void)hipFree(D.out);
      }
    }
    D.out = nullptr;
    D.out_cap = 0;
  }
  return SPT_OK;
}

extern "C" int32_t spt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" const char* spt_last_error(void) { return g_last_error.c_str(); }
