// spt_device.h — device-side building blocks of the counter-mode contract (gfx950).
//
// Every float operation here is spelled exactly as in the contract (DESIGN.md "Counter-mode
// contract", restated on the CPU in oracle/spt_oracle.c): explicit fmaf, IEEE '/' where the
// contract keeps a true division, integer-seeded Newton-Raphson reciprocal / rsqrt elsewhere,
// no fast-math and no implicit contraction (-ffp-contract=off), so the kernel reproduces the CPU
// statement of the same contract bit for bit.
//
// Cost model on gfx950 (tools/valu_rates.hip, measured): add/mul/fma/xor/cmp full rate (2 cyc per
// wave64 instruction per SIMD); v_mad_u64_u32, v_mul_lo/hi_u32, packed fp32 half rate; v_rcp /
// v_sqrt / v_sin quarter rate. A correctly rounded fp32 '/' or sqrtf is a ~30-cycle sequence;
// rcp_nr / rsq_nr below are 7 / 11 full-rate instructions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/spt.h"

namespace spt {

// ---- Philox4x32-R (Salmon et al. SC'11; R = SPT_PHILOX_ROUNDS = 7, include/spt.h), replaces
// erand48/rand() (utilities.h:26-51, smallpt.cpp:365-366,460,533-534). Fixed key
// (SPT_PHILOX_KEY0/1): the whole key schedule is compile-time, so each round is two
// v_mad_u64_u32 and two xors. Counter = (pixel, sample, vertex | stream << 31, seed).
constexpr uint32_t kPhM0 = 0xD2511F53u, kPhM1 = 0xCD9E8D57u;
constexpr uint32_t kPhW0 = 0x9E3779B9u, kPhW1 = 0xBB67AE85u;

struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  uint32_t k0 = SPT_PHILOX_KEY0, k1 = SPT_PHILOX_KEY1;
#pragma unroll
  for (int r = 0; r < SPT_PHILOX_ROUNDS; ++r) {
    const uint64_t p0 = (uint64_t)kPhM0 * c0;  // one v_mad_u64_u32 each (hi and lo together)
    const uint64_t p1 = (uint64_t)kPhM1 * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    k0 += kPhW0; k1 += kPhW1;
  }
  return u4{c0, c1, c2, c3};
}

// The same generator with the counter word c0 (the pixel) and c3 (the seed) fixed for a whole work
// unit: round 1's product M0 * c0 and its xor with c3 and the first key word are computed once per
// unit (PxKey), so each call saves one v_mad_u64_u32 and one v_xor. Bit-identical to
// philox4x32(pix, c1, c2, seed).
// Round 2 multiplies that same word (round 1's n2, per unit) by M1, so its product is per unit too:
// PxKey keeps hi(M1 * n2) ^ k0(round 2), lo(M1 * n2) and round 1's c3 = lo(M0 * pix), which saves a
// second v_mad_u64_u32 per call.
struct PxKey { uint32_t qhi, qlo, lo; };
__device__ __forceinline__ PxKey philox_pixel_key(uint32_t pix, uint32_t seed) {
  const uint64_t p0 = (uint64_t)kPhM0 * pix;
  const uint32_t n2 = (uint32_t)(p0 >> 32) ^ seed ^ (uint32_t)SPT_PHILOX_KEY1;
  const uint64_t q1 = (uint64_t)kPhM1 * n2;
  return PxKey{(uint32_t)(q1 >> 32) ^ (uint32_t)(SPT_PHILOX_KEY0 + kPhW0), (uint32_t)q1, (uint32_t)p0};
}
// a ^ b ^ k in ONE full-rate v_bitop3_b32 (tools/valu_rates: v_xor and v_bitop3 issue at the same
// rate), k a compile-time round key held in an SGPR: halves the xor count of a Philox round.
__device__ __forceinline__ uint32_t xor3k(uint32_t a, uint32_t b, uint32_t k) {
  uint32_t r;
  // (round 3 A/B: two VOP2 xors with the key as a literal instead -- no s_mov of the key into an
  // SGPR, 16 SALU fewer and 16 VALU more per call -- cost C3 +1.3 %: VALU issue is the binding cost)
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
}
__device__ __forceinline__ u4 philox_px(PxKey pk, uint32_t c1, uint32_t c2) {
  uint32_t k0 = SPT_PHILOX_KEY0, k1 = SPT_PHILOX_KEY1;
  // round 1: the pixel word's product is per unit (philox_pixel_key)
  const uint64_t p1 = (uint64_t)kPhM1 * c2;
  uint32_t c0 = xor3k((uint32_t)(p1 >> 32), c1, k0), c3 = pk.lo;
  c1 = (uint32_t)p1;
  k0 += kPhW0; k1 += kPhW1;
  // round 2: M1 * c2 is per unit as well (pk.qhi already holds its high word ^ k0)
  {
    const uint64_t p0 = (uint64_t)kPhM0 * c0;
    const uint32_t n0 = pk.qhi ^ c1;
    const uint32_t n2 = xor3k((uint32_t)(p0 >> 32), c3, k1);
    c0 = n0; c1 = pk.qlo; c2 = n2; c3 = (uint32_t)p0;
    k0 += kPhW0; k1 += kPhW1;
  }
#pragma unroll
  for (int r = 2; r < SPT_PHILOX_ROUNDS; ++r) {
    const uint64_t p0 = (uint64_t)kPhM0 * c0;
    const uint64_t q1 = (uint64_t)kPhM1 * c2;
    const uint32_t n0 = xor3k((uint32_t)(q1 >> 32), c1, k0);
    const uint32_t n2 = xor3k((uint32_t)(p0 >> 32), c3, k1);
    c0 = n0; c1 = (uint32_t)q1; c2 = n2; c3 = (uint32_t)p0;
    k0 += kPhW0; k1 += kPhW1;
  }
  return u4{c0, c1, c2, c3};
}

// A uniform [0, 1) float from the top 23 bits (contract v5, oracle u01): the float 1 + m 2^-23
// (bits 0x3F800000 | m) minus 1 -- an or and a subtract (rounds 1-4: shift, half-rate conversion,
// multiply)
__device__ __forceinline__ float u01(uint32_t v) { return __uint_as_float(0x3F800000u | (v >> 9)) - 1.0f; }
// 16-bit draw from the low bytes of two Philox words (RR and NEE-mix draws, camera jitter; see
// the kernel): (lo & 0xFF) | (hi & 0xFF) << 8 as ONE v_perm_b32 (bytes {hi:lo}[4], [0], 0, 0).
__device__ __forceinline__ uint32_t u16i(uint32_t lo, uint32_t hi) {
  return __builtin_amdgcn_perm(hi, lo, 0x0C0C0400u);
}
__device__ __forceinline__ float u16(uint32_t lo, uint32_t hi) { return (float)u16i(lo, hi) * 0x1p-16f; }

// ---- deterministic reciprocal / reciprocal square root (contract): integer seed + 3 Newton
// steps; max relative error 6e-8 / 1.3e-7 (oracle tests). rcp_nr(+-0) is NaN, which the
// intersection treats exactly like 1/0 = inf (no hit on a parallel plane).
__device__ __forceinline__ float rcp_nr(float x) {
  float y = __uint_as_float(0x7EF311C3u - __float_as_uint(x));
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float e = fmaf(-x, y, 1.0f);
    y = fmaf(e, y, y);
  }
  return y;
}
__device__ __forceinline__ float rsq_nr(float x) {
  float y = __uint_as_float(0x5F375A86u - (__float_as_uint(x) >> 1));
  const float h = 0.5f * x;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float hy = h * y;
    y = y * fmaf(-hy, y, 1.5f);
  }
  return y;
}

// The same with one Newton step (relative error < 1.8e-3, always below the root): the free-scale
// contract's normalize of the path directions (contract v7, oracle c_unit_dirs). Not the cosine
// sample's R, whose error would bias the sampled distribution.
__device__ __forceinline__ float rsq_nr1(float x) {
  const float y = __uint_as_float(0x5F375A86u - (__float_as_uint(x) >> 1));
  const float hy = (0.5f * x) * y;
  return y * fmaf(-hy, y, 1.5f);
}
// With two Newton steps (relative error < 5e-6): the cosine sample's R in the free-scale contract
// and the sphere root (oracle c_sphere).
__device__ __forceinline__ float rsq_nr2(float x) {
  float y = __uint_as_float(0x5F375A86u - (__float_as_uint(x) >> 1));
  const float h = 0.5f * x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float hy = h * y;
    y = y * fmaf(-hy, y, 1.5f);
  }
  return y;
}

// Materialise v here, unconditionally: LLVM turns `c ? a : expensive(b)` back into a branch around
// the expensive side, and each such branch costs exec-mask SALU, the loop's binding resource.
template <typename T>
__device__ __forceinline__ T keep(T v) {
  asm volatile("" : "+v"(v));
  return v;
}

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
// Vec::norm :50-52 as *this * rsq_nr(len2) (contract, oracle fnormalize; round 1 kept exactly-unit
// vectors unchanged with a compare + select, two VALU per normalize for a 2^-24 case).
__device__ __forceinline__ f3 normalize3(f3 v) {
  const float l2 = fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x));
  const float inv = rsq_nr(l2);
  return mk(v.x * inv, v.y * inv, v.z * inv);
}
// The free-scale contract's normalize (contract v7, oracle fnormalize_free): rsq with ONE Newton
// step, |d| = 1 within 1.8e-3 (rounds 1-4: two steps, 5e-6). The scale of a path direction places
// no geometry -- the hit point o + d t is the same real point -- it only moves the roundings that
// set the self-hit / leak statistics, which stay within 0.3 %.
__device__ __forceinline__ f3 normalize3_free(f3 v) {
  const float l2 = fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x));
  const float inv = rsq_nr1(l2);
  return mk(v.x * inv, v.y * inv, v.z * inv);
}
__device__ __forceinline__ f3 normalize_dir(f3 v, bool unit) { return unit ? normalize3(v) : normalize3_free(v); }
// operator% :56-58
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

// sin/cos(2*pi*xi), xi in [0,1): exact quarter-turn reduction, Taylor in r = 4*xi - rint(4*xi).
__device__ __forceinline__ void sincos2pi(float xi, float& s_out, float& c_out) {
  const float q = xi * 4.0f;
  const float kf = rintf(q);
  const float r = q - kf;
  const int k = (int)kf & 3;
  const float r2 = r * r;
  float ps = fmaf(r2, 0.000160441184787359821f, -0.00468175413531868810f);
  float pc = fmaf(r2, 0.000919260274839426030f, -0.0208634807633529609f);
  ps = fmaf(r2, ps, 0.0796926262461670451f);
  ps = fmaf(r2, ps, -0.645964097506246254f);
  ps = fmaf(r2, ps, 1.57079632679489662f);
  const float s = r * ps;
  pc = fmaf(r2, pc, 0.253669507901048014f);
  pc = fmaf(r2, pc, -1.23370055013616983f);
  const float c = fmaf(r2, pc, 1.0f);
  const float sa = (k & 1) ? c : s;   // k=0:( s, c) 1:( c,-s) 2:(-s,-c) 3:(-c, s)
  const float ca = (k & 1) ? s : c;
  s_out = (k & 2) ? -sa : sa;
  c_out = (k == 1 || k == 2) ? -ca : ca;
}

// The azimuth of random_scattering (:343) from one Philox word by octant symmetry (oracle
// spt_oracle_disk_dir): bits 31, 30 = signs of cos and sin, bit 29 = swap, bits 28..8 = theta in
// [0, pi/4) as quarter turns r = u * 2^-22 for the sincos2pi polynomials. No range reduction and no
// quadrant rotation: two sign-bit inserts and one conditional swap.
__device__ __forceinline__ void disk_dir(uint32_t ra, float& c_out, float& s_out) {
  // r = u * 2^-22 for the 21-bit u = bits 28..8: the float with bits 0x4B000000 | u is 2^23 + u,
  // so fma(2^23 + u, 2^-22, -2) is u * 2^-22 exactly (the bits of (float)u * 0x1p-22f, with a
  // full-rate v_or instead of a half-rate conversion and a multiply)
  const float r = fmaf(__uint_as_float(__builtin_amdgcn_ubfe(ra, 8, 21) | 0x4B000000u), 0x1p-22f, -2.0f);
  const float r2 = r * r;
  // minimax sin / cos on [0, pi/4], 4 terms each (oracle DD_*: within 1.3e-7 relative in fp32)
  float ps = fmaf(r2, -0.004601659253239632f, 0.07968003302812576f);
  float pc = fmaf(r2, -0.020417289808392525f, 0.2536032199859619f);
  ps = fmaf(r2, ps, -0.6459634900093079f);
  ps = fmaf(r2, ps, 1.5707963705062866f);
  const float sn = r * ps;
  pc = fmaf(r2, pc, -1.2336976528167725f);
  const float cs = fmaf(r2, pc, 1.0f);
  const bool sw = (ra & 0x20000000u) != 0u;
  const float c = sw ? sn : cs, s = sw ? cs : sn;
  c_out = __uint_as_float(__float_as_uint(c) ^ (ra & 0x80000000u));
  s_out = __uint_as_float(__float_as_uint(s) ^ ((ra << 1) & 0x80000000u));
}

// random_scattering :337-347 (cosine-weighted hemisphere about nl), before the final normalize
// (the kernel shares that normalize with the camera ray, :536). AXIS: nl is known to be
// axis-aligned (rect-only scenes); otherwise it is tested per lane, as the oracle does.
// uniform: the reference's commented-out uniform hemisphere (:352-359), radial sqrt(r2(2-r2)) and
// normal component 1-r2 (SPT_FLAG_UNIFORM_SCATTER; oracle c_cosine).
// unit: the unit-direction contract (rsq_nr) or the free-scale one (rsq_nr2; oracle c_unit_dirs).
template <bool AXIS = false>
__device__ __forceinline__ f3 cosine_vec(f3 nl, uint32_t ra, uint32_t rb, bool uniform, bool unit) {
  const float xi2 = u01(rb);
  float s, c;
  disk_dir(ra, c, s);  // the azimuth r1 = 2*pi*xi1 of :343
  float r2s, s1;
  if (uniform) {
    const float m = xi2 * (2.0f - xi2);
    r2s = m * (unit ? rsq_nr(m) : rsq_nr2(m));
    s1 = 1.0f - xi2;
  } else {
    // Contract (oracle c_cosine): sqrt(r2) and sqrt(1 - r2) of :343-347 scaled by 1/sqrt(1 - r2),
    // since the kernel normalizes the direction anyway: R = sqrt(r2 / (1 - r2)) with ONE rsqrt,
    // R = r2 * rsq(r2 * (1 - r2)) (r2 = 0 gives 0), and a normal component of exactly 1.
    const float q = xi2 * (1.0f - xi2);
    r2s = xi2 * (unit ? rsq_nr(q) : rsq_nr2(q));
    s1 = 1.0f;
  }
  const float cr = c * r2s, sr = s * r2s;
  // Contract: an axis-aligned normal (every rectangle's, :123,:166,:209) makes the frame of
  // :345-346 a signed permutation of the axes: (sx,0,0) -> (sx*s1, sr, -sx*cr);
  // (0,sy,0) -> (sr, sy*s1, sy*cr); (0,0,sz) -> (sr, -sz*cr, sz*s1) (oracle c_cosine). Written
  // with the normal's components as 0 / +-1 weights (round 5): six fmas and no compare or select,
  // the same values up to the sign of an exact zero, which nothing downstream reads (a zero
  // direction component's rcp_nr is NaN for either sign).
  if (AXIS || (fabsf(nl.x) + fabsf(nl.y) + fabsf(nl.z) == 1.0f &&
               ((int)(nl.x == 0.0f) + (int)(nl.y == 0.0f) + (int)(nl.z == 0.0f)) == 2)) {
    return mk(fmaf(nl.x, s1, fmaf(-fabsf(nl.x), sr, sr)),
              fmaf(fabsf(nl.x), sr, fmaf(nl.y, s1, -(nl.z * cr))),
              fmaf(nl.z, s1, (nl.y - nl.x) * cr));
  }
  const f3 a = fabsf(nl.x) > 0.1f ? mk(nl.z, 0.0f, -nl.x) : mk(0.0f, -nl.z, nl.y);
  const f3 u = normalize3(a);
  const f3 v = cross3(nl, u);
  return mk(fmaf(nl.x, s1, fmaf(v.x, sr, u.x * cr)), fmaf(nl.y, s1, fmaf(v.y, sr, u.y * cr)),
            fmaf(nl.z, s1, fmaf(v.z, sr, u.z * cr)));
}


// 1.31 fixed-point per-sample contribution (order-independent, exact integer accumulation):
// min(L/spp, 1) * 2^31 truncated (oracle c_fix). scale = inv_spp * 2^31 (exact), and
// RN(L * scale) = RN(L * inv_spp) * 2^31 (a power-of-two scaling commutes with rounding), so this is
// min(L * scale, 2^31) — one mul and one min. L >= 0 always (T, e >= 0); NaN -> 2^31 as fminf(NaN, 1).
__device__ __forceinline__ uint32_t fix31(float L, float scale) {
  return (uint32_t)fminf(L * scale, 2147483648.0f);
}

}  // namespace spt
