// spt_device.h — device-side building blocks of the counter-mode contract (gfx950).
//
// Every float operation here is spelled exactly as in the contract (DESIGN.md "Counter-mode
// contract"): explicit fmaf, IEEE correctly rounded '/' and sqrtf (built with
// -fhip-fp32-correctly-rounded-divide-sqrt -ffp-contract=off), no fast-math, so the kernel
// reproduces the CPU statement of the same contract bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spt {

// ---- Philox4x32-10 (Salmon et al. SC'11), replaces erand48/rand() (utilities.h:26-51,
// smallpt.cpp:365-366,460,533-534). Counter = (pixel, sample, vertex, stream), key = (seed, "SPT1").
constexpr uint32_t kPhM0 = 0xD2511F53u, kPhM1 = 0xCD9E8D57u;
constexpr uint32_t kPhW0 = 0x9E3779B9u, kPhW1 = 0xBB67AE85u;

struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(kPhM0, c0), lo0 = kPhM0 * c0;
    const uint32_t hi1 = __umulhi(kPhM1, c2), lo1 = kPhM1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += kPhW0; k1 += kPhW1;
  }
  return u4{c0, c1, c2, c3};
}

__device__ __forceinline__ float u01(uint32_t v) { return (float)(v >> 8) * 0x1p-24f; }

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
// Vec::norm :50-52 as *this * (1/sqrt(len2)).
__device__ __forceinline__ f3 normalize3(f3 v) {
  const float inv = 1.0f / sqrtf(fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x)));
  return mk(v.x * inv, v.y * inv, v.z * inv);
}
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

// random_scattering :337-347 (cosine-weighted hemisphere about nl).
__device__ __forceinline__ f3 cosine_dir(f3 nl, uint32_t ra, uint32_t rb) {
  const float xi1 = u01(ra), xi2 = u01(rb);
  float s, c;
  sincos2pi(xi1, s, c);
  const float r2s = sqrtf(xi2);
  const float s1 = sqrtf(1.0f - xi2);
  const f3 a = fabsf(nl.x) > 0.1f ? mk(nl.z, 0.0f, -nl.x) : mk(0.0f, -nl.z, nl.y);
  const f3 u = normalize3(a);
  const f3 v = cross3(nl, u);
  const float cr = c * r2s, sr = s * r2s;
  return normalize3(mk(fmaf(nl.x, s1, fmaf(v.x, sr, u.x * cr)),
                       fmaf(nl.y, s1, fmaf(v.y, sr, u.y * cr)),
                       fmaf(nl.z, s1, fmaf(v.z, sr, u.z * cr))));
}

// Fixed-point per-sample contribution (order-independent, exact integer accumulation).
__device__ __forceinline__ unsigned long long fix32(float L, float inv_spp) {
  float c = L * inv_spp;
  if (!(c >= 0.0f)) c = 0.0f;
  if (c > 1.0f) c = 1.0f;
  return (unsigned long long)(c * 4294967296.0f);
}

}  // namespace spt
