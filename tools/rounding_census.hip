// rounding_census.hip — are gfx950's v_rcp_f32 / v_rsq_f32 / v_sqrt_f32 correctly rounded?
// Exhaustive over every float in [1, 4) (all 2^23 significands of both exponent parities; the
// results for other binades are exact power-of-two scalings away from denormals and overflow).
// A hardware approximation the CPU can reproduce bit for bit (i.e. correctly rounded) could
// replace the contract's Newton-Raphson rcp_nr / rsq_nr. Exactness is checked with integer
// arithmetic: y = RN(1/x) iff x*(y - u/2) < 1 < x*(y + u/2) (u = ulp(y)), and the same for
// 1/sqrt(x) and sqrt(x) with squared bounds, all in 128-bit integers.
//   hipcc --offload-arch=gfx950 -O2 -fhip-fp32-correctly-rounded-divide-sqrt -o tools/rounding_census tools/rounding_census.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned __int128 u128;

// x = mx * 2^ex (mx 24-bit integer), y = my * 2^ey. Returns -1 if y too small, +1 if too large, 0 if
// y is the correctly rounded value of f(x) with f = 1/x (kind 0), 1/sqrt(x) (1), sqrt(x) (2).
__device__ int check(uint32_t xb, uint32_t yb, int kind) {
  const uint64_t mx = (xb & 0x7FFFFF) | 0x800000;
  const int ex = (int)((xb >> 23) & 0xFF) - 127 - 23;
  const uint64_t my = (yb & 0x7FFFFF) | 0x800000;
  const int ey = (int)((yb >> 23) & 0xFF) - 127 - 23;
  // bounds: lo = (2my - 1) * 2^(ey-1), hi = (2my + 1) * 2^(ey-1)
  const uint64_t lo = 2 * my - 1, hi = 2 * my + 1;
  const int e = ey - 1;
  // compare g(bound) with 1 (kinds 0, 1) or with x (kind 2), as integers scaled by powers of two
  auto cmp = [&](uint64_t b) -> int {  // sign of (value(b) - target)
    if (kind == 0) {  // x * b * 2^(ex + e) vs 1
      const u128 p = (u128)mx * b;
      const int s = ex + e;  // p * 2^s vs 1
      if (s >= 0) return 1;
      const int sh = -s;
      if (sh >= 127) return -1;
      const u128 one = (u128)1 << sh;
      return p > one ? 1 : (p < one ? -1 : 0);
    } else if (kind == 1) {  // x * b^2 * 2^(ex + 2e) vs 1
      const u128 p = (u128)mx * b * b;
      const int s = ex + 2 * e;
      if (s >= 0) return 1;
      const int sh = -s;
      if (sh >= 127) return -1;
      const u128 one = (u128)1 << sh;
      return p > one ? 1 : (p < one ? -1 : 0);
    } else {  // b^2 * 2^(2e) vs mx * 2^ex
      const u128 p = (u128)b * b;
      int s = 2 * e - ex;  // p * 2^s vs mx
      u128 l = p, r = mx;
      if (s >= 0) l <<= s; else r <<= -s;
      return l > r ? 1 : (l < r ? -1 : 0);
    }
  };
  // every comparison is increasing in b: y is the correctly rounded value iff the rounding
  // interval [lo, hi] of y brackets the exact result: cmp(lo) < 0 < cmp(hi)
  if (cmp(lo) >= 0) return 1;   // y too large
  if (cmp(hi) <= 0) return -1;  // y too small
  return 0;
}

__global__ void census(uint32_t base, uint32_t n, unsigned long long* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t xb = base + i;
  const float x = __uint_as_float(xb);
  const float r = __builtin_amdgcn_rcpf(x), q = __builtin_amdgcn_rsqf(x), s = __builtin_amdgcn_sqrtf(x);
  const int cr = check(xb, __float_as_uint(r), 0);
  const int cq = check(xb, __float_as_uint(q), 1);
  const int cs = check(xb, __float_as_uint(s), 2);
  // controls: IEEE division and sqrt (built with -fhip-fp32-correctly-rounded-divide-sqrt)
  if (check(xb, __float_as_uint(1.0f / x), 0)) atomicAdd(out + 6, 1ull);
  if (check(xb, __float_as_uint(sqrtf(x)), 2)) atomicAdd(out + 7, 1ull);
  // one correction step after the hardware approximation
  const float r1 = fmaf(fmaf(-x, r, 1.0f), r, r);
  if (check(xb, __float_as_uint(r1), 0)) atomicAdd(out + 8, 1ull);
  const float q1 = fmaf(q * 0.5f, fmaf(-x, q * q, 1.0f), q);            // h = y*y rounded
  if (check(xb, __float_as_uint(q1), 1)) atomicAdd(out + 9, 1ull);
  const float xq = x * q;                                                // h = x*y rounded
  const float q2 = fmaf(q * 0.5f, fmaf(-xq, q, 1.0f), q);
  if (check(xb, __float_as_uint(q2), 1)) atomicAdd(out + 10, 1ull);
  const float s1 = fmaf(fmaf(-s, s, x), 0.5f * __builtin_amdgcn_rcpf(s), s);  // sqrt + residual
  if (check(xb, __float_as_uint(s1), 2)) atomicAdd(out + 11, 1ull);
  if (cr) atomicAdd(out + (cr < 0 ? 0 : 1), 1ull);
  if (cq) atomicAdd(out + (cq < 0 ? 2 : 3), 1ull);
  if (cs) atomicAdd(out + (cs < 0 ? 4 : 5), 1ull);
}

int main(int argc, char** argv) {
  // default: [1, 4); with an argument, every binade from 2^-60 to 2^4 of both signs (the
  // reciprocal's exponent independence; rsq and sqrt are counted for positive inputs only)
  const bool wide = argc > 1;
  unsigned long long* d = nullptr;
  unsigned long long h[12] = {}, tot[12] = {};
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  uint64_t total = 0, total_pos = 0;
  const int e_lo = wide ? -60 : 0, e_hi = wide ? 4 : 2;  // binades [2^e, 2^(e+2)) in steps of 2
  for (int sign = 0; sign < (wide ? 2 : 1); ++sign) {
    for (int e = e_lo; e < e_hi; e += 2) {
      (void)hipMemset(d, 0, sizeof h);
      const uint32_t base = (sign ? 0x80000000u : 0u) | ((uint32_t)(127 + e) << 23), n = 1u << 24;
      hipLaunchKernelGGL(census, dim3((n + 255) / 256), dim3(256), 0, 0, base, n, d);
      if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      for (int k = 0; k < 12; ++k) {
        if (sign && k >= 2 && k != 6 && k != 8) continue;  // negative x: rcp only
        tot[k] += h[k];
      }
      total += n;
      if (!sign) total_pos += n;
    }
  }
  std::printf("floats checked: %llu (positive %llu), binades 2^%d .. 2^%d%s\n", (unsigned long long)total,
              (unsigned long long)total_pos, e_lo, e_hi, wide ? ", both signs" : "");
  std::printf("v_rcp_f32  not correctly rounded: %llu (too small %llu, too large %llu)\n", tot[0] + tot[1], tot[0], tot[1]);
  std::printf("v_rsq_f32  not correctly rounded: %llu (too small %llu, too large %llu)\n", tot[2] + tot[3], tot[2], tot[3]);
  std::printf("v_sqrt_f32 not correctly rounded: %llu (too small %llu, too large %llu)\n", tot[4] + tot[5], tot[4], tot[5]);
  std::printf("controls (must be 0): IEEE 1/x %llu, IEEE sqrtf %llu\n", tot[6], tot[7]);
  std::printf("after one correction: rcp %llu, rsq (y*y) %llu, rsq (x*y) %llu, sqrt %llu not CR\n",
              tot[8], tot[9], tot[10], tot[11]);
  (void)hipFree(d);
  return 0;
}
