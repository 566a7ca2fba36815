// issue_mix.hip — how much do SALU instructions and v_cmp->s_and->v_cndmask chains cost next to
// VALU work on gfx950? (design input for the intersect loop). 8 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N_ITER 2048

// 12 independent-ish VALU per "prim", plus S extra SALU
template <int S, int CHAIN>
__global__ void __launch_bounds__(256) k(float* out, float seed, int n) {
  float a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, t = 1e20f;
  int pos = -1;
  for (int i = 0; i < n; ++i) {
    if constexpr (CHAIN) {
      // the real pattern: 4 arith, 3 compares -> 2 s_and -> 2 cndmask  (~12 VALU incl. subs)
      const float tt = (a0 - seed) * a1;
      const float a = fmaf(a2, tt, a3), b = fmaf(a3, tt, a2);
      const bool ia = fabsf(a - seed) <= a1, ib = fabsf(b - a0) <= a2;
      const uint32_t kk = __float_as_uint(tt) - 1u;
      const bool acc = ((int)ia & (int)ib) & (kk < __float_as_uint(t));
      t = acc ? __uint_as_float(kk) : t;
      pos = acc ? i : pos;
      a0 += 1e-7f; a1 = a1 * 0.999f; a2 += tt * 1e-9f; a3 -= 1e-7f;
    } else {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(a1), "v"(a2));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(a2), "v"(a3));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(a3), "v"(a0));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(a0), "v"(a1));
      }
#pragma unroll
      for (int j = 0; j < S; ++j) asm volatile("s_and_b64 s[20:21], s[20:21], s[22:23]" ::: "s20", "s21", "scc");
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + t + (float)pos;
}

template <typename F> double time_it(F f) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  f(); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) f();
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1); return ms / 5;
}
int main() {
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8;
  float* buf; (void)hipMalloc(&buf, sizeof(float) * blocks * 256);
  const double waves_per_simd = blocks * 4.0 / (p.multiProcessorCount * 4);
  auto rep = [&](const char* name, double ms, double valu_per_iter) {
    const double cyc = ms * 1e-3 * 2.4e9 / (waves_per_simd * N_ITER);  // SIMD cycles per wave-iter
    printf("%-28s %7.3f ms  %6.1f SIMD-cycles per wave-iteration  (%.1f VALU -> %.2f cyc/VALU)\n",
           name, ms, cyc, valu_per_iter, cyc / valu_per_iter);
  };
#define RUN(S, C, NAME, V) rep(NAME, time_it([&] { hipLaunchKernelGGL((k<S, C>), dim3(blocks), dim3(256), 0, 0, buf, 1.0001f, N_ITER); }), V);
  RUN(0, 0, "12 fma", 12) RUN(2, 0, "12 fma + 2 salu", 12) RUN(5, 0, "12 fma + 5 salu", 12)
  RUN(8, 0, "12 fma + 8 salu", 12) RUN(12, 0, "12 fma + 12 salu", 12) RUN(0, 1, "rect-test pattern", 16)
  return 0;
}
