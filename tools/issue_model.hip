// issue_model.hip — what limits VALU issue on gfx950 for the render kernel's instruction mix?
// Each kernel runs N_ITER iterations of a fixed body at a chosen occupancy and reports SIMD cycles
// per body and per VALU. Bodies:
//   fmaC      : 16 v_fma_f32 in C independent chains (C = 1, 2, 4, 8): dependent-issue latency
//   salu S    : 16 fma (4 chains) + S s_and_b64: co-issue of SALU with VALU from other waves
//   cmpsel    : v_cmp_e64 -> s_and_b64 -> v_cndmask chains (the rect-test mask pattern)
//   cmpsel_v  : the same selects with the compare result kept in a VGPR (v_cndmask on vcc)
//   div       : a divergent if/else on a lane-varying predicate (s_and_saveexec / s_or exec)
//   smem      : 16 fma + one s_load_dword + s_waitcnt per body (params re-loaded in the loop)
//   mad64     : 8 v_mad_u64_u32 + 8 v_xor (Philox round pattern)
// Usage: issue_model [waves_per_simd]   (occupancy set by LDS padding per block)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define N_ITER 4096

#define FMA(a, b, c) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c))

template <int C>
__global__ void __launch_bounds__(256) k_fma(float* out, float s, int n) {
  float a[8], b = s * threadIdx.x, c = s + 1.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = b + j;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) FMA(a[j % C], b, c);
  }
  float r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r += a[j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int S>
__global__ void __launch_bounds__(256) k_salu(float* out, float s, int n) {
  float a0 = s * threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, b = s, c = s + 1;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { FMA(a0, b, c); FMA(a1, b, c); FMA(a2, b, c); FMA(a3, b, c); }
#pragma unroll
    for (int j = 0; j < S; ++j) asm volatile("s_and_b64 s[20:21], s[20:21], s[22:23]" ::: "s20", "s21", "scc");
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}

// 4 independent (cmp -> s_and -> cndmask) selects per body, 16 VALU + 4 SALU
template <int VCC>
__global__ void __launch_bounds__(256) k_cmpsel(float* out, float s, int n) {
  float a0 = s * threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, b = s, c = s + 1;
  for (int i = 0; i < n; ++i) {
    if constexpr (VCC) {
      asm volatile(
          "v_cmp_lt_f32 vcc, %0, %4\n v_cndmask_b32 %0, %0, %5, vcc\n"
          "v_cmp_lt_f32 vcc, %1, %4\n v_cndmask_b32 %1, %1, %5, vcc\n"
          "v_cmp_lt_f32 vcc, %2, %4\n v_cndmask_b32 %2, %2, %5, vcc\n"
          "v_cmp_lt_f32 vcc, %3, %4\n v_cndmask_b32 %3, %3, %5, vcc\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b), "v"(c) : "vcc");
    } else {
      asm volatile(
          "v_cmp_lt_f32 s[20:21], %0, %4\n v_cmp_lt_f32 s[22:23], %1, %4\n"
          "v_cmp_lt_f32 s[24:25], %2, %4\n v_cmp_lt_f32 s[26:27], %3, %4\n"
          "s_and_b64 s[20:21], s[20:21], s[22:23]\n s_and_b64 s[22:23], s[22:23], s[24:25]\n"
          "s_and_b64 s[24:25], s[24:25], s[26:27]\n s_and_b64 s[26:27], s[26:27], s[20:21]\n"
          "v_cndmask_b32 %0, %0, %5, s[20:21]\n v_cndmask_b32 %1, %1, %5, s[22:23]\n"
          "v_cndmask_b32 %2, %2, %5, s[24:25]\n v_cndmask_b32 %3, %3, %5, s[26:27]\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b), "v"(c)
          : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "scc");
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) { FMA(a0, b, c); FMA(a1, b, c); FMA(a2, b, c); FMA(a3, b, c); }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}

// divergent if/else around 8 fma each side (half the lanes each way): 16 VALU issued + exec SALU
__global__ void __launch_bounds__(256) k_div(float* out, float s, int n) {
  float a0 = s * threadIdx.x, a1 = a0 + 1, b = s, c = s + 1;
  const bool odd = (threadIdx.x & 1) != 0;
  for (int i = 0; i < n; ++i) {
    if (odd) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { FMA(a0, b, c); FMA(a1, b, c); }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) { FMA(a1, c, b); FMA(a0, c, b); }
    }
    asm volatile("" : "+v"(a0), "+v"(a1));
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1;
}

// 16 fma + a scalar reload of a parameter with its wait (the render loop's cptr pattern)
__global__ void __launch_bounds__(256) k_smem(float* out, const float* __restrict__ prm, float s, int n) {
  float a0 = s * threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  for (int i = 0; i < n; ++i) {
    const float* p = prm;
    asm volatile("" : "+s"(p));
    const float b = __builtin_nontemporal_load(p) ;  // uniform -> s_load
    float c = p[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { FMA(a0, b, c); FMA(a1, b, c); FMA(a2, b, c); FMA(a3, b, c); }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}

__global__ void __launch_bounds__(256) k_mad64(float* out, float s, int n) {
  uint32_t c0 = threadIdx.x, c1 = 7, c2 = 11, c3 = 13;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
      const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ 0x1234u, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ 0x5678u;
      c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3));
  }
  out[blockIdx.x * 256 + threadIdx.x] = (float)(c0 ^ c1 ^ c2 ^ c3);
}

template <typename F> double time_it(F f) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  f(); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) f();
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1); return ms / 5;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 8;  // waves per SIMD = blocks per CU (4 waves each)
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * wps;
  const double clk = p.clockRate * 1e3;
  float *buf, *prm; (void)hipMalloc(&buf, sizeof(float) * blocks * 256); (void)hipMalloc(&prm, 64);
  (void)hipMemset(prm, 0, 64);
  printf("waves/SIMD %d, CUs %d, clock %.0f MHz\n", wps, p.multiProcessorCount, clk * 1e-6);
  auto rep = [&](const char* name, double ms, double valu) {
    const double cyc = ms * 1e-3 * clk / (wps * (double)N_ITER);  // SIMD cycles per wave-body
    printf("%-22s %8.3f ms %7.1f SIMD-cyc/body  %5.1f VALU  %.2f cyc/VALU\n", name, ms, cyc, valu, cyc / valu);
  };
#define L(K, ...) time_it([&] { hipLaunchKernelGGL(K, dim3(blocks), dim3(256), 0, 0, __VA_ARGS__); })
  rep("fma 1 chain", L(k_fma<1>, buf, 1.0001f, N_ITER), 16);
  rep("fma 2 chains", L(k_fma<2>, buf, 1.0001f, N_ITER), 16);
  rep("fma 4 chains", L(k_fma<4>, buf, 1.0001f, N_ITER), 16);
  rep("fma 8 chains", L(k_fma<8>, buf, 1.0001f, N_ITER), 16);
  rep("16 fma + 4 salu", L(k_salu<4>, buf, 1.0001f, N_ITER), 16);
  rep("16 fma + 8 salu", L(k_salu<8>, buf, 1.0001f, N_ITER), 16);
  rep("16 fma + 16 salu", L(k_salu<16>, buf, 1.0001f, N_ITER), 16);
  rep("cmp->s_and->cndmask", L(k_cmpsel<0>, buf, 1.0001f, N_ITER), 16);
  rep("cmp->cndmask (vcc)", L(k_cmpsel<1>, buf, 1.0001f, N_ITER), 16);
  rep("divergent if/else 8+8", L(k_div, buf, 1.0001f, N_ITER), 16);
  rep("16 fma + s_load/wait", L(k_smem, buf, prm, 1.0001f, N_ITER), 16);
  rep("philox 4 rounds", L(k_mad64, buf, 1.0001f, N_ITER), 24);
  return 0;
}
