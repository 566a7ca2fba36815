// valu_rates.hip — measure per-instruction VALU throughput on gfx950 (design input for the
// render kernel: integer multiplies for the RNG, packed fp32, transcendentals, div/sqrt sequences).
// Each kernel runs 8 independent chains of N_ITER x UNROLL inline-asm instructions per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N_ITER 4096
#define OP8(S) S S S S S S S S

template <int K>
__global__ void __launch_bounds__(256) k_rate(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
  const uint32_t b = seed | 1;
  for (int i = 0; i < N_ITER; ++i) {
#define DO(INS) asm volatile(INS " %0, %0, %1" : "+v"(a0) : "v"(b)); asm volatile(INS " %0, %0, %1" : "+v"(a1) : "v"(b)); \
  asm volatile(INS " %0, %0, %1" : "+v"(a2) : "v"(b)); asm volatile(INS " %0, %0, %1" : "+v"(a3) : "v"(b)); \
  asm volatile(INS " %0, %0, %1" : "+v"(a4) : "v"(b)); asm volatile(INS " %0, %0, %1" : "+v"(a5) : "v"(b)); \
  asm volatile(INS " %0, %0, %1" : "+v"(a6) : "v"(b)); asm volatile(INS " %0, %0, %1" : "+v"(a7) : "v"(b));
#define DO1(INS) asm volatile(INS " %0, %0" : "+v"(a0)); asm volatile(INS " %0, %0" : "+v"(a1)); \
  asm volatile(INS " %0, %0" : "+v"(a2)); asm volatile(INS " %0, %0" : "+v"(a3)); \
  asm volatile(INS " %0, %0" : "+v"(a4)); asm volatile(INS " %0, %0" : "+v"(a5)); \
  asm volatile(INS " %0, %0" : "+v"(a6)); asm volatile(INS " %0, %0" : "+v"(a7));
#define DO3(INS) asm volatile(INS " %0, %0, %1, %0" : "+v"(a0) : "v"(b)); asm volatile(INS " %0, %0, %1, %0" : "+v"(a1) : "v"(b)); \
  asm volatile(INS " %0, %0, %1, %0" : "+v"(a2) : "v"(b)); asm volatile(INS " %0, %0, %1, %0" : "+v"(a3) : "v"(b)); \
  asm volatile(INS " %0, %0, %1, %0" : "+v"(a4) : "v"(b)); asm volatile(INS " %0, %0, %1, %0" : "+v"(a5) : "v"(b)); \
  asm volatile(INS " %0, %0, %1, %0" : "+v"(a6) : "v"(b)); asm volatile(INS " %0, %0, %1, %0" : "+v"(a7) : "v"(b));
    if constexpr (K == 0) { DO("v_add_u32") }
    if constexpr (K == 1) { DO("v_mul_lo_u32") }
    if constexpr (K == 2) { DO("v_mul_hi_u32") }
    if constexpr (K == 3) { DO("v_mul_u32_u24") }
    if constexpr (K == 4) { DO("v_mul_f32") }
    if constexpr (K == 5) { DO3("v_fma_f32") }
    if constexpr (K == 6) { DO1("v_sqrt_f32") }
    if constexpr (K == 7) { DO1("v_rcp_f32") }
    if constexpr (K == 8) { DO1("v_sin_f32") }
    if constexpr (K == 9) { DO("v_xor_b32") }
    if constexpr (K == 10) { DO3("v_or3_b32") }
    if constexpr (K == 11) { DO("v_mul_hi_u32_u24") }
    if constexpr (K == 12) { DO1("v_rsq_f32") }
    if constexpr (K == 13) { DO3("v_med3_f32") }
#define DOB(INS) asm volatile(INS " %0, %0, %1, %0 bitop3:0x96" : "+v"(a0) : "v"(b)); asm volatile(INS " %0, %0, %1, %0 bitop3:0x96" : "+v"(a1) : "v"(b)); \
  asm volatile(INS " %0, %0, %1, %0 bitop3:0x96" : "+v"(a2) : "v"(b)); asm volatile(INS " %0, %0, %1, %0 bitop3:0x96" : "+v"(a3) : "v"(b)); \
  asm volatile(INS " %0, %0, %1, %0 bitop3:0x96" : "+v"(a4) : "v"(b)); asm volatile(INS " %0, %0, %1, %0 bitop3:0x96" : "+v"(a5) : "v"(b)); \
  asm volatile(INS " %0, %0, %1, %0 bitop3:0x96" : "+v"(a6) : "v"(b)); asm volatile(INS " %0, %0, %1, %0 bitop3:0x96" : "+v"(a7) : "v"(b));
    if constexpr (K == 14) { DOB("v_bitop3_b32") }
    if constexpr (K == 15) { DO1("v_cvt_f32_u32") }
    if constexpr (K == 16) { DO3("v_add3_u32") }
    if constexpr (K == 17) { DO3("v_xad_u32") }
    if constexpr (K == 18) { DO3("v_perm_b32") }
    if constexpr (K == 19) { DO3("v_lshl_add_u32") }
    if constexpr (K == 20) { DO1("v_cvt_f32_ubyte0") }
    if constexpr (K == 21) { DO1("v_cvt_f32_ubyte1") }
    if constexpr (K == 22) { DO3("v_bfi_b32") }
    if constexpr (K == 23) { DO3("v_and_or_b32") }
    if constexpr (K == 24) { DO3("v_lshl_or_b32") }
    if constexpr (K == 25) { DO1("v_cvt_f32_i32") }
    if constexpr (K == 26) { DO3("v_bfe_u32") }
    if constexpr (K == 27) { DO("v_lshrrev_b32") }
    if constexpr (K == 28) { DO("v_mul_u32_u24") }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// 64-bit / packed forms need register pairs
template <int K>
__global__ void __launch_bounds__(256) k_rate64(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
  const uint64_t b = seed | 1;
  for (int i = 0; i < N_ITER; ++i) {
#define P(INS, X) asm volatile(INS : "+v"(X) : "v"(b));
    if constexpr (K == 0) {
#define M(X) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(X) : "v"(b));
      M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
#undef M
    }
    if constexpr (K == 1) {
#define M(X) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(X) : "v"(b));
      M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
#undef M
    }
    if constexpr (K == 2) {
#define M(X) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(X) : "v"(b));
      M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
#undef M
    }
    if constexpr (K == 3) {
#define M(X) { uint32_t lo = (uint32_t)X; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(X) : "v"(lo), "v"((uint32_t)b)); }
      M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
#undef M
    }
    if constexpr (K == 4) {
#define M(X) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(X) : "v"(b));
      M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
#undef M
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <typename F>
double time_it(F f) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) f();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  const int blocks = ncu * 8;  // 8 blocks x 4 waves = 32 waves/CU
  uint64_t* buf; (void)hipMalloc(&buf, sizeof(uint64_t) * blocks * 256);
  const double insts = (double)blocks * 4 * N_ITER * 8;  // wave-instructions
  auto report = [&](const char* name, double ms) {
    // cycles per wave-instruction per SIMD at 2.4 GHz nominal
    const double per_simd = insts / (ncu * 4);
    printf("%-22s %8.3f ms  %6.2f cyc/wave-instr/SIMD (@2.4GHz)  %7.2f T lane-ops/s\n", name, ms,
           ms * 1e-3 * 2.4e9 / per_simd, insts * 64 / (ms * 1e-3) / 1e12);
  };
#define R32(K, NAME) report(NAME, time_it([&] { hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, (uint32_t*)buf, 7u); }));
#define R64(K, NAME) report(NAME, time_it([&] { hipLaunchKernelGGL(k_rate64<K>, dim3(blocks), dim3(256), 0, 0, buf, 7u); }));
  R32(0, "v_add_u32") R32(1, "v_mul_lo_u32") R32(2, "v_mul_hi_u32") R32(3, "v_mul_u32_u24")
  R32(11, "v_mul_hi_u32_u24") R32(4, "v_mul_f32") R32(5, "v_fma_f32") R32(6, "v_sqrt_f32")
  R32(7, "v_rcp_f32") R32(12, "v_rsq_f32") R32(8, "v_sin_f32") R32(9, "v_xor_b32")
  R32(10, "v_or3_b32") R32(13, "v_med3_f32") R32(14, "v_bitop3_b32") R32(15, "v_cvt_f32_u32")
  R32(16, "v_add3_u32") R32(17, "v_xad_u32") R32(18, "v_perm_b32") R32(19, "v_lshl_add_u32")
  R32(20, "v_cvt_f32_ubyte0") R32(21, "v_cvt_f32_ubyte1") R32(22, "v_bfi_b32") R32(23, "v_and_or_b32")
  R32(24, "v_lshl_or_b32") R32(25, "v_cvt_f32_i32") R32(26, "v_bfe_u32") R32(27, "v_lshrrev_b32")
  R64(0, "v_pk_fma_f32") R64(1, "v_pk_mul_f32") R64(2, "v_pk_add_f32") R64(3, "v_mad_u64_u32")
  R64(4, "v_fma_f64")
  printf("CUs %d clock %d kHz\n", ncu, p.clockRate);
  return 0;
}
