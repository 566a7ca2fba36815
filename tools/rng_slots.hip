// rng_slots.hip — static issue cost of the per-vertex random words under the candidate generators
// of VERDICT r04 item 3(a) ("one Philox call per sample seeding a per-lane generator of erand48's
// class"). Compiled to ISA only; tools/rng_slots.sh counts each kernel's VALU slots with
// tools/isa_blocks.py and subtracts the empty kernel's. Each kernel does what the render kernel's
// generate block must do per wave-iteration for the same four 32-bit words per vertex:
//
//   philox  : philox_px(pk, s, ctr) — the product (spt_device.h), counter-based, no state
//   lcg48   : erand48's recurrence (a = 0x5DEECE66D, c = 0xB, mod 2^48), 4 steps, the top 32 bits
//             of each state; the state of a camera lane is re-seeded from (pk, s) by a 32-bit
//             finaliser (murmur3 fmix32) and selected per lane (camera and cosine lanes share a
//             wave, so the seed runs in every wave-iteration)
//   pcg32   : a 32-bit LCG with the PCG RXS-M-XS output permutation, 4 steps, the same seeding
//   xs32    : xorshift32, 4 steps (no output permutation: low bits linear), the same seeding
//
// The render kernel reads the words' low bytes (Russian roulette, NEE mix, jitter) as well as their
// top bits, so every generator must give 4 full-quality words.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../small-pathtracer_amd/csrc/spt_device.h"

using namespace spt;

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

struct In { uint32_t qhi, qlo, lo, s, ctr, cam, st0, st1; };

extern "C" __global__ void __launch_bounds__(256) k_empty(const In* in, uint4* out) {
  const In v = in[blockIdx.x * 256 + threadIdx.x];
  out[blockIdx.x * 256 + threadIdx.x] = make_uint4(v.qhi ^ v.s, v.qlo ^ v.ctr, v.lo ^ v.cam, v.st0 ^ v.st1);
}

extern "C" __global__ void __launch_bounds__(256) k_philox(const In* in, uint4* out) {
  const In v = in[blockIdx.x * 256 + threadIdx.x];
  const u4 r = philox_px(PxKey{v.qhi, v.qlo, v.lo}, v.s, v.ctr);
  out[blockIdx.x * 256 + threadIdx.x] = make_uint4(r.x, r.y, r.z, r.w);
}

extern "C" __global__ void __launch_bounds__(256) k_lcg48(const In* in, uint4* out) {
  const In v = in[blockIdx.x * 256 + threadIdx.x];
  // seed: lo = fmix32(pixel key ^ s * golden), hi = pixel key word (16 bits used)
  const uint32_t sl = fmix32(v.qlo ^ (v.s * 0x9E3779B9u));
  uint32_t lo = v.cam ? sl : v.st0, hi = v.cam ? v.qhi : v.st1;
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // x' = (0x5DEECE66D x + 0xB) mod 2^48: lo*a_lo + c as one 64-bit mad, the high 16 bits from
    // lo(a_lo) * hi + 5 * lo (mod 2^16 only) as two 24-bit mads
    const uint64_t p = (uint64_t)lo * 0xDEECE66Du + 0xBu;
    const uint32_t nh = (uint32_t)(p >> 32) + __umul24(0xE66Du, hi) + 5u * lo;
    lo = (uint32_t)p;
    hi = nh;
    w[i] = __builtin_amdgcn_alignbit(hi, lo, 16);  // bits 16..47
  }
  out[blockIdx.x * 256 + threadIdx.x] = make_uint4(w[0], w[1], w[2], w[3] ^ hi);
}

extern "C" __global__ void __launch_bounds__(256) k_pcg32(const In* in, uint4* out) {
  const In v = in[blockIdx.x * 256 + threadIdx.x];
  uint32_t x = v.cam ? fmix32(v.qlo ^ (v.s * 0x9E3779B9u)) : v.st0;
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x = x * 747796405u + 2891336453u;
    uint32_t z = ((x >> ((x >> 28u) + 4u)) ^ x) * 277803737u;
    w[i] = (z >> 22u) ^ z;
  }
  out[blockIdx.x * 256 + threadIdx.x] = make_uint4(w[0], w[1], w[2], w[3] ^ x);
}

extern "C" __global__ void __launch_bounds__(256) k_xs32(const In* in, uint4* out) {
  const In v = in[blockIdx.x * 256 + threadIdx.x];
  uint32_t x = v.cam ? fmix32(v.qlo ^ (v.s * 0x9E3779B9u)) | 1u : v.st0;
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    w[i] = x;
  }
  out[blockIdx.x * 256 + threadIdx.x] = make_uint4(w[0], w[1], w[2], w[3]);
}

// the 48-bit recurrence alone (state loaded, no seed, no select): the floor of lcg48
extern "C" __global__ void __launch_bounds__(256) k_lcg48_steps(const In* in, uint4* out) {
  const In v = in[blockIdx.x * 256 + threadIdx.x];
  uint32_t lo = v.st0, hi = v.st1;
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t p = (uint64_t)lo * 0xDEECE66Du + 0xBu;
    const uint32_t nh = (uint32_t)(p >> 32) + __umul24(0xE66Du, hi) + 5u * lo;
    lo = (uint32_t)p;
    hi = nh;
    w[i] = __builtin_amdgcn_alignbit(hi, lo, 16);
  }
  out[blockIdx.x * 256 + threadIdx.x] = make_uint4(w[0], w[1], w[2], w[3] ^ hi);
}
