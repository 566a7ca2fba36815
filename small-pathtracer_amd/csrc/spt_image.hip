// spt_image.hip — the reference's image output (/root/reference/src/smallpt.cpp:313-321 toInt/clamp,
// :548-551 the P3 writer) as a gfx950 encoder, plus binary P6 and linear PFM.
//
// The reference writes `fprintf(f, "%d %d %d ", toInt(r), toInt(g), toInt(b))` per pixel: ASCII
// P3, 6-12 bytes per pixel, ~200 MB of text at 4096². Here the framebuffer never leaves HBM until
// the bytes are final. P3 takes four short HBM-bound passes split at the toInt bytes (p6_write ->
// p3_lengths -> p3_offsets -> p3_text, below): the bytes, each 8192-value text block's length,
// the blocks' byte offsets, then the "%d " text assembled in LDS at the destination's 16-byte phase
// and written with 16-byte stores. (Rounds 1-3 used one pass with a decoupled look-back; at 4096^2
// it took 155.6 us against 132-136 us for the passes, profiles/r03_encoder.txt.)
// P6 / PFM are fixed-size: grid-stride float4 loops, one dword / float4 store per 4 values.
// toInt is the reference's double-precision formula exactly: a 256-entry threshold table computed
// on the host with that very formula (toInt is monotone in x) settles a v_log/v_exp estimate,
// which is never more than one step off. NaN prints as x86-64's int(NaN), INT_MIN, as the
// reference binary does.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/spt.h"

namespace spt_img {

constexpr int kThreads = 256;
constexpr int kMaxValueText = 12;                        // "-2147483648 "

struct Thresholds { float t[256]; };  // t[k] = smallest x with toInt(x) >= k; t[0] = -inf

// toInt :319-321 with the reference's own arithmetic (double pow, clamp, +.5, truncation).
static int ref_toInt(double x) { return (int)(std::pow(x < 0 ? 0 : x > 1 ? 1 : x, 1 / 2.2) * 255 + .5); }

static const Thresholds& thresholds() {
  static Thresholds T;
  static std::once_flag once;
  std::call_once(once, [] {
    T.t[0] = -INFINITY;
    for (int k = 1; k < 256; ++k) {  // smallest non-negative float bit pattern with toInt >= k
      uint32_t lo = 0, hi = 0x3F800000u;  // toInt(1.0f) = 255
      while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        float f;
        std::memcpy(&f, &mid, 4);
        if (ref_toInt((double)f) >= k) hi = mid; else lo = mid + 1;
      }
      std::memcpy(&T.t[k], &lo, 4);
    }
  });
  return T;
}

// toInt(x) = #{k >= 1 : x >= thr[k]}: a hardware estimate pow(x, 1/2.2)*255 + .5 (v_log/v_exp, a
// few ulps) lands within one step of the exact count; the table then settles it exactly
// (thresholds are >= ~1e-6 apart in relative terms, the estimate is ~1e-6 accurate).
__device__ __forceinline__ int dev_toInt(const float* __restrict__ thr, float x) {
  if (x != x) return (int)0x80000000;  // int(NaN) on x86-64 (cvttsd2si)
  const float xc = fminf(fmaxf(x, 0.0f), 1.0f);
  const float est = __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(xc) * (1.0f / 2.2f)) * 255.0f + 0.5f;
  int v = (int)fminf(fmaxf(est, 0.0f), 255.0f);
  if (v < 255 && x >= thr[v + 1]) ++v;  // thr[0] = -inf, so x >= thr[v] below always holds at v = 0
  else if (x < thr[v]) --v;
  return v;
}

// The same without branches (both table words read, selects instead of the if/else): one straight
// block per value instead of three exec-masked ones (round 3: the branchy form cost ~39 SALU per
// wave-value in the P3 encoder).
__device__ __forceinline__ int dev_toInt_bf(const float* __restrict__ thr, float x) {
  const float xc = fminf(fmaxf(x, 0.0f), 1.0f);
  const float est = __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(xc) * (1.0f / 2.2f)) * 255.0f + 0.5f;
  const int v = (int)fminf(fmaxf(est, 0.0f), 255.0f);
  const float hi = thr[min(v + 1, 255)], lo = thr[v];
  const int inc = (int)(v < 255) & (int)(x >= hi), dec = (inc ^ 1) & (int)(x < lo);
  return x != x ? (int)0x80000000 : v + inc - dec;
}

// "%d " of v in [0, 255] as one little-endian word of n = 2..4 bytes: the 3-digit text
// "hdd " shifted right past its leading zero digits (v / 10 as (v * 205) >> 11, exact below 1029).
__device__ __forceinline__ uint32_t text_word(int v, uint32_t& n) {
  const uint32_t u = (uint32_t)v, t = (u * 205u) >> 11, d0 = u - t * 10u;
  const uint32_t h = (t * 205u) >> 11, d1 = t - h * 10u;
  n = 2u + (uint32_t)(u >= 10u) + (uint32_t)(u >= 100u);
  return (0x20303030u + (h | d1 << 8 | d0 << 16)) >> (32u - 8u * n);
}

__device__ __forceinline__ uint32_t text_len(int v) {  // digits + the trailing space; -1: no value
  return v == -1 ? 0u : v < 0 ? 12u : v >= 100 ? 4u : v >= 10 ? 3u : 2u;
}

__device__ __forceinline__ uint32_t put_value(uint8_t* p, int v) {  // "%d " into LDS
  if (v < 0) {
    const char* s = "-2147483648 ";
    for (int i = 0; i < 12; ++i) p[i] = (uint8_t)s[i];
    return 12;
  }
  uint32_t n = 0;
  if (v >= 100) p[n++] = (uint8_t)('0' + v / 100);
  if (v >= 10) p[n++] = (uint8_t)('0' + (v / 10) % 10);
  p[n++] = (uint8_t)('0' + v % 10);
  p[n++] = (uint8_t)' ';
  return n;
}

__device__ __forceinline__ void load_thr(float* s_thr, const Thresholds& T) {
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_thr[i] = T.t[i];
  __syncthreads();
}

// Block-wide exclusive scan of one uint32 per thread (wave shuffles + LDS for wave totals).
template <int kBlockThreads>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_wave, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(incl, off, 64);
    if (lane >= off) incl += u;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  uint32_t base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kBlockThreads / 64; ++w) {
    const uint32_t t = s_wave[w];
    base += w < wave ? t : 0u;
    all += t;
  }
  *total = all;
  return base + incl - v;
}

// ---- P3 in passes (round 3). The round-1/2 single pass serialised each block's phases (ticket,
// loads, toInt, scan, look-back, staging, stores) and held 48 KB of LDS per 512-thread block (3
// blocks per CU). Split at the toInt bytes instead:
//   p6_write:   toInt of every value as one byte (the P6 kernel itself: coalesced float4 loads, dword
//               stores), and the encode's epoch in a NaN word if any value is NaN;
//   p3_lengths: each 8192-value text block's length from its bytes;
//   p3_offsets: one block scans the text-block lengths (header first) into byte offsets;
//   p3_text:    each 512-thread block formats 16 contiguous digits per thread ("%d " words), scans
//               the thread lengths, assembles its text in LDS at the destination's 16-byte phase
//               and writes it with 16-byte stores.
// HBM traffic per value: 4 B read + 1 B written, 1 B read, 1 B read + 2-4 B written, with no
// cross-block dependency inside a pass. (An image with a NaN, "-2147483648 ", takes an exact slow
// path in the last two passes: toInt again from the floats, byte stores.)
#ifndef SPT_TXT_THREADS
#define SPT_TXT_THREADS 512
#endif
constexpr int kTxtThreads = SPT_TXT_THREADS, kTxtVals = 16, kTxtBlockVals = kTxtThreads * kTxtVals;  // 8192
constexpr int kStageTxt = kTxtBlockVals * 4 + 32;  // every value <= "255 ", + the 16-byte phase

// Pass 1 is the P6 kernel itself (p6_write with a NaN word: the toInt bytes, 1 B per value, and the
// encode's epoch stored in *nan_word if any value is NaN). Pass 2, here: each 8192-value text
// block's length from its bytes (one 16-byte load per thread, block reduce). With a NaN in the
// image every block takes the exact slow path (toInt again from the floats).
// (Round 3: computing the lengths inside pass 1 -- one block per text block, persistent blocks, or
// the P6 loop with a per-wave atomic -- ran at 67-77 us at 4096^2, against 42 us for the P6 loop
// alone plus ~10 us for this pass.)
__device__ __forceinline__ bool nan_seen(const uint32_t* nan_word, uint32_t epoch) {
  return __hip_atomic_load(nan_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
}
__device__ __forceinline__ uint32_t digit_len(uint32_t b) {  // "%d " of a toInt byte
  return 2u + (uint32_t)(b >= 10u) + (uint32_t)(b >= 100u);
}

__global__ void __launch_bounds__(kTxtThreads)
p3_lengths(const uint4* __restrict__ digits, const float* __restrict__ rgb, uint32_t nv, Thresholds T,
           const uint32_t* __restrict__ nan_word, uint32_t epoch, uint32_t* __restrict__ blen) {
  __shared__ float s_thr[256];
  __shared__ uint32_t s_red[kTxtThreads / 64];
  const uint32_t v0 = blockIdx.x * (uint32_t)kTxtBlockVals + threadIdx.x * (uint32_t)kTxtVals;
  const uint32_t n_in = v0 < nv ? min((uint32_t)kTxtVals, nv - v0) : 0u;  // nv < 2^32
  uint32_t len = 0;
  if (nan_seen(nan_word, epoch)) {  // grid-uniform
    load_thr(s_thr, T);
#pragma unroll 1
    for (uint32_t i = 0; i < n_in; ++i) len += text_len(dev_toInt_bf(s_thr, rgb[v0 + i]));
  } else {
    uint4 q = make_uint4(0u, 0u, 0u, 0u);
    if (n_in) q = digits[v0 >> 4];  // the digits are padded to whole 16-byte groups
    const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < kTxtVals; ++i)
      len += (uint32_t)i < n_in ? digit_len((wd[i >> 2] >> (8 * (i & 3))) & 0xFFu) : 0u;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) len += __shfl_xor(len, off, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = len;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kTxtThreads / 64; ++w) t += s_red[w];
    blen[blockIdx.x] = t;
  }
}

// Exclusive scan of the text-block lengths into byte offsets (header first); *total = the length.
// Super-rounds of 8192 entries: each thread loads its 8 contiguous entries at once (one memory
// latency), one block scan of the thread sums, then the running carry.
constexpr int kScanThreads = 1024, kScanPer = 8;
__global__ void __launch_bounds__(kScanThreads)
p3_offsets(const uint32_t* __restrict__ blen, uint32_t nb, uint64_t header_len,
           uint64_t* __restrict__ offs, uint64_t* __restrict__ total) {
  __shared__ uint64_t s_wave[2][kScanThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t carry = header_len;
  int par = 0;
  for (uint32_t r0 = 0; r0 < nb; r0 += kScanThreads * kScanPer, par ^= 1) {
    const uint32_t b0 = r0 + threadIdx.x * kScanPer;
    uint32_t v[kScanPer];
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) v[i] = b0 + i < nb ? blen[b0 + i] : 0u;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) sum += v[i];
    uint64_t incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint64_t u = __shfl_up(incl, off, 64);
      if (lane >= off) incl += u;
    }
    if (lane == 63) s_wave[par][wave] = incl;  // (double-buffered: one barrier per round)
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
      const uint64_t t = s_wave[par][w];
      before += w < wave ? t : 0ull;
      all += t;
    }
    uint64_t run = carry + before + incl - sum;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
      if (b0 + i < nb) offs[b0 + i] = run;
      run += v[i];
    }
    carry += all;
  }
  if (threadIdx.x == 0) *total = carry;
}

// A text block holding a NaN (12-byte "-2147483648 "): toInt again from the floats (twice: lengths,
// then bytes; rolled loops keep the registers of the common path), byte stores.
__device__ __forceinline__ void p3_text_nan(const float* __restrict__ rgb, uint32_t nv, const float* s_thr,
                                            uint64_t dst, uint8_t* __restrict__ out, uint64_t cap,
                                            uint32_t* s_wave) {
  const uint32_t v0 = blockIdx.x * (uint32_t)kTxtBlockVals + threadIdx.x * (uint32_t)kTxtVals;
  const uint32_t n_in = v0 < nv ? min((uint32_t)kTxtVals, nv - v0) : 0u;
  uint32_t len = 0;
#pragma unroll 1
  for (uint32_t i = 0; i < n_in; ++i) len += text_len(dev_toInt_bf(s_thr, rgb[v0 + i]));
  uint32_t total;
  uint64_t q = dst + block_excl_scan<kTxtThreads>(len, s_wave, &total);
#pragma unroll 1
  for (uint32_t i = 0; i < n_in; ++i) {
    uint8_t b[12];
    const uint32_t n = put_value(b, dev_toInt_bf(s_thr, rgb[v0 + i]));
    for (uint32_t k = 0; k < n; ++k, ++q)
      if (q < cap) out[q] = b[k];
  }
}

__global__ void __launch_bounds__(kTxtThreads) __attribute__((amdgpu_waves_per_eu(8)))  // 4 blocks per CU
p3_text(const uint4* __restrict__ digits, const float* __restrict__ rgb, uint32_t nv, Thresholds T,
        const uint32_t* __restrict__ nan_word, uint32_t epoch, const uint64_t* __restrict__ offs,
        uint8_t* __restrict__ out, uint64_t cap) {
  __shared__ uint32_t s_wave[kTxtThreads / 64];
  __shared__ __attribute__((aligned(16))) uint32_t s_dw[kStageTxt / 4];
  uint8_t* const s_txt = (uint8_t*)s_dw;
  const uint64_t dst = offs[blockIdx.x];
  if (nan_seen(nan_word, epoch)) {  // grid-uniform
    load_thr((float*)s_dw, T);
    p3_text_nan(rgb, nv, (const float*)s_dw, dst, out, cap, s_wave);
    return;
  }
  const uint32_t v0 = blockIdx.x * (uint32_t)kTxtBlockVals + threadIdx.x * (uint32_t)kTxtVals;
  const uint32_t n_in = v0 < nv ? min((uint32_t)kTxtVals, nv - v0) : 0u;  // values here (nv < 2^32)
  uint4 q = make_uint4(0u, 0u, 0u, 0u);
  if (n_in) q = digits[v0 >> 4];  // the digits are padded to whole 16-byte groups
  const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
  uint32_t len = 0;
#pragma unroll
  for (int i = 0; i < kTxtVals; ++i)
    len += (uint32_t)i < n_in ? digit_len((wd[i >> 2] >> (8 * (i & 3))) & 0xFFu) : 0u;
  for (int i = threadIdx.x; i < kStageTxt / 16; i += kTxtThreads)  // OR-assembled staging starts at 0
    ((uint4*)s_dw)[i] = make_uint4(0u, 0u, 0u, 0u);
  uint32_t total;
  const uint32_t my = block_excl_scan<kTxtThreads>(len, s_wave, &total);  // (its barrier orders the zeroing)
  // Stage the text at the destination's 16-byte phase. Each value's "%d " word (2-4 bytes) is
  // appended to a 64-bit accumulator at the thread's byte offset and its low dword ORed into the
  // zeroed staging after every value (ds_or: a thread's first and last dword are shared with its
  // neighbours; re-ORing a growing dword is idempotent); the dword index advances once 32 bits are
  // full. Branch-free: a few VALU and one LDS op per value.
  const uint32_t phase = (uint32_t)(dst & 15u);
  const uint32_t o = phase + my;
  uint32_t di = o >> 2, nb = (o & 3u) * 8u;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < kTxtVals; ++i) {
    uint32_t n;
    const uint32_t wv = text_word((int)((wd[i >> 2] >> (8 * (i & 3))) & 0xFFu), n);
    acc |= (uint64_t)wv << nb;
    nb += (uint32_t)i < n_in ? 8u * n : 0u;
    atomicOr(&s_dw[di], (uint32_t)acc);
    const uint32_t full = nb >> 5;  // 0 or 1
    acc = full ? acc >> 32 : acc;
    nb -= full << 5;
    di += full;
  }
  if (nb) atomicOr(&s_dw[di], (uint32_t)acc);
  __syncthreads();
  if (dst + total > cap) {  // the host reports the error; write nothing past cap
    for (uint32_t i = threadIdx.x; i < total; i += kTxtThreads)
      if (dst + i < cap) out[dst + i] = s_txt[phase + i];
    return;
  }
  const uint64_t a0 = (dst + 15u) & ~15ull, a1 = (dst + total) & ~15ull;
  if (a0 >= a1) {
    for (uint32_t i = threadIdx.x; i < total; i += kTxtThreads) out[dst + i] = s_txt[phase + i];
    return;
  }
  const uint32_t head = (uint32_t)(a0 - dst), tail = (uint32_t)(dst + total - a1);
  if (threadIdx.x < head) out[dst + threadIdx.x] = s_txt[phase + threadIdx.x];
  if (threadIdx.x < tail) out[a1 + threadIdx.x] = s_txt[phase + (uint32_t)(a1 - dst) + threadIdx.x];
  const uint32_t n_q = (uint32_t)((a1 - a0) >> 4);
  const uint4* s_q = (const uint4*)(s_txt + phase + head);
  uint4* o_q = (uint4*)(out + a0);
  for (uint32_t i = threadIdx.x; i < n_q; i += kTxtThreads) o_q[i] = s_q[i];
}

// P6: header (padded to 16 bytes, see header()), then toInt bytes (the int's low byte, as a
// byte-writing port would store). Grid-stride over float4 chunks: 4 values -> one dword store.
__global__ void __launch_bounds__(kThreads)
p6_write(const float4* __restrict__ rgb, uint32_t n_vals, Thresholds T, uint32_t* __restrict__ out,
         uint32_t* __restrict__ nan_word, uint32_t epoch) {  // nan_word: P3's pass 1 (else null)
  __shared__ float s_thr[256];
  load_thr(s_thr, T);
  const uint32_t n4 = n_vals / 4;
  for (uint32_t c = blockIdx.x * kThreads + threadIdx.x; c < n4; c += gridDim.x * kThreads) {
    const float4 v = rgb[c];
    const int a = dev_toInt(s_thr, v.x), b = dev_toInt(s_thr, v.y), d = dev_toInt(s_thr, v.z),
              e = dev_toInt(s_thr, v.w);
    out[c] = (uint32_t)(uint8_t)a | (uint32_t)(uint8_t)b << 8 | (uint32_t)(uint8_t)d << 16 |
             (uint32_t)(uint8_t)e << 24;
    if (nan_word && (a | b | d | e) < 0) *nan_word = epoch;  // toInt >= 0 except int(NaN) = INT_MIN
  }
  if (blockIdx.x == 0 && threadIdx.x < (n_vals & 3u)) {  // ragged tail (n_vals % 4 values)
    const uint32_t i = n4 * 4 + threadIdx.x;
    const int a = dev_toInt(s_thr, ((const float*)rgb)[i]);
    ((uint8_t*)out)[i] = (uint8_t)a;
    if (nan_word && a < 0) *nan_word = epoch;
  }
}

// PFM: little-endian float RGB, scanlines bottom to top. Rows of 3w floats; when w % 4 == 0 a row
// is whole float4 chunks and the (16-byte padded) header keeps every store 16-byte aligned.
__global__ void __launch_bounds__(kThreads)
pfm_write4(const float4* __restrict__ rgb, uint32_t row4, uint32_t h, uint32_t m_row, uint32_t sh_row,
           float4* __restrict__ out) {
  const uint32_t n4 = row4 * h;
  for (uint32_t c = blockIdx.x * kThreads + threadIdx.x; c < n4; c += gridDim.x * kThreads) {
    const uint32_t y = (uint32_t)(((uint64_t)c * m_row) >> sh_row), r = c - y * row4;
    out[(h - 1 - y) * row4 + r] = rgb[c];
  }
}
__global__ void __launch_bounds__(kThreads)
pfm_write1(const float* __restrict__ rgb, uint32_t row, uint32_t h, uint32_t m_row, uint32_t sh_row,
           float* __restrict__ out) {
  const uint32_t n = row * h;
  for (uint32_t c = blockIdx.x * kThreads + threadIdx.x; c < n; c += gridDim.x * kThreads) {
    const uint32_t y = (uint32_t)(((uint64_t)c * m_row) >> sh_row), r = c - y * row;
    out[(h - 1 - y) * row + r] = rgb[c];
  }
}

// n / d = (n * m) >> sh for n < 2^31 (same construction as the render kernel's refill)
static void magic31(uint32_t d, uint32_t* m, uint32_t* sh) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  *m = (uint32_t)(((unsigned __int128)1 << (31 + l)) / d + 1);
  *sh = 31 + l;
}

// P3 is the reference's header exactly. P6 and PFM pad their header to a multiple of 16 bytes so
// the raster starts 16-byte aligned: P6 with spaces before the final newline of the size line
// (any whitespace may separate tokens in a PPM header), PFM with zeros in the scale ("-1.000...").
static std::string header(int w, int h, int format) {
  char b[96];
  if (format == SPT_IMAGE_P3) {
    std::snprintf(b, sizeof b, "P3\n%d %d\n%d\n", w, h, 255);  // :549
    return b;
  }
  if (format == SPT_IMAGE_P6) {
    std::string s = "P6\n" + std::to_string(w) + " " + std::to_string(h);
    while ((s.size() + 5) % 16) s += " ";
    return s + "\n255\n";
  }
  std::string s = "PF\n" + std::to_string(w) + " " + std::to_string(h) + "\n-1.0";
  while ((s.size() + 1) % 16) s += "0";
  return s + "\n";
}

}  // namespace spt_img

using namespace spt_img;

struct spt_encoder {
  int device = 0;
  uint8_t* scratch = nullptr;    // two-pass P3: offsets, block lengths, NaN word, digits
  size_t scratch_cap = 0;        // bytes
  uint32_t epoch = 0;            // P3 encodes so far: the NaN word holds the epoch of the last NaN
  uint64_t* total = nullptr;     // device word: encoded length
  uint64_t* h_total = nullptr;   // pinned mirror
};

void spt_set_last_error(const std::string& msg);  // spt_kernel.hip: spt_last_error() text
static spt_status img_fail(spt_status s, const std::string& m) {
  spt_set_last_error(m);
  return s;
}
#define IMG_HIP(call)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return img_fail(e_ == hipErrorOutOfMemory ? SPT_ERR_OOM : SPT_ERR_HIP,                 \
                      std::string(#call) + ": " + hipGetErrorString(e_));                    \
  } while (0)

extern "C" uint64_t spt_image_bound(int32_t w, int32_t h, int32_t format) {
  if (w <= 0 || h <= 0 || format < SPT_IMAGE_P3 || format > SPT_IMAGE_PFM) return 0;
  const uint64_t n = (uint64_t)w * (uint64_t)h;
  const uint64_t per = format == SPT_IMAGE_P3 ? 3 * kMaxValueText : format == SPT_IMAGE_P6 ? 3 : 12;
  return header(w, h, format).size() + n * per;
}

extern "C" spt_status spt_encoder_create(int32_t device, spt_encoder** out) {
  if (!out) return img_fail(SPT_ERR_INVALID_ARG, "null out");
  int count = 0;
  const hipError_t ce = hipGetDeviceCount(&count);
  if (ce != hipSuccess || count == 0)
    return img_fail(SPT_ERR_NO_DEVICE, std::string("no HIP device (") + hipGetErrorString(ce) + ")");
  if (device < 0 || device >= count) return img_fail(SPT_ERR_INVALID_ARG, "bad device ordinal");
  IMG_HIP(hipSetDevice(device));
  spt_encoder* e = new spt_encoder();
  e->device = device;
  hipError_t r = hipMalloc(&e->total, sizeof(uint64_t));
  if (r == hipSuccess) r = hipHostMalloc(&e->h_total, sizeof(uint64_t), hipHostMallocDefault);
  if (r != hipSuccess) {
    spt_encoder_destroy(e);
    return img_fail(SPT_ERR_OOM, "encoder alloc");
  }
  *out = e;
  return SPT_OK;
}

extern "C" spt_status spt_encoder_destroy(spt_encoder* e) {
  if (!e) return SPT_OK;
  (void)hipSetDevice(e->device);
  if (e->scratch) (void)hipFree(e->scratch);
  if (e->total) (void)hipFree(e->total);
  if (e->h_total) (void)hipHostFree(e->h_total);
  delete e;
  return SPT_OK;
}

extern "C" spt_status spt_encode_image(spt_encoder* e, const float* rgb_dev, int32_t w, int32_t h,
                                       int32_t format, uint8_t* out_dev, uint64_t cap,
                                       uint64_t* len_out, void* stream_v) {
  if (!e || !rgb_dev || !out_dev || !len_out) return img_fail(SPT_ERR_INVALID_ARG, "null argument");
  // 3 w h <= 2^32 - 8192: the text kernels' 32-bit value index of the last block cannot wrap
  if (w <= 0 || h <= 0 || 3ull * (uint64_t)w * (uint64_t)h > 0xFFFFFFFFull - kTxtBlockVals)
    return img_fail(SPT_ERR_INVALID_ARG, "bad image size");
  if (format < SPT_IMAGE_P3 || format > SPT_IMAGE_PFM) return img_fail(SPT_ERR_INVALID_ARG, "bad format");
  const std::string hd = header(w, h, format);
  // every argument check before any work is queued: a rejected call leaves out_dev and the
  // encoder's scratch as they were
  if (((uintptr_t)rgb_dev & 15u) != 0) return img_fail(SPT_ERR_INVALID_ARG, "framebuffer must be 16-byte aligned");
  if (format != SPT_IMAGE_P3 && ((uintptr_t)(out_dev + hd.size()) & 15u) != 0)
    return img_fail(SPT_ERR_INVALID_ARG, "output raster must be 16-byte aligned");
  IMG_HIP(hipSetDevice(e->device));
  hipStream_t stream = (hipStream_t)stream_v;
  const uint32_t n_pix = (uint32_t)((uint64_t)w * (uint64_t)h);
  const Thresholds& T = thresholds();
  uint64_t len;
  if (format == SPT_IMAGE_P3) {
    if (cap >= hd.size()) IMG_HIP(hipMemcpyAsync(out_dev, hd.data(), hd.size(), hipMemcpyHostToDevice, stream));
    // two passes around the toInt bytes: p6_write (+ NaN epoch) -> p3_lengths -> p3_offsets ->
    // p3_text, all on the stream
    const uint32_t nv = n_pix * 3;
    const uint32_t nbt = (uint32_t)(((uint64_t)nv + kTxtBlockVals - 1) / kTxtBlockVals);
    const size_t off_b = 0, len_b = off_b + 8ull * nbt, nan_b = len_b + 4ull * nbt;
    const size_t dig_b = (nan_b + 4 + 15) & ~size_t(15);
    const size_t need = dig_b + (((size_t)nv + 15) & ~size_t(15));
    if (need > e->scratch_cap) {
      if (e->scratch) IMG_HIP(hipFree(e->scratch));
      e->scratch = nullptr;
      e->scratch_cap = 0;
      IMG_HIP(hipMalloc(&e->scratch, need));
      IMG_HIP(hipMemsetAsync(e->scratch, 0, need, stream));  // the NaN word starts at epoch 0
      e->scratch_cap = need;
      e->epoch = 0;
    }
    const uint32_t epoch = ++e->epoch == 0 ? ++e->epoch : e->epoch;  // never 0 (the initial word)
    uint64_t* offs = (uint64_t*)(e->scratch + off_b);
    uint32_t* blen = (uint32_t*)(e->scratch + len_b);
    uint32_t* nan_word = (uint32_t*)(e->scratch + nan_b);
    uint8_t* digits = e->scratch + dig_b;
    const uint32_t grid1 = std::max(1u, std::min((nv / 4 + kThreads - 1) / kThreads, 2048u));
    hipLaunchKernelGGL(p6_write, dim3(grid1), dim3(kThreads), 0, stream, (const float4*)rgb_dev, nv, T,
                       (uint32_t*)digits, nan_word, epoch);
    IMG_HIP(hipGetLastError());
    hipLaunchKernelGGL(p3_lengths, dim3(nbt), dim3(kTxtThreads), 0, stream, (const uint4*)digits, rgb_dev,
                       nv, T, (const uint32_t*)nan_word, epoch, blen);
    IMG_HIP(hipGetLastError());
    hipLaunchKernelGGL(p3_offsets, dim3(1), dim3(kScanThreads), 0, stream, (const uint32_t*)blen, nbt,
                       (uint64_t)hd.size(), offs, e->total);
    IMG_HIP(hipGetLastError());
    hipLaunchKernelGGL(p3_text, dim3(nbt), dim3(kTxtThreads), 0, stream, (const uint4*)digits, rgb_dev,
                       nv, T, (const uint32_t*)nan_word, epoch, (const uint64_t*)offs, out_dev, cap);
    IMG_HIP(hipGetLastError());
    IMG_HIP(hipMemcpyAsync(e->h_total, e->total, sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
    IMG_HIP(hipStreamSynchronize(stream));  // the text length is data-dependent
    len = *e->h_total;
    *len_out = len;
    if (len > cap) return img_fail(SPT_ERR_INVALID_ARG, "output buffer too small (need " + std::to_string(len) + " bytes)");
  } else {
    len = hd.size() + (uint64_t)n_pix * (format == SPT_IMAGE_P6 ? 3 : 12);
    *len_out = len;
    if (len > cap) return img_fail(SPT_ERR_INVALID_ARG, "output buffer too small (need " + std::to_string(len) + " bytes)");
    IMG_HIP(hipMemcpyAsync(out_dev, hd.data(), hd.size(), hipMemcpyHostToDevice, stream));
    const uint32_t nv = n_pix * 3;
    // grid-stride loops over ~8 blocks per CU (the block prologue stages the toInt table)
    const uint32_t grid = std::max(1u, std::min((nv / 4 + kThreads - 1) / kThreads, 2048u));
    if (format == SPT_IMAGE_P6) {
      hipLaunchKernelGGL(p6_write, dim3(grid), dim3(kThreads), 0, stream, (const float4*)rgb_dev, nv, T,
                         (uint32_t*)(out_dev + hd.size()), (uint32_t*)nullptr, 0u);
    } else if (w % 4 == 0) {
      uint32_t m, sh;
      magic31((uint32_t)w * 3 / 4, &m, &sh);
      hipLaunchKernelGGL(pfm_write4, dim3(grid), dim3(kThreads), 0, stream, (const float4*)rgb_dev,
                         (uint32_t)w * 3 / 4, (uint32_t)h, m, sh, (float4*)(out_dev + hd.size()));
    } else {
      uint32_t m, sh;
      magic31((uint32_t)w * 3, &m, &sh);
      hipLaunchKernelGGL(pfm_write1, dim3(grid * 4), dim3(kThreads), 0, stream, rgb_dev, (uint32_t)w * 3,
                         (uint32_t)h, m, sh, (float*)(out_dev + hd.size()));
    }
    IMG_HIP(hipGetLastError());
  }
  return SPT_OK;
}

extern "C" spt_status spt_write_image(int32_t device, const float* rgb, int32_t w, int32_t h,
                                      int32_t format, const char* path) {
  if (!rgb || !path) return img_fail(SPT_ERR_INVALID_ARG, "null argument");
  spt_encoder* e = nullptr;
  spt_status st = spt_encoder_create(device, &e);
  if (st != SPT_OK) return st;
  hipPointerAttribute_t attr;
  const bool on_device = hipPointerGetAttributes(&attr, rgb) == hipSuccess &&
                         attr.type == hipMemoryTypeDevice;
  (void)hipGetLastError();
  const size_t n_f = 3ull * (size_t)w * (size_t)h;
  float* src = nullptr;
  uint8_t* dev_out = nullptr;
  std::vector<uint8_t> host;
  uint64_t cap = spt_image_bound(w, h, format), len = 0;
  hipError_t r = hipSuccess;
  if (!on_device) {
    r = hipMalloc(&src, n_f * sizeof(float));
    if (r == hipSuccess) r = hipMemcpy(src, rgb, n_f * sizeof(float), hipMemcpyHostToDevice);
  }
  if (r == hipSuccess) r = hipMalloc(&dev_out, cap);
  if (r != hipSuccess) st = img_fail(SPT_ERR_OOM, std::string("write_image: ") + hipGetErrorString(r));
  if (st == SPT_OK) st = spt_encode_image(e, on_device ? rgb : src, w, h, format, dev_out, cap, &len, nullptr);
  if (st == SPT_OK) {
    host.resize(len);
    r = hipMemcpy(host.data(), dev_out, len, hipMemcpyDeviceToHost);
    if (r != hipSuccess) st = img_fail(SPT_ERR_HIP, hipGetErrorString(r));
  }
  if (st == SPT_OK) {
    FILE* f = std::fopen(path, "wb");
    if (!f || std::fwrite(host.data(), 1, len, f) != len) st = img_fail(SPT_ERR_INVALID_ARG, std::string("cannot write ") + path);
    if (f) std::fclose(f);
  }
  if (src) (void)hipFree(src);
  if (dev_out) (void)hipFree(dev_out);
  spt_encoder_destroy(e);
  return st;
}
