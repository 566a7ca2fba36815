// spt_image.hip — the reference's image output (/root/reference/src/smallpt.cpp:313-321 toInt/clamp,
// :548-551 the P3 writer) as a gfx950 encoder, plus binary P6 and linear PFM.
//
// The reference writes `fprintf(f, "%d %d %d ", toInt(r), toInt(g), toInt(b))` per pixel: ASCII
// P3, 6-12 bytes per pixel, ~200 MB of text at 4096². Here the framebuffer never leaves HBM until
// the bytes are final: three HBM-bound byte passes over the fp32 framebuffer.
//   pass 1  per-block text length (4 pixels per thread, 1024 per block)
//   scan    exclusive scan of the block lengths (one block), + header length -> block offsets
//   pass 3  per-thread text into an LDS staging buffer placed at the destination's dword phase,
//           then aligned dword stores of the block's contiguous byte range (head/tail bytes apart)
// toInt is evaluated exactly as the reference's double-precision pow() by a 256-entry threshold
// table computed on the host with that very formula (toInt is monotone in x): the device counts
// the thresholds <= x with an 8-step binary search in LDS. NaN prints as x86-64's int(NaN),
// INT_MIN, as the reference binary does.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/spt.h"

namespace spt_img {

constexpr int kThreads = 256;
constexpr int kPixPerThread = 4;
constexpr int kPixPerBlock = kThreads * kPixPerThread;  // 1024
constexpr int kMaxValueText = 12;                        // "-2147483648 "
constexpr int kStageBytes = kPixPerBlock * 3 * kMaxValueText + 16;

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

__device__ __forceinline__ int dev_toInt(const float* __restrict__ thr, float x) {
  if (x != x) return (int)0x80000000;  // int(NaN) on x86-64 (cvttsd2si)
  int idx = 0;
#pragma unroll
  for (int step = 128; step >= 1; step >>= 1) idx = x >= thr[idx + step] ? idx + step : idx;
  return idx;
}

__device__ __forceinline__ uint32_t text_len(int v) {
  return v < 0 ? 12u : v >= 100 ? 4u : v >= 10 ? 3u : 2u;  // digits + the trailing space
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
  for (int i = threadIdx.x; i < 256; i += kThreads) s_thr[i] = T.t[i];
  __syncthreads();
}

// Block-wide exclusive scan of one uint32 per thread (wave shuffles + LDS for wave totals).
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
  for (int w = 0; w < kThreads / 64; ++w) {
    const uint32_t t = s_wave[w];
    base += w < wave ? t : 0u;
    all += t;
  }
  *total = all;
  return base + incl - v;
}

__global__ void __launch_bounds__(kThreads)
p3_lengths(const float* __restrict__ rgb, uint32_t n_pix, Thresholds T, uint32_t* __restrict__ block_len) {
  __shared__ float s_thr[256];
  __shared__ uint32_t s_wave[kThreads / 64];
  load_thr(s_thr, T);
  const uint64_t v0 = ((uint64_t)blockIdx.x * kPixPerBlock + (uint64_t)threadIdx.x * kPixPerThread) * 3;
  const uint64_t nv = (uint64_t)n_pix * 3;
  uint32_t len = 0;
#pragma unroll
  for (int i = 0; i < kPixPerThread * 3; ++i)
    if (v0 + i < nv) len += text_len(dev_toInt(s_thr, rgb[v0 + i]));
  uint32_t total;
  (void)block_excl_scan(len, s_wave, &total);
  if (threadIdx.x == 0) block_len[blockIdx.x] = total;
}

// Exclusive scan of the block lengths (one block of 1024 threads, sequential tiles with a carry).
__global__ void __launch_bounds__(1024)
scan_blocks(const uint32_t* __restrict__ block_len, uint64_t* __restrict__ block_off, uint32_t n,
            uint64_t header, uint64_t* __restrict__ total) {
  __shared__ uint64_t s[1024];
  uint64_t carry = header;
  for (uint32_t base = 0; base < n; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint64_t v = i < n ? block_len[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
      const uint64_t u = threadIdx.x >= (unsigned)off ? s[threadIdx.x - off] : 0;
      __syncthreads();
      s[threadIdx.x] += u;
      __syncthreads();
    }
    if (i < n) block_off[i] = carry + s[threadIdx.x] - v;
    const uint64_t tile = s[1023];
    __syncthreads();
    carry += tile;
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ void __launch_bounds__(kThreads)
p3_write(const float* __restrict__ rgb, uint32_t n_pix, Thresholds T,
         const uint64_t* __restrict__ block_off, uint8_t* __restrict__ out) {
  __shared__ float s_thr[256];
  __shared__ uint32_t s_wave[kThreads / 64];
  __shared__ __attribute__((aligned(16))) uint8_t s_txt[kStageBytes];
  load_thr(s_thr, T);
  const uint64_t v0 = ((uint64_t)blockIdx.x * kPixPerBlock + (uint64_t)threadIdx.x * kPixPerThread) * 3;
  const uint64_t nv = (uint64_t)n_pix * 3;
  int vals[kPixPerThread * 3];
  uint32_t len = 0;
#pragma unroll
  for (int i = 0; i < kPixPerThread * 3; ++i) {
    vals[i] = v0 + i < nv ? dev_toInt(s_thr, rgb[v0 + i]) : 0;
    len += v0 + i < nv ? text_len(vals[i]) : 0u;
  }
  uint32_t total;
  const uint32_t my = block_excl_scan(len, s_wave, &total);
  const uint64_t dst = block_off[blockIdx.x];
  const uint32_t phase = (uint32_t)(dst & 3u);  // stage at the destination's dword phase
  uint8_t* p = s_txt + phase + my;
#pragma unroll
  for (int i = 0; i < kPixPerThread * 3; ++i)
    if (v0 + i < nv) p += put_value(p, vals[i]);
  __syncthreads();
  // bytes [dst, dst + total) <- s_txt[phase, phase + total)
  const uint64_t a0 = (dst + 3u) & ~3ull, a1 = (dst + total) & ~3ull;  // aligned middle
  if (a0 >= a1) {
    for (uint32_t i = threadIdx.x; i < total; i += kThreads) out[dst + i] = s_txt[phase + i];
    return;
  }
  const uint32_t head = (uint32_t)(a0 - dst), tail = (uint32_t)(dst + total - a1);
  if (threadIdx.x < head) out[dst + threadIdx.x] = s_txt[phase + threadIdx.x];
  if (threadIdx.x < tail) out[a1 + threadIdx.x] = s_txt[phase + (uint32_t)(a1 - dst) + threadIdx.x];
  const uint32_t n_dw = (uint32_t)((a1 - a0) >> 2);
  const uint32_t* s_dw = (const uint32_t*)(s_txt + phase + head);  // dword-aligned in LDS
  uint32_t* o_dw = (uint32_t*)(out + a0);
  for (uint32_t i = threadIdx.x; i < n_dw; i += kThreads) o_dw[i] = s_dw[i];
}

// P6: header, then toInt bytes (unsigned char of the int, as a byte-writing port would store).
__global__ void __launch_bounds__(kThreads)
p6_write(const float* __restrict__ rgb, uint32_t n_pix, Thresholds T, uint8_t* __restrict__ out) {
  __shared__ float s_thr[256];
  load_thr(s_thr, T);
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < (uint64_t)n_pix * 3) out[i] = (uint8_t)dev_toInt(s_thr, rgb[i]);
}

// PFM: little-endian float RGB, scanlines bottom to top; the header is padded to a dword multiple
// so every float store is aligned.
__global__ void __launch_bounds__(kThreads)
pfm_write(const float* __restrict__ rgb, uint32_t w, uint32_t h, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint64_t row_f = (uint64_t)w * 3;
  if (i >= row_f * h) return;
  const uint64_t y = i / row_f, r = i - y * row_f;
  out[(h - 1 - y) * row_f + r] = __float_as_uint(rgb[i]);
}

static std::string header(int w, int h, int format) {
  char b[96];
  if (format == SPT_IMAGE_P3) std::snprintf(b, sizeof b, "P3\n%d %d\n%d\n", w, h, 255);  // :549
  else if (format == SPT_IMAGE_P6) std::snprintf(b, sizeof b, "P6\n%d %d\n255\n", w, h);
  else {
    std::string s = "PF\n" + std::to_string(w) + " " + std::to_string(h) + "\n-1.0";
    while ((s.size() + 1) % 4) s += "0";  // "-1.0", "-1.00", ... : data starts dword-aligned
    return s + "\n";
  }
  return b;
}

}  // namespace spt_img

using namespace spt_img;

struct spt_encoder {
  int device = 0;
  uint32_t* block_len = nullptr;
  uint64_t* block_off = nullptr;
  uint32_t cap_blocks = 0;
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
  if (e->block_len) (void)hipFree(e->block_len);
  if (e->block_off) (void)hipFree(e->block_off);
  if (e->total) (void)hipFree(e->total);
  if (e->h_total) (void)hipHostFree(e->h_total);
  delete e;
  return SPT_OK;
}

extern "C" spt_status spt_encode_image(spt_encoder* e, const float* rgb_dev, int32_t w, int32_t h,
                                       int32_t format, uint8_t* out_dev, uint64_t cap,
                                       uint64_t* len_out, void* stream_v) {
  if (!e || !rgb_dev || !out_dev || !len_out) return img_fail(SPT_ERR_INVALID_ARG, "null argument");
  if (w <= 0 || h <= 0 || (uint64_t)w * (uint64_t)h > 0xFFFFFFFFull / 3)
    return img_fail(SPT_ERR_INVALID_ARG, "bad image size");
  if (format < SPT_IMAGE_P3 || format > SPT_IMAGE_PFM) return img_fail(SPT_ERR_INVALID_ARG, "bad format");
  IMG_HIP(hipSetDevice(e->device));
  hipStream_t stream = (hipStream_t)stream_v;
  const uint32_t n_pix = (uint32_t)((uint64_t)w * (uint64_t)h);
  const std::string hd = header(w, h, format);
  const Thresholds& T = thresholds();
  uint64_t len;
  if (format == SPT_IMAGE_P3) {
    const uint32_t nb = (n_pix + kPixPerBlock - 1) / kPixPerBlock;
    if (nb > e->cap_blocks) {
      if (e->block_len) IMG_HIP(hipFree(e->block_len));
      if (e->block_off) IMG_HIP(hipFree(e->block_off));
      e->block_len = nullptr;
      e->block_off = nullptr;
      e->cap_blocks = 0;
      IMG_HIP(hipMalloc(&e->block_len, sizeof(uint32_t) * nb));
      IMG_HIP(hipMalloc(&e->block_off, sizeof(uint64_t) * nb));
      e->cap_blocks = nb;
    }
    hipLaunchKernelGGL(p3_lengths, dim3(nb), dim3(kThreads), 0, stream, rgb_dev, n_pix, T, e->block_len);
    IMG_HIP(hipGetLastError());
    hipLaunchKernelGGL(scan_blocks, dim3(1), dim3(1024), 0, stream, (const uint32_t*)e->block_len,
                       e->block_off, nb, (uint64_t)hd.size(), e->total);
    IMG_HIP(hipGetLastError());
    IMG_HIP(hipMemcpyAsync(e->h_total, e->total, sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
    IMG_HIP(hipStreamSynchronize(stream));  // the text length is data-dependent
    len = *e->h_total;
    *len_out = len;
    if (len > cap) return img_fail(SPT_ERR_INVALID_ARG, "output buffer too small (need " + std::to_string(len) + " bytes)");
    IMG_HIP(hipMemcpyAsync(out_dev, hd.data(), hd.size(), hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(p3_write, dim3(nb), dim3(kThreads), 0, stream, rgb_dev, n_pix, T,
                       (const uint64_t*)e->block_off, out_dev);
    IMG_HIP(hipGetLastError());
  } else {
    len = hd.size() + (uint64_t)n_pix * (format == SPT_IMAGE_P6 ? 3 : 12);
    *len_out = len;
    if (len > cap) return img_fail(SPT_ERR_INVALID_ARG, "output buffer too small (need " + std::to_string(len) + " bytes)");
    IMG_HIP(hipMemcpyAsync(out_dev, hd.data(), hd.size(), hipMemcpyHostToDevice, stream));
    const uint64_t nv = (uint64_t)n_pix * 3;
    const dim3 grid((unsigned)((nv + kThreads - 1) / kThreads));
    if (format == SPT_IMAGE_P6)
      hipLaunchKernelGGL(p6_write, grid, dim3(kThreads), 0, stream, rgb_dev, n_pix, T, out_dev + hd.size());
    else
      hipLaunchKernelGGL(pfm_write, grid, dim3(kThreads), 0, stream, rgb_dev, (uint32_t)w, (uint32_t)h,
                         (uint32_t*)(out_dev + hd.size()));
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
