// spt_multi.hip — multi-GPU row-tile sharding with ONE framebuffer gather over RCCL.
//
// The reference renders on one CPU thread (its only parallel construct is the commented-out
// OpenMP pragma at smallpt.cpp:526 over the row loop :528). Here rows are sharded across GPUs in
// tiles of tile_rows (tile t -> rank t % n, spt_shard_rows), each rank renders its rows into a
// compact buffer (spt_render_async), and rank 0 receives every other rank's buffer with one grouped
// ncclSend/ncclRecv per rank over xGMI, then de-interleaves the tiles into the image with one
// HBM-bound kernel. Pixels are disjoint, so there is no reduction (an ncclReduce over zero-padded
// full-size buffers would move n times the bytes). Because the counter RNG is keyed by the global
// pixel index and accumulation is integer, the gathered image is bit-identical to a 1-GPU render.
//
// Two ways in:
//   * one process per GPU (bench.py under torchrun): spt_comm_unique_id on rank 0, the id passed
//     to every rank by the caller (torch.distributed here), spt_comm_create(id, n, rank, device),
//     spt_gather_framebuffer after each rank's spt_render_async on the same stream;
//   * one process driving n GPUs (smallpt_amd --devices N): spt_render_multi.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/spt.h"

void spt_set_last_error(const std::string& msg);  // spt_kernel.hip
int spt_shard_row_count(const spt_params* p);     // spt_host.cpp

namespace {

constexpr int kMaxRanks = 64;
constexpr int kThreads = 256;

spt_status fail(spt_status s, const std::string& msg) {
  spt_set_last_error(msg);
  return s;
}
#define SPT_HIPM(call)                                                                    \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(e_ == hipErrorOutOfMemory ? SPT_ERR_OOM : SPT_ERR_HIP,                  \
                  std::string(#call) + ": " + hipGetErrorString(e_));                     \
  } while (0)
#define SPT_NCCL(call)                                                                    \
  do {                                                                                    \
    ncclResult_t r_ = (call);                                                             \
    if (r_ != ncclSuccess)                                                                \
      return fail(SPT_ERR_RCCL, std::string(#call) + ": " + ncclGetErrorString(r_));      \
  } while (0)

struct Sources { const float* p[kMaxRanks]; };

// The de-interleave's row map, shared by the kernel and the host plan (spt_deinterleave_source):
// image row r lies in tile t = r / T, which rank k = t % n rendered as its compact row
// j = (t / n) * T + r % T (spt_shard_rows lists a shard's rows in increasing order).
__host__ __device__ inline void row_source(int r, int n, int T, int* k, size_t* j) {
  const int t = r / T;
  *k = t % n;
  *j = (size_t)(t / n) * (size_t)T + (size_t)(r % T);
}

// image row r <- its rank's compact row (row_source). One block per image row, 16-byte vectors when
// a row is a multiple of them.
__global__ void __launch_bounds__(kThreads)
deinterleave_kernel(Sources src, int n, int T, int h, int row_floats, float* __restrict__ image) {
  const int r = blockIdx.x;
  if (r >= h) return;
  int k;
  size_t j;
  row_source(r, n, T, &k, &j);
  const float* __restrict__ s = src.p[k] + j * (size_t)row_floats;
  float* __restrict__ d = image + (size_t)r * (size_t)row_floats;
  if ((row_floats & 3) == 0 && ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
    const int nv = row_floats >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(s);
    float4* d4 = reinterpret_cast<float4*>(d);
    for (int i = threadIdx.x; i < nv; i += kThreads) d4[i] = s4[i];
  } else {
    for (int i = threadIdx.x; i < row_floats; i += kThreads) d[i] = s[i];
  }
}

spt_status check_layout(const spt_params* p, int32_t nranks) {
  if (!p) return fail(SPT_ERR_INVALID_ARG, "null params");
  if (nranks < 1 || nranks > kMaxRanks) return fail(SPT_ERR_INVALID_ARG, "nranks must be in [1, 64]");
  if (p->width <= 0 || p->height <= 0) return fail(SPT_ERR_INVALID_ARG, "bad image size");
  if (p->shard_count != nranks) return fail(SPT_ERR_INVALID_ARG, "params.shard_count != nranks");
  if (p->tile_rows < 0) return fail(SPT_ERR_INVALID_ARG, "negative tile_rows");
  return SPT_OK;
}

int tile_rows_of(const spt_params* p) { return p->tile_rows > 0 ? p->tile_rows : 8; }

size_t shard_floats(const spt_params* p, int k) {
  spt_params q = *p;
  q.shard_index = k;
  return 3ull * (size_t)spt_shard_row_count(&q) * (size_t)p->width;
}

}  // namespace

struct spt_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0, device = 0;
  float* gbuf = nullptr;  // rank 0: slots for ranks 1..n-1, `slot` floats each
  size_t gbuf_cap = 0;    // floats
};

extern "C" spt_status spt_deinterleave_rows(const spt_params* p, int32_t nranks,
                                            const float* const* shards_dev, float* image_dev,
                                            void* stream) {
  spt_status st = check_layout(p, nranks);
  if (st != SPT_OK) return st;
  if (!shards_dev || !image_dev) return fail(SPT_ERR_INVALID_ARG, "null buffer");
  Sources src{};
  for (int k = 0; k < nranks; ++k) {
    if (!shards_dev[k] && shard_floats(p, k) != 0) return fail(SPT_ERR_INVALID_ARG, "null shard");
    src.p[k] = shards_dev[k];
  }
  hipLaunchKernelGGL(deinterleave_kernel, dim3(p->height), dim3(kThreads), 0, (hipStream_t)stream,
                     src, (int)nranks, tile_rows_of(p), (int)p->height, 3 * (int)p->width, image_dev);
  SPT_HIPM(hipGetLastError());
  return SPT_OK;
}

// ---- the gather as pure host functions (CPU-testable: no device, no RCCL) ----

extern "C" uint64_t spt_gather_staging_floats(const spt_params* p, int32_t nranks) {
  if (check_layout(p, nranks) != SPT_OK) return 0;
  return nranks < 2 ? 0 : shard_floats(p, 0) * (uint64_t)(nranks - 1);
}

extern "C" int32_t spt_gather_plan(const spt_params* p, int32_t nranks, int32_t rank,
                                   spt_gather_op* ops, int32_t cap) {
  if (check_layout(p, nranks) != SPT_OK || rank < 0 || rank >= nranks || cap < 0 || (!ops && cap > 0))
    return -1;
  // slot = shard 0's floats: shard 0 owns tiles 0, n, 2n, ..., never fewer rows than another shard
  const uint64_t slot = shard_floats(p, 0);
  int32_t n = 0;
  auto put = [&](int32_t kind, int32_t peer, uint64_t count, uint64_t offset) {
    if (n < cap) ops[n] = spt_gather_op{kind, peer, count, offset};
    ++n;
  };
  if (rank != 0) {
    const uint64_t cnt = shard_floats(p, rank);
    if (cnt) put(SPT_GATHER_SEND, 0, cnt, 0);
  } else {
    for (int k = 1; k < nranks; ++k) {
      const uint64_t cnt = shard_floats(p, k);
      if (cnt) put(SPT_GATHER_RECV, k, cnt, (uint64_t)(k - 1) * slot);
    }
  }
  return n > cap ? -1 : n;
}

extern "C" spt_status spt_deinterleave_source(const spt_params* p, int32_t nranks, int32_t row,
                                              int32_t* rank, int32_t* compact_row) {
  spt_status st = check_layout(p, nranks);
  if (st != SPT_OK) return st;
  if (!rank || !compact_row || row < 0 || row >= p->height) return fail(SPT_ERR_INVALID_ARG, "bad row");
  int k;
  size_t j;
  row_source(row, nranks, tile_rows_of(p), &k, &j);
  *rank = k;
  *compact_row = (int32_t)j;
  return SPT_OK;
}

extern "C" spt_status spt_comm_unique_id(uint8_t id[SPT_COMM_ID_BYTES]) {
  if (!id) return fail(SPT_ERR_INVALID_ARG, "null id");
  static_assert(SPT_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId u;
  SPT_NCCL(ncclGetUniqueId(&u));
  std::memcpy(id, u.internal, SPT_COMM_ID_BYTES);
  return SPT_OK;
}

extern "C" spt_status spt_comm_create(const uint8_t id[SPT_COMM_ID_BYTES], int32_t nranks,
                                      int32_t rank, int32_t device, spt_comm** out) {
  if (!id || !out) return fail(SPT_ERR_INVALID_ARG, "null argument");
  if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks)
    return fail(SPT_ERR_INVALID_ARG, "bad nranks/rank");
  SPT_HIPM(hipSetDevice(device));
  ncclUniqueId u;
  std::memcpy(u.internal, id, SPT_COMM_ID_BYTES);
  spt_comm* c = new spt_comm();
  c->nranks = nranks; c->rank = rank; c->device = device;
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(SPT_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  *out = c;
  return SPT_OK;
}

extern "C" spt_status spt_comm_destroy(spt_comm* c) {
  if (!c) return SPT_OK;
  (void)hipSetDevice(c->device);
  if (c->gbuf) (void)hipFree(c->gbuf);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
  return SPT_OK;
}

namespace {

// The transfers of one gather as calls inside an open ncclGroupStart/End, executed from the pure
// host plan (spt_gather_plan): rank k > 0 sends its compact shard to rank 0; rank 0 posts one
// receive per other rank into that rank's slot of gbuf.
spt_status post_gather(spt_comm* c, const spt_params* p, const float* shard_dev, hipStream_t s) {
  spt_gather_op ops[kMaxRanks];
  const int n_ops = spt_gather_plan(p, c->nranks, c->rank, ops, kMaxRanks);
  if (n_ops < 0) return fail(SPT_ERR_INVALID_ARG, "gather plan");
  for (int i = 0; i < n_ops; ++i) {
    const spt_gather_op& o = ops[i];
    if (o.kind == SPT_GATHER_SEND) SPT_NCCL(ncclSend(shard_dev, o.count, ncclFloat32, o.peer, c->comm, s));
    else SPT_NCCL(ncclRecv(c->gbuf + o.offset, o.count, ncclFloat32, o.peer, c->comm, s));
  }
  return SPT_OK;
}

spt_status reserve_gbuf(spt_comm* c, size_t slot) {
  if (c->rank != 0 || c->nranks < 2) return SPT_OK;
  const size_t need = slot * (size_t)(c->nranks - 1);
  if (need <= c->gbuf_cap) return SPT_OK;
  SPT_HIPM(hipSetDevice(c->device));
  if (c->gbuf) SPT_HIPM(hipFree(c->gbuf));
  c->gbuf = nullptr;
  c->gbuf_cap = 0;
  SPT_HIPM(hipMalloc(&c->gbuf, need * sizeof(float)));
  c->gbuf_cap = need;
  return SPT_OK;
}

// Rank 0's de-interleave: shard 0 from its own render, shard k > 0 from where the plan's receive
// from k landed (a rank that owns no rows has no receive, and the de-interleave reads none of it).
spt_status deinterleave_on_root(spt_comm* c, const spt_params* p, const float* shard_dev,
                                float* image_dev, hipStream_t s) {
  std::vector<const float*> src((size_t)c->nranks, (const float*)c->gbuf);
  src[0] = shard_dev;
  spt_gather_op ops[kMaxRanks];
  const int n_ops = spt_gather_plan(p, c->nranks, 0, ops, kMaxRanks);
  if (n_ops < 0) return fail(SPT_ERR_INVALID_ARG, "gather plan");
  for (int i = 0; i < n_ops; ++i) src[(size_t)ops[i].peer] = c->gbuf + ops[i].offset;
  return spt_deinterleave_rows(p, c->nranks, src.data(), image_dev, s);
}

}  // namespace

extern "C" spt_status spt_comm_reserve(spt_comm* c, const spt_params* p) {
  if (!c) return fail(SPT_ERR_INVALID_ARG, "null comm");
  spt_status st = check_layout(p, c->nranks);
  if (st != SPT_OK) return st;
  return reserve_gbuf(c, shard_floats(p, 0));
}

extern "C" spt_status spt_gather_framebuffer(spt_comm* c, const spt_params* p,
                                             const float* shard_dev, float* image_dev,
                                             void* stream) {
  if (!c) return fail(SPT_ERR_INVALID_ARG, "null comm");
  spt_status st = check_layout(p, c->nranks);
  if (st != SPT_OK) return st;
  if (c->rank == 0 && !image_dev) return fail(SPT_ERR_INVALID_ARG, "rank 0 needs image_dev");
  if (!shard_dev && shard_floats(p, c->rank) != 0) return fail(SPT_ERR_INVALID_ARG, "null shard");
  const size_t slot = shard_floats(p, 0);  // shard 0 owns the most rows (tiles 0, n, 2n, ...)
  st = reserve_gbuf(c, slot);
  if (st != SPT_OK) return st;
  SPT_HIPM(hipSetDevice(c->device));
  const hipStream_t s = (hipStream_t)stream;
  if (c->nranks > 1) {
    SPT_NCCL(ncclGroupStart());
    st = post_gather(c, p, shard_dev, s);
    const ncclResult_t r = ncclGroupEnd();
    if (st != SPT_OK) return st;
    if (r != ncclSuccess) return fail(SPT_ERR_RCCL, std::string("ncclGroupEnd: ") + ncclGetErrorString(r));
  }
  if (c->rank == 0) return deinterleave_on_root(c, p, shard_dev, image_dev, s);
  return SPT_OK;
}

extern "C" spt_status spt_render_multi(const spt_prim* prims, int32_t n_prims, const spt_camera* cam,
                                       const spt_params* p_in, const int32_t* devices, int32_t n_dev,
                                       float* rgb_out, spt_stats* stats) {
  if (!prims || !cam || !p_in || !devices || !rgb_out)
    return fail(SPT_ERR_INVALID_ARG, "null argument");
  if (n_dev < 1 || n_dev > kMaxRanks) return fail(SPT_ERR_INVALID_ARG, "n_dev must be in [1, 64]");
  for (int i = 0; i < n_dev; ++i)
    for (int j = 0; j < i; ++j)
      if (devices[i] == devices[j]) return fail(SPT_ERR_INVALID_ARG, "duplicate device");
  spt_params base = *p_in;
  base.shard_index = 0;
  base.shard_count = n_dev;
  const size_t image_floats = 3ull * (size_t)base.width * (size_t)base.height;
  const size_t slot = shard_floats(&base, 0);

  struct Rank {
    spt_context* ctx = nullptr;
    hipStream_t stream = nullptr;
    float* shard = nullptr;
    spt_comm comm;
  };
  std::vector<Rank> R((size_t)n_dev);
  std::vector<ncclComm_t> comms((size_t)n_dev, nullptr);
  float* image = nullptr;
  spt_status st = SPT_OK;
  auto cleanup = [&]() {
    for (int k = 0; k < n_dev; ++k) {
      Rank& r = R[(size_t)k];
      (void)hipSetDevice(devices[k]);
      if (r.stream) (void)hipStreamSynchronize(r.stream);
      if (r.shard) (void)hipFree(r.shard);
      if (r.comm.gbuf) (void)hipFree(r.comm.gbuf);
      if (r.stream) (void)hipStreamDestroy(r.stream);
      if (r.ctx) spt_context_destroy(r.ctx);
      if (comms[(size_t)k]) (void)ncclCommDestroy(comms[(size_t)k]);
    }
    if (image) {
      (void)hipSetDevice(devices[0]);
      (void)hipFree(image);
    }
  };
  {
    const ncclResult_t r = ncclCommInitAll(comms.data(), n_dev, devices);
    if (r != ncclSuccess) {
      cleanup();
      return fail(SPT_ERR_RCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    }
  }
  // Every shard renders concurrently, one context and stream per device.
  for (int k = 0; k < n_dev && st == SPT_OK; ++k) {
    Rank& r = R[(size_t)k];
    spt_params q = base;
    q.shard_index = k;
    q.device = devices[k];
    r.comm.comm = comms[(size_t)k];
    r.comm.nranks = n_dev; r.comm.rank = k; r.comm.device = devices[k];
    st = spt_context_create(devices[k], &r.ctx);
    if (st != SPT_OK) break;
    if (hipSetDevice(devices[k]) != hipSuccess || hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&r.shard, std::max<size_t>(1, slot) * sizeof(float)) != hipSuccess) {
      st = fail(SPT_ERR_OOM, "shard buffer/stream");
      break;
    }
    if (k == 0) {
      if (hipMalloc(&image, image_floats * sizeof(float)) != hipSuccess) { st = fail(SPT_ERR_OOM, "image"); break; }
      st = reserve_gbuf(&r.comm, slot);
      if (st != SPT_OK) break;
    }
    if (shard_floats(&q, k) != 0) st = spt_render_async(r.ctx, prims, n_prims, cam, &q, r.shard, r.stream);
  }
  // One grouped gather over all devices of this process, then the de-interleave on device 0.
  if (st == SPT_OK && n_dev > 1) {
    if (ncclGroupStart() != ncclSuccess) st = fail(SPT_ERR_RCCL, "ncclGroupStart");
    for (int k = 0; k < n_dev && st == SPT_OK; ++k) {
      Rank& r = R[(size_t)k];
      spt_params q = base;
      st = post_gather(&r.comm, &q, r.shard, r.stream);
    }
    const ncclResult_t e = ncclGroupEnd();
    if (st == SPT_OK && e != ncclSuccess) st = fail(SPT_ERR_RCCL, std::string("ncclGroupEnd: ") + ncclGetErrorString(e));
  }
  if (st == SPT_OK) {
    (void)hipSetDevice(devices[0]);
    st = deinterleave_on_root(&R[0].comm, &base, R[0].shard, image, R[0].stream);
  }
  spt_stats tot{};
  for (int k = 0; k < n_dev && st == SPT_OK; ++k) {
    spt_params q = base;
    q.shard_index = k;
    if (shard_floats(&q, k) == 0) continue;
    spt_stats s{};
    st = spt_context_stats(R[(size_t)k].ctx, &s);
    tot.samples += s.samples; tot.path_rays += s.path_rays; tot.shadow_rays += s.shadow_rays;
    tot.vertices += s.vertices; tot.nee_events += s.nee_events; tot.nee_light_hits += s.nee_light_hits;
    tot.cosine_samples += s.cosine_samples; tot.misses += s.misses;
    tot.shadow_traced += s.shadow_traced; tot.sphere_vertices += s.sphere_vertices;
    tot.shadow_proven += s.shadow_proven;
    tot.flop += s.flop; tot.flop_executed += s.flop_executed;
    tot.kernel_ms = std::max(tot.kernel_ms, s.kernel_ms);
  }
  if (st == SPT_OK) {
    (void)hipSetDevice(devices[0]);
    if (hipStreamSynchronize(R[0].stream) != hipSuccess ||
        hipMemcpy(rgb_out, image, image_floats * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
      st = fail(SPT_ERR_HIP, "image copy");
  }
  if (st == SPT_OK && stats) *stats = tot;
  for (auto& r : R) r.comm.comm = nullptr;  // destroyed through comms[]
  cleanup();
  return st;
}
