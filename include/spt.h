/*
 * spt.h — C ABI of the MI355X-native smallpt sampling loop (small-pathtracer_amd).
 *
 * Drop-in boundary for the reference's per-pixel sampling loop
 *   /root/reference/src/smallpt.cpp:528-542  (main: row/col/sample loops, r += radiance()/spp, c[i] = clamp(r))
 * whose per-sample kernel is radiance() at :419-496 (live path tracer :444-480).
 * The reference has no plugin/operator/FFI API; its de-facto inputs are globals and locals:
 *   scene  Hitable *rect[NUMBER_OBJ]         :287-311   -> spt_prim[] (tagged flat records)
 *   camera Camera cam(LOOKFROM, ...)         :262-279, :521 -> spt_camera
 *   w, h, samps                              :507-508   -> spt_params.width/height/spp
 *   srand(time) / Xi={0,0,y^3}               :503, :530 -> spt_params.seed (counter-based Philox stream)
 * and its output is Vec *c (w*h RGB, clamped to [0,1], row-major, y=0 = top row) :510, :538,
 * consumed by the PPM writer :548-551 -> rgb_out (float, same layout/clamping).
 *
 * Conventions: extern "C", plain pointers and sizes, no exceptions cross the ABI, every entry
 * point returns an spt_status. Buffers are caller-owned. One spt_context per HIP device; calls on
 * different contexts may run concurrently, calls on one context must be serialised by the caller.
 */
#ifndef SPT_H_
#define SPT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPT_ABI_VERSION 5 /* 2: spt_stats gained shadow_traced, sphere_vertices, flop_executed;
                             3: shadow_proven; 4: spt_gather_plan, spt_deinterleave_source,
                             spt_gather_staging_floats, spt_shutdown; 5: SPT_FLAG_REFERENCE_LEAKS */

typedef enum spt_status {
  SPT_OK = 0,
  SPT_ERR_INVALID_ARG = 1, /* bad sizes, null pointers, unsupported scene/params */
  SPT_ERR_HIP = 2,         /* a HIP runtime call failed (spt_last_error() has the text) */
  SPT_ERR_NO_DEVICE = 3,   /* no usable gfx950 device */
  SPT_ERR_OOM = 4,         /* device allocation failed */
  SPT_ERR_UNSUPPORTED = 5, /* reserved: feature not implemented (not returned today) */
  SPT_ERR_RCCL = 6         /* an RCCL call of the multi-GPU gather failed (spt_last_error()) */
} spt_status;

/* Primitive kinds: the reference's Hitable subclasses (:92-254). */
typedef enum spt_kind {
  SPT_RECT_XY = 0, /* Rectangle_xy(x1,x2,y1,y2,z, e,c,refl)  :137-178, plane z=k  */
  SPT_RECT_XZ = 1, /* Rectangle_xz(x1,x2,z1,z2,y, e,c,refl)  :92-135,  plane y=k  */
  SPT_RECT_YZ = 2, /* Rectangle_yz(y1,y2,z1,z2,x, e,c,refl)  :180-221, plane x=k  */
  SPT_SPHERE = 3   /* Sphere(rad, p, e, c, refl)             :223-254             */
} spt_kind;

/* Refl_t :72-74. Only DIFF is live in the reference (:457); SPEC/REFR are commented out (:481-495). */
typedef enum spt_refl { SPT_DIFF = 0, SPT_SPEC = 1, SPT_REFR = 2 } spt_refl;

/* One scene primitive. geom[] holds the constructor arguments in the reference's order:
 *   RECT_XY: {x1, x2, y1, y2, z}   RECT_XZ: {x1, x2, z1, z2, y}   RECT_YZ: {y1, y2, z1, z2, x}
 *   SPHERE : {rad, px, py, pz, 0}
 * e = emission, c = colour (Vec e, c in the reference). Doubles mirror the reference constructors;
 * the device path rounds them to fp32 once per render. */
typedef struct spt_prim {
  int32_t kind;  /* spt_kind */
  int32_t refl;  /* spt_refl */
  double geom[5];
  double e[3];
  double c[3];
} spt_prim;

/* Camera :256-285 — the four vectors its constructor computes (:267-274). Build with
 * spt_camera_init() for the reference's constructor semantics (float vfov/aspect, tanf). */
typedef struct spt_camera {
  double origin[3];
  double lower_left_corner[3];
  double horizontal[3];
  double vertical[3];
} spt_camera;

/* Light-sample arithmetic of light_sampling() :363-369:  x = 32 + rand()*36/double(RAND_MAX).
 * With glibc (RAND_MAX = 2^31-1) rand()*36 overflows int32 and wraps, so the reference as built
 * on Linux samples x in [31,33], z in [62,64] (measured). GLIBC_WRAP reproduces that arithmetic
 * on a 31-bit draw; UNIFORM is the intended [x0, x0+dx] x [z0, z0+dz] (MinGW RAND_MAX=32767). */
typedef enum spt_light_mode { SPT_LIGHT_GLIBC_WRAP = 0, SPT_LIGHT_UNIFORM = 1 } spt_light_mode;

typedef struct spt_params {
  int32_t width, height, spp; /* :507-508 */
  uint32_t seed;              /* Philox4x32-7 counter word 3 (the key is the fixed SPT_PHILOX_KEY) */
  float nee_prob;             /* Q of :464 (`q < Q`): 1 = HEAD explicit light sampling, 0 = cosine only */
  int32_t rr_depth;           /* Russian roulette starts when ++depth > rr_depth  (:448, HEAD = 5) */
  int32_t max_depth;          /* 0 = unbounded (reference); >0 = path ends at this vertex depth */
  int32_t light_id;           /* primitive index treated as "the light" by NEE (:467, HEAD = 6) */
  float light_x0, light_dx;   /* light sample rect x0 + [0,dx] (:365)   HEAD 32, 36 */
  float light_z0, light_dz;   /* light sample rect z0 + [0,dz] (:366)   HEAD 63, 36 */
  float light_y;              /* sample plane y (:367)                  HEAD 81.6   */
  float light_area;           /* PDF area constant (:471)               HEAD 1296   */
  int32_t light_mode;         /* spt_light_mode */
  /* Row sharding (multi-GPU): tiles of tile_rows image rows, tile t rendered by shard t % shard_count.
   * The output of a shard holds only its rows, compacted in increasing row order (spt_shard_rows). */
  int32_t tile_rows;          /* 0 -> 8 */
  int32_t shard_index, shard_count;
  int32_t chunk;              /* samples per work unit (0 = auto). Never changes results. */
  int32_t device;             /* HIP device ordinal for spt_render() */
  uint32_t flags;             /* SPT_FLAG_* below; other bits must be 0 */
} spt_params;

/* random_scattering() draws from the reference's commented-out UNIFORM hemisphere code (:351-360:
 * dir = u cos(r1) sqrt(r2(2-r2)) + v sin(r1) sqrt(r2(2-r2)) + w (1-r2)) instead of the live
 * cosine-weighted code (:340-347); the estimator weight stays 1, as in the reference. */
#define SPT_FLAG_UNIFORM_SCATTER 1u
/* Leaked paths (a path ray that misses every primitive, :371-377) go on from the miss vertex --
 * the origin, with prim 0's material -- exactly as the reference's do. Without this flag the
 * contract's leak-end rule applies wherever the host can prove it (contract v6: the
 * scene has a closed room, the origin lies outside it, prim 0 does not emit and every emitter lies
 * inside): such a path ends at its first miss, which skips the reference's post-leak vertices (~4 %
 * of them in the HEAD scene) and changes the image's mean by ~8 ppm. */
#define SPT_FLAG_REFERENCE_LEAKS 4u
/* Kernel specialisation cap, flags bits 8-9 (A/B comparisons and tests; never changes a result:
 * every kernel computes the same contract bit for bit). AUTO (0) runs the most specialised kernel
 * the host can prove applicable to the scene and params; the others stop at that level. */
#define SPT_FLAG_KERNEL_LEVEL_MASK 0x300u
#define SPT_FLAG_KERNEL_LEVEL(l) (((uint32_t)(l) & 3u) << 8)
enum { SPT_KERNEL_LEVEL_AUTO = 0, SPT_KERNEL_LEVEL_GENERIC = 1, SPT_KERNEL_LEVEL_CORNELL = 2,
       SPT_KERNEL_LEVEL_CONST = 3 };

/* The counter RNG: Philox4x32 with SPT_PHILOX_ROUNDS rounds (7: the Random123 paper's smallest
 * Crush-resistant count for Philox4x32; its library default is 10), a fixed key (so the key
 * schedule is compile-time) and the counter ctr = (pixel = y*w + x, sample, vertex | stream << 31,
 * seed). */
#define SPT_PHILOX_ROUNDS 7
#define SPT_PHILOX_KEY0 0x53505430u /* "SPT0" */
#define SPT_PHILOX_KEY1 0x53505431u /* "SPT1" */

/* Per-render path statistics (counted in-kernel, summed once per wave). */
typedef struct spt_stats {
  uint64_t samples;        /* pixel-samples finished = camera rays */
  uint64_t path_rays;      /* rays traced through the scene for path vertices (incl. camera rays) */
  uint64_t shadow_rays;    /* NEE shadow rays of the reference: one per NEE event (:466). The kernel
                              traces only `shadow_traced` of them (below); the others cannot reach
                              the light and are rejected exactly by the light's own test */
  uint64_t vertices;       /* path vertices shaded (incl. terminal ones) */
  uint64_t nee_events;     /* NEE light samples taken (:465) */
  uint64_t nee_light_hits; /* ... whose shadow ray hit light_id (:470-472) */
  uint64_t cosine_samples; /* cosine-weighted scatter directions drawn (:337-347) */
  uint64_t misses;         /* path rays that hit nothing (reference: x = origin, id = 0, :373-374) */
  uint64_t shadow_traced;  /* NEE shadow rays that pass the light pre-test: the kernel resolves each
                              of them as the nearest-hit test of :466-467 -- by tracing it, or ... */
  uint64_t sphere_vertices;/* vertices on a sphere (Sphere::normal :246-253) */
  uint64_t shadow_proven;  /* ... of shadow_traced, those the HEAD NEE kernel proved to reach the
                              light without a trace (exact: the trace's result is implied by the
                              geometry; 0 in the other kernels) */
  double flop;             /* algorithmic FLOPs of the reference's work (model in spt_flops.h): every
                              shadow ray of :466 charged as a full scene test */
  double flop_executed;    /* the same model with only the traced shadow rays charged
                              (shadow_traced - shadow_proven) */
  double kernel_ms;        /* device time of the render kernel (HIP events) */
} spt_stats;

/* ---- host helpers mirroring the reference's host-side API ---- */
spt_status spt_default_params(spt_params* p); /* HEAD: w=h=512, spp=16, Q=1, rr 5, light 6, ... */
spt_status spt_camera_init(spt_camera* cam, const double lookfrom[3], const double lookat[3],
                           const double vup[3], float vfov_deg, float aspect); /* :262-275 */
/* rect[] :287-311 (17 primitives). *n_out = 17; fails if cap < 17. */
spt_status spt_scene_cornell(spt_prim* out, int32_t cap, int32_t* n_out);
/* The build-defined 32-sphere scene of config 5: room rects 0-6 of :288-294 + 32 DIFF spheres. */
spt_status spt_scene_spheres32(spt_prim* out, int32_t cap, int32_t* n_out);
/* The room and light of :288-294 plus smallpt's mirror (SPEC) and glass (REFR) balls at the places
 * of the spheres commented out at :296-297; shading = the commented-out code :481-495. 9 prims. */
spt_status spt_scene_cornell_specular(spt_prim* out, int32_t cap, int32_t* n_out);
/* The classic smallpt sphere box of the reference's older revision (the constants mined from the
 * shipped src/a.exe; its renders are the repository's image*.ppm): walls are
 * spheres of radius 1e5 (left x = 1e5+1 green, right x = -1e5+99 red, back, front (black), floor,
 * ceiling y = -1e5+81.6), two matte white (DIFF, .999) balls of radius 16.5 at (27,16.5,47) /
 * (73,16.5,78), and the light, a sphere of radius 600 at (50, 681.33, 81.6) with emission 12
 * (prim 8). 9 prims. Spheres of radius >= SPT_WIDE_SPHERE_RADIUS are intersected in fp64: an fp32
 * quadratic cannot hold a 1e5 wall to the scene's scale, and for the radius-600 light, whose cap
 * dips only 0.27 below the ceiling, r^2 - |q|^2 has an fp32 rounding step of ~0.03 (measured:
 * concentric rings and a washed-out ceiling around the cap). NEE (nee_prob > 0) samples the light
 * RECTANGLE of spt_params, which this scene does not have: render it with nee_prob = 0. */
spt_status spt_scene_smallpt_classic(spt_prim* out, int32_t cap, int32_t* n_out);
/* The same box with smallpt's original materials: the left ball a mirror (SPEC), the right one
 * glass (REFR; shading = the commented-out code :481-495). 9 prims. */
spt_status spt_scene_smallpt_mirror_glass(spt_prim* out, int32_t cap, int32_t* n_out);
#define SPT_WIDE_SPHERE_RADIUS 100.0 /* larger than the scenes' rooms (~100 units across) */
/* Rows rendered by this shard (params tile_rows/shard_index/shard_count), ascending. Returns count. */
int32_t spt_shard_rows(const spt_params* p, int32_t* rows_out, int32_t cap);

/* ---- rendering ---- */
/* One-shot drop-in for :528-542. rgb_out: caller-owned HOST buffer of shard_rows*w*3 floats
 * (linear, clamped to [0,1] per channel after the spp average, :538). stats may be NULL.
 * The library keeps one render context and device output buffer per device (params.device) between
 * calls, so repeated calls pay no context creation, allocation or cold launch; calls on one device
 * are serialised, calls on different devices may run concurrently. Thread-safe. */
spt_status spt_render(const spt_prim* prims, int32_t n_prims, const spt_camera* cam,
                      const spt_params* p, float* rgb_out, spt_stats* stats);
/* Releases spt_render's cached per-device contexts and buffers (the next spt_render re-creates
 * them). Call before unloading the library if its device memory must be returned earlier than
 * process exit. */
spt_status spt_shutdown(void);

typedef struct spt_context spt_context;
spt_status spt_context_create(int32_t device, spt_context** out);
spt_status spt_context_destroy(spt_context* ctx);
/* Enqueue a render on `stream` (a hipStream_t, NULL = default stream). rgb_dev: DEVICE buffer of
 * shard_rows*w*3 floats. No allocation once the context is large enough (spt_context_reserve) and
 * no host synchronisation, except that a second call before spt_context_stats() first waits for
 * the previous call's scene upload (the pinned staging buffers are reused). */
spt_status spt_context_reserve(spt_context* ctx, int32_t n_prims, const spt_params* p);
spt_status spt_render_async(spt_context* ctx, const spt_prim* prims, int32_t n_prims,
                            const spt_camera* cam, const spt_params* p, float* rgb_dev,
                            void* stream);
/* Synchronises the context's last render and returns its stats (SPT_ERR_INVALID_ARG before the
 * context's first render).
 * A render that hit the kernel's runaway-iteration guard returns SPT_ERR_HIP here and leaves its
 * rgb_dev all NaN (never a partial image). */
spt_status spt_context_stats(spt_context* ctx, spt_stats* out);

/* ---- multi-GPU: row-tile shards and ONE framebuffer gather over RCCL ----
 * The reference's only parallel construct is the OpenMP pragma over its row loop (:526-528). Here
 * rows are sharded in tiles of tile_rows across ranks (tile t -> rank t % n, spt_shard_rows);
 * every rank renders its rows with spt_render_async into a compact buffer, and rank 0 receives
 * all of them in one grouped ncclSend/ncclRecv over xGMI and de-interleaves the tiles into the
 * image (h*w*3 floats). The image is bit-identical for any rank count. */
#define SPT_COMM_ID_BYTES 128
typedef struct spt_comm spt_comm;
/* One process per GPU: rank 0 creates the id and the caller hands it to every rank (any channel). */
spt_status spt_comm_unique_id(uint8_t id[SPT_COMM_ID_BYTES]);
spt_status spt_comm_create(const uint8_t id[SPT_COMM_ID_BYTES], int32_t nranks, int32_t rank,
                           int32_t device, spt_comm** out);
spt_status spt_comm_destroy(spt_comm* comm);
/* Allocate rank 0's receive slots for renders of this size ahead of a timed loop (optional). */
spt_status spt_comm_reserve(spt_comm* comm, const spt_params* p);
/* The gather, enqueued on `stream` after this rank's render: shard_dev = the rank's compact rows
 * (spt_render_async's output for p with shard_index = rank), image_dev = the full image on rank 0
 * (ignored elsewhere). p->shard_count must equal nranks. No host synchronisation. */
spt_status spt_gather_framebuffer(spt_comm* comm, const spt_params* p, const float* shard_dev,
                                  float* image_dev, void* stream);
/* The de-interleave alone (rank 0's last step): shards_dev[k] = shard k's compact rows (device
 * pointers on the current device), image_dev = h*w*3 floats. */
spt_status spt_deinterleave_rows(const spt_params* p, int32_t nranks, const float* const* shards_dev,
                                 float* image_dev, void* stream);
/* The gather as pure host functions (no device, no RCCL; spt_gather_framebuffer executes exactly
 * this plan): the transfers `rank` posts inside the gather's ncclGroupStart/End. Rank k > 0 sends
 * its compact shard (count = its rows * w * 3 floats) to rank 0; rank 0 receives each rank k > 0
 * that owns rows into its staging buffer at offset (k - 1) * (shard 0's floats) -- shard 0 never
 * owns fewer rows than another shard. Returns the number of ops (<= cap), or -1 on bad arguments
 * or a too small cap. */
typedef struct spt_gather_op {
  int32_t kind;    /* SPT_GATHER_SEND or SPT_GATHER_RECV */
  int32_t peer;    /* the other rank */
  uint64_t count;  /* floats */
  uint64_t offset; /* RECV: float offset into rank 0's staging buffer; SEND: 0 */
} spt_gather_op;
enum { SPT_GATHER_SEND = 0, SPT_GATHER_RECV = 1 };
int32_t spt_gather_plan(const spt_params* p, int32_t nranks, int32_t rank, spt_gather_op* ops,
                        int32_t cap);
uint64_t spt_gather_staging_floats(const spt_params* p, int32_t nranks); /* rank 0's staging size */
/* Where rank 0's de-interleave reads image row `row`: shard *rank's compact row *compact_row (the
 * device kernel's own row map). */
spt_status spt_deinterleave_source(const spt_params* p, int32_t nranks, int32_t row, int32_t* rank,
                                   int32_t* compact_row);
/* One process driving n_dev GPUs (smallpt_amd --devices N): shard k renders on devices[k]
 * (distinct), the gather lands on devices[0], rgb_out = the full image on the host (h*w*3 floats).
 * p's shard fields are ignored. stats: summed over devices, kernel_ms = the slowest device's. */
spt_status spt_render_multi(const spt_prim* prims, int32_t n_prims, const spt_camera* cam,
                            const spt_params* p, const int32_t* devices, int32_t n_dev,
                            float* rgb_out, spt_stats* stats);

/* ---- image output (:313-321 toInt/clamp, :548-551 the P3 writer) ----
 * The encoder turns a DEVICE framebuffer (h*w*3 floats, row-major, y=0 top: what spt_render_async
 * writes) into file bytes on the GPU. P3 is byte-identical to the reference's fprintf loop
 * ("P3\n%d %d\n%d\n" then "%d %d %d " per pixel, toInt = int(pow(clamp(x), 1/2.2)*255 + .5) in
 * double); P6 is its binary form; PFM is the linear framebuffer ("PF", scale -1 = little endian,
 * scanlines bottom to top, header padded so the floats are dword-aligned). */
typedef enum spt_image_format { SPT_IMAGE_P3 = 0, SPT_IMAGE_P6 = 1, SPT_IMAGE_PFM = 2 } spt_image_format;
typedef struct spt_encoder spt_encoder;
uint64_t spt_image_bound(int32_t w, int32_t h, int32_t format); /* max encoded bytes (0 if invalid) */
spt_status spt_encoder_create(int32_t device, spt_encoder** out);
spt_status spt_encoder_destroy(spt_encoder* enc);
/* Encode on `stream` into out_dev (cap bytes). *len_out = encoded length. P3's length depends on
 * the data, so P3 synchronises `stream` once (after its passes); P6/PFM do not. rgb_dev must be
 * 16-byte aligned (SPT_ERR_INVALID_ARG otherwise; P6/PFM also need out_dev past the header 16-byte
 * aligned) and 3*w*h <= 2^32 - 8192; a call rejected for its arguments queues nothing and leaves
 * out_dev untouched. One encoder runs one encode at a time (its scratch is reused). */
spt_status spt_encode_image(spt_encoder* enc, const float* rgb_dev, int32_t w, int32_t h,
                            int32_t format, uint8_t* out_dev, uint64_t cap, uint64_t* len_out,
                            void* stream);
/* Encode (rgb: host or device pointer) and write the file. Replaces the writer of :548-551. */
spt_status spt_write_image(int32_t device, const float* rgb, int32_t w, int32_t h, int32_t format,
                           const char* path);

/* ---- introspection ---- */
int32_t spt_abi_version(void);
/* sha256[:16] of the kernel sources this library was built from (the Makefile's HASHED list; equals
 * the Python package's kernel_sources_sha16() over an unchanged tree). */
const char* spt_build_sources_sha16(void);
const char* spt_status_string(spt_status s);
const char* spt_last_error(void); /* thread-local text of the last failure */
int32_t spt_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* SPT_H_ */
