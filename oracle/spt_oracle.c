#define _GNU_SOURCE /* sincos() */
/*
 * spt_oracle.c — CPU ORACLE for the smallpt per-pixel sampling loop.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product links, calls or ships this file: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it, as the checker.
 *
 * Two restatements of /root/reference/src/smallpt.cpp (HEAD with the dead Q-learning return
 * :424-442 removed — SURVEY.md §8c):
 *
 *  1. COMPAT mode (spt_oracle_compat_render): fp64, the reference's own arithmetic and RNG streams —
 *     erand48 per image row seeded {0,0,(ushort)y^3} (:530, utilities.h:26-51) and glibc TYPE_3
 *     rand() seeded by srand(seed) just before the pixel loop (:503, :533-534, :365-366, :460).
 *     Built with -ffp-contract=off it reproduces the patched reference's PPM md5s bit for bit
 *     (pinned against oracle/_ref in tests/test_oracle_golden.py and tests/golden/).
 *
 *  2. COUNTER mode (spt_oracle_counter_render): the device path's contract — the same algorithm in
 *     fp32 with a counter-based Philox4x32-7 stream (fixed key; counter = pixel, sample,
 *     vertex | stream << 31, seed),
 *     an iterative bounce loop and fixed-point per-pixel accumulation. Every float operation is
 *     spelled out (explicit fmaf, correctly rounded div/sqrt, own sincos polynomial) so that the HIP
 *     kernel must reproduce it BIT-EXACTLY. See DESIGN.md "Counter-mode contract".
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/spt.h"
#include "../include/spt_flops.h"

/* ========================================================================================== */
/* COMPAT MODE (fp64)                                                                          */
/* ========================================================================================== */

typedef struct { double x, y, z; } dv; /* Vec :24-62 */

static inline dv dv3(double x, double y, double z) { dv r = {x, y, z}; return r; }
static inline dv dadd(dv a, dv b) { return dv3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline dv dsub(dv a, dv b) { return dv3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline dv dmul(dv a, double b) { return dv3(a.x * b, a.y * b, a.z * b); }
static inline dv dmulv(dv a, dv b) { return dv3(a.x * b.x, a.y * b.y, a.z * b.z); } /* mult :47 */
static inline double ddot(dv a, dv b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* :53 */
static inline dv dcross(dv a, dv b) { /* operator% :56-58 */
  return dv3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline dv dnorm(dv a) { return dmul(a, 1 / sqrt(a.x * a.x + a.y * a.y + a.z * a.z)); } /* :50 */

/* erand48 of utilities.h:26-51: x <- 0x5DEECE66D*x + 0xB mod 2^48, value x/2^48. */
static double o_erand48(unsigned short xs[3]) {
  uint64_t x = (uint64_t)xs[0] | ((uint64_t)xs[1] << 16) | ((uint64_t)xs[2] << 32);
  x = (x * 0x5DEECE66Dull + 0xBull) & 0xFFFFFFFFFFFFull;
  xs[0] = (unsigned short)x;
  xs[1] = (unsigned short)(x >> 16);
  xs[2] = (unsigned short)(x >> 32);
  return ldexp((double)xs[0], -48) + ldexp((double)xs[1], -32) + ldexp((double)xs[2], -16);
}

/* glibc random_r TYPE_3 (x^31 + x^3 + 1 additive feedback), i.e. what srand()/rand() compute.
 * Restated from the published algorithm (glibc stdlib/random_r.c, srandom_r + random_r). */
typedef struct { int32_t r[34]; int i; } o_glibc_rand;
static void o_srand(o_glibc_rand* g, unsigned seed) {
  int32_t r[344 + 34];
  int k;
  if (seed == 0) seed = 1;
  r[0] = (int32_t)seed;
  for (k = 1; k < 31; k++) {
    const int32_t hi = r[k - 1] / 127773, lo = r[k - 1] % 127773;
    int32_t word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    r[k] = word;
  }
  for (k = 31; k < 34; k++) r[k] = r[k - 31];
  for (k = 34; k < 344; k++) r[k] = (int32_t)((uint32_t)r[k - 31] + (uint32_t)r[k - 3]);
  for (k = 0; k < 34; k++) g->r[k] = r[310 + k]; /* last 34 values r[310..343] */
  g->i = 0;                                      /* ring index of r[310] */
}
static int32_t o_rand(o_glibc_rand* g) {
  /* r[n] = r[n-31] + r[n-3]; ring of the last 34 values, g->i points at r[n-34]. */
  const int i = g->i;
  const uint32_t v = (uint32_t)g->r[(i + 3) % 34] + (uint32_t)g->r[(i + 31) % 34];
  g->r[i] = (int32_t)v;
  g->i = (i + 1) % 34;
  return (int32_t)(v >> 1);
}
#define O_RAND_MAX 2147483647

typedef struct { int kind; double g[5]; dv e, c; } o_prim;

/* Rectangle_*::intersect :102-112, :145-155, :188-198 and Sphere::intersect :229-239. */
static double o_prim_intersect(const o_prim* P, dv o, dv d) {
  double t;
  float a, b;
  switch (P->kind) {
    case SPT_RECT_XZ: /* (x1,x2,z1,z2,y) */
      t = (P->g[4] - o.y) / d.y;
      a = (float)(o.x + d.x * t);
      b = (float)(o.z + d.z * t);
      if (a < P->g[0] || a > P->g[1] || b < P->g[2] || b > P->g[3] || t < 0) return 0;
      return t;
    case SPT_RECT_XY: /* (x1,x2,y1,y2,z) */
      t = (P->g[4] - o.z) / d.z;
      a = (float)(o.x + d.x * t);
      b = (float)(o.y + d.y * t);
      if (a < P->g[0] || a > P->g[1] || b < P->g[2] || b > P->g[3] || t < 0) return 0;
      return t;
    case SPT_RECT_YZ: /* (y1,y2,z1,z2,x) */
      t = (P->g[4] - o.x) / d.x;
      a = (float)(o.y + d.y * t);
      b = (float)(o.z + d.z * t);
      if (a < P->g[0] || a > P->g[1] || b < P->g[2] || b > P->g[3] || t < 0) return 0;
      return t;
    default: { /* SPHERE (rad, px, py, pz) */
      const dv op = dsub(dv3(P->g[1], P->g[2], P->g[3]), o);
      const double eps = 1e-4, bb = ddot(op, d);
      double det = bb * bb - ddot(op, op) + P->g[0] * P->g[0];
      if (det < 0) return 0;
      det = sqrt(det);
      return (t = bb - det) > eps ? t : ((t = bb + det) > eps ? t : 0);
    }
  }
}

typedef struct {
  const o_prim* prims;
  int n;
  int light_id;
  double qthr; /* the NEE-mix threshold of :464: `q < 1` (HEAD), `q < 0` (cosine-only), or any
                  other value (`q < 0.5`: oracle/build_ref.sh smallpt_q05) */
  int max_depth; /* 0: none (HEAD); D > 0: `if (depth + 1 >= D) return hit.e;` before :448
                    (oracle/build_ref.sh smallpt_sph16) */
  int uniform; /* random_scattering: 0 = cosine code :340-347, 1 = uniform code :352-359 */
  o_glibc_rand* g;
  uint64_t vertices, misses; /* radiance() calls and their misses (fidelity statistics) */
  uint64_t first_misses, vertices_pre; /* per sample: the first miss; vertices up to and with it */
  int leaked;                          /* the current sample's path has missed */
} o_scene;

/* intersect :323-335: strict `<` keeps the lowest index on ties; id untouched on a miss. */
static int o_intersect(const o_scene* S, dv o, dv d, double* t, int* id) {
  const double inf = *t = 1e20;
  int i;
  for (i = 0; i < S->n; i++) {
    const double dd = o_prim_intersect(&S->prims[i], o, d);
    if (dd != 0 && dd < *t) { *t = dd; *id = i; }
  }
  return *t < inf;
}

/* Hitable::normal :118-124 etc: geometric normal oriented against the ray. */
static dv o_normal(const o_prim* P, dv d, dv x) {
  dv n;
  switch (P->kind) {
    case SPT_RECT_XZ: n = dv3(0, 1, 0); break;
    case SPT_RECT_XY: n = dv3(0, 0, 1); break;
    case SPT_RECT_YZ: n = dv3(1, 0, 0); break;
    default: n = dnorm(dsub(x, dv3(P->g[1], P->g[2], P->g[3]))); break;
  }
  return ddot(n, d) < 0 ? n : dmul(n, (double)-1); /* n * -1 : Vec::operator*(int) */
}

/* random_scattering :337-361: cosine-weighted (live, :340-347) or the commented-out uniform
   hemisphere (:352-359, `uniform`). */
static dv o_random_scattering(dv nl, unsigned short* Xi, int uniform) {
  const double r1 = 2 * M_PI * o_erand48(Xi);
  const double r2 = o_erand48(Xi);
  const dv w = nl;
  const dv u = dnorm(dcross(fabs(w.x) > .1 ? dv3(0, 1, 0) : dv3(1, 0, 0), w));
  const dv v = dcross(w, u);
  /* libm calls as the reference binary makes them (objdump of oracle/_ref): g++ -O3 turns the
     cosine body's cos(r1)/sin(r1) into one glibc sincos() call, but keeps separate sin()/cos()
     calls in the uniform body; glibc's sincos and sin/cos differ in the last bit for some r1. */
  if (uniform) {
    double (*volatile cos_f)(double) = cos, (*volatile sin_f)(double) = sin;
    return dnorm(dadd(dadd(dmul(dmul(u, cos_f(r1)), sqrt(r2 * (2 - r2))),
                           dmul(dmul(v, sin_f(r1)), sqrt(r2 * (2 - r2)))),
                      dmul(w, 1 - r2)));
  }
  {
    const double r2s = sqrt(r2);
    double sr1, cr1;
    sincos(r1, &sr1, &cr1);
    return dnorm(dadd(dadd(dmul(dmul(u, cr1), r2s), dmul(dmul(v, sr1), r2s)),
                      dmul(w, sqrt(1 - r2))));
  }
}

/* light_sampling :363-369. rand()*36 is int arithmetic (wraps with glibc RAND_MAX=2^31-1). */
static dv o_light_sampling(const o_scene* S, dv hit) {
  const int32_t ax = (int32_t)((uint32_t)o_rand(S->g) * 36u);
  const double x_light = 32 + ax / (double)O_RAND_MAX;
  const int32_t az = (int32_t)((uint32_t)o_rand(S->g) * 36u);
  const double z_light = 63 + az / (double)O_RAND_MAX;
  return dsub(dv3(x_light, 81.6, z_light), hit);
}

/* radiance :419-480 (live path), recursive exactly as the reference (evaluation order matters). */
static dv o_radiance(const o_scene* S, dv ro, dv rd, int depth, unsigned short* Xi) {
  int id = 0;
  double t;
  dv x;
  ((o_scene*)S)->vertices++;
  if (!S->leaked) ((o_scene*)S)->vertices_pre++;
  if (!o_intersect(S, ro, rd, &t, &id)) { /* :371-377 */
    x = dv3(0, 0, 0);
    ((o_scene*)S)->misses++;
    if (!S->leaked) { ((o_scene*)S)->first_misses++; ((o_scene*)S)->leaked = 1; }
  }
  else x = dadd(ro, dmul(rd, t));
  {
    const o_prim* obj = &S->prims[id];
    const dv nl = o_normal(obj, rd, x);
    dv f = obj->c;
    const double p = f.x > f.y && f.x > f.z ? f.x : f.y > f.z ? f.y : f.z;
    dv d;
    double q, PDF_inverse = 1, BRDF = 1;
    if (S->max_depth > 0 && depth + 1 >= S->max_depth) return obj->e;
    if (++depth > 5 || !p) {
      if (o_erand48(Xi) < p) f = dmul(f, 1 / p);
      else return obj->e;
    }
    q = o_rand(S->g) / (double)O_RAND_MAX;
    if (q < S->qthr) {
      d = o_light_sampling(S, x);
      d = dnorm(d);
      o_intersect(S, x, d, &t, &id);
      if (id != S->light_id) {
        d = o_random_scattering(nl, Xi, S->uniform);
        d = dnorm(d);
        o_intersect(S, x, d, &t, &id);
      } else {
        d = dnorm(d);
        PDF_inverse = fabs((1296 * ddot(d, dv3(0, 1, 0))) / (t * t));
        d = dnorm(d);
        BRDF = fabs(ddot(d, nl) / M_PI);
      }
    } else {
      d = o_random_scattering(nl, Xi, S->uniform);
      d = dnorm(d);
      o_intersect(S, x, d, &t, &id);
    }
    d = dnorm(d);
    {
      const dv Li = o_radiance(S, x, d, depth, Xi);
      return dadd(obj->e, dmul(dmul(dmulv(f, Li), PDF_inverse), BRDF));
    }
  }
}

static o_prim o_from_spt(const spt_prim* s) {
  o_prim p;
  p.kind = s->kind;
  memcpy(p.g, s->geom, sizeof p.g);
  p.e = dv3(s->e[0], s->e[1], s->e[2]);
  p.c = dv3(s->c[0], s->c[1], s->c[2]);
  return p;
}

/* Camera ctor :262-275 (theta/half_height float, tan(float) resolves to tanf under libstdc++). */
void spt_oracle_camera(double out[12], const double lf[3], const double la[3], const double vup[3],
                       float vfov, float aspect) {
  const float theta = (float)(vfov * M_PI / 180);
  const float half_height = tanf(theta / 2);
  const float half_width = aspect * half_height;
  const dv origin = dv3(lf[0], lf[1], lf[2]);
  const dv w = dnorm(dsub(dv3(la[0], la[1], la[2]), origin));
  const dv u = dnorm(dcross(w, dv3(vup[0], vup[1], vup[2])));
  const dv v = dcross(u, w);
  const dv llc = dadd(dsub(dsub(origin, dmul(u, (double)half_width)), dmul(v, (double)half_height)), w);
  const dv hor = dmul(u, (double)(half_width * 2));
  const dv ver = dmul(v, (double)(half_height * 2));
  const double vals[12] = {origin.x, origin.y, origin.z, llc.x, llc.y, llc.z,
                           hor.x,    hor.y,    hor.z,    ver.x, ver.y, ver.z};
  memcpy(out, vals, sizeof vals);
}

/* main() :502-542 with the HEAD scene, srand(seed) and the state-space build skipped.
 * flags: bit 1 = uniform random_scattering (:352-359); bit 2 = row streams {0, seed, y^3}
 * instead of :530's {0, 0, y^3} (oracle/build_ref.sh *_xs): without it every seed repeats the
 * same scattering/RR draws and only rand() varies, so seed-to-seed differences understate the
 * estimator's noise. qthr: the threshold of :464 (1 = HEAD NEE, 0 = cosine-only). max_depth: 0
 * or the depth cap D of the capped builds. c_out: w*h*3 doubles (clamped, row-major, y=0 top).
 * stats (may be NULL): {vertices, misses, first misses, vertices up to the first miss} over all
 * radiance() calls (4 words). Returns 0. */
int spt_oracle_compat_render_ex(const spt_prim* prims, int n, int w, int h, int spp, unsigned seed,
                                int flags, double qthr, int max_depth, double* c_out,
                                uint64_t* stats) {
  o_prim* P = (o_prim*)malloc(sizeof(o_prim) * (size_t)n);
  o_glibc_rand g;
  o_scene S;
  double cam[12];
  const double lf[3] = {50, 40, 168}, la[3] = {50, 40, 5}, up[3] = {0, 1, 0};
  int i, y;
  dv origin, llc, hor, ver;
  for (i = 0; i < n; i++) P[i] = o_from_spt(&prims[i]);
  S.prims = P; S.n = n; S.light_id = 6; S.qthr = qthr; S.max_depth = max_depth;
  S.uniform = (flags >> 1) & 1; S.g = &g;
  S.vertices = S.misses = S.first_misses = S.vertices_pre = 0;
  S.leaked = 0;
  o_srand(&g, seed);
  spt_oracle_camera(cam, lf, la, up, 65, (float)w / (float)h);
  origin = dv3(cam[0], cam[1], cam[2]);
  llc = dv3(cam[3], cam[4], cam[5]);
  hor = dv3(cam[6], cam[7], cam[8]);
  ver = dv3(cam[9], cam[10], cam[11]);
  for (y = 0, i = 0; y < h; y++) {
    unsigned short x, Xi[3];
    Xi[0] = 0; Xi[1] = (flags & 4) ? (unsigned short)seed : 0; Xi[2] = (unsigned short)(y * y * y);
    for (x = 0; x < w; x++) {
      dv r = dv3(0, 0, 0);
      int s;
      for (s = 0; s < spp; s++) {
        const float u = (float)(x - 0.5 + o_rand(&g) / (double)O_RAND_MAX) / (float)w;
        const float v = (float)((h - y - 1) - 0.5 + o_rand(&g) / (double)O_RAND_MAX) / (float)h;
        const dv d = dsub(dadd(dadd(llc, dmul(hor, (double)u)), dmul(ver, (double)v)), origin);
        dv L;
        S.leaked = 0;
        L = o_radiance(&S, origin, dnorm(d), 0, Xi);
        r = dadd(r, dmul(L, 1. / spp));
      }
      c_out[3 * i + 0] = r.x < 0 ? 0 : r.x > 1 ? 1 : r.x;
      c_out[3 * i + 1] = r.y < 0 ? 0 : r.y > 1 ? 1 : r.y;
      c_out[3 * i + 2] = r.z < 0 ? 0 : r.z > 1 ? 1 : r.z;
      i++;
    }
  }
  if (stats) { stats[0] = S.vertices; stats[1] = S.misses; stats[2] = S.first_misses; stats[3] = S.vertices_pre; }
  free(P);
  return 0;
}
/* nee: bit 0 = `q < 1` (HEAD) vs `q < 0`; bits 1, 2 as the flags above. */
int spt_oracle_compat_render_stats(const spt_prim* prims, int n, int w, int h, int spp,
                                   unsigned seed, int nee, double* c_out, uint64_t* stats) {
  return spt_oracle_compat_render_ex(prims, n, w, h, spp, seed, nee, (nee & 1) ? 1.0 : 0.0, 0,
                                     c_out, stats);
}
int spt_oracle_compat_render(const spt_prim* prims, int n, int w, int h, int spp, unsigned seed,
                             int nee, double* c_out) {
  return spt_oracle_compat_render_stats(prims, n, w, h, spp, seed, nee, c_out, NULL);
}

/* toInt :319-321 + the P3 writer :548-551 (byte-identical format). */
static int o_toInt(double x) { return (int)(pow(x < 0 ? 0 : x > 1 ? 1 : x, 1 / 2.2) * 255 + .5); }
int spt_oracle_write_ppm_d(const char* path, int w, int h, const double* c) {
  FILE* f = fopen(path, "w");
  int i;
  if (!f) return 1;
  fprintf(f, "P3\n%d %d\n%d\n", w, h, 255);
  for (i = 0; i < w * h; i++)
    fprintf(f, "%d %d %d ", o_toInt(c[3 * i]), o_toInt(c[3 * i + 1]), o_toInt(c[3 * i + 2]));
  fclose(f);
  return 0;
}
int spt_oracle_write_ppm_f(const char* path, int w, int h, const float* c) {
  FILE* f = fopen(path, "w");
  int i;
  if (!f) return 1;
  fprintf(f, "P3\n%d %d\n%d\n", w, h, 255);
  for (i = 0; i < w * h; i++)
    fprintf(f, "%d %d %d ", o_toInt(c[3 * i]), o_toInt(c[3 * i + 1]), o_toInt(c[3 * i + 2]));
  fclose(f);
  return 0;
}

/* The same files in memory (test checker for the GPU encoder, spt_image.hip): format 0 = P3 exactly
   as :549-551, 1 = P6 (bytes of toInt; header padded with spaces to 16 bytes), 2 = PFM
   (little-endian floats, bottom-to-top scanlines, scale "-1.0" padded with zeros so the data
   starts 16-byte aligned). Returns the length, or
   the needed length if cap is too small (nothing written then). */
size_t spt_oracle_encode_image(const float* c, int w, int h, int format, unsigned char* out,
                               size_t cap) {
  char hd[96];
  size_t n = 0, i;
  const size_t np = (size_t)w * (size_t)h;
  if (format == 0) {
    size_t need = (size_t)snprintf(hd, sizeof hd, "P3\n%d %d\n%d\n", w, h, 255);
    char buf[48];
    for (i = 0; i < np; i++)
      need += (size_t)snprintf(buf, sizeof buf, "%d %d %d ", o_toInt(c[3 * i]), o_toInt(c[3 * i + 1]),
                               o_toInt(c[3 * i + 2]));
    if (need > cap) return need;
    n = (size_t)snprintf(hd, sizeof hd, "P3\n%d %d\n%d\n", w, h, 255);
    memcpy(out, hd, n);
    for (i = 0; i < np; i++) {
      const int k = snprintf(buf, sizeof buf, "%d %d %d ", o_toInt(c[3 * i]), o_toInt(c[3 * i + 1]),
                             o_toInt(c[3 * i + 2]));
      memcpy(out + n, buf, (size_t)k);
      n += (size_t)k;
    }
    return n;
  }
  if (format == 1) {
    n = (size_t)snprintf(hd, sizeof hd, "P6\n%d %d", w, h);
    while ((n + 5) % 16) hd[n++] = ' ';  /* header padded to 16 bytes (legal PPM whitespace) */
    memcpy(hd + n, "\n255\n", 5);
    n += 5;
    if (n + 3 * np > cap) return n + 3 * np;
    memcpy(out, hd, n);
    for (i = 0; i < 3 * np; i++) out[n + i] = (unsigned char)o_toInt(c[i]);
    return n + 3 * np;
  }
  {
    int y;
    n = (size_t)snprintf(hd, sizeof hd, "PF\n%d %d\n-1.0", w, h);
    while ((n + 1) % 16) hd[n++] = '0';
    hd[n++] = '\n';
    if (n + 12 * np > cap) return n + 12 * np;
    memcpy(out, hd, n);
    for (y = 0; y < h; y++)
      memcpy(out + n + (size_t)(h - 1 - y) * (size_t)w * 12, c + (size_t)y * (size_t)w * 3,
             (size_t)w * 12);
    return n + 12 * np;
  }
}

/* Exposed for known-answer tests. */
double spt_oracle_erand48(unsigned short xs[3]) { return o_erand48(xs); }
void spt_oracle_glibc_rand(unsigned seed, int n, int32_t* out) {
  o_glibc_rand g;
  int i;
  o_srand(&g, seed);
  for (i = 0; i < n; i++) out[i] = o_rand(&g);
}
double spt_oracle_prim_intersect(const spt_prim* s, const double o[3], const double d[3]) {
  const o_prim p = o_from_spt(s);
  return o_prim_intersect(&p, dv3(o[0], o[1], o[2]), dv3(d[0], d[1], d[2]));
}

/* ========================================================================================== */
/* COUNTER MODE (fp32) — the device contract                                                   */
/* ========================================================================================== */

/* Philox4x32-R (Salmon et al., SC'11; Random123 constants): R = 10 for the KATs, SPT_PHILOX_ROUNDS = 7 in the contract. */
#define PH_M0 0xD2511F53u
#define PH_M1 0xCD9E8D57u
#define PH_W0 0x9E3779B9u
#define PH_W1 0xBB67AE85u
/* Philox4x32 with R rounds (Salmon et al. SC'11, the Random123 round function). R = 10 is
 * Random123's default (checked against its known-answer vectors); the counter-mode contract uses
 * R = SPT_PHILOX_ROUNDS = 7, the paper's smallest Crush-resistant round count for Philox4x32
 * (round 3: three rounds fewer per vertex are 18 VALU issue slots, -3.5 % kernel time at C3). */
void spt_oracle_philox_r(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4],
                         int rounds) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  int r;
  for (r = 0; r < rounds; r++) {
    const uint64_t p0 = (uint64_t)PH_M0 * c0, p1 = (uint64_t)PH_M1 * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += PH_W0;
    k1 += PH_W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
void spt_oracle_philox(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  spt_oracle_philox_r(ctr_in, key_in, out, 10);
}
/* The contract's generator (c_path): Philox4x32-SPT_PHILOX_ROUNDS. */
static void c_philox(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  spt_oracle_philox_r(ctr_in, key_in, out, SPT_PHILOX_ROUNDS);
}

typedef struct { float x, y, z; } fv;
static inline fv fv3(float x, float y, float z) { fv r = {x, y, z}; return r; }
static inline uint32_t u16i(uint32_t lo, uint32_t hi) { return (lo & 0xFFu) | ((hi & 0xFFu) << 8); }
static inline float u16(uint32_t lo, uint32_t hi) { return (float)u16i(lo, hi) * 0x1p-16f; }
static inline float fdot(fv a, fv b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
/* Deterministic reciprocal / rsqrt of the contract: integer seed + 3 Newton steps (only IEEE
 * fma/mul and integer ops, so every platform computes the same bits). */
static inline float asf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t asu(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
/* Contract v5: a uniform [0, 1) float from the top 23 bits of a Philox word, built as the float
 * 1 + m * 2^-23 (bits 0x3F800000 | m) minus 1 -- exact; on the GPU an or and a subtract instead of a
 * shift, a half-rate conversion and a multiply (rounds 1-4: (v >> 8) * 2^-24). */
static inline float u01(uint32_t v) { return asf(0x3F800000u | (v >> 9)) - 1.0f; }
float spt_oracle_rcp_nr(float x) {
  float y = asf(0x7EF311C3u - asu(x));
  int i;
  for (i = 0; i < 3; i++) {
    const float e = fmaf(-x, y, 1.0f);
    y = fmaf(e, y, y);
  }
  return y;
}
float spt_oracle_rsq_nr(float x) {
  float y = asf(0x5F375A86u - (asu(x) >> 1));
  const float h = 0.5f * x;
  int i;
  for (i = 0; i < 3; i++) {
    const float hy = h * y;
    y = y * fmaf(-hy, y, 1.5f);
  }
  return y;
}
/* The same reciprocal square root with two Newton steps (relative error < 5e-6): the sphere root
 * (c_sphere) and the free-scale cosine sample's R (rounds 1-4 also its normalize, now
 * spt_oracle_rsq_nr1). */
float spt_oracle_rsq_nr2(float x) {
  float y = asf(0x5F375A86u - (asu(x) >> 1));
  const float h = 0.5f * x;
  int i;
  for (i = 0; i < 2; i++) {
    const float hy = h * y;
    y = y * fmaf(-hy, y, 1.5f);
  }
  return y;
}
/* Contract v7: the free-scale contract's normalize of the path directions takes ONE Newton step
 * (relative error < 1.8e-3, from below; rounds 1-4 took two). The scale places no geometry, it
 * only moves the roundings behind the self-hit / leak statistics: measured on this oracle, 128x96
 * @ 16, 12 seeds, NEE, first misses +0.25 % (0.6 sigma); with the bare seed (3.4e-2) +2.3 % (5
 * sigma), so not that. The cosine sample's R keeps two steps: its error biases the sampled
 * distribution (one step: image mean +1.2e-4 at C3). */
float spt_oracle_rsq_nr1(float x) {
  const float y = asf(0x5F375A86u - (asu(x) >> 1));
  const float hy = (0.5f * x) * y;
  return y * fmaf(-hy, y, 1.5f);
}
static inline fv fnormalize_free(fv v) {
  const float l2 = fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x));
  const float inv = spt_oracle_rsq_nr1(l2);
  return fv3(v.x * inv, v.y * inv, v.z * inv);
}
/* Vec::norm :50-52 as v * rsq_nr(len2). (Round 1 returned exactly-unit vectors unchanged, as the
 * reference's fp64 1/sqrt(1) does; rsq_nr(1) is 1 - 2^-24, and the select cost every normalize two
 * VALU on the GPU for vectors that occur with probability ~2^-24.) */
static inline fv fnormalize(fv v) {
  const float l2 = fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x));
  const float inv = spt_oracle_rsq_nr(l2);
  return fv3(v.x * inv, v.y * inv, v.z * inv);
}
static inline fv fcross(fv a, fv b) {
  return fv3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

/* sin(2*pi*xi), cos(2*pi*xi) for xi in [0,1): exact quarter-turn reduction + Taylor polynomials
 * in r = 4*xi - k (|r| <= 1/2, i.e. |theta| <= pi/4). Coefficients (pi/2)^n/n!. */
#define SC_S1 1.57079632679489662f
#define SC_S3 -0.645964097506246254f
#define SC_S5 0.0796926262461670451f
#define SC_S7 -0.00468175413531868810f
#define SC_S9 0.000160441184787359821f
#define SC_C2 -1.23370055013616983f
#define SC_C4 0.253669507901048014f
#define SC_C6 -0.0208634807633529609f
#define SC_C8 0.000919260274839426030f
void spt_oracle_sincos2pi(float xi, float* s_out, float* c_out) {
  const float q = xi * 4.0f;
  const float kf = rintf(q);
  const float r = q - kf;
  const int k = (int)kf & 3;
  const float r2 = r * r;
  float ps = fmaf(r2, SC_S9, SC_S7), pc = fmaf(r2, SC_C8, SC_C6), s, c;
  ps = fmaf(r2, ps, SC_S5);
  ps = fmaf(r2, ps, SC_S3);
  ps = fmaf(r2, ps, SC_S1);
  s = r * ps;
  pc = fmaf(r2, pc, SC_C4);
  pc = fmaf(r2, pc, SC_C2);
  c = fmaf(r2, pc, 1.0f);
  switch (k) {
    case 0: *s_out = s; *c_out = c; break;
    case 1: *s_out = c; *c_out = -s; break;
    case 2: *s_out = -s; *c_out = -c; break;
    default: *s_out = -c; *c_out = s; break;
  }
}

/* The azimuth of random_scattering (:343, r1 = 2*pi*xi) in the contract: (cos phi, sin phi) from
 * one 32-bit word by octant symmetry. Bits 31, 30 = signs of cos and sin, bit 29 = swap, bits 28..8
 * = theta in [0, pi/4) (21 bits; theta = u * (pi/2) * 2^-22, the sincos2pi polynomials in quarter
 * turns r = u * 2^-22 < 1/2). Uniform on the circle like 2*pi*xi (8 octants x 2^21 angles), without
 * the quarter-turn reduction or a quadrant rotation. */
/* The azimuth polynomials (contract, round 3): minimax fits on theta in [0, pi/4] (r in [0, 1/2]
 * quarter turns) with one term fewer than the Taylor sums above -- sin r(s1 + s3 r^2 + s5 r^4 +
 * s7 r^6), cos 1 + r^2(c2 + c4 r^2 + c6 r^4) -- whose fp32 evaluation is within 1.3e-7 relative of
 * sin/cos (the 5-term Taylor forms: 1.6e-7 / 1.2e-7), two fma fewer per cosine sample. */
#define DD_S1 1.5707963705062866f
#define DD_S3 -0.6459634900093079f
#define DD_S5 0.07968003302812576f
#define DD_S7 -0.004601659253239632f
#define DD_C2 -1.2336976528167725f
#define DD_C4 0.2536032199859619f
#define DD_C6 -0.020417289808392525f
void spt_oracle_disk_dir(uint32_t ra, float* c_out, float* s_out) {
  const float r = (float)((ra >> 8) & 0x1FFFFFu) * 0x1p-22f;
  const float r2 = r * r;
  float ps = fmaf(r2, DD_S7, DD_S5), pc = fmaf(r2, DD_C6, DD_C4), sn, cs, t;
  ps = fmaf(r2, ps, DD_S3);
  ps = fmaf(r2, ps, DD_S1);
  sn = r * ps;
  pc = fmaf(r2, pc, DD_C2);
  cs = fmaf(r2, pc, 1.0f);
  if (ra & 0x20000000u) { t = cs; cs = sn; sn = t; }
  *c_out = asf(asu(cs) ^ (ra & 0x80000000u));
  *s_out = asf(asu(sn) ^ ((ra << 1) & 0x80000000u));
}

typedef struct {
  int kind;
  float k;                 /* rect: plane coordinate */
  float ma, ha, mb, hb;    /* rect: in-plane bounds as |a - ma| <= ha, |b - mb| <= hb */
  float rad2, px, py, pz;  /* sphere */
  float inv_r;             /* sphere: 1/r (float division), the normal is (x - p) * inv_r */
  double drad2, dpx, dpy, dpz; /* sphere in fp64 (wide: radius >= SPT_WIDE_SPHERE_RADIUS) */
  int wide;
  fv e, c;
  float pmax;
  int refl;                /* spt_refl: DIFF, SPEC, REFR */
} c_prim;

/* Rect bounds [lo, hi] of :106 as |a - mid| <= half with mid = (lo+hi)/2, half = (hi-lo)/2
 * (double, rounded once to float): one subtract + one compare per axis on the GPU. Differs from
 * the two float compares only within an ulp of an edge. Degenerate (hi < lo) rects: half = -1. */
static void c_rect_mid(double lo, double hi, float* mid, float* half) {
  *mid = (float)((lo + hi) * 0.5);
  *half = hi >= lo ? (float)((hi - lo) * 0.5) : -1.0f;
}

/* One rectangle test of the counter-mode intersection: a single rectangle (k0 == k1, id0 == id1) or
 * a PARALLEL PAIR — two rectangles of one kind with bit-identical in-plane bounds on different
 * planes k0 < k1 (a box's opposite faces, the room's opposite walls). Per ray only the pair's plane
 * that can be hit first is tested (c_intersect). */
typedef struct {
  int kind;
  float k0, k1, ma, ha, mb, hb;
  int id0, id1;
  int pos0, pos1; /* grouped positions of the two planes (the nearest-hit key's low bits, c_key) */
} c_test;

typedef struct {
  const c_prim* prims;
  int n;
  const spt_params* P;
  uint32_t key[2];
  const c_test* tests; /* rect tests in contract order (c_build_tests) */
  int n_tests;
  int pos2idx[64];      /* grouped position -> primitive index: rects XY, XZ, YZ (index order
                           inside a kind), then spheres (narrow, then wide, index order) */
  int n_rect;           /* rectangles = the first sphere's position */
  int light_pos;        /* grouped position of P->light_id (-1: none) */
  int room[3];          /* tests of the scene's room (c_find_room), -1 = none */
  int n_box;            /* boxes standing on the room's floor (c_find_boxes) */
  int box[21][3];       /* their tests: XY pair (planes z), YZ pair (planes x), XZ top */
  unsigned char in_box[64]; /* test index -> 1 if it is part of a box */
  int leak_end;         /* c_find_leak_end: a path ends at its first miss */
  /* the early-resolve clauses of an edited HEAD-topology scene (c_find_early_clauses; the host's
     choice in spt_render_async, the kernel's early_geo_proven) */
  float eb_top[2], eb_sgn[2], eb_bnd[2];
  int eb_z[2];
  /* ... and its room clause (round 6: the room and the light may be edited too): the vertex lies in
     [lo, hi] per axis as (bits(v) - er_lo) <= er_span on the float bits (lo >= +0), y below the
     light plane */
  uint32_t er_lo[3], er_span[3];
  int unit;     /* c_unit_dirs: 1 = unit directions, 0 = the free-scale contract */
  float nee_c;  /* free-scale NEE weight constant: light_area / pi, rounded once */
} c_ctx;

/* Contract: the precision of ray directions. Unit directions (normalised with rsq_nr) where
 * something needs |d| = 1 to fp32 accuracy: the sphere quadratic (:229-239 assumes |d| = 1) and
 * the REFR Fresnel terms (:485-491 treat d.nl as a cosine). Otherwise (rectangles, DIFF/SPEC) the
 * FREE-SCALE contract:
 *  - path directions (camera ray, cosine sample) are normalised with one Newton step
 *    (rsq_nr1, |d| = 1 within 1.8e-3; contract v7, rounds 1-4: two). They must stay unit to ~1e-3:
 *    the self-hit / leak rate of the
 *    rect tests depends on |d| (measured, 256x192 @ 64 cosine-only: misses per sample 0.458 at
 *    |d| = 1 +- 1e-3, but 0.67 at |d| = 0.75 or 1.5 and 0.71 at 1.25), as on the reference's fp64
 *    unit vectors;
 *  - the NEE shadow vector light_vec - hit (:367) is not normalised at all: the shadow ray only
 *    asks whether its nearest hit is the light (:466-467), which does not depend on the scale, and
 *    the weight :471-472 is written without the length (c_nee_weight). */
static int c_unit_dirs(const spt_prim* s, int n) {
  int i;
  for (i = 0; i < n; i++)
    if (s[i].kind == SPT_SPHERE || s[i].refl == SPT_REFR) return 1;
  return 0;
}
static int c_build_tests(const c_prim* P, int n, int light_id, c_test* T);
static void c_find_room(c_ctx* C, const spt_prim* s);
static void c_find_boxes(c_ctx* C, const spt_prim* s);
static void c_find_leak_end(c_ctx* C, const spt_prim* s);
static void c_find_early_clauses(c_ctx* C);
static int g_unit_override = -1; /* test hook: -1 = the contract (c_unit_dirs), 0/1 = forced */
void spt_oracle_set_unit_dirs(int mode) { g_unit_override = mode; }
static void c_ctx_init(c_ctx* C, const spt_prim* prims, const c_prim* CP, int n, const spt_params* P,
                       c_test* CT) {
  C->prims = CP; C->n = n; C->P = P; C->key[0] = SPT_PHILOX_KEY0; C->key[1] = SPT_PHILOX_KEY1;
  C->n_tests = c_build_tests(CP, n, P->light_id, CT);
  C->tests = CT;
  {
    int i, kind, pos = 0;
    for (kind = SPT_RECT_XY; kind <= SPT_RECT_YZ; kind++)
      for (i = 0; i < n; i++)
        if (CP[i].kind == kind) C->pos2idx[pos++] = i;
    C->n_rect = pos;
    for (kind = 0; kind < 2; kind++) /* narrow spheres, then wide ones */
      for (i = 0; i < n; i++)
        if (CP[i].kind == SPT_SPHERE && CP[i].wide == kind) C->pos2idx[pos++] = i;
  }
  c_find_room(C, prims);
  c_find_boxes(C, prims);
  c_find_leak_end(C, prims);
  c_find_early_clauses(C);
  {
    int i;
    C->light_pos = -1;
    for (i = 0; i < n; i++)
      if (C->pos2idx[i] == P->light_id) C->light_pos = i;
  }
  C->unit = g_unit_override >= 0 ? g_unit_override : c_unit_dirs(prims, n);
  C->nee_c = (float)((double)P->light_area / 3.14159265358979323846);
}

/* Contract: the rect test list. Kinds in the order XY, XZ, YZ; inside a kind, rectangles in index
 * order, each paired with the first later unpaired rectangle of its kind whose (ma, ha, mb, hb) are
 * bit-identical and whose plane differs (a test is ordered by its first member's index). The light
 * (P->light_id) is never paired. Returns the number of tests written to T (<= n). */
static int g_pairs = 1;
/* Test hook: 0 = no pairing (every rectangle tested on its own: the per-rectangle form the pair
 * rule must reproduce), 1 = the contract. Not thread-safe against a running render. */
void spt_oracle_set_pairs(int on) { g_pairs = on != 0; }
/* Test hook: 0 = boxes tested face by face (as pairs and a top), 1 = the contract (c_find_boxes). */
static int g_boxes = 1;
void spt_oracle_set_boxes(int on) { g_boxes = on != 0; }
static int c_build_tests(const c_prim* P, int n, int light_id, c_test* T) {
  int used[64] = {0}, gpos[64], nt = 0, kind, i, j, g = 0;
  for (kind = SPT_RECT_XY; kind <= SPT_RECT_YZ; kind++)
    for (i = 0; i < n; i++)
      if (P[i].kind == kind) gpos[i] = g++;
  for (kind = SPT_RECT_XY; kind <= SPT_RECT_YZ; kind++) {
    for (i = 0; i < n; i++) {
      const c_prim* A = &P[i];
      c_test* t;
      if (A->kind != kind || used[i]) continue;
      used[i] = 1;
      t = &T[nt++];
      t->kind = kind;
      t->k0 = t->k1 = A->k;
      t->ma = A->ma; t->ha = A->ha; t->mb = A->mb; t->hb = A->hb;
      t->id0 = t->id1 = i;
      t->pos0 = t->pos1 = gpos[i];
      if (i == light_id) continue;
      if (!g_pairs) continue; /* diagnostic: every rectangle tested on its own */
      for (j = i + 1; j < n; j++) {
        const c_prim* B = &P[j];
        if (B->kind != kind || used[j] || j == light_id) continue;
        if (asu(B->ma) != asu(A->ma) || asu(B->ha) != asu(A->ha) || asu(B->mb) != asu(A->mb) ||
            asu(B->hb) != asu(A->hb) || asu(B->k) == asu(A->k) || !(B->k == B->k) || !(A->k == A->k))
          continue;
        used[j] = 1;
        if (A->k < B->k) { t->k1 = B->k; t->id1 = j; t->pos1 = gpos[j]; }
        else { t->k0 = B->k; t->id0 = j; t->pos0 = gpos[j]; t->k1 = A->k; t->id1 = i; t->pos1 = gpos[i]; }
        break;
      }
    }
  }
  return nt;
}

/* Contract v5: the scene's ROOM, if it has one -- three parallel pairs, one per kind, that close a
 * box: the XY pair's planes z = {z1, z2}, the XZ pair's y = {y1, y2} and the YZ pair's x = {x1, x2}
 * are exactly (in the caller's doubles) the other pairs' in-plane bounds (the reference's walls
 * :288-293: x [1, 99], y [0, 81.6], z [0, 170]). The first such triple in test order. */
static int c_same_range(double a1, double a2, double b1, double b2) {
  const double lo = a1 < a2 ? a1 : a2, hi = a1 < a2 ? a2 : a1;
  return lo == b1 && hi == b2;
}
static void c_find_room(c_ctx* C, const spt_prim* s) {
  int a, b, c;
  C->room[0] = C->room[1] = C->room[2] = -1;
  for (a = 0; a < C->n_tests; a++) {
    const c_test* A = &C->tests[a]; /* XY: bounds x (geom 0,1), y (geom 2,3); planes z */
    if (A->kind != SPT_RECT_XY || A->id0 == A->id1) continue;
    for (b = 0; b < C->n_tests; b++) {
      const c_test* B = &C->tests[b]; /* XZ: bounds x, z; planes y */
      if (B->kind != SPT_RECT_XZ || B->id0 == B->id1) continue;
      for (c = 0; c < C->n_tests; c++) {
        const c_test* D = &C->tests[c]; /* YZ: bounds y, z; planes x */
        const double* ga = s[A->id0].geom, *gb = s[B->id0].geom, *gd = s[D->id0].geom;
        if (D->kind != SPT_RECT_YZ || D->id0 == D->id1) continue;
        if (!c_same_range(s[D->id0].geom[4], s[D->id1].geom[4], ga[0], ga[1]) ||
            !c_same_range(s[D->id0].geom[4], s[D->id1].geom[4], gb[0], gb[1]) ||
            !c_same_range(s[B->id0].geom[4], s[B->id1].geom[4], ga[2], ga[3]) ||
            !c_same_range(s[B->id0].geom[4], s[B->id1].geom[4], gd[0], gd[1]) ||
            !c_same_range(s[A->id0].geom[4], s[A->id1].geom[4], gb[2], gb[3]) ||
            !c_same_range(s[A->id0].geom[4], s[A->id1].geom[4], gd[2], gd[3]))
          continue;
        C->room[0] = a; C->room[1] = b; C->room[2] = c;
        return;
      }
    }
  }
}

/* Contract v6 (round 4): a BOX is a parallel XY pair, a parallel YZ pair and a single XZ top (not
 * the light, none of them the room's) that close an axis-aligned box standing on the room's floor:
 * the YZ planes are the x bounds of the XY pair and of the top, the XY planes the z bounds of the
 * YZ pair and of the top, both pairs span y from the floor plane (the room's lower XZ plane) to
 * the top's plane, and the floor's bounds contain the box's footprint -- compared on the caller's
 * doubles. The reference's two boxes (:298-308) qualify. Found in test order, each test used once.
 * c_intersect tests a box as one slab candidate (the faces' in-plane compares are gone); the
 * bottom is the floor plane, reported as the floor. */
static void c_find_boxes(c_ctx* C, const spt_prim* s) {
  int a, b, c, used[64] = {0};
  double floor_k, gf[4];
  C->n_box = 0;
  memset(C->in_box, 0, sizeof C->in_box);
  if (!g_pairs || !g_boxes || C->room[0] < 0) return;
  {
    const c_test* F = &C->tests[C->room[1]];
    floor_k = s[F->id0].geom[4] < s[F->id1].geom[4] ? s[F->id0].geom[4] : s[F->id1].geom[4];
    memcpy(gf, s[F->id0].geom, sizeof gf); /* floor bounds: x (0, 1), z (2, 3) */
  }
  for (a = 0; a < C->n_tests; a++) {
    const c_test* A = &C->tests[a]; /* XY pair: bounds x (geom 0,1), y (2,3); planes z */
    if (A->kind != SPT_RECT_XY || A->id0 == A->id1 || a == C->room[0] || used[a]) continue;
    for (b = 0; b < C->n_tests; b++) {
      const c_test* D = &C->tests[b]; /* YZ pair: bounds y (0,1), z (2,3); planes x */
      if (D->kind != SPT_RECT_YZ || D->id0 == D->id1 || b == C->room[2] || used[b]) continue;
      for (c = 0; c < C->n_tests; c++) {
        const c_test* T = &C->tests[c]; /* XZ single: bounds x (0,1), z (2,3); plane y */
        const double *ga = s[A->id0].geom, *gd = s[D->id0].geom, *gt;
        double xa, xb, za, zb;
        if (T->kind != SPT_RECT_XZ || T->id0 != T->id1 || T->id0 == C->P->light_id || used[c]) continue;
        gt = s[T->id0].geom;
        if (!c_same_range(s[D->id0].geom[4], s[D->id1].geom[4], ga[0], ga[1]) ||
            !c_same_range(s[D->id0].geom[4], s[D->id1].geom[4], gt[0], gt[1]) ||
            !c_same_range(s[A->id0].geom[4], s[A->id1].geom[4], gd[2], gd[3]) ||
            !c_same_range(s[A->id0].geom[4], s[A->id1].geom[4], gt[2], gt[3]) ||
            !c_same_range(floor_k, gt[4], ga[2], ga[3]) || !c_same_range(floor_k, gt[4], gd[0], gd[1]) ||
            !(gt[4] > floor_k))
          continue;
        xa = ga[0]; xb = ga[1]; za = gd[2]; zb = gd[3];
        if (!(gf[0] <= xa && xb <= gf[1] && gf[2] <= za && zb <= gf[3])) continue;
        used[a] = used[b] = used[c] = 1;
        C->in_box[a] = C->in_box[b] = C->in_box[c] = 1;
        C->box[C->n_box][0] = a; C->box[C->n_box][1] = b; C->box[C->n_box][2] = c;
        C->n_box++;
        break;
      }
      if (used[a]) break;
    }
  }
}

/* Contract v6 (round 4): LEAKED PATHS END AT THEIR FIRST MISS. A missed ray's vertex is the origin
 * with id 0 (:373-374) and the reference's path goes on from there, outside the room. When the
 * scene has a room (c_find_room), the origin lies strictly outside the room's box, prim 0 does not
 * emit, and every emitter lies strictly inside the box (its plane strictly between the room's
 * walls, its bounds within them; a sphere with its whole ball), such a path ends at the miss vertex
 * as if Russian roulette had ended it (its emission, prim 0's, is zero). What that drops: nothing
 * outside the room emits and a ray from outside meets a wall first, so the rest of a leaked path
 * collects light only if a later vertex on a wall's outer face rounds back into the room (the
 * leak's own mechanism in reverse) and its NEE ray then reaches the light: measured, 8 ppm of the
 * image's mean at 256x192 @ 64 (207 of 49 152 pixels differ by one sample each; cosine-only: none),
 * for 4 % fewer vertices -- the reference's post-leak wandering (tests/test_oracle.py, P2
 * re-checked). spt_params.flags SPT_FLAG_REFERENCE_LEAKS (and the test hook
 * spt_oracle_set_leak_end(0)) restores the reference's behaviour; with the rule on, statistics count
 * first misses. */
static int g_leak_end = 1;
void spt_oracle_set_leak_end(int on) { g_leak_end = on != 0; }
static void c_find_leak_end(c_ctx* C, const spt_prim* s) {
  double lo[3], hi[3]; /* room box per axis x, y, z from the room pairs' planes (doubles) */
  int i, a;
  C->leak_end = 0;
  if (!g_leak_end || (C->P->flags & SPT_FLAG_REFERENCE_LEAKS) || C->room[0] < 0) return;
  for (a = 0; a < 3; a++) { /* room[0] XY pair: planes z; room[1] XZ: y; room[2] YZ: x */
    const c_test* T = &C->tests[C->room[a]];
    const double k0 = s[T->id0].geom[4], k1 = s[T->id1].geom[4];
    const int ax = a == 0 ? 2 : (a == 1 ? 1 : 0);
    lo[ax] = k0 < k1 ? k0 : k1;
    hi[ax] = k0 < k1 ? k1 : k0;
  }
  if (!(0.0 < lo[0] || 0.0 > hi[0] || 0.0 < lo[1] || 0.0 > hi[1] || 0.0 < lo[2] || 0.0 > hi[2])) return;
  if (s[0].e[0] != 0.0 || s[0].e[1] != 0.0 || s[0].e[2] != 0.0) return;
  for (i = 0; i < C->n; i++) {
    const double* g = s[i].geom;
    int pa, ua, va; /* plane axis and the two bound axes */
    if (s[i].e[0] == 0.0 && s[i].e[1] == 0.0 && s[i].e[2] == 0.0) continue;
    if (s[i].kind == SPT_SPHERE) {
      for (a = 0; a < 3; a++)
        if (!(g[1 + a] - g[0] > lo[a] && g[1 + a] + g[0] < hi[a])) return;
      continue;
    }
    switch (s[i].kind) {
      case SPT_RECT_XY: pa = 2; ua = 0; va = 1; break;
      case SPT_RECT_XZ: pa = 1; ua = 0; va = 2; break;
      default: pa = 0; ua = 1; va = 2; break;
    }
    if (!(g[4] > lo[pa] && g[4] < hi[pa] && g[0] >= lo[ua] && g[1] <= hi[ua] && g[2] >= lo[va] &&
          g[3] <= hi[va]))
      return;
  }
  C->leak_end = 1;
}

/* Contract v5: the nearest-hit key of a candidate at t on the plane (or sphere) with grouped
 * position pos: the float bits of t with the low 6 bits replaced by pos, so an unsigned minimum
 * ranks the candidates (negatives -- a plane's zero distance is -2^-149, c_plane_t, a sphere
 * without a root -0 -- and NaN rank last; kKeyNone = tmin 1e20 of :324). A candidate's t is
 * ranked to 64 ulps; ties and near-ties inside that resolve to the lower position (the reference:
 * strict `<` over rect[] :328, ties to the lower index). On the GPU a key is one v_bitop3 and the
 * running minimum one v_min_u32 -- no compare and lane-mask select per candidate. */
static inline uint32_t c_key(float t, int pos) { return (asu(t) | 63u) ^ (uint32_t)(63 - pos); }
#define C_KEY_NONE (asu(1e20f) | 63u) /* tmin = 1e20 (:324): no hit */
/* A plane's distance in contract v5: t = (k - o_a) * inv_a as one fma with -2^-149 added. That is
 * the rounded product except when the product is an exact rounding tie (then the lower neighbour)
 * and turns a zero distance (the origin on the plane: :106 `t<0`, :328 `d != 0` reject it) into
 * -2^-149, which ranks last like every negative t: the key needs no "minus one" to put +0 last. */
#define C_NEG_TINY (-0x1p-149f)
static inline float c_plane_t_fma(float n, float inv) { return fmaf(n, inv, C_NEG_TINY); }
/* The same value without the fma's denormal addend (an x86 microcode assist of ~100+ cycles per
 * call: it made this restatement 10x slower). The product p = n * inv is exact in double. For a
 * normal p the fma rounds p - 2^-149, which can differ from round(p) only when p lies exactly
 * midway between two floats (p is a multiple of a 2^-46-relative unit, so nothing else lies within
 * 2^-149 of a midpoint): the fma then returns the lower neighbour. p == 0 gives -2^-149; tiny and
 * huge p (float denormal range, overflow) and NaN take the fma itself. Checked against
 * c_plane_t_fma on constructed ties and random operands (spt_oracle_plane_t_mismatches). */
static inline float c_plane_t(float n, float inv) {
  const double p = (double)n * (double)inv;
  const double ap = fabs(p);
  float r, lo;
  if (!(ap >= 0x1p-125 && ap <= 0x1p127)) return p == 0.0 ? C_NEG_TINY : c_plane_t_fma(n, inv);
  r = (float)p; /* normal, nonzero: its neighbours are one step of the bit pattern away */
  lo = (double)r > p ? asf(p > 0.0 ? asu(r) - 1u : asu(r) + 1u) : r;
  return (double)lo != p && p - (double)lo == (double)asf(p > 0.0 ? asu(lo) + 1u : asu(lo) - 1u) - p ? lo : r;
}

/* Test hook (round 5): the plane distance as ONE fma of the ray-constant o * inv,
 * t = fma(k, inv, -(o * inv)), instead of (k - o) * inv -- the candidate that would take the
 * per-plane subtraction out of the trace. 0 = the contract. */
static int g_fused_planes = 0;
void spt_oracle_set_fused_planes(int on) { g_fused_planes = on != 0; }
static inline float c_pt(float k, float o, float inv) {
  return g_fused_planes ? fmaf(k, inv, -(o * inv)) : c_plane_t(k - o, inv);
}
/* Test hook: how many of the n (num[i], inv[i]) give different bits from the fma form. */
int spt_oracle_plane_t_mismatches(const float* num, const float* inv, int n) {
  int i, bad = 0;
  for (i = 0; i < n; i++) {
    const float a = c_plane_t(num[i], inv[i]), b = c_plane_t_fma(num[i], inv[i]);
    uint32_t ua, ub;
    memcpy(&ua, &a, 4);
    memcpy(&ub, &b, 4);
    bad += ua != ub;
  }
  return bad;
}
static inline uint32_t c_umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
static inline int32_t c_imin(int32_t a, int32_t b) { return a < b ? a : b; }
static inline int32_t c_imax(int32_t a, int32_t b) { return a > b ? a : b; }

/* The counter-mode scene intersection (intersect :323-335). inv = rcp_nr(d) once per ray.
 * The rect tests (c_build_tests) run in their contract order — kind XY, XZ, YZ — then the spheres
 * in index order, with the reference's strict `<` (:328), so the first test in THAT order wins a
 * tie of exactly equal t (the reference: lowest index; they differ only for bit-identical t from
 * two different planes). id is left untouched on a miss; returns 1 on hit, *t = 1e20f on a miss.
 *
 * A parallel pair tests one plane per ray: with n_i = k_i - o_a, the plane k0 when the ray moves
 * up the axis (inv_a > 0) from below it (n0 > 0), or down the axis (inv_a <= 0, incl. NaN) from
 * anywhere not above k1 (n1 >= 0); otherwise k1. That is the plane of the pair that is ahead and
 * nearer; the other one can only be the nearest hit of the two through the box's interior, i.e.
 * when the first plane's test is missed within an ulp of an edge. Every test then computes
 * t = n * inv_a exactly as a single rectangle (the same bits as testing that plane alone). */
/* A wide sphere (the 1e5 walls and the radius-600 light of the classic smallpt box) in fp64: the
 * cancellation-free quadratic with explicit fma, IEEE division and sqrt, the fp32 contract's
 * epsilon, t rounded to float. The quadratic keeps a = d.d (the fp32-normalised d is not exactly
 * unit; assuming |d| = 1 puts an error (|d|^2 - 1) * b^2 ~ 1e3 into a radius-1e5 discriminant):
 * t = k -+ sqrt(det / a), k = (op.d) / a, det = r^2 - |op - k d|^2. */
static float c_sphere_wide(const c_prim* P, fv o, fv d) {
  const double ox = P->dpx - (double)o.x, oy = P->dpy - (double)o.y, oz = P->dpz - (double)o.z;
  const double dx = d.x, dy = d.y, dz = d.z;
  const double a = fma(dz, dz, fma(dy, dy, dx * dx));
  const double k = fma(oz, dz, fma(oy, dy, ox * dx)) / a;
  const double qx = fma(-k, dx, ox), qy = fma(-k, dy, oy), qz = fma(-k, dz, oz);
  const double det = P->drad2 - fma(qz, qz, fma(qy, qy, qx * qx));
  double sd, t1, t2;
  if (!(det >= 0.0)) return -0.0f;
  sd = sqrt(det / a);
  t1 = k - sd;
  t2 = k + sd;
  return (float)(t1 > 2e-3 ? t1 : (t2 > 2e-3 ? t2 : -0.0)); /* -0: no root (ranks last) */
}

/* A narrow sphere in fp32: det = b^2 - op.op + r^2 (:233, as one fma), the nearest root beyond
 * the fp32 epsilon 2e-3; 0 = no hit. The root of det is det * rsq_nr2(det) (the contract's
 * reciprocal square root with two Newton steps, 5e-6 relative: 3e-5 in t at r = 6, far below the
 * epsilon; det = 0 gives 0), not an IEEE sqrtf: on the GPU the correctly rounded square root is an
 * ~18-slot sequence, rsq_nr2 10 (round 2 took det * rsq_nr(det), 13). Pinned against the
 * reference's own fp64 Sphere by the sph/sph16 P2 runs. */
static float c_sphere(const c_prim* P, fv o, fv d) {
  const fv op = fv3(P->px - o.x, P->py - o.y, P->pz - o.z);
  const float bb = fdot(op, d);
  const float det = fmaf(bb, bb, P->rad2 - fdot(op, op)); /* :233's b*b - op.op + rad*rad */
  float sd, t1, t2;
  if (!(det >= 0.0f)) return -0.0f;
  sd = det * spt_oracle_rsq_nr2(det); /* two Newton steps (round 3): 5e-6 relative */
  t1 = bb - sd;
  t2 = bb + sd;
  return t1 > 2e-3f ? t1 : (t2 > 2e-3f ? t2 : -0.0f); /* -0: no root (ranks last) */
}

/* Does the light itself accept the ray (o, d)? Its own test, exactly as inside c_intersect (the
 * light is never paired). The device traces a NEE shadow ray only when this holds or the vertex
 * lies on the light (id kept on a miss); otherwise the nearest hit cannot be the light (:467).
 * Counts spt_stats.shadow_traced; never changes a result. */
static int c_light_accepts(const c_ctx* C, fv o, fv d) {
  const int l = C->P->light_id;
  const c_prim* P;
  if (l < 0 || l >= C->n) return 0;
  P = &C->prims[l];
  if (P->kind == SPT_SPHERE)
    return c_key(P->wide ? c_sphere_wide(P, o, d) : c_sphere(P, o, d), C->light_pos) < C_KEY_NONE;
  {
    float oa, da, tt, a, b;
    switch (P->kind) {
      case SPT_RECT_XY: oa = o.z; da = d.z; break;
      case SPT_RECT_XZ: oa = o.y; da = d.y; break;
      default: oa = o.x; da = d.x; break;
    }
    tt = c_pt(P->k, oa, spt_oracle_rcp_nr(da)); /* as inside c_intersect (contract v5) */
    switch (P->kind) {
      case SPT_RECT_XY: a = fmaf(d.x, tt, o.x - P->ma); b = fmaf(d.y, tt, o.y - P->mb); break;
      case SPT_RECT_XZ: a = fmaf(d.x, tt, o.x - P->ma); b = fmaf(d.z, tt, o.z - P->mb); break;
      default: a = fmaf(d.y, tt, o.y - P->ma); b = fmaf(d.z, tt, o.z - P->mb); break;
    }
    return fabsf(a) <= P->ha && fabsf(b) <= P->hb && c_key(tt, C->light_pos) < C_KEY_NONE;
  }
}

/* The HEAD NEE kernel's early resolve (spt_kernel.hip early_nee_proven), restated so the tests can
 * check it against c_intersect: for the HEAD scene (rect[] :287-311, light index 6 at y = 81.5), a
 * shadow ray (o, d) whose light test accepts and whose origin meets these conditions is claimed
 * to have the light as its nearest hit at the light's own t (*tl). Test-only: spt_oracle_proof_*
 * count the claims and any claim c_intersect contradicts; never changes a result. */
static int g_proof_on; /* 1: the HEAD scene (boxes); 2: spheres below g_proof_y0 - 1 in the HEAD room;
                          3: an edited HEAD-topology rect[] (c_find_early_clauses) */
static float g_proof_y0;
static uint64_t g_proof_n, g_proof_bad;
/* The clauses of early_geo_proven (spt_kernel.hip) for a scene with a room (c_find_room), two boxes
 * (c_find_boxes) and an XZ light, as the host picks them (spt_render_async, early_geo_setup):
 *  - room: the vertex in the room's box, y below the light plane: X0 <= x <= X1, Y0 <= y < y_L,
 *    Z0 <= z <= Z1 (uint compares of the float bits, so X0, Y0, Z0 >= 0). From inside, the room's
 *    slab candidate is its exit face; with the light's rectangle >= 1 inside the side walls, the
 *    ceiling >= 0.05 above the light plane and the room < 1000 across, every exit face lies beyond
 *    the light crossing by a relative margin >= 5e-5, far above the keys' 2^-17 resolution (HEAD:
 *    31 / 63 units and 0.1 above; the literal kernel's early_nee_proven is this clause for HEAD);
 *  - the light plane y_L at most 81.5 = the reference's sample plane y = 81.6 (:367) less 0.1, so
 *    the crossing lies on the segment from the vertex to its light sample (x in [31, 33), z in
 *    [62, 64): the reference's wrapped samples), and at least 1 above the floor;
 *  - per box, a top >= 0.5 below the light plane, and the clause its position allows: x0 >= 33 ->
 *    clear for x <= x0 (the segment to the sample stays at x <= x0), x1 <= 31 for x >= x1, z0 >= 64
 *    for z <= z0, z1 <= 62 for z >= z1; always: a vertex at or above its top (the ray rises).
 * A scene that fails any condition gets no clause: +inf / -inf (nothing is resolved early). */
static void c_find_early_clauses(c_ctx* C) {
  int b, a, ok = C->n_box == 2 && C->room[0] >= 0;
  const int l = C->P->light_id;
  float lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0}, yl = 0;
  for (b = 0; b < 2; b++) {
    C->eb_top[b] = INFINITY; C->eb_sgn[b] = 1.0f; C->eb_bnd[b] = -INFINITY; C->eb_z[b] = 0;
  }
  for (a = 0; a < 3; a++) C->er_lo[a] = C->er_span[a] = 0;
  if (ok && (l < 0 || l >= C->n || C->prims[l].kind != SPT_RECT_XZ)) ok = 0;
  if (ok) {
    const c_prim* L = &C->prims[l];
    for (a = 0; a < 3; a++) { /* room tests: XY pair (planes z), XZ (y), YZ (x) */
      const c_test* R = &C->tests[C->room[a]];
      const int ax = a == 0 ? 2 : (a == 1 ? 1 : 0);
      lo[ax] = R->k0 < R->k1 ? R->k0 : R->k1;
      hi[ax] = R->k0 < R->k1 ? R->k1 : R->k0;
      ok = ok && lo[ax] >= 0.0f && hi[ax] - lo[ax] <= 1000.0f;
    }
    yl = L->k;
    ok = ok && L->ha >= 0.0f && L->hb >= 0.0f && L->ma - L->ha >= lo[0] + 1.0f &&
         L->ma + L->ha <= hi[0] - 1.0f && L->mb - L->hb >= lo[2] + 1.0f &&
         L->mb + L->hb <= hi[2] - 1.0f && yl >= lo[1] + 1.0f && yl <= 81.5f && hi[1] >= yl + 0.05f;
  }
  for (b = 0; ok && b < 2; b++) {
    const c_test *XY = &C->tests[C->box[b][0]], *YZ = &C->tests[C->box[b][1]], *T = &C->tests[C->box[b][2]];
    const float z0 = XY->k0 < XY->k1 ? XY->k0 : XY->k1, z1 = XY->k0 < XY->k1 ? XY->k1 : XY->k0;
    const float x0 = YZ->k0 < YZ->k1 ? YZ->k0 : YZ->k1, x1 = YZ->k0 < YZ->k1 ? YZ->k1 : YZ->k0;
    if (!(T->k0 <= yl - 0.5f)) { ok = 0; break; } /* top >= 0.5 below the light plane */
    C->eb_top[b] = T->k0;
    if (x0 >= 33.0f) { C->eb_sgn[b] = 1.0f; C->eb_bnd[b] = x0; C->eb_z[b] = 0; }
    else if (x1 <= 31.0f) { C->eb_sgn[b] = -1.0f; C->eb_bnd[b] = -x1; C->eb_z[b] = 0; }
    else if (z0 >= 64.0f) { C->eb_sgn[b] = 1.0f; C->eb_bnd[b] = z0; C->eb_z[b] = 1; }
    else if (z1 <= 62.0f) { C->eb_sgn[b] = -1.0f; C->eb_bnd[b] = -z1; C->eb_z[b] = 1; }
  }
  if (!ok) {
    for (b = 0; b < 2; b++) { C->eb_top[b] = INFINITY; C->eb_sgn[b] = 1.0f; C->eb_bnd[b] = -INFINITY; }
    return;
  }
  for (a = 0; a < 3; a++) {
    const float top = a == 1 ? nextafterf(yl, 0.0f) : hi[a]; /* y < y_L */
    C->er_lo[a] = asu(lo[a]);
    C->er_span[a] = asu(top) - asu(lo[a]);
  }
}
/* The light's own test on (o, d) as in c_intersect (c_light_accepts), with its t (an XZ light). */
static int c_light_test_xz(const c_ctx* C, fv o, fv d, float* tt_out) {
  const c_prim* L = &C->prims[C->P->light_id];
  const float tt = c_pt(L->k, o.y, spt_oracle_rcp_nr(d.y));
  const float a = fmaf(d.x, tt, o.x - L->ma), b = fmaf(d.z, tt, o.z - L->mb);
  *tt_out = tt;
  return fabsf(a) <= L->ha && fabsf(b) <= L->hb && c_key(tt, C->light_pos) < C_KEY_NONE;
}
static int c_early_nee_proven(const c_ctx* C, fv o, fv d, float* tl) {
  const float tt = c_pt(81.5f, o.y, spt_oracle_rcp_nr(d.y));
  const float a = fmaf(d.x, tt, o.x - 50.0f), b = fmaf(d.z, tt, o.z - 79.5f);
  const int acc = fabsf(a) <= 18.0f && fabsf(b) <= 16.5f && c_key(tt, 8) < C_KEY_NONE;
  const int room = asu(o.x) - asu(1.0f) <= asu(99.0f) - asu(1.0f) && asu(o.z) <= asu(170.0f) &&
                   asu(o.y) < asu(81.5f);
  /* (round 4: "x_L < 63", a < 13, dropped as in the kernel: below y = 25 the reference's light
     samples, x in [31, 33), cross y = 81.5 at x_L < 33.2; the proof tests check the claims) */
  const int short_box = o.y >= 25.0f || o.x <= 63.0f;
  const int tall_box = o.y >= 50.0f || o.z >= 62.0f;
  *tl = tt;
  if (g_proof_on == 2) return acc && room && o.y > g_proof_y0; /* spt_kernel.hip early_room_proven */
  if (g_proof_on == 3) { /* spt_kernel.hip early_geo_proven (an edited HEAD-topology rect[]) */
    int b, a, ok = c_light_test_xz(C, o, d, tl);
    const float v3[3] = {o.x, o.y, o.z};
    for (a = 0; a < 3; a++) ok = ok && asu(v3[a]) - C->er_lo[a] <= C->er_span[a];
    for (b = 0; b < 2; b++) {
      const float v = C->eb_z[b] ? o.z : o.x;
      ok = ok && (o.y >= C->eb_top[b] || v * C->eb_sgn[b] <= C->eb_bnd[b]);
    }
    return ok;
  }
  return acc && room && short_box && tall_box;
}
/* Test hook (the shadow-ray slot model): the light-accepted shadow rays that the HEAD
 * early resolve leaves to a trace (proof mode 1), by outcome and by why the predicate failed.
 *  [0] reached the light  [1] blocked
 *  [2] reached, vertex outside the room box (rounded through its wall)  [3] blocked, same
 *  [4] blocked by the vertex's own primitive (a self-hit)  [5] blocked, own prim, vertex outside
 *  [6] reached, short-box clause failed (tall ok)  [7] reached, tall failed (short ok)  [8] both
 *  [9] blocked, vertex's own axis coordinate outside the room's range, all others inside */
static uint64_t g_census[16];
static void c_shadow_census(const c_ctx* C, fv o, fv d, int vid, int hid) {
  const int reached = hid == C->P->light_id;
  const int room = asu(o.x) - asu(1.0f) <= asu(99.0f) - asu(1.0f) && asu(o.z) <= asu(170.0f) &&
                   asu(o.y) < asu(81.5f);
  const int short_box = o.y >= 25.0f || o.x <= 63.0f, tall_box = o.y >= 50.0f || o.z >= 62.0f;
  (void)d;
  __atomic_fetch_add(&g_census[reached ? 0 : 1], 1, __ATOMIC_RELAXED);
  if (!room) __atomic_fetch_add(&g_census[reached ? 2 : 3], 1, __ATOMIC_RELAXED);
  if (!reached && hid == vid) __atomic_fetch_add(&g_census[room ? 4 : 5], 1, __ATOMIC_RELAXED);
  if (reached && room)
    __atomic_fetch_add(&g_census[!short_box && tall_box ? 6 : (short_box && !tall_box ? 7 : 8)], 1,
                       __ATOMIC_RELAXED);
}
void spt_oracle_shadow_census(uint64_t out[16]) {
  int i;
  for (i = 0; i < 16; i++) { out[i] = g_census[i]; g_census[i] = 0; }
}
void spt_oracle_proof_check(int on, float y0) {
  g_proof_on = on;
  g_proof_y0 = y0;
  g_proof_n = g_proof_bad = 0;
}
/* Test hook: the contract's nearest hit for n rays (o, d: 3 floats each) in the scene; t_out = 1e20
 * and id_out = -1 on a miss. */
static void c_prims_from_spt(const spt_prim* s, int n, c_prim* P);
static int c_intersect(const c_ctx* C, fv o, fv d, float* t, int* id);
int spt_oracle_intersect_batch(const spt_prim* prims, int n, const spt_params* P, const float* o,
                               const float* d, int nrays, float* t_out, int32_t* id_out) {
  c_prim CP[64];
  c_test CT[64];
  c_ctx C;
  int r;
  if (n < 1 || n > 64) return -1;
  c_prims_from_spt(prims, n, CP);
  c_ctx_init(&C, prims, CP, n, P, CT);
  for (r = 0; r < nrays; r++) {
    int id = -1;
    float t;
    c_intersect(&C, fv3(o[3 * r], o[3 * r + 1], o[3 * r + 2]), fv3(d[3 * r], d[3 * r + 1], d[3 * r + 2]), &t, &id);
    t_out[r] = t;
    id_out[r] = id;
  }
  return 0;
}
/* Test hook: the number of contract-v6 boxes c_find_boxes finds in the scene (-1: bad input). */
int spt_oracle_scene_boxes(const spt_prim* prims, int n, const spt_params* P) {
  c_prim CP[64];
  c_test CT[64];
  c_ctx C;
  if (n < 1 || n > 64) return -1;
  c_prims_from_spt(prims, n, CP);
  c_ctx_init(&C, prims, CP, n, P, CT);
  return C.n_box;
}
void spt_oracle_proof_counts(uint64_t out[2]) {
  out[0] = g_proof_n;
  out[1] = g_proof_bad;
}

/* Contract v5 (round 4). Every candidate is ranked by its key (c_key) and the nearest hit is the
 * smallest key:
 *  - a rect test gives one key per plane, t = (k - o_a) * inv_a; a parallel PAIR's candidate is
 *    the smaller of its two planes' keys -- the smaller positive t, which is exactly the plane the
 *    rounds-1-4 pair rule chose (the one ahead and nearer; the planes of a pair are >= 25 units
 *    apart, far more than the keys' 64 ulps) -- and its in-plane test is evaluated at the chosen
 *    t (c_plane_t: the distance as one fma with -2^-149). Accepted iff |a| <= half and
 *    |b| <= half there (:104-106);
 *  - the ROOM (c_find_room) and the BOXES (c_find_boxes) are slabs (contract v6): per axis the
 *    two planes' keys as signed integers bound the slab interval, the candidate is the entry (the
 *    largest interval start) -- or from inside the exit face (the smallest interval end), the
 *    nearest positive plane -- accepted iff entry <= exit. For an origin in the room that is the
 *    wall the per-wall tests find; it differs from them only for rays grazing an edge within
 *    rounding and it needs no in-plane compare at all (v5: the room's nearest plane accepted
 *    within its box widened by 2^-8);
 *  - spheres: key(t, position) of the nearest root beyond the epsilon (0 = no root, ranked last).
 * The hit's t is the winner's own t, recomputed from its plane / sphere (the same bits as in its
 * key). id is left untouched on a miss; returns 1 on hit, *t = 1e20f on a miss. */
static int c_intersect(const c_ctx* C, fv o, fv d, float* t, int* id) {
  const float ix = spt_oracle_rcp_nr(d.x), iy = spt_oracle_rcp_nr(d.y), iz = spt_oracle_rcp_nr(d.z);
  uint32_t tmin = C_KEY_NONE;
  int i, pos;
  for (i = 0; i < C->n_tests; i++) {
    const c_test* T = &C->tests[i];
    float oa, ia, tb, a, b;
    uint32_t kp;
    const int room = i == C->room[0] || i == C->room[1] || i == C->room[2] || C->in_box[i];
    switch (T->kind) {
      case SPT_RECT_XY: oa = o.z; ia = iz; break;
      case SPT_RECT_XZ: oa = o.y; ia = iy; break;
      default: oa = o.x; ia = ix; break;
    }
    if (room) continue; /* below */
    {
      const float t0 = c_pt(T->k0, oa, ia);
      if (T->id0 != T->id1) {
        const float t1 = c_pt(T->k1, oa, ia);
        kp = c_umin(c_key(t0, T->pos0), c_key(t1, T->pos1));
        tb = asf(c_umin(asu(t0), asu(t1)));
      } else {
        kp = c_key(t0, T->pos0);
        tb = t0;
      }
    }
    /* in-plane offsets from the rectangle's centre, a = d_b * t + (o_b - mid_b) in one fma */
    switch (T->kind) {
      case SPT_RECT_XY: a = fmaf(d.x, tb, o.x - T->ma); b = fmaf(d.y, tb, o.y - T->mb); break;
      case SPT_RECT_XZ: a = fmaf(d.x, tb, o.x - T->ma); b = fmaf(d.z, tb, o.z - T->mb); break;
      default: a = fmaf(d.y, tb, o.y - T->ma); b = fmaf(d.z, tb, o.z - T->mb); break;
    }
    if (fabsf(a) <= T->ha && fabsf(b) <= T->hb) tmin = c_umin(tmin, kp);
  }
  if (C->room[0] >= 0) { /* the room as a slab (contract v6), like a box below: from inside it is
                           * the exit face, the nearest positive plane of the three pairs */
    int32_t en = INT32_MIN, ex = INT32_MAX;
    int r;
    for (r = 0; r < 3; r++) {
      const c_test* T = &C->tests[C->room[r]];
      const float oa = r == 0 ? o.z : (r == 1 ? o.y : o.x), ia = r == 0 ? iz : (r == 1 ? iy : ix);
      const int32_t k0 = (int32_t)c_key(c_pt(T->k0, oa, ia), T->pos0);
      const int32_t k1 = (int32_t)c_key(c_pt(T->k1, oa, ia), T->pos1);
      en = c_imax(en, c_imin(k0, k1));
      ex = c_imin(ex, c_imax(k0, k1));
    }
    if (en <= ex) tmin = c_umin(tmin, c_umin((uint32_t)en, (uint32_t)ex));
  }
  /* Boxes (contract v6): per axis the keys of the two planes as signed integers -- for t >= 0 the
   * integer order is the order of t, and every negative t is a negative integer -- the slab
   * interval [min, max] (y: the floor and the top); the entry is the largest interval start, the
   * exit the smallest interval end, and the box is crossed iff entry <= exit. Its candidate is the
   * entry, or the exit when the origin lies inside the box (a negative entry): the face the ray
   * leaves through, as the per-face test finds it (a vertex rounded into a box self-hits its face,
   * like the reference's). As unsigned keys that is min(entry, exit); an exit behind the origin is
   * negative and ranks last. */
  for (i = 0; i < C->n_box; i++) {
    const c_test *Z = &C->tests[C->box[i][0]], *X = &C->tests[C->box[i][1]], *Y = &C->tests[C->box[i][2]];
    const c_test* F = &C->tests[C->room[1]];
    const int32_t kx0 = (int32_t)c_key(c_pt(X->k0, o.x, ix), X->pos0);
    const int32_t kx1 = (int32_t)c_key(c_pt(X->k1, o.x, ix), X->pos1);
    const int32_t kz0 = (int32_t)c_key(c_pt(Z->k0, o.z, iz), Z->pos0);
    const int32_t kz1 = (int32_t)c_key(c_pt(Z->k1, o.z, iz), Z->pos1);
    const int32_t ky0 = (int32_t)c_key(c_pt(F->k0, o.y, iy), F->pos0);
    const int32_t ky1 = (int32_t)c_key(c_pt(Y->k0, o.y, iy), Y->pos0);
    const int32_t en = c_imax(c_imax(c_imin(kx0, kx1), c_imin(kz0, kz1)), c_imin(ky0, ky1));
    const int32_t ex = c_imin(c_imin(c_imax(kx0, kx1), c_imax(kz0, kz1)), c_imax(ky0, ky1));
    if (en <= ex) tmin = c_umin(tmin, c_umin((uint32_t)en, (uint32_t)ex));
  }
  /* Spheres: narrow (fp32) ones, then the wide (fp64) ones, each in index order (their positions) */
  for (i = C->n_rect; i < C->n; i++) {
    const c_prim* P = &C->prims[C->pos2idx[i]];
    tmin = c_umin(tmin, c_key(P->wide ? c_sphere_wide(P, o, d) : c_sphere(P, o, d), i));
  }
  if (!(tmin < C_KEY_NONE)) {
    *t = 1e20f;
    return 0;
  }
  pos = (int)(tmin & 63u);
  *id = C->pos2idx[pos];
  {
    const c_prim* H = &C->prims[*id];
    switch (H->kind) {
      case SPT_RECT_XY: *t = c_pt(H->k, o.z, iz); break;
      case SPT_RECT_XZ: *t = c_pt(H->k, o.y, iy); break;
      case SPT_RECT_YZ: *t = c_pt(H->k, o.x, ix); break;
      default: *t = H->wide ? c_sphere_wide(H, o, d) : c_sphere(H, o, d);
    }
  }
  return 1;
}

/* random_scattering in the contract: cosine (:340-347), or with `uniform` the commented-out
   uniform hemisphere (:352-359): radial sqrt(r2*(2-r2)) and normal component (1-r2). */
static fv c_cosine(fv nl, uint32_t ra, uint32_t rb, int uniform, int unit) {
  const float xi2 = u01(rb);
  float s, c;
  fv a, u, v;
  float r2s, s1, cr, sr;
  spt_oracle_disk_dir(ra, &c, &s); /* the azimuth r1 = 2*pi*xi1 of :343 */
  if (uniform) {
    const float m = xi2 * (2.0f - xi2);
    r2s = m * (unit ? spt_oracle_rsq_nr(m) : spt_oracle_rsq_nr2(m));
    s1 = 1.0f - xi2;
  } else {
    /* (cos, sin) * sqrt(r2) and sqrt(1 - r2) (:343-347) scaled by 1 / sqrt(1 - r2): the direction
       is normalized below anyway, so the contract takes R = sqrt(r2 / (1 - r2)) with ONE rsqrt,
       R = r2 * rsq(r2 * (1 - r2)), and a normal component of exactly 1. */
    const float q = xi2 * (1.0f - xi2);
    r2s = xi2 * (unit ? spt_oracle_rsq_nr(q) : spt_oracle_rsq_nr2(q));
    s1 = 1.0f;
  }
  cr = c * r2s;
  sr = s * r2s;
  if ((nl.y == 0.0f && nl.z == 0.0f && fabsf(nl.x) == 1.0f) ||
      (nl.x == 0.0f && nl.z == 0.0f && fabsf(nl.y) == 1.0f) ||
      (nl.x == 0.0f && nl.y == 0.0f && fabsf(nl.z) == 1.0f)) {
    /* Contract: an axis-aligned normal (every rectangle's, smallpt.cpp:123,:166,:209) makes the
       frame of :345-346 a signed permutation of the axes, so the direction is written out:
       nl = (sx,0,0) -> (sx*s1, sr, -sx*cr); (0,sy,0) -> (sr, sy*s1, sy*cr);
       (0,0,sz) -> (sr, -sz*cr, sz*s1). Same values as the general formula below up to the sign
       of exact zeros. Round 5: written with the normal's components as 0 / +-1 weights, six fmas
       and no compare (the kernel's cosine_vec), the values of the case-by-case form up to the sign
       of an exact zero. */
    const fv r = fv3(fmaf(nl.x, s1, fmaf(-fabsf(nl.x), sr, sr)),
                     fmaf(fabsf(nl.x), sr, fmaf(nl.y, s1, -(nl.z * cr))),
                     fmaf(nl.z, s1, (nl.y - nl.x) * cr));
    return unit ? fnormalize(r) : fnormalize_free(r);
  }
  a = fabsf(nl.x) > 0.1f ? fv3(nl.z, 0.0f, -nl.x) : fv3(0.0f, -nl.z, nl.y);
  u = fnormalize(a);
  v = fcross(nl, u);
  {
    const fv r = fv3(fmaf(nl.x, s1, fmaf(v.x, sr, u.x * cr)), fmaf(nl.y, s1, fmaf(v.y, sr, u.y * cr)),
                     fmaf(nl.z, s1, fmaf(v.z, sr, u.z * cr)));
    return unit ? fnormalize(r) : fnormalize_free(r);
  }
}

/* The hit point's plane distance n / d_a (:103, n = k - o_a) in the contract: one Markstein
 * correction of the intersection's t = n * rcp_nr(d_a) — r = n - t*d_a is exact (fma), then
 * t + r * rcp_nr(d_a). Equal to the IEEE quotient in all of 2e8 sampled cases, which matters: where
 * x = o + d*t lands relative to the plane sets the self-hit / leak rate (see spt_oracle_plane_k). */
static float c_hit_t(float n, float da, float t) {
  return fmaf(fmaf(-t, da, n), spt_oracle_rcp_nr(da), t);
}
/* n / d in the contract where the reference divides once per event (the NEE pdf :471):
 * n * rcp_nr(d), within ~1 ulp of the quotient. (Round 1 added a Markstein correction to the IEEE
 * quotient; the pdf only weights a sample, it places no geometry, and the correction cost the GPU
 * two VALU per loop iteration.) */
static float c_div(float n, float d) { return n * spt_oracle_rcp_nr(d); }

/* PDF_inverse * BRDF of :471-472 for a NEE shadow ray (x, d) whose nearest hit is the light at
 * t. Unit directions: |area * d.y / t^2| * |d.nl / pi| as written. Free-scale (c_unit_dirs): d is
 * light_vec itself; with dl = d/|d| and the distance t|d| the same quantity is
 * (area/pi) |d.y| |d.nl| / (t^2 (d.d)^2), with no square root, rounded as written here. */
static float c_nee_weight(const c_ctx* C, fv d, fv nl, float t) {
  if (C->unit) {
    const float pdf = fabsf(c_div(C->P->light_area * d.y, t * t));
    const float brdf = fabsf(fdot(d, nl) * 0.318309886183790672f);
    return pdf * brdf;
  }
  {
    const float num = fabsf(d.y) * fabsf(fdot(d, nl));
    const float vv = fdot(d, d);
    return (num * C->nee_c) * spt_oracle_rcp_nr((t * t) * (vv * vv));
  }
}

typedef struct {
  uint64_t samples, path_rays, shadow_rays, vertices, nee_events, nee_light_hits, cosine_samples,
      misses, shadow_traced, sphere_vertices;
} c_stats;

/* A pending REFR branch (:494-495 at depth <= 2 returns reflection*Re + refraction*Tr): the
   refraction child is traced after the reflection subtree (depth-first), into the same L. */
typedef struct {
  fv o, d, T;
  int depth;
  uint32_t branch;
} c_node;

/* light_sampling :365-366 as built with glibc: x0 + rand()*dx/RAND_MAX with rand()*dx computed in
 * int32, which wraps. For dx = 2^a * odd (1 <= a <= 24) the wrapped product of
 * a uniform draw is uniform on the 2^(25-a) points x0 - 1 + m 2^(a-24), m in [0, 2^(25-a)) (an odd
 * factor permutes the residues), so contract v5 takes m from the top 25 - a bits of the Philox word:
 * fma(m, 2^(a-24), x0 - 1). (Rounds 1-4 multiplied a 24-bit draw by 2^7 dx and wrapped it: the same
 * lattice, points drawn in another order; the GPU's HEAD kernel now builds the float from the bits
 * with one or, dx = 36 = 4 * 9.) Odd dx keeps the rounds-1-4 arithmetic. */
static float c_wrap_sample(uint32_t r, uint32_t dx, float x0) {
  int a = 0;
  while (a < 32 && dx != 0 && !((dx >> a) & 1u)) a++;
  if (dx != 0 && a >= 1 && a <= 24) return fmaf((float)(r >> (7 + a)), ldexpf(1.0f, a - 24), x0 - 1.0f);
  return fmaf((float)(int32_t)(((r >> 8) << 7) * dx), 0x1p-31f, x0);
}

/* One path of the counter-mode contract; returns L. */
static fv c_path(const c_ctx* C, uint32_t pix, uint32_t s, int px, int py, const float cam[12],
                 c_stats* st) {
  const spt_params* P = C->P;
  uint32_t ctr[4], r[4], rl[4];
  fv o, d, T = fv3(1, 1, 1), L = fv3(0, 0, 0);
  int depth = 0, carried = 0, c_hit = 0, c_id = 0, sp = 0;
  uint32_t branch = 0; /* path-tree position: bit k-1 set = refraction child of the split at depth k */
  c_node stack[2];
  float c_t = 0;
  /* Camera ray :533-536. The jitter comes from the low bytes of vertex 1's Philox call (16 bits
   * each), so a sample start costs no extra RNG call; 1/w, 1/h are rounded once. */
  ctr[0] = pix; ctr[1] = s; ctr[2] = 1; ctr[3] = P->seed;
  c_philox(ctr, C->key, r);
  {
    /* Contract v5: d = llc + hor*su + ver*sv - origin with su = (x - 0.5 + ju 2^-16) / w,
     * sv = (h - y - 1 - 0.5 + jv 2^-16) / h (:533-536) as, per component c,
     *   fma(Fv, Cv_c, fma(Fu, Cu_c, P_c)),  Fu = 2^23 + ju, Fv = 2^23 + jv (exact floats),
     *   Au_c = hor_c * (1/w), Av_c = ver_c * (1/h), Cu_c = Au_c 2^-16, Cv_c = Av_c 2^-16,
     *   P_c = fma(Au_c, fx, fma(Av_c, fy, llc_c - origin_c)), fx = x - 0.5 - 128, fy = h-y-1-0.5 - 128
     * (the -128 cancels the 2^23 2^-16 = 128 inside Fu * Cu). P_c is per pixel: on the GPU a camera
     * ray costs one fma per component after the jitter bits (rounds 1-4: jitter, scale, fma chain,
     * subtract). */
    const float inv_w = 1.0f / (float)P->width, inv_h = 1.0f / (float)P->height;
    const float fx = ((float)px - 0.5f) - 128.0f, fy = ((float)(P->height - py - 1) - 0.5f) - 128.0f;
    const float Fu = asf(0x4B000000u | u16i(r[0], r[1])), Fv = asf(0x4B000000u | u16i(r[2], r[3]));
    float v[3];
    int c;
    for (c = 0; c < 3; c++) {
      const float Au = cam[6 + c] * inv_w, Av = cam[9 + c] * inv_h;
      const float Pc = fmaf(Au, fx, fmaf(Av, fy, cam[3 + c] - cam[c]));
      v[c] = fmaf(Fv, Av * 0x1p-16f, fmaf(Fu, Au * 0x1p-16f, Pc));
    }
    o = fv3(cam[0], cam[1], cam[2]);
    d = fv3(v[0], v[1], v[2]);
    d = C->unit ? fnormalize(d) : fnormalize_free(d);
  }
  st->samples++;
  for (;;) {
    int id = 0, hit;
    float t;
    fv x, nl, gn, f, e;
    const c_prim* H;
    if (carried) {
      hit = c_hit; t = c_t; id = hit ? c_id : 0;
      carried = 0;
    } else {
      hit = c_intersect(C, o, d, &t, &id);
      st->path_rays++;
    }
    H = &C->prims[id];
    if (!hit) { x = fv3(0, 0, 0); st->misses++; }
    else {
      /* hittingPoint :375 x = o + d*t with the plane distance re-derived as the reference does
       * (:103, (k - o_a)/d_a, one correctly rounded division per vertex, then mul + add): this
       * sets how often x lands beyond the plane, i.e. the reference's self-hit/leak rate. */
      float tr = t;
      if (H->kind == SPT_RECT_XY) tr = c_hit_t(H->k - o.z, d.z, t);
      else if (H->kind == SPT_RECT_XZ) tr = c_hit_t(H->k - o.y, d.y, t);
      else if (H->kind == SPT_RECT_YZ) tr = c_hit_t(H->k - o.x, d.x, t);
      x = fv3(o.x + d.x * tr, o.y + d.y * tr, o.z + d.z * tr);
    }
    st->vertices++;
    switch (H->kind) { /* gn: the unoriented (geometric) normal `n` of :482-491 */
      case SPT_RECT_XY: nl = d.z < 0.0f ? fv3(0, 0, 1) : fv3(0, 0, -1); gn = fv3(0, 0, 1); break;
      case SPT_RECT_XZ: nl = d.y < 0.0f ? fv3(0, 1, 0) : fv3(0, -1, 0); gn = fv3(0, 1, 0); break;
      case SPT_RECT_YZ: nl = d.x < 0.0f ? fv3(1, 0, 0) : fv3(-1, 0, 0); gn = fv3(1, 0, 0); break;
      default: {
        st->sphere_vertices++;
        /* Sphere::normal :248, (x - p).norm(), as (x - p) * (1/r): the hit point lies on the
         * sphere to ~1e-7, so this is the unit normal without a reciprocal square root */
        gn = fv3((x.x - H->px) * H->inv_r, (x.y - H->py) * H->inv_r, (x.z - H->pz) * H->inv_r);
        nl = fdot(gn, d) < 0.0f ? gn : fv3(-gn.x, -gn.y, -gn.z);
      }
    }
    f = H->c;
    e = H->e;
    ++depth;
    /* One Philox call per vertex: top 24 bits of r0..r3 = light x, light z, scatter xi1, xi2;
     * the low bytes form a 16-bit RR draw (r0, r1) and a 16-bit NEE-mix draw (r2, r3) — except at
     * vertex 1, whose low bytes were the camera jitter: its RR / NEE-mix draws (only needed when
     * rr_depth < 1 or 0 < nee_prob < 1) come from stream 1. */
    ctr[0] = pix; ctr[1] = s; ctr[2] = (uint32_t)depth | (branch << 24); ctr[3] = P->seed;
    c_philox(ctr, C->key, r);
    rl[0] = r[0]; rl[1] = r[1]; rl[2] = r[2]; rl[3] = r[3];
    if (depth == 1) {
      ctr[2] = 1u | 0x80000000u; /* stream 1 */
      c_philox(ctr, C->key, rl);
    }
    {
      const float p = H->pmax;
      int term = 0;
      if (P->max_depth > 0 && depth >= P->max_depth) term = 1;
      else if (!hit && C->leak_end) term = 1; /* a leaked path ends at its first miss (v6) */
      else if (depth > P->rr_depth || p == 0.0f) {
        if (!(p > 0.0f)) term = 1;
        else {
          int keep = 1;
          if (p < 1.0f) keep = u16(rl[0], rl[1]) < p;
          if (keep) {
            const float ip = 1.0f / p;
            f = fv3(f.x * ip, f.y * ip, f.z * ip);
          } else term = 1;
        }
      }
      if (term) {
        L = fv3(fmaf(T.x, e.x, L.x), fmaf(T.y, e.y, L.y), fmaf(T.z, e.z, L.z));
        if (sp > 0) { /* the pending refraction child of a REFR split */
          --sp;
          o = stack[sp].o; d = stack[sp].d; T = stack[sp].T;
          depth = stack[sp].depth; branch = stack[sp].branch;
          continue;
        }
        return L;
      }
    }
    if (H->refl != SPT_DIFF) {
      /* SPEC :481-482 and REFR :484-495 (smallpt's commented-out code, fp32): no NEE; the RR of
         :448 above already ran. reflRay direction r.d - n*2*n.dot(r.d), not renormalised. */
      const fv Tf = fv3(T.x * f.x, T.y * f.y, T.z * f.z);
      const float k2 = 2.0f * fdot(gn, d);
      const fv refl = fv3(d.x - gn.x * k2, d.y - gn.y * k2, d.z - gn.z * k2);
      L = fv3(fmaf(T.x, e.x, L.x), fmaf(T.y, e.y, L.y), fmaf(T.z, e.z, L.z));
      o = x;
      T = Tf;
      if (H->refl == SPT_REFR) {
        const int into = fdot(gn, nl) > 0.0f;                       /* :485 */
        const float nnt = into ? 1.0f / 1.5f : 1.5f / 1.0f;          /* nc=1, nt=1.5 :486 */
        const float ddn = fdot(d, nl);
        const float cos2t = 1.0f - nnt * nnt * (1.0f - ddn * ddn);
        if (!(cos2t < 0.0f)) {                                       /* else TIR :487-488 */
          const float kk = (into ? 1.0f : -1.0f) * (ddn * nnt + sqrtf(cos2t));
          const fv tdir = fnormalize(fv3(d.x * nnt - gn.x * kk, d.y * nnt - gn.y * kk,
                                         d.z * nnt - gn.z * kk));   /* :489 */
          const float a = 1.5f - 1.0f, b = 1.5f + 1.0f, R0 = a * a / (b * b);
          const float c = 1.0f - (into ? -ddn : fdot(tdir, gn));
          const float Re = R0 + (1.0f - R0) * c * c * c * c * c, Tr = 1.0f - Re;
          const float Pp = 0.25f + 0.5f * Re, RP = Re / Pp, TP = Tr / (1.0f - Pp);  /* :491 */
          if (depth > 2) { /* Russian roulette between the two :492-493 */
            if (u16(rl[2], rl[3]) < Pp) { T = fv3(Tf.x * RP, Tf.y * RP, Tf.z * RP); d = refl; }
            else { T = fv3(Tf.x * TP, Tf.y * TP, Tf.z * TP); d = tdir; }
          } else { /* both :494-495: reflection now, refraction later */
            stack[sp].o = x; stack[sp].d = tdir;
            stack[sp].T = fv3(Tf.x * Tr, Tf.y * Tr, Tf.z * Tr);
            stack[sp].depth = depth; stack[sp].branch = branch | (1u << (depth - 1));
            ++sp;
            T = fv3(Tf.x * Re, Tf.y * Re, Tf.z * Re);
            d = refl;
          }
          continue;
        }
      }
      d = refl;
      continue;
    }
    {
      int nee;
      float w = 1.0f;
      fv dn;
      if (P->nee_prob >= 1.0f) nee = 1;
      else if (P->nee_prob <= 0.0f) nee = 0;
      else nee = u16(rl[2], rl[3]) < P->nee_prob;
      if (nee) {
        float xl, zl, ts;
        int ids = id, sh;
        fv dl;
        if (P->light_mode == SPT_LIGHT_GLIBC_WRAP) {
          xl = c_wrap_sample(r[0], (uint32_t)P->light_dx, P->light_x0);
          zl = c_wrap_sample(r[1], (uint32_t)P->light_dz, P->light_z0);
        } else {
          xl = fmaf(u01(r[0]), P->light_dx, P->light_x0);
          zl = fmaf(u01(r[1]), P->light_dz, P->light_z0);
        }
        dl = fv3(xl - x.x, P->light_y - x.y, zl - x.z); /* light_vec :367 */
        if (C->unit) dl = fnormalize(dl);              /* else free-scale (c_unit_dirs) */
        if (id == P->light_id || c_light_accepts(C, x, dl)) st->shadow_traced++;
        sh = c_intersect(C, x, dl, &ts, &ids);
        if (g_proof_on) {
          float tl;
          if (c_early_nee_proven(C, x, dl, &tl)) {
            __atomic_fetch_add(&g_proof_n, 1, __ATOMIC_RELAXED);
            if (!sh || ids != P->light_id || asu(ts) != asu(tl))
              __atomic_fetch_add(&g_proof_bad, 1, __ATOMIC_RELAXED);
          } else if (g_proof_on == 1 && c_light_accepts(C, x, dl)) {
            c_shadow_census(C, x, dl, id, sh ? ids : -1);
          }
        }
        st->nee_events++;
        st->shadow_rays++;
        if (ids == P->light_id) {
          st->nee_light_hits++;
          w = c_nee_weight(C, dl, nl, ts);
          dn = dl;
          carried = 1; c_hit = sh; c_t = ts; c_id = ids;
        } else {
          dn = c_cosine(nl, r[2], r[3], (P->flags & SPT_FLAG_UNIFORM_SCATTER) != 0, C->unit);
          st->cosine_samples++;
        }
      } else {
        dn = c_cosine(nl, r[2], r[3], (P->flags & SPT_FLAG_UNIFORM_SCATTER) != 0, C->unit);
        st->cosine_samples++;
      }
      L = fv3(fmaf(T.x, e.x, L.x), fmaf(T.y, e.y, L.y), fmaf(T.z, e.z, L.z));
      T = fv3((T.x * f.x) * w, (T.y * f.y) * w, (T.z * f.z) * w);
      o = x;
      d = dn;
    }
  }
}

/* 1.31 fixed-point per-sample contribution: min(L/spp, 1) * 2^31 truncated, negatives -> 0
 * (fminf(NaN, 1) = 1). Integer sums are order-independent: results never depend on the GPU's
 * unit size, lane or queue order, or the GPU count. */
static inline uint64_t c_fix(float L, float inv_spp) {
  const float v = fminf(L * inv_spp, 1.0f) * 2147483648.0f;
  return v >= 0.0f ? (uint64_t)(uint32_t)v : 0u;
}

/* Contract: the fp32 plane coordinate of a rectangle. The reference has no epsilon on rectangles
 * (:103-106), so a hit point rounded to the far side of its plane self-hits and the path leaks out
 * of the room. How often the computed x = o + d*((k-o)/d) lands beyond k depends on the last
 * significand bit of k at the working precision (measured: odd 2.4 %, even 0.09 % of hits, in
 * fp32 and fp64 alike). k exactly representable in fp32: used as is (same statistics as fp64).
 * Otherwise the neighbouring float whose last significand bit equals the double's: (float)81.6
 * rounds to an odd significand where the double 81.6 is even, which made the fp32 ceiling leak 26x
 * as often as the reference's and darkened the image by 0.5 %. */
float spt_oracle_plane_k(double k) {
  const float f = (float)k;
  int e32, e64;
  double m32, m64;
  if ((double)f == k || !isfinite(k)) return f;
  m32 = frexp((double)f, &e32); /* f = m32 * 2^e32, 0.5 <= |m32| < 1 */
  m64 = frexp(k, &e64);
  {
    const uint32_t bit32 = (uint32_t)(uint64_t)ldexp(fabs(m32), 24) & 1u;
    const uint32_t bit64 = (uint32_t)(uint64_t)ldexp(fabs(m64), 53) & 1u;
    if (bit32 == bit64) return f;
  }
  return nextafterf(f, (double)f < k ? INFINITY : -INFINITY);
}

static void c_prims_from_spt(const spt_prim* s, int n, c_prim* out) {
  int i;
  for (i = 0; i < n; i++) {
    c_prim* P = &out[i];
    memset(P, 0, sizeof *P);
    P->kind = s[i].kind;
    if (s[i].kind == SPT_SPHERE) {
      P->rad2 = (float)s[i].geom[0] * (float)s[i].geom[0];
      P->px = (float)s[i].geom[1]; P->py = (float)s[i].geom[2]; P->pz = (float)s[i].geom[3];
      P->inv_r = 1.0f / (float)s[i].geom[0];
      P->wide = s[i].geom[0] >= SPT_WIDE_SPHERE_RADIUS;
      P->drad2 = s[i].geom[0] * s[i].geom[0];
      P->dpx = s[i].geom[1]; P->dpy = s[i].geom[2]; P->dpz = s[i].geom[3];
    } else {
      c_rect_mid(s[i].geom[0], s[i].geom[1], &P->ma, &P->ha);
      c_rect_mid(s[i].geom[2], s[i].geom[3], &P->mb, &P->hb);
      P->k = spt_oracle_plane_k(s[i].geom[4]);
    }
    P->e = fv3((float)s[i].e[0], (float)s[i].e[1], (float)s[i].e[2]);
    P->c = fv3((float)s[i].c[0], (float)s[i].c[1], (float)s[i].c[2]);
    P->pmax = P->c.x > P->c.y && P->c.x > P->c.z ? P->c.x : P->c.y > P->c.z ? P->c.y : P->c.z;
    P->refl = s[i].refl;
  }
}

/* Render the rows listed in rows[0..nrows) (image row indices, y=0 top) of the counter-mode contract.
 * rgb_out: nrows*w*3 floats. stats_out: 10 uint64 in spt_stats order (may be NULL).
 * threads <= 0: all OpenMP threads. Deterministic for any thread count. */
int spt_oracle_counter_render(const spt_prim* prims, int n, const spt_camera* cam,
                              const spt_params* P, const int32_t* rows, int nrows, float* rgb_out,
                              uint64_t* stats_out, int threads) {
  c_prim* CP;
  c_ctx C;
  c_test CT[64];
  float camf[12];
  const float inv_spp = 1.0f / (float)P->spp;
  c_stats tot;
  int i, ri;
  if (n <= 0 || n > 64) return -1; /* the C ABI's limit (spt_render: n_prims in [1, 64]) */
  CP = (c_prim*)malloc(sizeof(c_prim) * (size_t)n);
  memset(&tot, 0, sizeof tot);
  c_prims_from_spt(prims, n, CP);
  c_ctx_init(&C, prims, CP, n, P, CT);
  for (i = 0; i < 3; i++) {
    camf[i] = (float)cam->origin[i];
    camf[3 + i] = (float)cam->lower_left_corner[i];
    camf[6 + i] = (float)cam->horizontal[i];
    camf[9 + i] = (float)cam->vertical[i];
  }
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#else
  (void)threads;
#endif
#pragma omp parallel
  {
    c_stats st;
    memset(&st, 0, sizeof st);
#pragma omp for schedule(dynamic, 1)
    for (ri = 0; ri < nrows; ri++) {
      const int y = rows[ri];
      int x;
      for (x = 0; x < P->width; x++) {
        const uint32_t pix = (uint32_t)y * (uint32_t)P->width + (uint32_t)x;
        uint64_t acc[3] = {0, 0, 0};
        int s, ch;
        for (s = 0; s < P->spp; s++) {
          const fv L = c_path(&C, pix, (uint32_t)s, x, y, camf, &st);
          acc[0] += c_fix(L.x, inv_spp);
          acc[1] += c_fix(L.y, inv_spp);
          acc[2] += c_fix(L.z, inv_spp);
        }
        for (ch = 0; ch < 3; ch++) {
          float v = (float)acc[ch] * 0x1p-31f;
          rgb_out[((size_t)ri * (size_t)P->width + (size_t)x) * 3 + (size_t)ch] = v > 1.0f ? 1.0f : v;
        }
      }
    }
#pragma omp critical
    {
      tot.samples += st.samples; tot.path_rays += st.path_rays; tot.shadow_rays += st.shadow_rays;
      tot.vertices += st.vertices; tot.nee_events += st.nee_events;
      tot.nee_light_hits += st.nee_light_hits; tot.cosine_samples += st.cosine_samples;
      tot.misses += st.misses; tot.shadow_traced += st.shadow_traced;
      tot.sphere_vertices += st.sphere_vertices;
    }
  }
  if (stats_out) {
    stats_out[0] = tot.samples; stats_out[1] = tot.path_rays; stats_out[2] = tot.shadow_rays;
    stats_out[3] = tot.vertices; stats_out[4] = tot.nee_events; stats_out[5] = tot.nee_light_hits;
    stats_out[6] = tot.cosine_samples; stats_out[7] = tot.misses;
    stats_out[8] = tot.shadow_traced; stats_out[9] = tot.sphere_vertices;
  }
  free(CP);
  return 0;
}

/* The counter-mode contract at a list of pixels (pixel = y * w + x, any order): rgb_out npix*3
 * floats in list order, stats_out as spt_oracle_counter_render. Lets the GPU tests check a sample of
 * pixels of a full-workload render (C4/C5: 1024-4096 spp) in seconds. */
int spt_oracle_counter_render_pixels(const spt_prim* prims, int n, const spt_camera* cam,
                                     const spt_params* P, const uint32_t* pixels, int npix,
                                     float* rgb_out, uint64_t* stats_out, int threads) {
  c_prim* CP;
  c_ctx C;
  c_test CT[64];
  float camf[12];
  const float inv_spp = 1.0f / (float)P->spp;
  c_stats tot;
  int i, pi;
  if (n <= 0 || n > 64 || P->width <= 0) return -1;
  CP = (c_prim*)malloc(sizeof(c_prim) * (size_t)n);
  memset(&tot, 0, sizeof tot);
  c_prims_from_spt(prims, n, CP);
  c_ctx_init(&C, prims, CP, n, P, CT);
  for (i = 0; i < 3; i++) {
    camf[i] = (float)cam->origin[i];
    camf[3 + i] = (float)cam->lower_left_corner[i];
    camf[6 + i] = (float)cam->horizontal[i];
    camf[9 + i] = (float)cam->vertical[i];
  }
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#else
  (void)threads;
#endif
#pragma omp parallel
  {
    c_stats st;
    memset(&st, 0, sizeof st);
#pragma omp for schedule(dynamic, 1)
    for (pi = 0; pi < npix; pi++) {
      const uint32_t pix = pixels[pi];
      const int x = (int)(pix % (uint32_t)P->width), y = (int)(pix / (uint32_t)P->width);
      uint64_t acc[3] = {0, 0, 0};
      int s, ch;
      for (s = 0; s < P->spp; s++) {
        const fv L = c_path(&C, pix, (uint32_t)s, x, y, camf, &st);
        acc[0] += c_fix(L.x, inv_spp);
        acc[1] += c_fix(L.y, inv_spp);
        acc[2] += c_fix(L.z, inv_spp);
      }
      for (ch = 0; ch < 3; ch++) {
        const float v = (float)acc[ch] * 0x1p-31f;
        rgb_out[(size_t)pi * 3 + (size_t)ch] = v > 1.0f ? 1.0f : v;
      }
    }
#pragma omp critical
    {
      tot.samples += st.samples; tot.path_rays += st.path_rays; tot.shadow_rays += st.shadow_rays;
      tot.vertices += st.vertices; tot.nee_events += st.nee_events;
      tot.nee_light_hits += st.nee_light_hits; tot.cosine_samples += st.cosine_samples;
      tot.misses += st.misses; tot.shadow_traced += st.shadow_traced;
      tot.sphere_vertices += st.sphere_vertices;
    }
  }
  if (stats_out) {
    stats_out[0] = tot.samples; stats_out[1] = tot.path_rays; stats_out[2] = tot.shadow_rays;
    stats_out[3] = tot.vertices; stats_out[4] = tot.nee_events; stats_out[5] = tot.nee_light_hits;
    stats_out[6] = tot.cosine_samples; stats_out[7] = tot.misses;
    stats_out[8] = tot.shadow_traced; stats_out[9] = tot.sphere_vertices;
  }
  free(CP);
  return 0;
}

int spt_oracle_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ========================================================================================== */
/* Oracle-side scene / params (restated independently of the product's host helpers)           */
/* ========================================================================================== */

static void o_set(spt_prim* p, int kind, double a, double b, double c, double d, double k, double e,
                  double cr, double cg, double cb) {
  memset(p, 0, sizeof *p);
  p->kind = kind; p->refl = SPT_DIFF;
  p->geom[0] = a; p->geom[1] = b; p->geom[2] = c; p->geom[3] = d; p->geom[4] = k;
  p->e[0] = p->e[1] = p->e[2] = e;
  p->c[0] = cr; p->c[1] = cg; p->c[2] = cb;
}

/* rect[] of :287-311. */
int spt_oracle_scene_cornell(spt_prim* o) {
  o_set(&o[0], SPT_RECT_XY, 1, 99, 0, 81.6, 0, 0, .75, .75, .75);    /* Front  :288 */
  o_set(&o[1], SPT_RECT_XY, 1, 99, 0, 81.6, 170, 0, .75, .75, .75);  /* Back   :289 */
  o_set(&o[2], SPT_RECT_YZ, 0, 81.6, 0, 170, 1, 0, .25, .75, .25);   /* Left   :290 */
  o_set(&o[3], SPT_RECT_YZ, 0, 81.6, 0, 170, 99, 0, .75, .25, .25);  /* Right  :291 */
  o_set(&o[4], SPT_RECT_XZ, 1, 99, 0, 170, 0, 0, .75, .75, .75);     /* Bottom :292 */
  o_set(&o[5], SPT_RECT_XZ, 1, 99, 0, 170, 81.6, 0, .75, .75, .75);  /* Top    :293 */
  o_set(&o[6], SPT_RECT_XZ, 32, 68, 63, 96, 81.5, 12, 0, 0, 0);      /* Light  :294 */
  o_set(&o[7], SPT_RECT_XY, 12, 42, 0, 50, 32, 0, 1, 1, 1);          /* Tall box :300-304 */
  o_set(&o[8], SPT_RECT_XY, 12, 42, 0, 50, 62, 0, 1, 1, 1);
  o_set(&o[9], SPT_RECT_YZ, 0, 50, 32, 62, 12, 0, 1, 1, 1);
  o_set(&o[10], SPT_RECT_YZ, 0, 50, 32, 62, 42, 0, 1, 1, 1);
  o_set(&o[11], SPT_RECT_XZ, 12, 42, 32, 62, 50, 0, 1, 1, 1);
  o_set(&o[12], SPT_RECT_XY, 63, 88, 0, 25, 63, 0, 1, 1, 1);         /* Short box :306-310 */
  o_set(&o[13], SPT_RECT_XY, 63, 88, 0, 25, 88, 0, 1, 1, 1);
  o_set(&o[14], SPT_RECT_YZ, 0, 25, 63, 88, 63, 0, 1, 1, 1);
  o_set(&o[15], SPT_RECT_YZ, 0, 25, 63, 88, 88, 0, 1, 1, 1);
  o_set(&o[16], SPT_RECT_XZ, 63, 88, 63, 88, 25, 0, 1, 1, 1);
  return 17;
}

/* HEAD constants: :507-508 (512x512 @ 16), :464 (Q=1), :448 (5), :467 (6), :365-367, :471. */
void spt_oracle_default_params(spt_params* p) {
  memset(p, 0, sizeof *p);
  p->width = 512; p->height = 512; p->spp = 16; p->seed = 1;
  p->nee_prob = 1.0f; p->rr_depth = 5; p->max_depth = 0; p->light_id = 6;
  p->light_x0 = 32; p->light_dx = 36; p->light_z0 = 63; p->light_dz = 36;
  p->light_y = 81.6f; p->light_area = 1296; p->light_mode = SPT_LIGHT_GLIBC_WRAP;
  p->tile_rows = 8; p->shard_index = 0; p->shard_count = 1;
}

void spt_oracle_camera_spt(spt_camera* c, float aspect) {
  double v[12];
  const double lf[3] = {50, 40, 168}, la[3] = {50, 40, 5}, up[3] = {0, 1, 0};
  int i;
  spt_oracle_camera(v, lf, la, up, 65, aspect);
  for (i = 0; i < 3; i++) {
    c->origin[i] = v[i]; c->lower_left_corner[i] = v[3 + i];
    c->horizontal[i] = v[6 + i]; c->vertical[i] = v[9 + i];
  }
}
