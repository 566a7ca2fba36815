// spt_host.cpp — host-side helpers of the C ABI (include/spt.h) that mirror the reference's
// host API: HEAD parameters, the Camera constructor, the rect[] scene, and the row-tile sharding.
#include <cmath>
#include <cstring>

#include "../../include/spt.h"

namespace {

void set_prim(spt_prim* p, int kind, double a, double b, double c, double d, double k, double e,
              double cr, double cg, double cb) {
  std::memset(p, 0, sizeof *p);
  p->kind = kind;
  p->refl = SPT_DIFF;
  p->geom[0] = a; p->geom[1] = b; p->geom[2] = c; p->geom[3] = d; p->geom[4] = k;
  p->e[0] = p->e[1] = p->e[2] = e;
  p->c[0] = cr; p->c[1] = cg; p->c[2] = cb;
}

struct V { double x, y, z; };
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V mul(V a, double b) { return {a.x * b, a.y * b, a.z * b}; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V norm(V a) { return mul(a, 1 / std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z)); }

}  // namespace

extern "C" spt_status spt_default_params(spt_params* p) {
  if (!p) return SPT_ERR_INVALID_ARG;
  std::memset(p, 0, sizeof *p);
  p->width = 512; p->height = 512; p->spp = 16;  // :507-508
  p->seed = 1;
  p->nee_prob = 1.0f;                             // :464 `q < 1`
  p->rr_depth = 5;                                // :448
  p->max_depth = 0;
  p->light_id = 6;                                // :467
  p->light_x0 = 32; p->light_dx = 36;             // :365
  p->light_z0 = 63; p->light_dz = 36;             // :366
  p->light_y = 81.6f;                             // :367
  p->light_area = 1296;                           // :471
  p->light_mode = SPT_LIGHT_GLIBC_WRAP;
  p->tile_rows = 8;
  p->shard_index = 0; p->shard_count = 1;
  p->chunk = 0; p->device = 0; p->flags = 0;
  return SPT_OK;
}

// Camera::Camera :262-275. theta and half_height are float; tan(float) is tanf under libstdc++.
extern "C" spt_status spt_camera_init(spt_camera* cam, const double lookfrom[3],
                                      const double lookat[3], const double vup[3], float vfov,
                                      float aspect) {
  if (!cam || !lookfrom || !lookat || !vup) return SPT_ERR_INVALID_ARG;
  const float theta = (float)(vfov * M_PI / 180);
  const float half_height = std::tan(theta / 2);
  const float half_width = aspect * half_height;
  const V origin{lookfrom[0], lookfrom[1], lookfrom[2]};
  const V w = norm(sub(V{lookat[0], lookat[1], lookat[2]}, origin));
  const V u = norm(cross(w, V{vup[0], vup[1], vup[2]}));
  const V v = cross(u, w);
  const V llc = add(sub(sub(origin, mul(u, half_width)), mul(v, half_height)), w);
  const V hor = mul(u, half_width * 2);
  const V ver = mul(v, half_height * 2);
  const V vals[4] = {origin, llc, hor, ver};
  double* outs[4] = {cam->origin, cam->lower_left_corner, cam->horizontal, cam->vertical};
  for (int i = 0; i < 4; ++i) {
    outs[i][0] = vals[i].x; outs[i][1] = vals[i].y; outs[i][2] = vals[i].z;
  }
  return SPT_OK;
}

// rect[] :287-311.
extern "C" spt_status spt_scene_cornell(spt_prim* o, int32_t cap, int32_t* n_out) {
  if (!o || !n_out || cap < 17) return SPT_ERR_INVALID_ARG;
  set_prim(&o[0], SPT_RECT_XY, 1, 99, 0, 81.6, 0, 0, .75, .75, .75);    // Front
  set_prim(&o[1], SPT_RECT_XY, 1, 99, 0, 81.6, 170, 0, .75, .75, .75);  // Back
  set_prim(&o[2], SPT_RECT_YZ, 0, 81.6, 0, 170, 1, 0, .25, .75, .25);   // Left
  set_prim(&o[3], SPT_RECT_YZ, 0, 81.6, 0, 170, 99, 0, .75, .25, .25);  // Right
  set_prim(&o[4], SPT_RECT_XZ, 1, 99, 0, 170, 0, 0, .75, .75, .75);     // Bottom
  set_prim(&o[5], SPT_RECT_XZ, 1, 99, 0, 170, 81.6, 0, .75, .75, .75);  // Top
  set_prim(&o[6], SPT_RECT_XZ, 32, 68, 63, 96, 81.5, 12, 0, 0, 0);      // Light
  set_prim(&o[7], SPT_RECT_XY, 12, 42, 0, 50, 32, 0, 1, 1, 1);          // Tall box
  set_prim(&o[8], SPT_RECT_XY, 12, 42, 0, 50, 62, 0, 1, 1, 1);
  set_prim(&o[9], SPT_RECT_YZ, 0, 50, 32, 62, 12, 0, 1, 1, 1);
  set_prim(&o[10], SPT_RECT_YZ, 0, 50, 32, 62, 42, 0, 1, 1, 1);
  set_prim(&o[11], SPT_RECT_XZ, 12, 42, 32, 62, 50, 0, 1, 1, 1);
  set_prim(&o[12], SPT_RECT_XY, 63, 88, 0, 25, 63, 0, 1, 1, 1);         // Short box
  set_prim(&o[13], SPT_RECT_XY, 63, 88, 0, 25, 88, 0, 1, 1, 1);
  set_prim(&o[14], SPT_RECT_YZ, 0, 25, 63, 88, 63, 0, 1, 1, 1);
  set_prim(&o[15], SPT_RECT_YZ, 0, 25, 63, 88, 88, 0, 1, 1, 1);
  set_prim(&o[16], SPT_RECT_XZ, 63, 88, 63, 88, 25, 0, 1, 1, 1);
  *n_out = 17;
  return SPT_OK;
}

// Config 5's build-defined scene: the room and light of :288-294 (light stays index 6, :467) and
// 32 DIFF spheres (r = 6, Sphere :223-254) on an 8 x 4 floor grid with a fixed colour table.
extern "C" spt_status spt_scene_spheres32(spt_prim* o, int32_t cap, int32_t* n_out) {
  if (!o || !n_out || cap < 39) return SPT_ERR_INVALID_ARG;
  int32_t n17 = 0;
  spt_prim room[17];
  spt_scene_cornell(room, 17, &n17);
  for (int i = 0; i < 7; ++i) o[i] = room[i];
  static const double pal[8][3] = {{.75, .25, .25}, {.25, .75, .25}, {.25, .25, .75}, {.75, .75, .25},
                                   {.25, .75, .75}, {.75, .25, .75}, {.9, .9, .9},   {.6, .45, .3}};
  int n = 7;
  for (int row = 0; row < 4; ++row) {
    for (int col = 0; col < 8; ++col) {
      spt_prim* p = &o[n];
      std::memset(p, 0, sizeof *p);
      p->kind = SPT_SPHERE;
      p->refl = SPT_DIFF;
      p->geom[0] = 6.0;                       // radius
      p->geom[1] = 1.0 + 98.0 * (col + 0.5) / 8.0;  // x
      p->geom[2] = 6.0;                       // resting on the floor y = 0
      p->geom[3] = 30.0 + 30.0 * row;         // z = 30, 60, 90, 120
      const double* c = pal[(row * 3 + col) % 8];
      p->c[0] = c[0]; p->c[1] = c[1]; p->c[2] = c[2];
      ++n;
    }
  }
  *n_out = n;
  return SPT_OK;
}

// smallpt's mirror and glass balls in the HEAD room: the room and light of :288-294 (light stays
// index 6) plus the two spheres commented out at :296-297 with smallpt's materials (Sphere
// (16.5, (27,16.5,47), c .999, SPEC) "Mirr" and (16.5, (73,16.5,78), c .999, REFR) "Glas"), whose
// shading is the commented-out SPEC/REFR code :481-495.
extern "C" spt_status spt_scene_cornell_specular(spt_prim* o, int32_t cap, int32_t* n_out) {
  if (!o || !n_out || cap < 9) return SPT_ERR_INVALID_ARG;
  int32_t n17 = 0;
  spt_prim room[17];
  spt_scene_cornell(room, 17, &n17);
  for (int i = 0; i < 7; ++i) o[i] = room[i];
  const double ctr[2][3] = {{27, 16.5, 47}, {73, 16.5, 78}};
  for (int k = 0; k < 2; ++k) {
    spt_prim* p = &o[7 + k];
    std::memset(p, 0, sizeof *p);
    p->kind = SPT_SPHERE;
    p->refl = k == 0 ? SPT_SPEC : SPT_REFR;
    p->geom[0] = 16.5;
    p->geom[1] = ctr[k][0]; p->geom[2] = ctr[k][1]; p->geom[3] = ctr[k][2];
    p->c[0] = p->c[1] = p->c[2] = .999;
  }
  *n_out = 9;
  return SPT_OK;
}

// The classic smallpt sphere box. The shipped image*.ppm of the reference's
// older revision show its two r = 16.5 balls as matte white DIFF spheres (colour .999, the .rdata
// constant); `mirror_glass` gives them smallpt's original SPEC / REFR materials instead.
static spt_status classic_box(spt_prim* o, int32_t cap, int32_t* n_out, bool mirror_glass) {
  if (!o || !n_out || cap < 9) return SPT_ERR_INVALID_ARG;
  struct S { double r, x, y, z, e, c0, c1, c2; int refl; };
  const int ball0 = mirror_glass ? SPT_SPEC : SPT_DIFF, ball1 = mirror_glass ? SPT_REFR : SPT_DIFF;
  const S sc[9] = {
      {1e5, 1e5 + 1, 40.8, 81.6, 0, .25, .75, .25, SPT_DIFF},   // left (green)
      {1e5, -1e5 + 99, 40.8, 81.6, 0, .75, .25, .25, SPT_DIFF}, // right (red)
      {1e5, 50, 40.8, 1e5, 0, .75, .75, .75, SPT_DIFF},         // back
      {1e5, 50, 40.8, -1e5 + 170, 0, 0, 0, 0, SPT_DIFF},        // front
      {1e5, 50, 1e5, 81.6, 0, .75, .75, .75, SPT_DIFF},         // floor
      {1e5, 50, -1e5 + 81.6, 81.6, 0, .75, .75, .75, SPT_DIFF}, // ceiling
      {16.5, 27, 16.5, 47, 0, .999, .999, .999, ball0},         // left ball (smallpt: mirror)
      {16.5, 73, 16.5, 78, 0, .999, .999, .999, ball1},         // right ball (smallpt: glass)
      {600, 50, 681.6 - .27, 81.6, 12, 0, 0, 0, SPT_DIFF}};     // light
  for (int k = 0; k < 9; ++k) {
    spt_prim* p = &o[k];
    std::memset(p, 0, sizeof *p);
    p->kind = SPT_SPHERE;
    p->refl = sc[k].refl;
    p->geom[0] = sc[k].r;
    p->geom[1] = sc[k].x; p->geom[2] = sc[k].y; p->geom[3] = sc[k].z;
    p->e[0] = p->e[1] = p->e[2] = sc[k].e;
    p->c[0] = sc[k].c0; p->c[1] = sc[k].c1; p->c[2] = sc[k].c2;
  }
  *n_out = 9;
  return SPT_OK;
}

extern "C" spt_status spt_scene_smallpt_classic(spt_prim* o, int32_t cap, int32_t* n_out) {
  return classic_box(o, cap, n_out, false);
}

extern "C" spt_status spt_scene_smallpt_mirror_glass(spt_prim* o, int32_t cap, int32_t* n_out) {
  return classic_box(o, cap, n_out, true);
}

// Row-tile sharding: tile t (rows [t*T, t*T+T)) belongs to shard t % shard_count; a shard's rows
// are listed in increasing order (the order of its compact output buffer).
extern "C" int32_t spt_shard_rows(const spt_params* p, int32_t* rows_out, int32_t cap) {
  if (!p || p->height <= 0 || p->shard_count < 1) return 0;
  const int T = p->tile_rows > 0 ? p->tile_rows : 8;
  int32_t n = 0;
  for (int tile = p->shard_index; tile * T < p->height; tile += p->shard_count) {
    for (int r = tile * T; r < tile * T + T && r < p->height; ++r) {
      if (rows_out && n < cap) rows_out[n] = r;
      ++n;
    }
  }
  return n;
}

int spt_shard_row_count(const spt_params* p) { return spt_shard_rows(p, nullptr, 0); }

extern "C" int32_t spt_abi_version(void) { return SPT_ABI_VERSION; }
#ifndef SPT_SOURCES_SHA16
#define SPT_SOURCES_SHA16 "unknown"
#endif
extern "C" const char* spt_build_sources_sha16(void) { return SPT_SOURCES_SHA16; }

extern "C" const char* spt_status_string(spt_status s) {
  switch (s) {
    case SPT_OK: return "ok";
    case SPT_ERR_INVALID_ARG: return "invalid argument";
    case SPT_ERR_HIP: return "HIP runtime error";
    case SPT_ERR_NO_DEVICE: return "no usable gfx950 device";
    case SPT_ERR_OOM: return "device out of memory";
    case SPT_ERR_UNSUPPORTED: return "unsupported feature";
    case SPT_ERR_RCCL: return "RCCL error";
  }
  return "unknown status";
}
