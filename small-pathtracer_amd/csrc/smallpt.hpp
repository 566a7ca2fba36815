// smallpt.hpp — C++ host mirror of the reference's host-side API over the C ABI (include/spt.h).
// A reference user keeps writing the same scene/camera code (same class names, constructor
// argument orders and semantics: /root/reference/src/smallpt.cpp:24-321) and calls render()
// where the reference ran its pixel loop (:528-542).
#pragma once
#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/spt.h"

namespace smallpt_amd {

struct Vec {  // :24-62
  double x, y, z;
  Vec(double x_ = 0, double y_ = 0, double z_ = 0) : x(x_), y(y_), z(z_) {}
  Vec operator+(const Vec& b) const { return Vec(x + b.x, y + b.y, z + b.z); }
  Vec operator-(const Vec& b) const { return Vec(x - b.x, y - b.y, z - b.z); }
  Vec operator*(double b) const { return Vec(x * b, y * b, z * b); }
  Vec mult(const Vec& b) const { return Vec(x * b.x, y * b.y, z * b.z); }
  Vec& norm() { return *this = *this * (1 / std::sqrt(x * x + y * y + z * z)); }
  double dot(const Vec& b) const { return x * b.x + y * b.y + z * b.z; }
  Vec operator%(const Vec& b) const { return Vec(y * b.z - z * b.y, z * b.x - x * b.z, x * b.y - y * b.x); }
};

enum Refl_t { DIFF = SPT_DIFF, SPEC = SPT_SPEC, REFR = SPT_REFR };  // :72-74

inline spt_prim make_prim(int kind, double a, double b, double c, double d, double k, Vec e, Vec col,
                          Refl_t refl) {
  spt_prim p{};
  p.kind = kind;
  p.refl = refl;
  p.geom[0] = a; p.geom[1] = b; p.geom[2] = c; p.geom[3] = d; p.geom[4] = k;
  p.e[0] = e.x; p.e[1] = e.y; p.e[2] = e.z;
  p.c[0] = col.x; p.c[1] = col.y; p.c[2] = col.z;
  return p;
}
// Constructors with the reference's argument orders (:97-98, :142, :185, :228).
inline spt_prim Rectangle_xz(double x1, double x2, double z1, double z2, double y, Vec e, Vec c, Refl_t r) {
  return make_prim(SPT_RECT_XZ, x1, x2, z1, z2, y, e, c, r);
}
inline spt_prim Rectangle_xy(double x1, double x2, double y1, double y2, double z, Vec e, Vec c, Refl_t r) {
  return make_prim(SPT_RECT_XY, x1, x2, y1, y2, z, e, c, r);
}
inline spt_prim Rectangle_yz(double y1, double y2, double z1, double z2, double x, Vec e, Vec c, Refl_t r) {
  return make_prim(SPT_RECT_YZ, y1, y2, z1, z2, x, e, c, r);
}
inline spt_prim Sphere(double rad, Vec p, Vec e, Vec c, Refl_t r) {
  return make_prim(SPT_SPHERE, rad, p.x, p.y, p.z, 0, e, c, r);
}

const Vec LOOKFROM = Vec(50, 40, 168);  // :65

class Camera {  // :256-285
 public:
  Camera(Vec lookfrom, Vec lookat, Vec vup, float vfov, float aspect) {
    const double lf[3] = {lookfrom.x, lookfrom.y, lookfrom.z};
    const double la[3] = {lookat.x, lookat.y, lookat.z};
    const double up[3] = {vup.x, vup.y, vup.z};
    if (spt_camera_init(&cam_, lf, la, up, vfov, aspect) != SPT_OK) throw std::runtime_error("camera");
    origin = Vec(cam_.origin[0], cam_.origin[1], cam_.origin[2]);
    lower_left_corner = Vec(cam_.lower_left_corner[0], cam_.lower_left_corner[1], cam_.lower_left_corner[2]);
    horizontal = Vec(cam_.horizontal[0], cam_.horizontal[1], cam_.horizontal[2]);
    vertical = Vec(cam_.vertical[0], cam_.vertical[1], cam_.vertical[2]);
  }
  Vec get_ray_dir(float s, float t) const {
    return lower_left_corner + horizontal * s + vertical * t - origin;
  }
  const spt_camera& abi() const { return cam_; }
  Vec origin, lower_left_corner, horizontal, vertical;

 private:
  spt_camera cam_{};
};

inline std::vector<spt_prim> cornell_scene() {  // rect[] :287-311
  return {
      Rectangle_xy(1, 99, 0, 81.6, 0, Vec(), Vec(.75, .75, .75), DIFF),      // Front
      Rectangle_xy(1, 99, 0, 81.6, 170, Vec(), Vec(.75, .75, .75), DIFF),    // Back
      Rectangle_yz(0, 81.6, 0, 170, 1, Vec(), Vec(.25, .75, .25), DIFF),     // Left
      Rectangle_yz(0, 81.6, 0, 170, 99, Vec(), Vec(.75, .25, .25), DIFF),    // Right
      Rectangle_xz(1, 99, 0, 170, 0, Vec(), Vec(.75, .75, .75), DIFF),       // Bottom
      Rectangle_xz(1, 99, 0, 170, 81.6, Vec(), Vec(.75, .75, .75), DIFF),    // Top
      Rectangle_xz(32, 68, 63, 96, 81.5, Vec(12, 12, 12), Vec(), DIFF),      // Light
      Rectangle_xy(12, 42, 0, 50, 32, Vec(), Vec(1, 1, 1), DIFF),            // Tall box
      Rectangle_xy(12, 42, 0, 50, 62, Vec(), Vec(1, 1, 1), DIFF),
      Rectangle_yz(0, 50, 32, 62, 12, Vec(), Vec(1, 1, 1), DIFF),
      Rectangle_yz(0, 50, 32, 62, 42, Vec(), Vec(1, 1, 1), DIFF),
      Rectangle_xz(12, 42, 32, 62, 50, Vec(), Vec(1, 1, 1), DIFF),
      Rectangle_xy(63, 88, 0, 25, 63, Vec(), Vec(1, 1, 1), DIFF),            // Short box
      Rectangle_xy(63, 88, 0, 25, 88, Vec(), Vec(1, 1, 1), DIFF),
      Rectangle_yz(0, 25, 63, 88, 63, Vec(), Vec(1, 1, 1), DIFF),
      Rectangle_yz(0, 25, 63, 88, 88, Vec(), Vec(1, 1, 1), DIFF),
      Rectangle_xz(63, 88, 63, 88, 25, Vec(), Vec(1, 1, 1), DIFF),
  };
}

// The HEAD room and light (:288-294) with smallpt's Mirr/Glas balls at :296-297 (SPEC / REFR).
inline std::vector<spt_prim> cornell_specular_scene() {
  std::vector<spt_prim> s = cornell_scene();
  s.resize(7);
  s.push_back(Sphere(16.5, Vec(27, 16.5, 47), Vec(), Vec(1, 1, 1) * .999, SPEC));  // Mirr
  s.push_back(Sphere(16.5, Vec(73, 16.5, 78), Vec(), Vec(1, 1, 1) * .999, REFR));  // Glas
  return s;
}

// The classic smallpt sphere box of the reference's older revision (the shipped image*.ppm; the
// constants of src/a.exe, spt_scene_smallpt_classic): 1e5-radius walls, light sphere = prim 8.
inline std::vector<spt_prim> smallpt_classic_scene() {
  std::vector<spt_prim> s(9);
  int32_t n = 0;
  spt_scene_smallpt_classic(s.data(), 9, &n);
  s.resize(n);
  return s;
}

// The same box with smallpt's mirror (SPEC) and glass (REFR) balls.
inline std::vector<spt_prim> smallpt_mirror_glass_scene() {
  std::vector<spt_prim> s(9);
  int32_t n = 0;
  spt_scene_smallpt_mirror_glass(s.data(), 9, &n);
  s.resize(n);
  return s;
}

// Config 5's 32-sphere scene (spt_scene_spheres32).
inline std::vector<spt_prim> spheres32_scene() {
  std::vector<spt_prim> s(64);
  int32_t n = 0;
  spt_scene_spheres32(s.data(), 64, &n);
  s.resize(n);
  return s;
}

inline double clamp(double x) { return x < 0 ? 0 : x > 1 ? 1 : x; }                 // :314-316
inline int toInt(double x) { return int(std::pow(clamp(x), 1 / 2.2) * 255 + .5); }  // :319-321

// P3 writer :548-551 (byte-identical output; this one also closes the file).
// The writer of :548-551 (ASCII P3, "%d %d %d " per pixel, toInt :319-321), encoded on the GPU
// (spt_write_image): byte-identical to the reference's fprintf loop. P6 / PFM via `format`.
inline int write_ppm(const char* path, int w, int h, const float* c, int device = 0,
                     int format = SPT_IMAGE_P3) {
  return spt_write_image(device, c, w, h, format, path) == SPT_OK ? 0 : 1;
}

// The drop-in for the pixel loop :528-542: linear clamped RGB, row-major, y=0 top.
inline std::vector<float> render(const std::vector<spt_prim>& scene, const Camera& cam,
                                 const spt_params& p, spt_stats* stats = nullptr) {
  std::vector<float> c(3ull * (size_t)spt_shard_rows(&p, nullptr, 0) * (size_t)p.width);
  const spt_status s = spt_render(scene.data(), (int32_t)scene.size(), &cam.abi(), &p, c.data(), stats);
  if (s != SPT_OK)
    throw std::runtime_error(std::string(spt_status_string(s)) + ": " + spt_last_error());
  return c;
}

// The same drop-in on several GPUs of one process: row tiles sharded over `devices`, one RCCL
// gather to devices[0] (spt_render_multi). Bit-identical to render().
inline std::vector<float> render_multi(const std::vector<spt_prim>& scene, const Camera& cam,
                                       const spt_params& p, const std::vector<int32_t>& devices,
                                       spt_stats* stats = nullptr) {
  std::vector<float> c(3ull * (size_t)p.height * (size_t)p.width);
  const spt_status s = spt_render_multi(scene.data(), (int32_t)scene.size(), &cam.abi(), &p,
                                        devices.data(), (int32_t)devices.size(), c.data(), stats);
  if (s != SPT_OK)
    throw std::runtime_error(std::string(spt_status_string(s)) + ": " + spt_last_error());
  return c;
}

}  // namespace smallpt_amd
