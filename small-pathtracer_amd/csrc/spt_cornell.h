// spt_cornell.h — the reference's HEAD scene (rect[] of /root/reference/src/smallpt.cpp:287-311)
// as compile-time intersection geometry, in the kernel's grouped order (XY, XZ, YZ; index order
// inside a kind). The render kernel specialised on it reads every rectangle bound as an
// instruction literal: no scalar loads or waits in the intersect loop. The host runs that kernel
// only when the uploaded scene's grouped geometry equals this table bit for bit (spt_kernel.hip,
// cornell_const_match), so the table is an optimisation, never a substitute for the caller's scene.
#pragma once
#include <stdint.h>

namespace spt {

struct CRect { float k, ma, ha, mb, hb; int idx; };

// Same rounding as build_geo()/rect_mid() on the host: bounds rounded once from double.
constexpr CRect crect(double a1, double a2, double b1, double b2, double k, int idx) {
  return CRect{(float)k, (float)((a1 + a2) * 0.5), a2 >= a1 ? (float)((a2 - a1) * 0.5) : -1.0f,
               (float)((b1 + b2) * 0.5), b2 >= b1 ? (float)((b2 - b1) * 0.5) : -1.0f, idx};
}

// Rectangle_xy(x1,x2,y1,y2,z) :97-98; Rectangle_xz(x1,x2,z1,z2,y) :142; Rectangle_yz(y1,y2,z1,z2,x) :185
constexpr CRect kCornellRects[17] = {
    // XY (plane z): Front, Back, tall box z=32/62, short box z=63/88
    crect(1, 99, 0, 81.6, 0, 0), crect(1, 99, 0, 81.6, 170, 1), crect(12, 42, 0, 50, 32, 7),
    crect(12, 42, 0, 50, 62, 8), crect(63, 88, 0, 25, 63, 12), crect(63, 88, 0, 25, 88, 13),
    // XZ (plane y): Bottom, Top, Light, tall box top, short box top
    crect(1, 99, 0, 170, 0, 4), crect(1, 99, 0, 170, 81.6, 5), crect(32, 68, 63, 96, 81.5, 6),
    crect(12, 42, 32, 62, 50, 11), crect(63, 88, 63, 88, 25, 16),
    // YZ (plane x): Left, Right, tall box x=12/42, short box x=63/88
    crect(0, 81.6, 0, 170, 1, 2), crect(0, 81.6, 0, 170, 99, 3), crect(0, 50, 32, 62, 12, 9),
    crect(0, 50, 32, 62, 42, 10), crect(0, 25, 63, 88, 63, 14), crect(0, 25, 63, 88, 88, 15)};
constexpr int kCornellNXY = 6, kCornellNXZ = 5, kCornellNYZ = 6, kCornellLightPos = 8;

}  // namespace spt
