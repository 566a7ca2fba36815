// spt_cornell.h — the reference's HEAD scene (rect[] of /root/reference/src/smallpt.cpp:287-311)
// as compile-time intersection geometry, in the kernel's grouped order (XY, XZ, YZ; index order
// inside a kind). The render kernel specialised on it reads every rectangle bound as an
// instruction literal: no scalar loads or waits in the intersect loop. The host runs that kernel
// only when the uploaded scene's grouped geometry equals this table bit for bit (spt_kernel.hip,
// cornell_const_match), so the table is an optimisation, never a substitute for the caller's scene.
#pragma once
#include <stdint.h>

namespace spt {

struct CRect {
  float k, ma, ha, mb, hb;
  int idx;
  double a1, a2, b1, b2, kd;  // the constructor's doubles (the room rule compares them exactly)
};

constexpr double pow2i(int e) {
  double r = 1;
  for (; e > 0; --e) r *= 2;
  for (; e < 0; ++e) r *= 0.5;
  return r;
}
constexpr int floor_log2(double a) {  // a > 0, finite
  int e = 0;
  for (; a >= 2; a *= 0.5) ++e;
  for (; a < 1; a *= 2) --e;
  return e;
}
// Last bit of the prec-bit significand of a normal a != 0.
constexpr unsigned last_sig_bit(double a, int prec) {
  a = a < 0 ? -a : a;
  return (unsigned)((unsigned long long)(a * pow2i(prec - 1 - floor_log2(a))) & 1ull);
}

// The contract's fp32 plane coordinate of a rectangle (oracle spt_oracle_plane_k):
// k itself when fp32 holds it exactly, otherwise the neighbouring float whose last significand bit
// equals the double's. The reference has no epsilon on rectangles (:103-106); how often a hit point
// rounds to the far side of its plane (and the path leaks out) follows that last bit — round-to-
// nearest (float)81.6 is odd where the double is even, and leaked 26x as often at the ceiling.
constexpr float plane_k(double k) {
  const float f = (float)k;
  if ((double)f == k || !(k - k == 0) || !(k > 0x1p-100 || k < -0x1p-100) || k > 0x1p100 ||
      k < -0x1p100)
    return f;
  if (last_sig_bit((double)f, 24) == last_sig_bit(k, 53)) return f;
  const double af = f < 0 ? -(double)f : (double)f;
  const bool outward = ((double)f < k) == (f > 0);  // step away from zero?
  double ulp = pow2i(floor_log2(af) - 23);
  if (!outward && af == pow2i(floor_log2(af))) ulp *= 0.5;  // below a power of two
  return (float)((double)f + ((double)f < k ? ulp : -ulp));
}
static_assert(plane_k(81.6) == 81.600006103515625f && plane_k(81.5) == 81.5f &&
                  plane_k(-81.6) == -81.600006103515625f && plane_k(0.1) == 0.099999994039535522f,
              "plane_k");

// Same rounding as build_geo()/rect_mid() on the host: bounds rounded once from double.
constexpr CRect crect(double a1, double a2, double b1, double b2, double k, int idx) {
  return CRect{plane_k(k), (float)((a1 + a2) * 0.5), a2 >= a1 ? (float)((a2 - a1) * 0.5) : -1.0f,
               (float)((b1 + b2) * 0.5), b2 >= b1 ? (float)((b2 - b1) * 0.5) : -1.0f, idx,
               a1, a2, b1, b2, k};
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
constexpr int cornell_pos_of(int idx) {
  for (int i = 0; i < 17; ++i)
    if (kCornellRects[i].idx == idx) return i;
  return -1;
}
constexpr int kCornellPosOfPrim0 = cornell_pos_of(0);  // Front (:288), XY
static_assert(kCornellPosOfPrim0 == 0, "prim 0 is the first XY rect");

// The contract's rect tests over the grouped list (oracle c_build_tests): inside each kind group,
// in order, a rectangle pairs with the first later unpaired one of bit-identical bounds on a
// different plane (never the light); singles have k0 == k1, pos0 == pos1. axis: 2 = z (XY),
// 1 = y (XZ), 0 = x (YZ). pos*: grouped positions.
struct CTest { float k0, k1, ma, ha, mb, hb; int pos0, pos1, axis; };
struct CTestList { CTest t[17]; int n; };
constexpr bool same_bits(float a, float b) { return a == b && (a != 0.0f || (1.0f / a == 1.0f / b)); }
constexpr CTestList cornell_tests() {
  CTestList L{};
  bool used[17] = {};
  const int grp[4] = {0, kCornellNXY, kCornellNXY + kCornellNXZ, kCornellNXY + kCornellNXZ + kCornellNYZ};
  for (int g = 0; g < 3; ++g) {
    for (int i = grp[g]; i < grp[g + 1]; ++i) {
      if (used[i]) continue;
      used[i] = true;
      const CRect& A = kCornellRects[i];
      CTest t{A.k, A.k, A.ma, A.ha, A.mb, A.hb, i, i, 2 - g};
      if (i != kCornellLightPos) {
        for (int j = i + 1; j < grp[g + 1]; ++j) {
          const CRect& B = kCornellRects[j];
          if (used[j] || j == kCornellLightPos || !same_bits(A.ma, B.ma) || !same_bits(A.ha, B.ha) ||
              !same_bits(A.mb, B.mb) || !same_bits(A.hb, B.hb) || same_bits(A.k, B.k))
            continue;
          used[j] = true;
          if (A.k < B.k) { t.k1 = B.k; t.pos1 = j; }
          else { t.k0 = B.k; t.pos0 = j; t.k1 = A.k; t.pos1 = i; }
          break;
        }
      }
      L.t[L.n++] = t;
    }
  }
  return L;
}
constexpr CTestList kCornellTests = cornell_tests();
static_assert(kCornellTests.n == 10, "HEAD scene: 7 parallel pairs + light + 2 box tops");

// The room of contract v5 (oracle c_find_room): the first XY, XZ, YZ pair tests (in test order)
// whose planes are exactly the other pairs' in-plane bounds. HEAD: Front/Back, Bottom/Top,
// Left/Right (:288-293).
constexpr bool same_range(double k1, double k2, double b1, double b2) {
  return (k1 < k2 ? k1 : k2) == b1 && (k1 < k2 ? k2 : k1) == b2;
}
struct CRoom { int t[3]; };  // tests (XY, XZ, YZ)
constexpr CRoom cornell_room() {
  CRoom R{{-1, -1, -1}};
  const CTestList& L = kCornellTests;
  for (int a = 0; a < L.n; ++a) {
    if (L.t[a].axis != 2 || L.t[a].pos0 == L.t[a].pos1) continue;
    for (int b = 0; b < L.n; ++b) {
      if (L.t[b].axis != 1 || L.t[b].pos0 == L.t[b].pos1) continue;
      for (int c = 0; c < L.n; ++c) {
        if (L.t[c].axis != 0 || L.t[c].pos0 == L.t[c].pos1) continue;
        const CRect& A0 = kCornellRects[L.t[a].pos0];  // XY: bounds x, y; planes z
        const CRect& A1 = kCornellRects[L.t[a].pos1];
        const CRect& B0 = kCornellRects[L.t[b].pos0];  // XZ: bounds x, z; planes y
        const CRect& B1 = kCornellRects[L.t[b].pos1];
        const CRect& D0 = kCornellRects[L.t[c].pos0];  // YZ: bounds y, z; planes x
        const CRect& D1 = kCornellRects[L.t[c].pos1];
        // bounds from each pair's k0 member (the oracle's c_test.id0)
        if (!same_range(D0.kd, D1.kd, A0.a1, A0.a2) || !same_range(D0.kd, D1.kd, B0.a1, B0.a2) ||
            !same_range(B0.kd, B1.kd, A0.b1, A0.b2) || !same_range(B0.kd, B1.kd, D0.a1, D0.a2) ||
            !same_range(A0.kd, A1.kd, B0.b1, B0.b2) || !same_range(A0.kd, A1.kd, D0.b1, D0.b2))
          continue;
        R.t[0] = a; R.t[1] = b; R.t[2] = c;
        return R;
      }
    }
  }
  return R;
}
constexpr CRoom kCornellRoomDef = cornell_room();
constexpr int kCornellRoom[3] = {kCornellRoomDef.t[0], kCornellRoomDef.t[1], kCornellRoomDef.t[2]};
static_assert(kCornellRoom[0] == 0 && kCornellRoom[1] == 3 && kCornellRoom[2] == 7,
              "HEAD room: Front/Back, Bottom/Top, Left/Right");

// The boxes of contract v6 (oracle c_find_boxes): an XY pair, a YZ pair and an XZ top (none of
// them the room's, the top not the light) closing a box that stands on the room's floor and lies
// inside its bounds, compared on the constructor's doubles; searched in test order. HEAD: the tall
// and the short box (:298-308).
struct CBoxes { int n; int t[4][3]; };  // tests: XY pair (planes z), YZ pair (planes x), XZ top
constexpr CBoxes cornell_boxes() {
  CBoxes B{};
  const CTestList& L = kCornellTests;
  bool used[17] = {};
  const CRect& F0 = kCornellRects[L.t[kCornellRoom[1]].pos0];  // the floor: the room's lower XZ plane
  const CRect& F1 = kCornellRects[L.t[kCornellRoom[1]].pos1];
  const double floor_k = F0.kd < F1.kd ? F0.kd : F1.kd;
  for (int a = 0; a < L.n; ++a) {
    const CTest& A = L.t[a];
    if (A.axis != 2 || A.pos0 == A.pos1 || a == kCornellRoom[0] || used[a]) continue;
    for (int b = 0; b < L.n && !used[a]; ++b) {
      const CTest& D = L.t[b];
      if (D.axis != 0 || D.pos0 == D.pos1 || b == kCornellRoom[2] || used[b]) continue;
      for (int c = 0; c < L.n; ++c) {
        const CTest& T = L.t[c];
        if (T.axis != 1 || T.pos0 != T.pos1 || T.pos0 == kCornellLightPos || used[c]) continue;
        const CRect &A0 = kCornellRects[A.pos0], &A1 = kCornellRects[A.pos1];
        const CRect &D0 = kCornellRects[D.pos0], &D1 = kCornellRects[D.pos1], &T0 = kCornellRects[T.pos0];
        if (!same_range(D0.kd, D1.kd, A0.a1, A0.a2) || !same_range(D0.kd, D1.kd, T0.a1, T0.a2) ||
            !same_range(A0.kd, A1.kd, D0.b1, D0.b2) || !same_range(A0.kd, A1.kd, T0.b1, T0.b2) ||
            !same_range(floor_k, T0.kd, A0.b1, A0.b2) || !same_range(floor_k, T0.kd, D0.a1, D0.a2) ||
            !(T0.kd > floor_k))
          continue;
        if (!(F0.a1 <= A0.a1 && A0.a2 <= F0.a2 && F0.b1 <= D0.b1 && D0.b2 <= F0.b2)) continue;
        used[a] = used[b] = used[c] = true;
        B.t[B.n][0] = a; B.t[B.n][1] = b; B.t[B.n][2] = c;
        ++B.n;
        break;
      }
    }
  }
  return B;
}
constexpr CBoxes kCornellBoxes = cornell_boxes();
static_assert(kCornellBoxes.n == 2 && kCornellBoxes.t[0][0] == 1 && kCornellBoxes.t[0][1] == 8 &&
                  kCornellBoxes.t[0][2] == 5 && kCornellBoxes.t[1][0] == 2 &&
                  kCornellBoxes.t[1][1] == 9 && kCornellBoxes.t[1][2] == 6,
              "HEAD boxes: tall (z 32/62, x 12/42, top 50), short (z 63/88, x 63/88, top 25)");
constexpr bool cornell_in_box(int j) {
  for (int b = 0; b < kCornellBoxes.n; ++b)
    for (int r = 0; r < 3; ++r)
      if (kCornellBoxes.t[b][r] == j) return true;
  return false;
}

}  // namespace spt
