// wk_device.h -- register-resident 2-D rigid-body primitives (device side).
//
// Every polygon is a fixed-size register array (Poly<N>): all loops are unrolled
// with compile-time indices, so no per-env data ever spills to scratch.  Runtime
// vertex choices (significant vertex / face, ContactPoints.cs:79-113) are resolved
// with unrolled compare-select chains instead of indexed loads.
#pragma once
#include <float.h>
#include "wk_common.h"

namespace wk {

#define DEV __device__ __forceinline__

struct V2 { float x, y; };
DEV V2 mk(float x, float y) { V2 r; r.x = x; r.y = y; return r; }
DEV V2 vadd(V2 a, V2 b) { return mk(a.x + b.x, a.y + b.y); }
DEV V2 vsub(V2 a, V2 b) { return mk(a.x - b.x, a.y - b.y); }
DEV V2 vmul(V2 a, float s) { return mk(a.x * s, a.y * s); }
// MonoGame Vector2 operator /(Vector2, float): multiply by the reciprocal
DEV V2 vdiv(V2 a, float d) { float f = 1.0f / d; return mk(a.x * f, a.y * f); }
DEV V2 vneg(V2 a) { return mk(-a.x, -a.y); }
DEV float vdot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
DEV float vlen(V2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
DEV V2 vnormalize(V2 a) {
  float val = 1.0f / sqrtf(a.x * a.x + a.y * a.y);
  return mk(a.x * val, a.y * val);
}

// System.Math.Min/Max(float, float) (IEEE 754:2019 minimum/maximum)
DEV float net_minf(float x, float y) {
  if (x != y) { if (!__builtin_isnan(x)) return x < y ? x : y; return x; }
  return __builtin_signbit(x) ? x : y;
}
DEV float net_maxf(float x, float y) {
  if (x != y) { if (!__builtin_isnan(x)) return y < x ? x : y; return x; }
  return __builtin_signbit(y) ? x : y;
}

// Matrix.Clip(m, 1, -1) (Walker/PPO/Matrix.cs:377-405)
DEV float clip1(float x) {
  if (x >= 1.0f) return 1.0f;
  if (x <= -1.0f) return -1.0f;
  return x;
}

// RigidBody.WrapAngle (Bodies/RigidBody.cs:132-140): MathF.PI / MathF.Tau
DEV float wrap_angle(float a) {
  const float PI_F = 3.14159265358979323846f, TAU_F = 6.28318530717958647692f;
  if (a > PI_F) return a - TAU_F;
  if (a < -PI_F) return a + TAU_F;
  return a;
}

template <int N>
struct Poly {
  float x[N], y[N];
  float cx, cy;
};
struct Dyn { float vx, vy, w, th; };
struct Mat { float im, ii, e, mu; };
struct Body {
  float cx, cy;
  Dyn* d;
  float im, ii;
};

// Skeleton.FindCentroid (Skeleton.cs:100-113)
template <int N>
DEV void find_centroid(Poly<N>& p) {
  float sx = 0.0f, sy = 0.0f;
#pragma unroll
  for (int i = 0; i < N; i++) { sx = sx + p.x[i]; sy = sy + p.y[i]; }
  V2 c = vdiv(mk(sx, sy), (float)N);
  p.cx = c.x;
  p.cy = c.y;
}

// Environment.CreateFloor (Environment.cs:219-223); centroid (500, 975) exactly
DEV void floor_poly(Poly<4>& f) {
  f.x[0] = -50.0f;  f.y[0] = 1050.0f;
  f.x[1] = -50.0f;  f.y[1] = 900.0f;
  f.x[2] = 1050.0f; f.y[2] = 900.0f;
  f.x[3] = 1050.0f; f.y[3] = 1050.0f;
  find_centroid(f);
}

// Skeleton.Move (Skeleton.cs:76-85)
template <int N>
DEV void move(Poly<N>& p, V2 d) {
#pragma unroll
  for (int i = 0; i < N; i++) { p.x[i] = p.x[i] + d.x; p.y[i] = p.y[i] + d.y; }
  p.cx = p.cx + d.x;
  p.cy = p.cy + d.y;
}

// Skeleton.Rotate (Skeleton.cs:89-97): XNA CreateRotationZ uses (float)Math.Cos/Sin of
// the double-promoted angle; Vector2.Transform(p, M) = (p.x*M11 + p.y*M21 + M41, ...)
template <int N>
DEV void rotate(Poly<N>& p, float angle) {
  double sd, cd;
  sincos((double)angle, &sd, &cd);
  const float c = (float)cd, s = (float)sd;
  const float m11 = c, m12 = s, m21 = -s, m22 = c;
#pragma unroll
  for (int i = 0; i < N; i++) {
    float px = p.x[i] - p.cx, py = p.y[i] - p.cy;
    float tx = (px * m11) + (py * m21) + 0.0f;
    float ty = (px * m12) + (py * m22) + 0.0f;
    p.x[i] = tx + p.cx;
    p.y[i] = ty + p.cy;
  }
}

// BoundingBox.FindSignificantCorners + IsColliding (Skeleton.cs:133-176)
template <int N>
DEV void aabb(const Poly<N>& p, float& mnx, float& mny, float& mxx, float& mxy) {
  float maxX = -FLT_MAX, maxY = -FLT_MAX, minX = FLT_MAX, minY = FLT_MAX;
#pragma unroll
  for (int i = 0; i < N; i++) {
    if (p.x[i] > maxX) maxX = p.x[i];
    if (p.y[i] > maxY) maxY = p.y[i];
    if (p.x[i] < minX) minX = p.x[i];
    if (p.y[i] < minY) minY = p.y[i];
  }
  mnx = minX; mny = minY; mxx = maxX; mxy = maxY;
}
template <int NA, int NB>
DEV bool aabb_overlap(const Poly<NA>& a, const Poly<NB>& b) {
  float a0x, a0y, a1x, a1y, b0x, b0y, b1x, b1y;
  aabb(a, a0x, a0y, a1x, a1y);
  aabb(b, b0x, b0y, b1x, b1y);
  return a0x < b1x && a1x > b0x && a0y < b1y && a1y > b0y;
}

// ---------------- SAT (Bodies/Physics/SATCollision.cs:15-104) ----------------
template <int NA, int NB>
DEV void project2(float ax, float ay, const Poly<NA>& A, const Poly<NB>& B, float& amin,
                  float& amax, float& bmin, float& bmax) {
  amin = FLT_MAX; amax = -FLT_MAX; bmin = FLT_MAX; bmax = -FLT_MAX;
#pragma unroll
  for (int i = 0; i < NA; i++) {
    float p = ax * A.x[i] + ay * A.y[i];
    if (p < amin) amin = p;
    if (p > amax) amax = p;
  }
#pragma unroll
  for (int i = 0; i < NB; i++) {
    float p = ax * B.x[i] + ay * B.y[i];
    if (p < bmin) bmin = p;
    if (p > bmax) bmax = p;
  }
}

// AxisChecks(vectorA = P's edges, vectorB = Q): projections of P then Q on each axis
template <int NP, int NQ>
DEV bool axis_checks(const Poly<NP>& P, const Poly<NQ>& Q, V2& normal, float& depth) {
#pragma unroll
  for (int i = 0; i < NP; i++) {
    const int i1 = (i + 1) % NP;
    float ex = P.x[i1] - P.x[i], ey = P.y[i1] - P.y[i];
    V2 axis = mk(-ey, ex);
    if (axis.x == 0.0f && axis.y == 0.0f) continue;
    axis = vnormalize(axis);
    float pmin, pmax, qmin, qmax;
    project2(axis.x, axis.y, P, Q, pmin, pmax, qmin, qmax);
    float temp = net_minf(qmax - pmin, pmax - qmin);
    bool overlapping = (pmin < qmax) && (qmin < pmax);
    if (!overlapping) return false;
    if (temp >= depth) continue;
    depth = temp;
    normal = axis;
  }
  return true;
}

template <int NA, int NB>
DEV bool sat(const Poly<NA>& A, const Poly<NB>& B, V2& normal, float& depth) {
  normal = mk(0.0f, 0.0f);
  depth = FLT_MAX;
  bool result = axis_checks(A, B, normal, depth) && axis_checks(B, A, normal, depth);
  V2 dir = mk(B.cx - A.cx, B.cy - A.cy);
  if (vdot(dir, normal) > 0.0f) normal = vmul(normal, -1.0f);
  return result;
}

// ---------------- contact points (ContactPoints.cs:13-134) ----------------
// Runtime vertex select as a bit-mask OR over compile-time registers.  (A compare/select
// chain gets folded by LLVM into a load through a selected address, which pins the
// whole per-env state in scratch memory.)
template <int N>
DEV V2 pick(const Poly<N>& p, int i) {
  uint32_t bx = 0u, by = 0u;
#pragma unroll
  for (int k = 0; k < N; k++) {
    const uint32_t m = (i == k) ? 0xffffffffu : 0u;
    bx |= m & __float_as_uint(p.x[k]);
    by |= m & __float_as_uint(p.y[k]);
  }
  return mk(__uint_as_float(bx), __uint_as_float(by));
}

// GetSignificantFace (:79-94) with GetSignificantVertex (:97-113)
template <int N>
DEV void significant_face(const Poly<N>& P, V2 n, V2& fa, V2& fb, V2& fmax) {
  int index = -1;
  float mind = FLT_MAX;
#pragma unroll
  for (int i = 0; i < N; i++) {
    float p = P.x[i] * n.x + P.y[i] * n.y;
    if (p < mind) { index = i; mind = p; }
  }
  // index == -1 (all projections NaN / >= MaxValue) keeps Vector2.Zero as the vertex
  V2 sig = pick(P, index);
  const int ia = (index + 1) % N;
  const int ib = ((index - 1) % N + N) % N;  // ContactPoints.Mod (:131-134)
  V2 va = pick(P, ia), vb = pick(P, ib);
  V2 after = vnormalize(vsub(sig, va));
  V2 before = vnormalize(vsub(sig, vb));
  if (vdot(n, before) >= vdot(n, after)) { fa = sig; fb = vb; }
  else { fa = va; fb = sig; }
  fmax = sig;
}

// ClipVectors (:56-76)
DEV int clip_vectors(V2 a, V2 b, V2 n, float offset, V2& o0, V2& o1) {
  int cnt = 0;
  float da = vdot(a, n) - offset;
  float db = vdot(b, n) - offset;
  if (da >= 0.0f) { o0 = a; cnt = 1; }
  if (db >= 0.0f) { if (cnt == 0) o0 = b; else o1 = b; cnt++; }
  if (da * db < 0.0f) {
    V2 edge = vsub(b, a);
    float location = da / (da - db);
    edge = vmul(edge, location);
    edge = vadd(edge, a);
    if (cnt == 0) o0 = edge; else o1 = edge;
    cnt++;
  }
  return cnt;
}

template <int NA, int NB>
DEV int contact_points(const Poly<NA>& A, const Poly<NB>& B, V2 normal, V2& c0, V2& c1) {
  V2 ra, rb, rmax, ia, ib, imax;
  significant_face(A, normal, ra, rb, rmax);
  V2 rf = vsub(rb, ra);
  significant_face(B, vneg(normal), ia, ib, imax);
  V2 iv = vsub(ib, ia);
  if (fabsf(vdot(rf, normal)) > fabsf(vdot(iv, normal))) {
    V2 t;
    t = ra; ra = ia; ia = t;
    t = rb; rb = ib; ib = t;
    t = rmax; rmax = imax; imax = t;
    rf = vsub(rb, ra);
  }
  rf = vnormalize(rf);
  float offset = vdot(rf, ra);
  V2 p0 = mk(0.0f, 0.0f), p1 = mk(0.0f, 0.0f);
  if (clip_vectors(ia, ib, rf, offset, p0, p1) < 2) return 0;
  offset = vdot(rf, rb);
  V2 q0 = mk(0.0f, 0.0f), q1 = mk(0.0f, 0.0f);
  if (clip_vectors(p0, p1, vneg(rf), -offset, q0, q1) < 2) return 0;
  V2 refn = mk(rf.y, -rf.x);
  float maximum = vdot(refn, rmax);
  int cnt = 2;
  // List.Remove(First()) / Remove(Last()) (:42-50)
  if (vdot(refn, q0) - maximum < 0.0f) { q0 = q1; cnt = 1; }
  V2 last = cnt == 2 ? q1 : q0;
  if (vdot(refn, last) - maximum < 0.0f) {
    // Remove(Last()) deletes the first element equal to it: from [q0, q1] that leaves
    // q0's value (q1 itself, or q0 == q1); from [q1] it leaves nothing
    cnt = cnt == 2 ? 1 : 0;
  }
  c0 = q0;
  c1 = q1;
  return cnt;
}

// ---------------- impulses (Bodies/Physics/Impulses.cs:57-115) ----------------
DEV float calc_impulse(const Body& A, const Body& B, V2 contact, float force, V2 normal, V2& rA,
                       V2& rB) {
  rA = mk(contact.x - A.cx, contact.y - A.cy);
  V2 pA = mk(-rA.y, rA.x);
  float ctcA = vdot(normal, pA);
  rB = mk(contact.x - B.cx, contact.y - B.cy);
  V2 pB = mk(-rB.y, rB.x);
  float ctcB = vdot(normal, pB);
  V2 aVel = vadd(mk(A.d->vx, A.d->vy), vmul(pA, A.d->w));
  V2 bVel = vadd(mk(B.d->vx, B.d->vy), vmul(pB, B.d->w));
  V2 vel = vsub(bVel, aVel);
  float vdn = vdot(vel, normal);
  float j = -force * vdn;
  float denom = (A.im + B.im) + ((ctcA * ctcA) * A.ii) + ((ctcB * ctcB) * B.ii);
  return j / denom;
}

template <bool BSTATIC>
DEV void apply_impulses(Body& A, Body& B, V2 normal, float impulse, V2 rA, V2 rB) {
  V2 J = vmul(normal, impulse);
  V2 va = vsub(mk(A.d->vx, A.d->vy), vmul(J, A.im));
  A.d->vx = va.x;
  A.d->vy = va.y;
  if (!BSTATIC) {
    V2 vb = vadd(mk(B.d->vx, B.d->vy), vmul(J, B.im));
    B.d->vx = vb.x;
    B.d->vy = vb.y;
  }
  V2 pA = mk(-rA.y, rA.x);
  A.d->w = A.d->w - (vdot(pA, J) * A.ii);
  if (!BSTATIC) {
    V2 pB = mk(-rB.y, rB.x);
    B.d->w = B.d->w + (vdot(pB, J) * B.ii);
  }
}

}  // namespace wk
