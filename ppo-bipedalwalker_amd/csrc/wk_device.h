// wk_device.h -- register-resident 2-D rigid-body primitives (device side).
//
// Every polygon is a fixed-size register array (Poly<N>): all loops are unrolled
// with compile-time indices, so no per-env data ever spills to scratch.  Runtime
// vertex choices (significant vertex / face, ContactPoints.cs:79-113) are resolved
// with unrolled compare-select chains instead of indexed loads.
#pragma once
#include <float.h>
#include "wk_common.h"
#include "wk_sincos_small.h"


namespace wk {

#define DEV __device__ __forceinline__

struct V2 { float x, y; };
typedef float pf2 __attribute__((ext_vector_type(2)));
DEV V2 mk(float x, float y) { V2 r; r.x = x; r.y = y; return r; }
DEV V2 vadd(V2 a, V2 b) { return mk(a.x + b.x, a.y + b.y); }
DEV V2 vsub(V2 a, V2 b) { return mk(a.x - b.x, a.y - b.y); }
DEV V2 vmul(V2 a, float s) { return mk(a.x * s, a.y * s); }
// MonoGame Vector2 operator /(Vector2, float): multiply by the reciprocal
DEV V2 vdiv(V2 a, float d) { float f = 1.0f / d; return mk(a.x * f, a.y * f); }
DEV V2 vneg(V2 a) { return mk(-a.x, -a.y); }
DEV float vdot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
// Correctly rounded sqrt / reciprocal without the library's rescaling and special-value
// fixups.  For x in [2^-96, 2^126] HIP's sqrtf (v_sqrt_f32 plus a one-ulp round-to-nearest
// correction) equals sqrt_core below; for a divisor in [2^-48, 2^64] the reciprocal
// needs only v_rcp_f32 and one Newton step (rcp_core).  Both are checked bit for bit
// against sqrtf and 1.0f/x over every non-negative float (tests/cpp/fastmath_check.hip).
// Inputs outside [2^-96, 2^126] (never produced by walker-scale geometry) take the
// library path.
// On [2^-96, 2^126] the correctly rounded sqrt is also v_rsq_f32 y, s0 = x y and one FMA
// correction s0 + (x - s0^2) (y / 2): 5 instructions instead of HIP's 9 (v_sqrt_f32 and
// both neighbours' residuals).  Exhaustive: scripts/probe/sqrt_variants.hip, and the GPU
// test's tests/cpp/fastmath_check.hip.
DEV float sqrt_core(float x) {
  const float y = __builtin_amdgcn_rsqf(x);
  const float s0 = x * y;
  const float e = __builtin_fmaf(-s0, s0, x);
  return __builtin_fmaf(e, 0.5f * y, s0);
}
// v_rcp_f32 plus one Newton-Raphson step already equals the correctly rounded 1/d on
// the whole domain (exhaustive: scripts/probe/fastmath_variants.hip, and the GPU test)
DEV float rcp_core(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}
DEV bool fast_domain(float x) { return x >= 0x1p-96f && x <= 0x1p126f; }
DEV float sqrt_rn(float x) {
  if (__builtin_expect(!fast_domain(x), 0)) return sqrtf(x);
  return sqrt_core(x);
}
// 1.0f / sqrtf(x) with both roundings
DEV float rsqrt_rn(float x) {
  if (__builtin_expect(!fast_domain(x), 0)) return 1.0f / sqrtf(x);
  return rcp_core(sqrt_core(x));
}
// Normalize for an edge of a walker polygon or the floor: rigid bodies keep their edge
// lengths (7.5 .. 1100), so |e|^2 is inside the fast domain for every finite state and
// the guard branch is dropped; a zero edge (masked by the caller) or a non-finite state
// (already a fault) are the only inputs outside it.
DEV V2 vnormalize_edge(V2 a) {
  const float val = rcp_core(sqrt_core(a.x * a.x + a.y * a.y));
  return mk(a.x * val, a.y * val);
}
DEV float vlen(V2 a) { return sqrt_rn(a.x * a.x + a.y * a.y); }
DEV V2 vnormalize(V2 a) {
  float val = rsqrt_rn(a.x * a.x + a.y * a.y);
  return mk(a.x * val, a.y * val);
}

// System.Math.Min/Max(float, float) (IEEE 754:2019 minimum/maximum: a NaN operand gives
// NaN, -0 < +0).  gfx950 has them as one instruction (v_minimum3_f32 / v_maximum3_f32); the
// compare-and-select restatement (the oracle's net_minf) compiled to two branches.
DEV float net_minf(float x, float y) { return __builtin_elementwise_minimum(x, y); }
DEV float net_maxf(float x, float y) { return __builtin_elementwise_maximum(x, y); }

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
  const pf2 dx = {d.x, d.x}, dy = {d.y, d.y};
#pragma unroll
  for (int i = 0; i + 1 < N; i += 2) {
    const pf2 x = pf2{p.x[i], p.x[i + 1]} + dx, y = pf2{p.y[i], p.y[i + 1]} + dy;
    p.x[i] = x.x; p.x[i + 1] = x.y; p.y[i] = y.x; p.y[i + 1] = y.y;
  }
  if (N & 1) { p.x[N - 1] = p.x[N - 1] + d.x; p.y[N - 1] = p.y[N - 1] + d.y; }
  p.cx = p.cx + d.x;
  p.cy = p.cy + d.y;
}

// Skeleton.Rotate (Skeleton.cs:89-97): XNA CreateRotationZ uses (float)Math.Cos/Sin of
// the double-promoted angle; Vector2.Transform(p, M) = (p.x*M11 + p.y*M21 + M41, ...)
// |angle| <= 0.25 (every substep rotation in practice: w * dt with dt = 1/3000 s) takes
// the short Taylor form, proven equal after the (float) rounding to the C library's
// sin / cos for every float in range (tests/cpp/sincos_small_check.c, exhaustive).
template <int N>
DEV void rotate(Poly<N>& p, float angle) {
  double sd, cd;
  if (__builtin_fabsf(angle) <= 0.25f) wk_sincos_small((double)angle, &sd, &cd);
  else sincos((double)angle, &sd, &cd);
  const float c = (float)cd, s = (float)sd;
  const float m11 = c, m12 = s, m21 = -s, m22 = c;
  const pf2 cx = {p.cx, p.cx}, cy = {p.cy, p.cy}, z2 = {0.0f, 0.0f};
  const pf2 a11 = {m11, m11}, a12 = {m12, m12}, a21 = {m21, m21}, a22 = {m22, m22};
#pragma unroll
  for (int i = 0; i + 1 < N; i += 2) {
    const pf2 px = pf2{p.x[i], p.x[i + 1]} - cx, py = pf2{p.y[i], p.y[i + 1]} - cy;
    const pf2 tx = ((px * a11) + (py * a21)) + z2;
    const pf2 ty = ((px * a12) + (py * a22)) + z2;
    const pf2 x = tx + cx, y = ty + cy;
    p.x[i] = x.x; p.x[i + 1] = x.y; p.y[i] = y.x; p.y[i + 1] = y.y;
  }
  if (N & 1) {
    const int i = N - 1;
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
  // IsColliding only compares these, so v_max/v_min (which may pick the other signed
  // zero of a +0/-0 tie) give the same verdict as the sequential compare-and-replace
  float maxX = -FLT_MAX, maxY = -FLT_MAX, minX = FLT_MAX, minY = FLT_MAX;
#pragma unroll
  for (int i = 0; i < N; i++) {
    maxX = __builtin_fmaxf(maxX, p.x[i]);
    maxY = __builtin_fmaxf(maxY, p.y[i]);
    minX = __builtin_fminf(minX, p.x[i]);
    minY = __builtin_fminf(minY, p.y[i]);
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
  // min/max by value (v_min/v_max): a +0/-0 tie may keep the other zero than the
  // sequential compare-and-replace, which cannot change AxisChecks -- an overlapping
  // axis has bmax - amin > 0 and amax - bmin > 0, so no zero reaches depth.
  amin = FLT_MAX; amax = -FLT_MAX; bmin = FLT_MAX; bmax = -FLT_MAX;
#pragma unroll
  for (int i = 0; i < NA; i++) {
    float p = ax * A.x[i] + ay * A.y[i];
    amin = __builtin_fminf(amin, p);
    amax = __builtin_fmaxf(amax, p);
  }
#pragma unroll
  for (int i = 0; i < NB; i++) {
    float p = ax * B.x[i] + ay * B.y[i];
    bmin = __builtin_fminf(bmin, p);
    bmax = __builtin_fmaxf(bmax, p);
  }
}

// Projection of a polygon on an axis, min and max by value (see project2).  Vertex pairs go
// through v_pk_mul_f32 / v_pk_add_f32: two IEEE fp32 products / sums per instruction, the
// same per-element operations as ax * x + ay * y (no FMA: -ffp-contract=off).  Measured
// (bench A/B on one box): -2 % rollout time; Skeleton.Move / Rotate over vertex pairs
// (move, rotate) another -0.7 %; packing per (x, y) pair instead cost +25 % (register
// shuffles), packing the contact-face projections changed nothing.
template <int N>
DEV void proj_minmax(const Poly<N>& P, float ax, float ay, float& mn, float& mx) {
  float v[N];
  const pf2 a2 = {ax, ax}, b2 = {ay, ay};
#pragma unroll
  for (int i = 0; i + 1 < N; i += 2) {
    const pf2 q = (a2 * pf2{P.x[i], P.x[i + 1]}) + (b2 * pf2{P.y[i], P.y[i + 1]});
    v[i] = q.x;
    v[i + 1] = q.y;
  }
  if (N & 1) v[N - 1] = ax * P.x[N - 1] + ay * P.y[N - 1];
  mn = FLT_MAX; mx = -FLT_MAX;
#pragma unroll
  for (int i = 0; i < N; i++) { mn = __builtin_fminf(mn, v[i]); mx = __builtin_fmaxf(mx, v[i]); }
}

// P's projections onto P's OWN edge axis I, when P is a walker pole (Pole.FromSize,
// Objects/RigidBodies/Pole.cs:18-34: vertices (a, h) (0, h) (-a, h) (-a, -h) (0, -h) (a, -h)
// about the centroid, a = 7.5, h = 26.25, moved and rotated rigidly).  Axis I = Normalize((-e.y,
// e.x)) of edge I is the inward normal, so the edge's own vertices (and the ones collinear with
// it) are the minimum and the opposite edge's vertices the maximum: for edges 0 / 1 min over
// {0, 1, 2} and max over {3, 4, 5}, for 3 / 4 the reverse, for edge 2 min over {2, 3} and max
// over {5, 0}, for edge 5 the reverse.  Every other vertex is at least a = 7.5 px (the
// midpoints 1, 4 for the short edges) from the group it is left out of, while the projections
// carry ~1e-4 px of rounding and a rigid body's vertices drift from their shape by rounding only
// (<< 1 px over the 50,000 substeps of the longest episode; a reset rebuilds the template), so
// the minimum / maximum over the group is the minimum / maximum over all six, bit for bit --
// 2 min/max instructions instead of 6 per own axis (12 own axes per leg-leg SAT).
// (I: the edge index, a constant once the axis loop is unrolled)
DEV void pole_own_minmax(const Poly<6>& P, int I, float ax, float ay, float& mn, float& mx) {
  float v[6];
  const pf2 a2 = {ax, ax}, b2 = {ay, ay};
#pragma unroll
  for (int i = 0; i < 6; i += 2) {
    const pf2 q = (a2 * pf2{P.x[i], P.x[i + 1]}) + (b2 * pf2{P.y[i], P.y[i + 1]});
    v[i] = q.x;
    v[i + 1] = q.y;
  }
  if (I == 0 || I == 1) {
    mn = __builtin_fminf(__builtin_fminf(v[0], v[1]), v[2]);
    mx = __builtin_fmaxf(__builtin_fmaxf(v[3], v[4]), v[5]);
  } else if (I == 3 || I == 4) {
    mn = __builtin_fminf(__builtin_fminf(v[3], v[4]), v[5]);
    mx = __builtin_fmaxf(__builtin_fmaxf(v[0], v[1]), v[2]);
  } else if (I == 2) {
    mn = __builtin_fminf(v[2], v[3]);
    mx = __builtin_fmaxf(v[5], v[0]);
  } else {
    mn = __builtin_fminf(v[5], v[0]);
    mx = __builtin_fmaxf(v[2], v[3]);
  }
}

// AxisChecks(vectorA = P's edges, vectorB = Q): projections of P then Q on each axis.
// Branch-free: every axis is evaluated -- the loop's early `return false` only cuts
// short a result whose normal / depth the caller discards -- a zero-length edge is
// skipped by predication, and the first strict minimum wins exactly as in the loop.
// (On an overlapping axis both differences are > 0, so Math.Min == v_min there.)
// (Packing two axes per instruction measured 1.7x slower -- each packed result needed a
// wait state before use; two vertices per instruction, proj_minmax, is the packing kept.)
// FLOORQ: Q is the flat floor box {x in (-50, 1050)} x {y in (900, 1050)}, all four
// corner combinations.  Round-to-nearest addition is monotonic in each operand, so
// min over corners of fl(fl(ax x) + fl(ay y)) = fl(min_x fl(ax x) + min_y fl(ay y)) (and
// likewise max): the box projects in 4 products, 2 min, 2 max, 2 adds instead of a
// 4-vertex loop -- the same values (a zero's sign aside, which no overlapping axis sees).
//
// Verdict algebra: fl(a - b) > 0 iff a > b, so a finite axis overlaps iff temp =
// min(qmax - pmin, pmax - qmin) > 0, and a NaN temp (Math.Min propagates it; IsOverlapping's
// compares are then false) separates and keeps depth NaN (see below); and a depth or
// normal is only ever used when no axis separates, so an axis may be taken on temp < depth
// alone -- whenever a separating axis exists the caller discards both.  ZE: P may have a
// zero edge (a rough-floor segment); a walker polygon's rigid edges never vanish.
//
// AX (optional): the normalised axes, kept for the contact faces (see EdgeAxes).
template <int N> struct EdgeAxes { float x[N], y[N]; };
// NE: only P's first NE edges (the quad mapping's halves of an axis list).
// POLE: P is a walker pole in its template vertex order (or that order rotated by 3, see
// sat_floor_split): its own projections use pole_own_minmax.
template <int NP, int NQ, bool FLOORQ = false, bool ZE = false, int NE = NP, bool POLE = false>
DEV void axis_pass(const Poly<NP>& P, const Poly<NQ>& Q, bool& sep, V2& normal, float& depth,
                   EdgeAxes<NP>* AX = nullptr) {
  static_assert(!POLE || NP == 6, "pole vertex groups");
#pragma unroll
  for (int i = 0; i < NE; i++) {
    const int i1 = (i + 1) % NP;
    const float ex = P.x[i1] - P.x[i], ey = P.y[i1] - P.y[i];
    V2 axis = mk(-ey, ex);
    const bool valid = !ZE || !(axis.x == 0.0f && axis.y == 0.0f);
    axis = vnormalize_edge(axis);  // garbage for a zero edge: masked by `valid`
    if (AX) { AX->x[i] = axis.x; AX->y[i] = axis.y; }
    float pmin, pmax, qmin, qmax;
    if constexpr (POLE) pole_own_minmax(P, i, axis.x, axis.y, pmin, pmax);
    else proj_minmax(P, axis.x, axis.y, pmin, pmax);
    if constexpr (FLOORQ) {
      const float x0 = axis.x * -50.0f, x1 = axis.x * 1050.0f;
      const float y0 = axis.y * 900.0f, y1 = axis.y * 1050.0f;
      qmin = __builtin_fminf(x0, x1) + __builtin_fminf(y0, y1);
      qmax = __builtin_fmaxf(x0, x1) + __builtin_fmaxf(y0, y1);
    } else {
      proj_minmax(Q, axis.x, axis.y, qmin, qmax);
    }
    const float temp = net_minf(qmax - pmin, pmax - qmin);
    // (no per-axis separation flag: an axis separates iff !(temp > 0), and depth ends as the
    // minimum temp over the valid axes, so the callers test depth > 0 once -- see sat()).
    // depth is the NaN-propagating minimum (one instruction, like the select it replaces): a
    // NaN temp -- a non-finite vertex, where IsOverlapping's compares are false and
    // AxisChecks returns false -- leaves depth NaN and the verdict depth > 0 false
    const bool take = valid && temp < depth;
    depth = valid ? net_minf(depth, temp) : depth;
    normal.x = take ? axis.x : normal.x;
    normal.y = take ? axis.y : normal.y;
  }
}

// SAT of A against the static floor (Environment.CreateFloor, Environment.cs:219-223).
// The floor's four edge normals normalise to exactly (1,+0), (-0,1), (-1,+0), (-0,-1)
// and its own projections onto them are constants; A's projections onto them
// (1*x + 0*y, ...) equal A's bounding-box extents in value -- at most a zero's sign
// differs, which never reaches depth on an overlapping axis -- so the floor's half of
// AxisChecks needs no vertex loop.  Same verdict, normal and depth bits as sat().
DEV void floor_axis(float pmin, float pmax, float qmin, float qmax, float nx, float ny, bool& sep,
                    V2& normal, float& depth) {
  const float temp = net_minf(qmax - pmin, pmax - qmin);
  const bool take = temp < depth;  // see axis_pass (separation: the caller's depth > 0)
  depth = net_minf(depth, temp);
  normal.x = take ? nx : normal.x;
  normal.y = take ? ny : normal.y;
}
template <int NA, bool POLE = false>  // POLE: A is a walker pole (see pole_own_minmax)
DEV bool sat_floor(const Poly<NA>& A, const Poly<4>& F, float mnx, float mny, float mxx,
                   float mxy, V2& normal, float& depth, EdgeAxes<NA>* AX = nullptr) {
  normal = mk(0.0f, 0.0f);
  depth = FLT_MAX;
  bool sep = false;
  axis_pass<NA, 4, true, false, NA, POLE>(A, F, sep, normal, depth, AX);
  floor_axis(-50.0f, 1050.0f, mnx, mxx, 1.0f, 0.0f, sep, normal, depth);
  floor_axis(900.0f, 1050.0f, mny, mxy, -0.0f, 1.0f, sep, normal, depth);
  floor_axis(-1050.0f, 50.0f, -mxx, -mnx, -1.0f, 0.0f, sep, normal, depth);
  floor_axis(-1050.0f, -900.0f, -mxy, -mny, -0.0f, -1.0f, sep, normal, depth);
  V2 dir = mk(F.cx - A.cx, F.cy - A.cy);
  if (vdot(dir, normal) > 0.0f) normal = vmul(normal, -1.0f);
  return depth > 0.0f;  // (see sat)
}

// POLES: a Poly<6> operand is a walker pole (its own projections by pole_own_minmax); the
// scene kernel's hexagon props never come here (they take the generic axis_pass_g)
template <int NA, int NB, bool BZE = false, bool POLES = false>
DEV bool sat(const Poly<NA>& A, const Poly<NB>& B, V2& normal, float& depth,
             EdgeAxes<NA>* AXA = nullptr, EdgeAxes<NB>* AXB = nullptr) {
  normal = mk(0.0f, 0.0f);
  depth = FLT_MAX;
  bool sep = false;
  axis_pass<NA, NB, false, false, NA, POLES && NA == 6>(A, B, sep, normal, depth, AXA);
  axis_pass<NB, NA, false, BZE, NB, POLES && NB == 6>(B, A, sep, normal, depth, AXB);
  V2 dir = mk(B.cx - A.cx, B.cy - A.cy);
  if (vdot(dir, normal) > 0.0f) normal = vmul(normal, -1.0f);
  // AxisChecks returns false at the first axis whose projections do not overlap, i.e. with
  // !(temp > 0) (verdict algebra in axis_pass).  depth is the minimum temp over every valid
  // axis (take = temp < depth), so for a finite state "no axis separates" is exactly
  // depth > 0 -- one compare here instead of one per axis.
  return depth > 0.0f;
}

// ---------------- SAT, axes split over an L-lane row (L in {4, 8, 16}) ----------------
// Lane `sub` of the walker's row owns axis `sub` (A's edges first, then B's, the order
// of AxisChecks(A, B) && AxisChecks(B, A)).  The sequential loop's result is exactly:
// false if any axis separates; otherwise the smallest depth, ties to the lowest axis
// index (strict '<' in AxisChecks keeps the first).  That is an order-independent
// lexicographic min over (depth, index), reduced across the row with DPP.
DEV int dpp_i(int v, int ctrl_sel) {
  switch (ctrl_sel) {
    case 0: return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    case 1: return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    case 2: return __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    default: return __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false); // row_mirror
  }
}
DEV float dpp_f(float v, int c) { return __int_as_float(dpp_i(__float_as_int(v), c)); }

template <int L>
DEV void row_reduce(int& sep, float& depth, int& idx, float& nx, float& ny) {
  constexpr int steps = L == 16 ? 4 : (L == 8 ? 3 : 2);
#pragma unroll
  for (int s = 0; s < steps; s++) {
    const int osep = dpp_i(sep, s), oidx = dpp_i(idx, s);
    const float od = dpp_f(depth, s), onx = dpp_f(nx, s), ony = dpp_f(ny, s);
    sep |= osep;
    const bool take = (od < depth) || (od == depth && oidx < idx);
    depth = take ? od : depth;
    idx = take ? oidx : idx;
    nx = take ? onx : nx;
    ny = take ? ony : ny;
  }
}

// candidate edge endpoints of axis k: A's edges 0..NA-1 then B's edges
template <int NA, int NB>
DEV void edge_of(const Poly<NA>& A, const Poly<NB>& B, int k, V2& p0, V2& p1) {
  uint32_t x0 = 0u, y0 = 0u, x1 = 0u, y1 = 0u;
#pragma unroll
  for (int i = 0; i < NA + NB; i++) {
    const uint32_t m = (k == i) ? 0xffffffffu : 0u;
    const bool fa = i < NA;
    const int a = fa ? i : i - NA;
    const int b = fa ? (a + 1) % NA : (a + 1) % NB;
    const float sx = fa ? A.x[fa ? a : 0] : B.x[fa ? 0 : a];
    const float sy = fa ? A.y[fa ? a : 0] : B.y[fa ? 0 : a];
    const float ex = fa ? A.x[fa ? b : 0] : B.x[fa ? 0 : b];
    const float ey = fa ? A.y[fa ? b : 0] : B.y[fa ? 0 : b];
    x0 |= m & __float_as_uint(sx); y0 |= m & __float_as_uint(sy);
    x1 |= m & __float_as_uint(ex); y1 |= m & __float_as_uint(ey);
  }
  p0 = mk(__uint_as_float(x0), __uint_as_float(y0));
  p1 = mk(__uint_as_float(x1), __uint_as_float(y1));
}

template <int L, int NA, int NB>
DEV bool sat_row(const Poly<NA>& A, const Poly<NB>& B, int sub, V2& normal, float& depth) {
  static_assert(NA + NB <= L, "one axis per lane");
  int sep = 0, idx = 1 << 20;
  float d = FLT_MAX, nx = 0.0f, ny = 0.0f;
  if (sub < NA + NB) {
    V2 p0, p1;
    edge_of(A, B, sub, p0, p1);
    const float ex = p1.x - p0.x, ey = p1.y - p0.y;
    V2 axis = mk(-ey, ex);
    if (!(axis.x == 0.0f && axis.y == 0.0f)) {
      axis = vnormalize(axis);
      float amin, amax, bmin, bmax;
      project2(axis.x, axis.y, A, B, amin, amax, bmin, bmax);
      float temp;
      bool overlapping;
      if (sub < NA) {  // AxisChecks(A, B): projectionA = A
        temp = net_minf(bmax - amin, amax - bmin);
        overlapping = (amin < bmax) && (bmin < amax);
      } else {         // AxisChecks(B, A): projectionA = B
        temp = net_minf(amax - bmin, bmax - amin);
        overlapping = (bmin < amax) && (amin < bmax);
      }
      if (!overlapping) sep = 1;
      d = temp; idx = sub; nx = axis.x; ny = axis.y;
    }
  }
  row_reduce<L>(sep, d, idx, nx, ny);
  normal = idx < (1 << 20) ? mk(nx, ny) : mk(0.0f, 0.0f);
  depth = d;
  const bool result = sep == 0;
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

// GetSignificantFace (:79-94) with GetSignificantVertex (:97-113).  One pass: the
// sequential argmin (first strict minimum) carries the vertex and both neighbours along
// as bit-masked copies (v_bfi), so no runtime-indexed pick is needed.  With no
// projection below MaxValue (index -1) the reference keeps Vector2.Zero and takes the
// neighbours (index + 1) % N = 0 and Mod(index - 1, N) = N - 2.
DEV uint32_t bsel(uint32_t m, float a, uint32_t b) { return (m & __float_as_uint(a)) | (~m & b); }
template <int N, bool SAFE = false>
DEV void significant_face(const Poly<N>& P, V2 n, V2& fa, V2& fb, V2& fmax) {
  float mind = FLT_MAX;
  uint32_t sx = 0u, sy = 0u;
  uint32_t ax = __float_as_uint(P.x[0]), ay = __float_as_uint(P.y[0]);
  uint32_t bx = __float_as_uint(P.x[N - 2]), by = __float_as_uint(P.y[N - 2]);
#pragma unroll
  for (int i = 0; i < N; i++) {
    const float p = P.x[i] * n.x + P.y[i] * n.y;
    const bool lt = p < mind;
    const uint32_t m = lt ? 0xffffffffu : 0u;
    mind = lt ? p : mind;
    sx = bsel(m, P.x[i], sx);
    sy = bsel(m, P.y[i], sy);
    ax = bsel(m, P.x[(i + 1) % N], ax);
    ay = bsel(m, P.y[(i + 1) % N], ay);
    bx = bsel(m, P.x[(i + N - 1) % N], bx);
    by = bsel(m, P.y[(i + N - 1) % N], by);
  }
  const V2 sig = mk(__uint_as_float(sx), __uint_as_float(sy));
  const V2 va = mk(__uint_as_float(ax), __uint_as_float(ay));
  const V2 vb = mk(__uint_as_float(bx), __uint_as_float(by));
  // SAFE: the polygon may have a zero edge, whose Normalize is NaN (and the compare false)
  V2 after = SAFE ? vnormalize(vsub(sig, va)) : vnormalize_edge(vsub(sig, va));
  V2 before = SAFE ? vnormalize(vsub(sig, vb)) : vnormalize_edge(vsub(sig, vb));
  const bool first = vdot(n, before) >= vdot(n, after);
  fa = first ? sig : va;
  fb = first ? vb : sig;
  fmax = sig;
}

// The same face from the SAT's normalised axes (no new normalisation).  Axis i of P is
// vnormalize_edge((-ey, ex)) of edge e_i = v_{i+1} - v_i, i.e. (-ey val, ex val) with
// val = 1 / |e_i| (the squared length sums the same two exact squares, so val is
// Normalize's): e_i's Normalize is (axis.y, -axis.x) bit for bit, and a negated vector
// normalises to the negated result.  So after = Normalize(v_i - v_{i+1}) = -ê_i and
// before = Normalize(v_i - v_{i-1}) = ê_{i-1}; the face direction Normalize(fb - fa) is
// -before (face [sig, prev]) or after (face [next, sig]), returned in fdir.  (With no
// projection below MaxValue -- a NaN normal, already a fault -- the reference's Zero
// vertex is not on an edge; the result then differs from the reference's NaNs only in value.)
template <int N>
DEV void significant_face_ax(const Poly<N>& P, const EdgeAxes<N>& AX, V2 n, V2& fa, V2& fb,
                             V2& fmax, V2& fdir) {
  float mind = FLT_MAX;
  uint32_t sx = 0u, sy = 0u;
  uint32_t ax = __float_as_uint(P.x[0]), ay = __float_as_uint(P.y[0]);
  uint32_t bx = __float_as_uint(P.x[N - 2]), by = __float_as_uint(P.y[N - 2]);
  uint32_t ex = __float_as_uint(AX.x[N - 1]), ey = __float_as_uint(AX.y[N - 1]);  // axis i
  uint32_t px = __float_as_uint(AX.x[N - 2]), py = __float_as_uint(AX.y[N - 2]);  // axis i-1
#pragma unroll
  for (int i = 0; i < N; i++) {
    const float p = P.x[i] * n.x + P.y[i] * n.y;
    const bool lt = p < mind;
    const uint32_t m = lt ? 0xffffffffu : 0u;
    mind = lt ? p : mind;
    sx = bsel(m, P.x[i], sx);
    sy = bsel(m, P.y[i], sy);
    ax = bsel(m, P.x[(i + 1) % N], ax);
    ay = bsel(m, P.y[(i + 1) % N], ay);
    bx = bsel(m, P.x[(i + N - 1) % N], bx);
    by = bsel(m, P.y[(i + N - 1) % N], by);
    ex = bsel(m, AX.x[i], ex);
    ey = bsel(m, AX.y[i], ey);
    px = bsel(m, AX.x[(i + N - 1) % N], px);
    py = bsel(m, AX.y[(i + N - 1) % N], py);
  }
  const V2 sig = mk(__uint_as_float(sx), __uint_as_float(sy));
  const V2 va = mk(__uint_as_float(ax), __uint_as_float(ay));
  const V2 vb = mk(__uint_as_float(bx), __uint_as_float(by));
  const V2 after = mk(-__uint_as_float(ey), __uint_as_float(ex));    // -(axis_i.y, -axis_i.x)
  const V2 before = mk(__uint_as_float(py), -__uint_as_float(px));  // (axis_{i-1}.y, -axis_{i-1}.x)
  const bool first = vdot(n, before) >= vdot(n, after);
  fa = first ? sig : va;
  fb = first ? vb : sig;
  fmax = sig;
  fdir = first ? vneg(before) : after;
}
// significant_face_ax through LDS (the pair mapping's contact faces): instead of carrying the
// vertex, both neighbours and two axes through ten bit-select chains over the N vertices, the
// lane writes its polygon and axes as N float4 records (x, y, axis x, axis y) into its own LDS
// column rec[k * S] (S: the block's lanes, so a wave's 16-byte accesses hit distinct banks), finds
// the first strict minimum's index, and reads the three records it needs.  The same index rule as
// significant_face_ax: with no projection below MaxValue (index -1) the vertex is Vector2.Zero,
// its neighbours are vertices 0 and N - 2 and its axes N - 1 and N - 2 (the wrapped indices).
template <int N, int S>
DEV void significant_face_lds(const Poly<N>& P, const EdgeAxes<N>& AX, V2 n, float4* rec, V2& fa,
                              V2& fb, V2& fmax, V2& fdir) {
#pragma unroll
  for (int k = 0; k < N; k++) rec[k * S] = make_float4(P.x[k], P.y[k], AX.x[k], AX.y[k]);
  float mind = FLT_MAX;
  int idx = -1;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const float p = P.x[i] * n.x + P.y[i] * n.y;
    const bool lt = p < mind;
    mind = lt ? p : mind;
    idx = lt ? i : idx;
  }
  const int ie = idx < 0 ? N - 1 : idx;           // axis i (-1 wraps to N - 1)
  const int inx = idx == N - 1 ? 0 : idx + 1;      // vertex i + 1 (-1 -> 0)
  const int ipv = idx <= 0 ? idx + N - 1 : idx - 1;  // vertex and axis i - 1 (-1 -> N - 2)
  __builtin_amdgcn_wave_barrier();  // (the lane reads only its own column: no other lane's data)
  const float4 re = rec[ie * S], rn = rec[inx * S], rp = rec[ipv * S];
  const V2 sig = idx < 0 ? mk(0.0f, 0.0f) : mk(re.x, re.y);
  const V2 va = mk(rn.x, rn.y);
  const V2 vb = mk(rp.x, rp.y);
  const V2 after = mk(-re.w, re.z);    // -(axis_i.y, -axis_i.x)
  const V2 before = mk(rp.w, -rp.z);   // (axis_{i-1}.y, -axis_{i-1}.x)
  const bool first = vdot(n, before) >= vdot(n, after);
  fa = first ? sig : va;
  fb = first ? vb : sig;
  fmax = sig;
  fdir = first ? vneg(before) : after;
}

// the flat floor's normalised edges (Environment.cs:219-223): (0,-150), (1100,0), (0,150),
// (-1100,0) normalise to exactly (+0,-1), (1,+0), (+0,1), (-1,+0); as axes (-ey, ex) * val
DEV EdgeAxes<4> floor_axes() {
  EdgeAxes<4> a;
  a.x[0] = 1.0f;  a.y[0] = 0.0f;    // edge (+0,-1)
  a.x[1] = -0.0f; a.y[1] = 1.0f;    // edge (1,+0)
  a.x[2] = -1.0f; a.y[2] = 0.0f;    // edge (+0,1)
  a.x[3] = -0.0f; a.y[3] = -1.0f;   // edge (-1,+0)
  return a;
}

// ClipVectors (:56-76), branch-free: the kept points in order [a], [b], [crossing]
DEV int clip_vectors(V2 a, V2 b, V2 n, float offset, V2& o0, V2& o1) {
  const float da = vdot(a, n) - offset;
  const float db = vdot(b, n) - offset;
  const bool ka = da >= 0.0f, kb = db >= 0.0f, kx = da * db < 0.0f;
  const float location = da / (da - db);  // used only when kx (then da != db)
  const V2 edge = vadd(vmul(vsub(b, a), location), a);
  const V2 second = kb ? b : edge;          // the point after a when a is kept
  V2 r0 = ka ? a : (kb ? b : edge);
  V2 r1 = ka ? second : edge;               // only meaningful when two are kept
  const bool has0 = ka || kb || kx;
  const bool has1 = ka ? (kb || kx) : (kb && kx);
  o0 = has0 ? r0 : o0;
  o1 = has1 ? r1 : o1;
  return (int)ka + (int)kb + (int)kx;
}

// GetContactPoints (:13-53) from the two significant faces (A's on the normal, B's on its
// negation: vertices a, b, the max vertex and the normalised face direction)
DEV int contact_clip(V2 ra, V2 rb, V2 rmax, V2 rd, V2 ia, V2 ib, V2 imax, V2 id, V2 normal,
                     V2& c0, V2& c1) {
  V2 rf = vsub(rb, ra);
  V2 iv = vsub(ib, ia);
  if (fabsf(vdot(rf, normal)) > fabsf(vdot(iv, normal))) {  // selects, not a branch
    V2 t;
    t = ra; ra = ia; ia = t;
    t = rb; rb = ib; ib = t;
    t = rmax; rmax = imax; imax = t;
    rd = id;
  }
  rf = rd;  // Normalize(rb - ra)
  float offset = vdot(rf, ra);
  V2 p0 = mk(0.0f, 0.0f), p1 = mk(0.0f, 0.0f);
  const int k1 = clip_vectors(ia, ib, rf, offset, p0, p1);
  offset = vdot(rf, rb);
  V2 q0 = mk(0.0f, 0.0f), q1 = mk(0.0f, 0.0f);
  const int k2 = clip_vectors(p0, p1, vneg(rf), -offset, q0, q1);
  if (k1 < 2 || k2 < 2) return 0;
  V2 refn = mk(rf.y, -rf.x);
  float maximum = vdot(refn, rmax);
  int cnt = 2;
  if (vdot(refn, q0) - maximum < 0.0f) { q0 = q1; cnt = 1; }
  V2 last = cnt == 2 ? q1 : q0;
  if (vdot(refn, last) - maximum < 0.0f) cnt = cnt == 2 ? 1 : 0;
  c0 = q0;
  c1 = q1;
  return cnt;
}
// GetContactPoints with both polygons' SAT axes kept: the faces' directions come normalised
template <int NA, int NB, int S = 0>  // S > 0: both faces through LDS (one column, in turn)
DEV int contact_points_ax(const Poly<NA>& A, const EdgeAxes<NA>& AXA, const Poly<NB>& B,
                          const EdgeAxes<NB>& AXB, V2 normal, V2& c0, V2& c1,
                          float4* rec = nullptr) {
  V2 ra, rb, rmax, rd, ia, ib, imax, id;
  if constexpr (S > 0) {
    significant_face_lds<NA, S>(A, AXA, normal, rec, ra, rb, rmax, rd);
    __builtin_amdgcn_wave_barrier();  // (A's records read before B's overwrite them: same lane)
    significant_face_lds<NB, S>(B, AXB, vneg(normal), rec, ia, ib, imax, id);
  } else {
    significant_face_ax(A, AXA, normal, ra, rb, rmax, rd);
    significant_face_ax(B, AXB, vneg(normal), ia, ib, imax, id);
  }
  return contact_clip(ra, rb, rmax, rd, ia, ib, imax, id, normal, c0, c1);
}
// significant_face_ax(floor_poly, floor_axes(), n) for the flat floor box, vertices
// (-50,1050), (-50,900), (1050,900), (1050,1050): the same four projections and first strict
// minimum, then the vertex, its neighbours and the two axes are constants selected by the
// index's two bits (b1 b0) instead of ten bit-select chains -- the same values whenever a
// minimum exists (a NaN normal, already a fault, takes index 0).
DEV void floor_face_ax(V2 n, V2& fa, V2& fb, V2& fmax, V2& fdir) {
  const float xa = -50.0f * n.x, xb = 1050.0f * n.x, ya = 1050.0f * n.y, yb = 900.0f * n.y;
  const float p[4] = {xa + ya, xa + yb, xb + yb, xb + ya};
  float mind = FLT_MAX;
  bool b0 = false, b1 = false;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const bool lt = p[i] < mind;
    mind = lt ? p[i] : mind;
    b0 = lt ? (i & 1) != 0 : b0;
    b1 = lt ? (i >> 1) != 0 : b1;
  }
  const bool bx = b0 != b1;
  const V2 sig = mk(b1 ? 1050.0f : -50.0f, bx ? 900.0f : 1050.0f);  // vertex idx
  const V2 va = mk(bx ? 1050.0f : -50.0f, b1 ? 1050.0f : 900.0f);   // vertex idx + 1
  const V2 vb = mk(bx ? -50.0f : 1050.0f, b1 ? 900.0f : 1050.0f);   // vertex idx - 1
  const float ex = b0 ? -0.0f : (b1 ? -1.0f : 1.0f), ey = b0 ? (b1 ? -1.0f : 1.0f) : 0.0f;
  const float px = b0 ? (b1 ? -1.0f : 1.0f) : -0.0f, py = b0 ? 0.0f : (b1 ? 1.0f : -1.0f);
  const V2 after = mk(-ey, ex);
  const V2 before = mk(py, -px);
  const bool first = vdot(n, before) >= vdot(n, after);
  fa = first ? sig : va;
  fb = first ? vb : sig;
  fmax = sig;
  fdir = first ? vneg(before) : after;
}
template <int NA, int S = 0>  // S > 0: A's face through LDS (significant_face_lds, column rec)
DEV int contact_points_floor(const Poly<NA>& A, const EdgeAxes<NA>& AXA, V2 normal, V2& c0,
                             V2& c1, float4* rec = nullptr) {
  V2 ra, rb, rmax, rd, ia, ib, imax, id;
  if constexpr (S > 0) significant_face_lds<NA, S>(A, AXA, normal, rec, ra, rb, rmax, rd);
  else significant_face_ax(A, AXA, normal, ra, rb, rmax, rd);
  floor_face_ax(vneg(normal), ia, ib, imax, id);
  return contact_clip(ra, rb, rmax, rd, ia, ib, imax, id, normal, c0, c1);
}

template <int NA, int NB, bool SAFE = false>
DEV int contact_points(const Poly<NA>& A, const Poly<NB>& B, V2 normal, V2& c0, V2& c1) {
  V2 ra, rb, rmax, ia, ib, imax;
  significant_face(A, normal, ra, rb, rmax);
  V2 rf = vsub(rb, ra);
  significant_face<NB, SAFE>(B, vneg(normal), ia, ib, imax);
  V2 iv = vsub(ib, ia);
  if (fabsf(vdot(rf, normal)) > fabsf(vdot(iv, normal))) {  // selects, not a branch
    V2 t;
    t = ra; ra = ia; ia = t;
    t = rb; rb = ib; ib = t;
    t = rmax; rmax = imax; imax = t;
    rf = vsub(rb, ra);
  }
  rf = SAFE ? vnormalize(rf) : vnormalize_edge(rf);  // rb - ra: an edge of the reference face
  float offset = vdot(rf, ra);
  V2 p0 = mk(0.0f, 0.0f), p1 = mk(0.0f, 0.0f);
  const int k1 = clip_vectors(ia, ib, rf, offset, p0, p1);
  offset = vdot(rf, rb);
  V2 q0 = mk(0.0f, 0.0f), q1 = mk(0.0f, 0.0f);
  const int k2 = clip_vectors(p0, p1, vneg(rf), -offset, q0, q1);
  if (k1 < 2 || k2 < 2) return 0;  // the second clip ran on whatever the first left
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
