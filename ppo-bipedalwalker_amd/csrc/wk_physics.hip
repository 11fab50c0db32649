// wk_physics.hip -- fused batched env-step kernel for gfx950 (one walker per lane).
//
// One launch runs K whole Environment.Update steps (Environment.cs:64-92) for every
// walker: optional policy sampling (PPOAgent.SampleActions, PPOAgent.cs:381-398),
// Clip + Joint.SetTorque (Environment.cs:78, Joint.cs:56-61), Iterations substeps of
// StepObjects (Environment.cs:126-143: Joint.Step Joint.cs:31-41, RigidBody.Step
// Bodies/RigidBody.cs:54-61 with the AABB broadphase Skeleton.cs:133-140, SAT
// Bodies/Physics/SATCollision.cs:15-104, contact clipping ContactPoints.cs:13-134 and
// impulses Impulses.cs:12-115), Walker.Update (Walker.cs:49-54), CalculateReward
// (Environment.cs:148-154), terminal checks (:106-117), GetState (Walker.cs:132-152)
// and auto-reset (Environment.cs:167-180, Walker.cs:212-223).
//
// All walker state lives in VGPRs for the whole launch; HBM is touched only to load
// and store the 112-float SoA state once per launch and to write per-step outputs.
// Arithmetic is restated op-for-op in IEEE fp32 with -ffp-contract=off so the
// trajectories are bit-identical to the CPU oracle (MonoGame Vector2 semantics:
// v / f == v * (1/f); rotation via (float)cos/sin of the double-promoted angle).
#include "wk_common.h"
#include "wk_device.h"
#include "wk_kernels.h"
#include "wk_mfma_layout.h"
#include "wk_region_prof.h"

// Build parts (the Makefile compiles this file eight times, in parallel): kernels are
// templates instantiated where the host shims at the end launch them, so each part holds the
// shims of one family -- 1: the pair side kernels, 8: the quad side kernels (the default
// scheduler), 5: both on the rough floor, 2 and 4: the scene-prop kernel (given actions / policy),
// 6 and 7: the same on the rough floor, 3: the rest (1- and 16-lane kernels, the counting replay,
// init, obs, policy, returns).  0: all.
#ifndef WK_PHYS_PART
#define WK_PHYS_PART 0
#endif
#define WK_PART(k) (WK_PHYS_PART == 0 || WK_PHYS_PART == (k))

// two waves per SIMD for the one- and 16-lane kernels (three: 168 VGPRs, spills, slower)
#define WK_ENV_WPE __attribute__((amdgpu_waves_per_eu(2, 2)))

namespace wk {

struct EnvState {
  Poly<6> lll, llu, rll, rlu;
  Poly<5> body;
  Dyn dlll, dllu, dbody, drll, drlu;
  bool clll, cllu, cbody, crll, crlu;
  float torque[4];
  float posx, posy, prevx, prevy;
  int steps, episodes;
  bool post, terminal;
};

// Pole.FromSize (Objects/RigidBodies/Pole.cs:18-34) + FindCentroid (Skeleton.cs:100-113)
DEV void make_pole(Poly<6>& p, float cx, float cy) {
  float adjustment = 0.1f * 75.0f;
  float h = adjustment * 3.5f;
  p.x[0] = cx + adjustment; p.y[0] = cy + h;
  p.x[1] = cx;              p.y[1] = cy + h;
  p.x[2] = cx - adjustment; p.y[2] = cy + h;
  p.x[3] = cx - adjustment; p.y[3] = cy - h;
  p.x[4] = cx;              p.y[4] = cy - h;
  p.x[5] = cx + adjustment; p.y[5] = cy - h;
  find_centroid(p);
}

DEV void zero_dyn(Dyn& d) { d.vx = 0.0f; d.vy = 0.0f; d.w = 0.0f; d.th = 0.0f; }

// Walker.CreateCreature / Reset + Environment.InitialState
DEV void make_template(EnvState& s, float dx) {
  float px = 125.0f + dx, py = 800.0f;
  s.body.x[0] = px + 20; s.body.y[0] = py + 20;
  s.body.x[1] = px;      s.body.y[1] = py + 20;
  s.body.x[2] = px - 20; s.body.y[2] = py + 20;
  s.body.x[3] = px - 20; s.body.y[3] = py - 20;
  s.body.x[4] = px + 20; s.body.y[4] = py - 20;
  find_centroid(s.body);
  make_pole(s.llu, px + 0.0f, py + 30.0f);
  make_pole(s.lll, px + 0.0f, py + 60.0f);
  make_pole(s.rlu, px + 0.0f, py + 30.0f);
  make_pole(s.rll, px + 0.0f, py + 60.0f);
  zero_dyn(s.dlll); zero_dyn(s.dllu); zero_dyn(s.dbody); zero_dyn(s.drll); zero_dyn(s.drlu);
  s.clll = s.cllu = s.cbody = s.crll = s.crlu = false;
#pragma unroll
  for (int j = 0; j < 4; j++) s.torque[j] = 0.0f;
  s.steps = 0;
  s.terminal = false;
  // InitialState -> Walker.Update: prev = (125, 800); pos = Body centroid
  s.prevx = px; s.prevy = py;
  s.posx = s.body.cx; s.posy = s.body.cy;
}

template <int N>
DEV void load_poly(Poly<N>& p, const float* __restrict__ st, int b, int e, int n) {
#pragma unroll
  for (int i = 0; i < N; i++) {
    p.x[i] = st[(size_t)e * NSTATE + (b * BSTRIDE + 2 * i)];
    p.y[i] = st[(size_t)e * NSTATE + (b * BSTRIDE + 2 * i + 1)];
  }
  p.cx = st[(size_t)e * NSTATE + (b * BSTRIDE + F_CX)];
  p.cy = st[(size_t)e * NSTATE + (b * BSTRIDE + F_CY)];
}
DEV void load_dyn(Dyn& d, bool& col, const float* __restrict__ st, int b, int e, int n) {
  d.vx = st[(size_t)e * NSTATE + (b * BSTRIDE + F_VX)];
  d.vy = st[(size_t)e * NSTATE + (b * BSTRIDE + F_VY)];
  d.w = st[(size_t)e * NSTATE + (b * BSTRIDE + F_W)];
  d.th = st[(size_t)e * NSTATE + (b * BSTRIDE + F_TH)];
  col = st[(size_t)e * NSTATE + (b * BSTRIDE + F_COL)] != 0.0f;
}
template <int N>
DEV void store_body(const Poly<N>& p, const Dyn& d, bool col, float* __restrict__ st, int b, int e,
                    int n) {
#pragma unroll
  for (int i = 0; i < 6; i++) {
    st[(size_t)e * NSTATE + (b * BSTRIDE + 2 * i)] = i < N ? p.x[i < N ? i : 0] : 0.0f;
    st[(size_t)e * NSTATE + (b * BSTRIDE + 2 * i + 1)] = i < N ? p.y[i < N ? i : 0] : 0.0f;
  }
  st[(size_t)e * NSTATE + (b * BSTRIDE + F_CX)] = p.cx;
  st[(size_t)e * NSTATE + (b * BSTRIDE + F_CY)] = p.cy;
  st[(size_t)e * NSTATE + (b * BSTRIDE + F_VX)] = d.vx;
  st[(size_t)e * NSTATE + (b * BSTRIDE + F_VY)] = d.vy;
  st[(size_t)e * NSTATE + (b * BSTRIDE + F_W)] = d.w;
  st[(size_t)e * NSTATE + (b * BSTRIDE + F_TH)] = d.th;
  st[(size_t)e * NSTATE + (b * BSTRIDE + F_COL)] = col ? 1.0f : 0.0f;
  st[(size_t)e * NSTATE + (b * BSTRIDE + 19)] = 0.0f;
}

DEV void load_state(EnvState& s, const float* __restrict__ st, int e, int n) {
  load_poly(s.lll, st, LLL, e, n);
  load_poly(s.llu, st, LLU, e, n);
  load_poly(s.body, st, BODY, e, n);
  load_poly(s.rll, st, RLL, e, n);
  load_poly(s.rlu, st, RLU, e, n);
  load_dyn(s.dlll, s.clll, st, LLL, e, n);
  load_dyn(s.dllu, s.cllu, st, LLU, e, n);
  load_dyn(s.dbody, s.cbody, st, BODY, e, n);
  load_dyn(s.drll, s.crll, st, RLL, e, n);
  load_dyn(s.drlu, s.crlu, st, RLU, e, n);
#pragma unroll
  for (int j = 0; j < 4; j++) s.torque[j] = st[(size_t)e * NSTATE + (S_TORQUE + j)];
  s.posx = st[(size_t)e * NSTATE + S_POS];
  s.posy = st[(size_t)e * NSTATE + (S_POS + 1)];
  s.prevx = st[(size_t)e * NSTATE + S_PREV];
  s.prevy = st[(size_t)e * NSTATE + (S_PREV + 1)];
  s.steps = (int)st[(size_t)e * NSTATE + S_STEPS];
  s.post = st[(size_t)e * NSTATE + S_POSTRESET] != 0.0f;
  s.terminal = st[(size_t)e * NSTATE + S_TERMINAL] != 0.0f;
  s.episodes = (int)st[(size_t)e * NSTATE + S_EPISODES];
}

DEV void store_state(const EnvState& s, float* __restrict__ st, int e, int n) {
  store_body(s.lll, s.dlll, s.clll, st, LLL, e, n);
  store_body(s.llu, s.dllu, s.cllu, st, LLU, e, n);
  store_body(s.body, s.dbody, s.cbody, st, BODY, e, n);
  store_body(s.rll, s.drll, s.crll, st, RLL, e, n);
  store_body(s.rlu, s.drlu, s.crlu, st, RLU, e, n);
#pragma unroll
  for (int j = 0; j < 4; j++) st[(size_t)e * NSTATE + (S_TORQUE + j)] = s.torque[j];
  st[(size_t)e * NSTATE + S_POS] = s.posx;
  st[(size_t)e * NSTATE + (S_POS + 1)] = s.posy;
  st[(size_t)e * NSTATE + S_PREV] = s.prevx;
  st[(size_t)e * NSTATE + (S_PREV + 1)] = s.prevy;
  st[(size_t)e * NSTATE + S_STEPS] = (float)s.steps;
  st[(size_t)e * NSTATE + S_POSTRESET] = s.post ? 1.0f : 0.0f;
  st[(size_t)e * NSTATE + S_TERMINAL] = s.terminal ? 1.0f : 0.0f;
  st[(size_t)e * NSTATE + S_EPISODES] = (float)s.episodes;
}

// Walker.GetState (Walker.cs:132-152)
DEV void get_obs(const EnvState& s, float o[12]) {
  o[0] = s.body.x[1] / 900.0f;
  o[1] = s.body.y[1] / 500.0f;
  o[2] = s.llu.x[2] / 900.0f;
  o[3] = s.llu.y[2] / 500.0f;
  o[4] = s.rlu.x[2] / 900.0f;
  o[5] = s.rlu.y[2] / 500.0f;
  o[6] = s.dbody.vx / 60.0f;
  o[7] = s.dbody.vy / 60.0f;
  o[8] = s.dlll.th;
  o[9] = s.dllu.th;
  o[10] = s.drll.th;
  o[11] = s.drlu.th;
}

// ---------------- quad mapping helpers (L = 4: two lanes per leg) ----------------
// The lane pair of a leg (halves 0 and 1: quad_perm [2,3,0,1] partners) holds the same leg
// state and splits the heavy halves of its pairs; each half ends with the other's results
// (DPP) combined in the reference's order, so both hold identical values throughout.
DEV float hswap(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}
// per-lane selects as bit masks: a ?: between register copies can be folded by LLVM into a
// load through a selected address, which moves the polygons to scratch memory (cf. pick)
DEV float fsel(uint32_t m, float a, float b) { return __uint_as_float(bsel(m, a, __float_as_uint(b))); }
template <int N>
DEV Poly<N> psel(bool c, const Poly<N>& a, const Poly<N>& b) {
  const uint32_t m = c ? 0xffffffffu : 0u;
  Poly<N> r;
#pragma unroll
  for (int i = 0; i < N; i++) { r.x[i] = fsel(m, a.x[i], b.x[i]); r.y[i] = fsel(m, a.y[i], b.y[i]); }
  r.cx = fsel(m, a.cx, b.cx);
  r.cy = fsel(m, a.cy, b.cy);
  return r;
}
// AxisChecks(A's edges, B) on half 0 and AxisChecks(B's edges, A) on half 1, then
// SATCollision's order: A's axes first, B's best only when strictly smaller (axis_pass
// takes on temp < depth, so the sequential result is the first strict minimum over A's axes
// then B's).  P / AXP: this half's own polygon and its normalised axes (for its face).
template <int N>
DEV bool sat_split(const Poly<N>& A, const Poly<N>& B, int half, V2& normal, float& depth,
                   Poly<N>& P, EdgeAxes<N>& AXP) {
  P = psel(half != 0, B, A);
  const Poly<N> Q = psel(half != 0, A, B);
  bool sep = false;
  V2 nn = mk(0.0f, 0.0f);
  float dd = FLT_MAX;
  axis_pass<N, N, false, false, N, N == 6>(P, Q, sep, nn, dd, &AXP);  // (P: a walker pole)
  const float dd_o = hswap(dd), nx_o = hswap(nn.x), ny_o = hswap(nn.y);
  const float dA = half ? dd_o : dd, dB = half ? dd : dd_o;
  const V2 nA = half ? mk(nx_o, ny_o) : nn, nB = half ? nn : mk(nx_o, ny_o);
  const bool takeB = dB < dA;
  depth = net_minf(dA, dB);  // (a NaN on either half stays NaN: no collision, see axis_pass)
  normal = takeB ? nB : nA;
  const V2 dir = mk(B.cx - A.cx, B.cy - A.cy);
  if (vdot(dir, normal) > 0.0f) normal = vmul(normal, -1.0f);
  return depth > 0.0f;  // (no axis separates: see sat in wk_device.h)
}
// GetContactPoints with the two faces split: half 0 A's on the normal, half 1 B's on its
// negation (each from its own SAT axes), exchanged, then the clipping in both
template <int N, int FS = 0>  // FS > 0: the face through LDS (significant_face_lds, column frec)
DEV int contacts_split(const Poly<N>& P, const EdgeAxes<N>& AXP, int half, V2 normal, V2& c0,
                       V2& c1, float4* frec = nullptr) {
  V2 fa, fb, fm, fd;
  if constexpr (FS > 0) significant_face_lds<N, FS>(P, AXP, half ? vneg(normal) : normal, frec, fa, fb, fm, fd);
  else significant_face_ax(P, AXP, half ? vneg(normal) : normal, fa, fb, fm, fd);
  const V2 oa = mk(hswap(fa.x), hswap(fa.y)), ob = mk(hswap(fb.x), hswap(fb.y));
  const V2 om = mk(hswap(fm.x), hswap(fm.y)), od = mk(hswap(fd.x), hswap(fd.y));
  const bool h = half != 0;
  return contact_clip(h ? oa : fa, h ? ob : fb, h ? om : fm, h ? od : fd,
                      h ? fa : oa, h ? fb : ob, h ? fm : om, h ? fd : od, normal, c0, c1);
}
// SAT of a leg segment against the flat floor with the segment's six axes split three and
// three (half 1 walks the segment from vertex 3: its edges 0..2 are edges 3..5, the same
// vertex set projected), then the floor's four closed-form axes in both; every axis of A
// ends up in AX on both halves (for A's contact face)
DEV bool sat_floor_split(const Poly<6>& A, const Poly<4>& F, float mnx, float mny, float mxx,
                         float mxy, int half, V2& normal, float& depth, EdgeAxes<6>& AX) {
  Poly<6> R;
  const uint32_t hm = half ? 0xffffffffu : 0u;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    R.x[i] = fsel(hm, A.x[(i + 3) % 6], A.x[i]);
    R.y[i] = fsel(hm, A.y[(i + 3) % 6], A.y[i]);
  }
  R.cx = A.cx;
  R.cy = A.cy;
  bool sep = false;
  V2 nn = mk(0.0f, 0.0f);
  float dd = FLT_MAX;
  EdgeAxes<6> own;
  axis_pass<6, 4, true, false, 3, true>(R, F, sep, nn, dd, &own);  // (R: the pole, maybe rotated by 3)
  const float dd_o = hswap(dd), nx_o = hswap(nn.x), ny_o = hswap(nn.y);
  const float d0 = half ? dd_o : dd, d1 = half ? dd : dd_o;
  const V2 n0 = half ? mk(nx_o, ny_o) : nn, n1 = half ? nn : mk(nx_o, ny_o);
  const bool take1 = d1 < d0;
  depth = net_minf(d0, d1);
  normal = take1 ? n1 : n0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float ox = hswap(own.x[i]), oy = hswap(own.y[i]);
    AX.x[i] = half ? ox : own.x[i];
    AX.y[i] = half ? oy : own.y[i];
    AX.x[i + 3] = half ? own.x[i] : ox;
    AX.y[i + 3] = half ? own.y[i] : oy;
  }
  floor_axis(-50.0f, 1050.0f, mnx, mxx, 1.0f, 0.0f, sep, normal, depth);
  floor_axis(900.0f, 1050.0f, mny, mxy, -0.0f, 1.0f, sep, normal, depth);
  floor_axis(-1050.0f, 50.0f, -mxx, -mnx, -1.0f, 0.0f, sep, normal, depth);
  floor_axis(-1050.0f, -900.0f, -mxy, -mny, -0.0f, -1.0f, sep, normal, depth);
  V2 dir = mk(F.cx - A.cx, F.cy - A.cy);
  if (vdot(dir, normal) > 0.0f) normal = vmul(normal, -1.0f);
  return depth > 0.0f;  // (see sat in wk_device.h)
}

// RigidBody.ResolveCollisions body for one (this=A, other=B) candidate
// (Bodies/RigidBody.cs:66-96); B may be the static floor.  GENERIC: B is a static floor
// polygon other than the flat box (a rough-floor segment): its bounding box, SAT and
// contact faces are evaluated in general, with Vector2.Normalize's NaN for a zero edge.
// H = 2: the quad mapping (sub = this lane's half): SAT axes and contact faces split over
// the leg's two lanes (leg-leg and leg-floor pairs of Poly<6> segments).
// FS > 0: the contact faces through this lane's LDS column frec (stride FS, the pair mapping)
template <int NA, int NB, bool BSTATIC, bool TRACE, int L, bool GENERIC = false, int H = 1, int FS = 0>
DEV void resolve_pair(Poly<NA>& A, Dyn& dA, const Mat& mA, Poly<NB>& B, Dyn& dB, const Mat& mB,
                      bool& colA, PairTraceDev* tr, int pi, int sub, RegionProf* rp = nullptr,
                      uint32_t* ec = nullptr, float4* frec = nullptr) {
  static_assert(H == 1 || (L == 1 && !GENERIC && NA == 6 && NB == (BSTATIC ? 4 : 6)),
                "the quad split covers leg-leg and leg-floor pairs");
  static_assert(!BSTATIC || NB == 4, "the static body is the floor");
  static_assert(!GENERIC || BSTATIC, "generic static floor polygon");
  constexpr bool FLAT = BSTATIC && !GENERIC;
  constexpr int EVK = !BSTATIC ? 0 : (NA == 5 ? 2 : 1);  // leg-leg, leg-floor, torso-floor
  float mnx, mny, mxx, mxy;  // A's bounding box (the floor pass of sat_floor reuses it)
  aabb(A, mnx, mny, mxx, mxy);
  bool ov;
  if constexpr (FLAT) {
    ov = mnx < 1050.0f && mxx > -50.0f && mny < 1050.0f && mxy > 900.0f;  // floor box
  } else {
    float b0x, b0y, b1x, b1y;
    aabb(B, b0x, b0y, b1x, b1y);
    ov = mnx < b1x && mxx > b0x && mny < b1y && mxy > b0y;
  }
  rp_mark(rp, RP_AABB_LL + EVK, ov ? 1.0f : 0.0f);
  if (!ov) return;
  if (ec) ec[EV_AABB_LL + EVK]++;
  if (TRACE && tr && pi >= 0) tr->aabb_hit[pi] = 1;
  if (BSTATIC) colA = true;  // body._isFloor -> Collided = true (:75)
  V2 n;
  float depth;
  bool hit;
  // the one- and two-lane mappings keep both polygons' SAT axes for the contact faces
  constexpr bool KEEP = L == 1 && !GENERIC;
  EdgeAxes<NA> axa;
  EdgeAxes<NB> axb;
  Poly<NA> own;  // H = 2 leg-leg: this half's polygon (A or B) and its axes (in axa)
  if constexpr (H == 2 && FLAT) hit = sat_floor_split(A, B, mnx, mny, mxx, mxy, sub, n, depth, axa);
  else if constexpr (H == 2) hit = sat_split(A, B, sub, n, depth, own, axa);
  else if constexpr (L > 1) hit = sat_row<L>(A, B, sub, n, depth);
  // (a Poly<6> here is always a walker pole: A is a leg segment or the torso, B a leg segment
  // or a floor; scene props resolve in wk_scene.inc)
  else if constexpr (FLAT) hit = sat_floor<NA, NA == 6>(A, B, mnx, mny, mxx, mxy, n, depth, &axa);
  else if constexpr (KEEP) hit = sat<NA, NB, false, true>(A, B, n, depth, &axa, &axb);
  else hit = sat<NA, NB, GENERIC, true>(A, B, n, depth);
  rp_mark(rp, RP_SAT_LL + EVK, depth, n.x, n.y, hit ? 1.0f : 0.0f);
  if (!hit) return;
  if (ec) ec[EV_SAT_LL + EVK]++;
  V2 c0, c1;
  int nc;
  if constexpr (H == 2 && !BSTATIC) nc = contacts_split<NA, FS>(own, axa, sub, n, c0, c1, frec);
  else if constexpr (KEEP && FLAT) nc = contact_points_floor<NA, FS>(A, axa, n, c0, c1, frec);
  else if constexpr (KEEP) nc = contact_points_ax<NA, NB, FS>(A, axa, B, axb, n, c0, c1, frec);
  else nc = contact_points<NA, NB, GENERIC>(A, B, n, c0, c1);
  rp_mark(rp, RP_CON_LL + EVK, c0.x, c0.y, c1.x, c1.y, (float)nc);
  if (TRACE && tr && pi >= 0) {
    tr->sat_hit[pi] = 1;
    tr->n_contacts[pi] = (uint8_t)nc;
    tr->normal[pi][0] = n.x;
    tr->normal[pi][1] = n.y;
    tr->depth[pi] = depth;
    if (nc > 0) { tr->contact[pi][0][0] = c0.x; tr->contact[pi][0][1] = c0.y; }
    if (nc > 1) { tr->contact[pi][1][0] = c1.x; tr->contact[pi][1][1] = c1.y; }
  }
  // MoveObjects (:99-113): A is never static here
  if (BSTATIC) {
    move(A, vmul(n, depth));
  } else {
    move(A, vdiv(vmul(n, depth), 2.0f));
    move(B, vdiv(vmul(vneg(n), depth), 2.0f));
  }
  // Impulses.ResolveCollisions (Impulses.cs:12-28)
  if (ec) ec[EV_CONTACTS] += (uint32_t)nc;
  if (nc == 0) return;
  if (ec) ec[EV_IMP_LL + EVK]++;
  float e = net_maxf(mA.e, mB.e);
  float mu = net_minf(mA.mu, mB.mu);
  V2 contact = nc == 2 ? vdiv(vadd(c0, c1), 2.0f) : c0;
  Body bA{A.cx, A.cy, &dA, mA.im, mA.ii};
  Body bB{B.cx, B.cy, &dB, mB.im, mB.ii};
  V2 rA, rB, rAF, rBF;
  V2 tangent = mk(-n.y, n.x);
  float j, jf;
  if constexpr (H == 2) {  // the normal impulse on half 0, the friction impulse on half 1
    const uint32_t hm = sub ? 0xffffffffu : 0u;
    const float mine = calc_impulse(bA, bB, contact, fsel(hm, mu, 1.0f + e),
                                    mk(fsel(hm, tangent.x, n.x), fsel(hm, tangent.y, n.y)), rA, rB);
    const float other = hswap(mine);
    j = fsel(hm, other, mine);
    jf = fsel(hm, mine, other);
    rAF = rA;  // (the lever arms do not depend on the direction)
    rBF = rB;
  } else {
    j = calc_impulse(bA, bB, contact, 1.0f + e, n, rA, rB);
    jf = calc_impulse(bA, bB, contact, mu, tangent, rAF, rBF);
  }
  if (TRACE && tr && pi >= 0) { tr->impulse[pi][0] = j; tr->impulse[pi][1] = jf; }
  apply_impulses<BSTATIC>(bA, bB, n, j, rA, rB);
  apply_impulses<BSTATIC>(bA, bB, tangent, jf, rAF, rBF);
  rp_mark(rp, RP_IMP_LL + EVK, dA.vx, dA.vy, dA.w, dB.vx, dB.vy, dB.w);
}

// Joint.Step (Objects/RigidBodies/Joint.cs:31-41); ResolveJoint swaps the bodies (:40)
template <int NA, int NB, int IA, int IB, bool TRACE>
DEV void joint_step(Poly<NA>& A, Dyn& dA, const Mat& mA, Poly<NB>& B, Dyn& dB, const Mat& mB,
                    PairTraceDev* tr, int ji, uint32_t* ec = nullptr) {
  V2 ab = vsub(mk(B.x[IB], B.y[IB]), mk(A.x[IA], A.y[IA]));
  float depth = vlen(ab);
  if (depth < 0.1f) return;
  if (ec) ec[EV_JOINT]++;
  // ab.Normalize(): ab * (1 / sqrt(x^2 + y^2)), and that sqrt is depth (same correctly
  // rounded sqrt of the same sum); rcp_core is 1.0f / d bit for bit on [2^-48, 2^64]
  const float rinv = depth <= 0x1p63f ? rcp_core(depth) : 1.0f / depth;
  ab = mk(ab.x * rinv, ab.y * rinv);
  move(A, vdiv(vmul(ab, depth), 2.0f));
  move(B, vdiv(vmul(vneg(ab), depth), 2.0f));
  V2 contact = vdiv(vadd(mk(A.x[IA], A.y[IA]), mk(B.x[IB], B.y[IB])), 2.0f);
  Body bJ{B.cx, B.cy, &dB, mB.im, mB.ii};  // manifold.BodyA = joint body B
  Body bI{A.cx, A.cy, &dA, mA.im, mA.ii};  // manifold.BodyB = joint body A
  V2 rA, rB;
  float j = calc_impulse(bJ, bI, contact, 1.0f + 1.0f, ab, rA, rB);
  if (TRACE && tr) { tr->joint_depth[ji] = depth; tr->joint_impulse[ji] = j; }
  apply_impulses<false>(bJ, bI, ab, j, rA, rB);
}

// RigidBody.StepLinearVelocity + StepAngularVelocity (RigidBody.cs:116-140)
template <int N>
DEV void integrate(Poly<N>& P, Dyn& D, float dt, float adx, float ady) {
  D.vx = D.vx + adx;
  D.vy = D.vy + ady;
  move(P, mk(D.vx * dt, D.vy * dt));
  D.th = D.th + D.w * dt;
  D.th = wrap_angle(D.th);
  rotate(P, D.w * dt);
}

// Environment.CreateRoughFloor (Environment.cs:230-261), segment k of 10 (movement 120):
// {(x, 1050), previousVector, (x, y), (x + 120, 1050)} with x = -50 + 120 k; the first
// previousVector is (-50, 800 + draw 0), so segment 0 has three vertices on x = -50 (and
// a zero edge when draws 0 and 1 are equal).  All coordinates are small integers (exact).
DEV void rough_segment(Poly<4>& f, int k, float yprev, float y) {
  const float x = -50.0f + 120.0f * (float)k;
  f.x[0] = x;                         f.y[0] = 1050.0f;
  f.x[1] = k == 0 ? x : x - 120.0f;   f.y[1] = yprev;
  f.x[2] = x;                         f.y[2] = y;
  f.x[3] = x + 120.0f;                f.y[3] = 1050.0f;
  find_centroid(f);
}

// a walker part's candidate pair(s) against the floor: the flat box (Environment.cs:211-226)
// or, with RoughFloor, the 10 static segments in list order (ter: this walker's 11 terrain
// heights in LDS, stride TS)
template <int N, bool TRACE, int L, bool ROUGH, int TS = 64>
DEV void floor_pairs(Poly<N>& P, Dyn& D, const Mat& m, bool& col, PairTraceDev* tr, int pi,
                     int sub, const float* ter, uint32_t* ec = nullptr) {
  Dyn dfl;
  zero_dyn(dfl);
  const Mat mf{0.0f, 0.0f, 0.3f, 1.0f};  // Metal, static: inverse mass/inertia 0
  if constexpr (ROUGH) {
    // Only the segments whose x-extent can reach the part's are visited: segment k spans
    // [x_k - 120, x_k + 120] (k = 0: from x_0), x_k = -50 + 120 k, so a segment with
    // x_k + 120 <= mnx or x_k - 120 >= mxx fails the pair's own bounding-box test; the range
    // below keeps one more segment on each side (rounding of the bound itself), so every
    // segment it leaves out is more than 100 px clear.  In list order as before; once the
    // part has moved (a resolved pair) the remaining segments are all visited, as the full
    // loop would test them against the moved part.  A non-finite or huge box: every segment.
    // With the lane order by start offset a part spans 3-5 segments of the 10.
    float mnx, mny, mxx, mxy;
    aabb(P, mnx, mny, mxx, mxy);
    int k = 0, kend = 9;
    if (mnx >= -1.0e6f && mxx <= 1.0e6f) {
      k = max(0, (int)floorf((mnx - 70.0f) * (1.0f / 120.0f)) - 1);
      kend = min(9, (int)floorf((mxx + 170.0f) * (1.0f / 120.0f)) + 1);
    }
#pragma unroll 1
    for (; k <= kend; k++) {
      Poly<4> seg;
      rough_segment(seg, k, ter[k * TS], ter[(k + 1) * TS]);
      const float cx0 = P.cx, cy0 = P.cy;
      resolve_pair<N, 4, true, TRACE, L, true>(P, D, m, seg, dfl, mf, col, tr, -1, sub, nullptr, ec);
      if (!(P.cx == cx0 && P.cy == cy0)) kend = 9;
    }
  } else {
    Poly<4> fl;
    floor_poly(fl);
    resolve_pair<N, 4, true, TRACE, L>(P, D, m, fl, dfl, mf, col, tr, pi, sub, nullptr, ec);
  }
}

// one substep of Environment.StepObjects (:130-142); ec: event counters (counting replay)
template <bool TRACE, int L, bool ROUGH>
DEV void substep(EnvState& s, const Mat& mp, const Mat& mb, float dt, float adx, float ady,
                 PairTraceDev* tr, int sub, const float* ter, uint32_t* ec = nullptr) {
  // joints: [bodyJointLeft, bodyJointRight, leftJoint, rightJoint] (Walker.cs:182-187)
  joint_step<5, 6, 1, 4, TRACE>(s.body, s.dbody, mb, s.llu, s.dllu, mp, tr, 0, ec);
  joint_step<5, 6, 1, 4, TRACE>(s.body, s.dbody, mb, s.rlu, s.drlu, mp, tr, 1, ec);
  joint_step<6, 6, 2, 3, TRACE>(s.llu, s.dllu, mp, s.lll, s.dlll, mp, tr, 2, ec);
  joint_step<6, 6, 2, 3, TRACE>(s.rlu, s.drlu, mp, s.rll, s.drll, mp, tr, 3, ec);
  // bodies in list order; the floor's own step is a no-op (static, zero velocity).
  // Episode 0 lists the floor last, every later episode first (Walker.cs:212-234):
  // that only changes the order of each leg segment's candidate pairs.
  integrate(s.lll, s.dlll, dt, adx, ady);
#pragma unroll 1
  for (int q = 0; q < 2; q++) {
    if ((q == 0) == s.post) floor_pairs<6, TRACE, L, ROUGH>(s.lll, s.dlll, mp, s.clll, tr, 1, sub, ter, ec);
    else resolve_pair<6, 6, false, TRACE, L>(s.lll, s.dlll, mp, s.llu, s.dllu, mp, s.clll, tr, 0, sub, nullptr, ec);
  }
  integrate(s.llu, s.dllu, dt, adx, ady);
#pragma unroll 1
  for (int q = 0; q < 2; q++) {
    if ((q == 0) == s.post) floor_pairs<6, TRACE, L, ROUGH>(s.llu, s.dllu, mp, s.cllu, tr, 3, sub, ter, ec);
    else resolve_pair<6, 6, false, TRACE, L>(s.llu, s.dllu, mp, s.lll, s.dlll, mp, s.cllu, tr, 2, sub, nullptr, ec);
  }
  integrate(s.body, s.dbody, dt, adx, ady);
  floor_pairs<5, TRACE, L, ROUGH>(s.body, s.dbody, mb, s.cbody, tr, 4, sub, ter, ec);
  integrate(s.rll, s.drll, dt, adx, ady);
#pragma unroll 1
  for (int q = 0; q < 2; q++) {
    if ((q == 0) == s.post) floor_pairs<6, TRACE, L, ROUGH>(s.rll, s.drll, mp, s.crll, tr, 6, sub, ter, ec);
    else resolve_pair<6, 6, false, TRACE, L>(s.rll, s.drll, mp, s.rlu, s.drlu, mp, s.crll, tr, 5, sub, nullptr, ec);
  }
  integrate(s.rlu, s.drlu, dt, adx, ady);
#pragma unroll 1
  for (int q = 0; q < 2; q++) {
    if ((q == 0) == s.post) floor_pairs<6, TRACE, L, ROUGH>(s.rlu, s.drlu, mp, s.crlu, tr, 8, sub, ter, ec);
    else resolve_pair<6, 6, false, TRACE, L>(s.rlu, s.drlu, mp, s.rll, s.drll, mp, s.crlu, tr, 7, sub, nullptr, ec);
  }
  if (ec) ec[EV_SUBSTEPS]++;
}

// ---------------- policy (fused, weights read with wave-uniform scalar loads) ----------
// DenseLayer.FeedForward (DenseLayer.cs:82-98): z_j = (sum_k W[j][k] x[k], in order) + b_j
DEV void actor_mean(const float* __restrict__ W, const float s[12], float mean[4]) {
  float h1[64];
#pragma unroll
  for (int j = 0; j < 64; j++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 12; k++) acc = acc + W[OFF_A_W1 + j * 12 + k] * s[k];
    float z = acc + W[OFF_A_B1 + j];
    h1[j] = net_maxf(0.2f * z, z);
  }
  float z3[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 2
  for (int j = 0; j < 64; j++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 64; k++) acc = acc + W[OFF_A_W2 + j * 64 + k] * h1[k];
    float z = acc + W[OFF_A_B2 + j];
    float h2 = net_maxf(0.2f * z, z);
#pragma unroll
    for (int d = 0; d < 4; d++) z3[d] = z3[d] + W[OFF_A_W3 + d * 64 + j] * h2;
  }
#pragma unroll
  for (int d = 0; d < 4; d++) mean[d] = tanhf(z3[d] + W[OFF_A_B3 + d]);
}

DEV float critic_value(const float* __restrict__ W, const float s[12]) {
  float v = 0.0f;
#pragma unroll 4
  for (int j = 0; j < 64; j++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 12; k++) acc = acc + W[OFF_C_W1 + j * 12 + k] * s[k];
    float z = acc + W[OFF_C_B1 + j];
    float h = net_maxf(0.2f * z, z);
    v = v + W[OFF_C_W2 + j] * h;
  }
  return v + W[OFF_C_B2];
}

// NormalDistribution.BoxMullerTransform (NormalDistribution.cs:12-19) with Philox draws
DEV void sample_actions(const EnvParams& P, float lp_const, uint32_t gid, uint32_t t,
                        const float mean[4], float act[4], float logp[4]) {
  const float PI_F = 3.14159265358979323846f;
#pragma unroll
  for (int d = 0; d < 4; d++) {
    U4 o = philox(P.seed, gid, t, (uint32_t)d, ST_ACT);
    float u1 = next_double_f(o.x, o.y);
    float u2 = next_double_f(o.z, o.w);
    if (u1 == 0.0f) u1 = 1.0f;
    float z = sqrtf(-2.0f * logf(u1)) * sinf(2.0f * PI_F * u2);
    act[d] = mean[d] + (P.std_ * z);
  }
#pragma unroll
  for (int d = 0; d < 4; d++) {
    // LogProbabilityDensity (:24-32); lp_const = -ln(std) - ln(sqrt(2 pi)) (host libm)
    float fraction = (act[d] - mean[d]) / P.std_;
    fraction *= fraction;
    fraction /= 2.0f;
    logp[d] = lp_const - fraction;
  }
}

// Row-parallel policy for L = 16 lanes per walker: lane `sub` owns neurons 4*sub..4*sub+3
// of every 64-wide layer (each neuron's sum stays sequential in k, so the values are
// bit-identical to actor_mean / critic_value); activations cross lanes through a
// 192-float LDS slice per walker.  Lanes 0..3 own one action dimension each (output
// neuron, Philox draw, log-density), lane 4 the critic output; results are broadcast
// back to the row.
DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

DEV void policy_row(const EnvParams& P, const float* __restrict__ W, float lp_const,
                    uint32_t gid, uint32_t t, const float obs[12], int sub, int row_base,
                    float* __restrict__ h, bool want_value, float act[4], float logp[4],
                    float& value) {
  float* h1 = h;
  float* h2 = h + 64;
  float* hc = h + 128;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int j = sub * 4 + q;
    float za = 0.0f, zc = 0.0f;
#pragma unroll
    for (int k = 0; k < 12; k++) {
      za = za + W[OFF_A_W1 + j * 12 + k] * obs[k];
      zc = zc + W[OFF_C_W1 + j * 12 + k] * obs[k];
    }
    za = za + W[OFF_A_B1 + j];
    zc = zc + W[OFF_C_B1 + j];
    h1[j] = net_maxf(0.2f * za, za);
    hc[j] = net_maxf(0.2f * zc, zc);
  }
  wave_lds_sync();
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int j = sub * 4 + q;
    float z = 0.0f;
#pragma unroll 16
    for (int k = 0; k < 64; k++) z = z + W[OFF_A_W2 + j * 64 + k] * h1[k];
    z = z + W[OFF_A_B2 + j];
    h2[j] = net_maxf(0.2f * z, z);
  }
  wave_lds_sync();
  // output neurons: lanes 0..3 actor (W3 row d on h2), lane 4 critic (Wc2 on hc)
  const int d = sub & 3;
  const bool vlane = sub == 4;
  const float* wrow = vlane ? (W + OFF_C_W2) : (W + OFF_A_W3 + d * 64);
  const float* xin = vlane ? hc : h2;
  float zo = 0.0f;
#pragma unroll 16
  for (int k = 0; k < 64; k++) zo = zo + wrow[k] * xin[k];
  zo = zo + (vlane ? W[OFF_C_B2] : W[OFF_A_B3 + d]);
  const float mean = tanhf(zo);
  // SampleActions for dimension d (PPOAgent.cs:381-398; NormalDistribution.cs:12-32)
  const float PI_F = 3.14159265358979323846f;
  U4 o = philox(P.seed, gid, t, (uint32_t)d, ST_ACT);
  float u1 = next_double_f(o.x, o.y);
  const float u2 = next_double_f(o.z, o.w);
  if (u1 == 0.0f) u1 = 1.0f;
  const float zn = sqrtf(-2.0f * logf(u1)) * sinf(2.0f * PI_F * u2);
  const float a = mean + (P.std_ * zn);
  float fraction = (a - mean) / P.std_;
  fraction *= fraction;
  fraction /= 2.0f;
  const float lp = lp_const - fraction;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    act[q] = __shfl(a, row_base + q);
    logp[q] = __shfl(lp, row_base + q);
  }
  value = want_value ? __shfl(zo, row_base + 4) : 0.0f;
  wave_lds_sync();  // the slice is rewritten by the next env-step
}

// WK_FAULT_NONFINITE: x * 0 is NaN exactly for a NaN or infinite x, so the sum over every
// vertex, centroid and velocity of the walker stays 0 iff all are finite (once per env-step)
template <int N>
DEV float nonfinite_acc(const Poly<N>& p, const Dyn& d) {
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < N; i++) acc += p.x[i] * 0.0f + p.y[i] * 0.0f;
  return acc + (p.cx * 0.0f + p.cy * 0.0f) + (d.vx * 0.0f + d.vy * 0.0f) + (d.w * 0.0f + d.th * 0.0f);
}
DEV bool state_finite(const EnvState& s) {
  const float acc = nonfinite_acc(s.lll, s.dlll) + nonfinite_acc(s.llu, s.dllu) +
                    nonfinite_acc(s.rll, s.drll) + nonfinite_acc(s.rlu, s.drlu) +
                    nonfinite_acc(s.body, s.dbody);
  return acc == 0.0f;
}

// L lanes per walker (a "row"): the Gauss-Seidel chain runs replicated in every lane of
// the row (bit-identical state), SAT axes are split one per lane (sat_row); lane 0 of
// the row owns all stores.  L = 1 is the plain one-walker-per-lane mapping.
// COUNT (one lane per walker, flat floor, given actions): the counting replay -- the same
// physics with per-lane event counters summed into A.counts (SURVEY 8(d) F_counted).
// Pacing of co-resident waves (k_env_side's pair mapping: two 4-wave blocks per CU; k_env_step:
// two 64-lane blocks per SIMD).  The SIMD arbitrates VALU issue between its co-resident waves by
// priority, then age (MI355X_MICROARCH.md, "Two waves per SIMD"): at equal priority the older
// block's waves issue first, so in the 65,536-walker rollout they finished their 64 env-steps in
// ~25 ms while the younger block's waves, left the spare slots, ran on alone for another ~14 ms at
// one wave per SIMD (per-wave clocks, scripts/r06_wave_clock.py, profiles/r06_wave_clock.txt).
// Each wave publishes (launch, env-step) in its SIMD's slot once per env-step -- an atomic max
// from one lane -- and runs at priority 1 while the slot says another wave there is ahead, 0
// otherwise, so the waves keep pace and share the SIMD to the end.  Scheduling only: no result
// depends on it.
DEV void pace_partner(unsigned long long* pace, uint32_t seq, int k) {
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);  // HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // XCC_ID[3:0]
  const uint32_t slot = (((((xcc & 7u) * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u +
                          ((hw >> 8) & 15u)) * 4u) + ((hw >> 4) & 3u);  // (XCC, SE, SH, CU, SIMD)
  const unsigned long long tag = ((unsigned long long)seq << 32) | (uint32_t)k;
  unsigned long long prev = 0;
  if ((threadIdx.x & 63) == 0) prev = atomicMax(&pace[slot], tag);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(prev >> 32), 0);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)prev, 0);
  if ((((unsigned long long)hi << 32) | lo) > tag) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

template <bool POLICY, bool RECORD, bool TRACE, int L, bool ROUGH, bool COUNT = false>
__global__ __launch_bounds__(64) WK_ENV_WPE void k_env_step(EnvParams P, StepArgs A) {
  static_assert(!COUNT || (L == 1 && !POLICY && !TRACE), "counting replay");
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = tid / L, sub = tid % L;
  const int n = P.n_env;
  if (e >= n) return;  // whole rows exit together
  const bool leader = sub == 0;
  __shared__ float pol_lds[(L == 16 && POLICY) ? 4 * 192 : 1];
  // the walker's rough-floor heights 800 + Random.Next(0, 100), [draw][walker of block]:
  // each lane writes and later reads only its own walker's column (no barrier needed)
  __shared__ float ter_lds[ROUGH ? 11 * 64 : 1];
  float* ter = ter_lds + (threadIdx.x / L);
  if constexpr (ROUGH) {
#pragma unroll 1
    for (int i = 0; i < 11; i++)
      ter[i * 64] = 800.0f + (float)terrain_draw(P.seed, (uint32_t)(P.env_offset + e), i);
  }
  EnvState s;
  load_state(s, A.st, e, n);
  const float dx = A.dxoff[e];
  const MatConst mc = material(A.mat[e]);
  const Mat mp{mc.inv_mass, 0.001f * mc.inv_mass, mc.restitution, mc.friction};
  const Mat mb{mc.inv_mass, 0.0003f, mc.restitution, mc.friction};  // Walker.cs:168
  const float dt = P.dt_sub;
  const float adx = 0.0f * dt, ady = 980.0f * dt;  // _acceleration * deltaTime
  const uint32_t gid = (uint32_t)(P.env_offset + e);
  uint32_t t = A.rng_t[e];
  uint32_t fault = 0;
  uint32_t ecnt[NEV];
#pragma unroll
  for (int i = 0; i < NEV; i++) ecnt[i] = 0u;
  uint32_t* const ec = COUNT ? ecnt : nullptr;

#pragma unroll 1
  for (int k = 0; k < A.k_steps; k++) {
    float a[4], lp[4], obs[12];
    if (A.pace) pace_partner(A.pace, A.pace_seq, k);  // (lane 0 always holds a walker)
    if (POLICY) {
      get_obs(s, obs);
      float v = 0.0f;
      if constexpr (L == 16) {
        policy_row(P, A.W, A.lp_const, gid, t, obs, sub, threadIdx.x & ~15,
                   pol_lds + (threadIdx.x >> 4) * 192, RECORD, a, lp, v);
      } else {
        float mean[4];
        actor_mean(A.W, obs, mean);
        sample_actions(P, A.lp_const, gid, t, mean, a, lp);
        if (RECORD) v = critic_value(A.W, obs);
      }
      if (RECORD) {
        if (leader) {
          const size_t idx = (size_t)(A.t0 + k) * n + e;
#pragma unroll
          for (int i = 0; i < 12; i++) A.traj_s[idx * 12 + i] = obs[i];
#pragma unroll
          for (int d = 0; d < 4; d++) {
            A.traj_a[idx * 4 + d] = a[d];
            A.traj_lp[idx * 4 + d] = lp[d];
          }
          A.traj_v[idx] = v;
        }
      }
    } else {
#pragma unroll
      for (int d = 0; d < 4; d++) a[d] = A.actions[((size_t)k * n + e) * 4 + d];
    }
    // Environment.Update (:71-78)
    s.steps++;
    float ac[4];
#pragma unroll
    for (int d = 0; d < 4; d++) ac[d] = clip1(a[d]);
    // Joint.SetTorque on joints [Body-LLU, Body-RLU, LLU-LLL, RLU-RLL]: child w += 5*change
    {
      float c;
      c = ac[0] - s.torque[0]; s.torque[0] = ac[0]; s.dllu.w = s.dllu.w + c * 5.0f;
      c = ac[1] - s.torque[1]; s.torque[1] = ac[1]; s.drlu.w = s.drlu.w + c * 5.0f;
      c = ac[2] - s.torque[2]; s.torque[2] = ac[2]; s.dlll.w = s.dlll.w + c * 5.0f;
      c = ac[3] - s.torque[3]; s.torque[3] = ac[3]; s.drll.w = s.drll.w + c * 5.0f;
    }
    // StepObjects
    const uint32_t lf0 = ecnt[EV_AABB_LF], ll0 = ecnt[EV_SAT_LL];
#pragma unroll 1
    for (int it = 0; it < P.iterations; it++) {
      PairTraceDev* tr = nullptr;
      if (TRACE && leader) {
        tr = A.trace + ((size_t)e * P.iterations + it);
        PairTraceDev z = {};
        *tr = z;
      }
      substep<TRACE, L, ROUGH>(s, mp, mb, dt, adx, ady, tr, sub, ter, ec);
    }
    if (COUNT) {
      ecnt[EV_ENV_STEPS]++;
      ecnt[EV_STEPS_LF] += ecnt[EV_AABB_LF] != lf0 ? 1u : 0u;
      ecnt[EV_STEPS_SATLL] += ecnt[EV_SAT_LL] != ll0 ? 1u : 0u;
    }
    // Walker.Update
    s.prevx = s.posx; s.prevy = s.posy;
    s.posx = s.body.cx; s.posy = s.body.cy;
    if (s.cbody || s.cllu || s.crlu) s.terminal = true;
    // CalculateReward
    float reward = 0.0f;
    float dX = s.posx - s.prevx;
    float yb = s.body.y[1];
    reward = reward + ((dX > 0.0f && ((yb / 500.0f) < 1.6f)) ? dX : 0.0f);
    reward = reward - (((yb / 500.0f) > 1.65f) ? -0.1f : 0.0f);
    bool terminal = false;
    if (s.terminal || s.steps > P.max_timesteps) {
      if (s.terminal) reward -= 40.0f;
      terminal = true;
    }
    if (s.posx > 900.0f) {
      reward += 80.0f;
      terminal = true;
    }
    if (!state_finite(s)) fault |= 1u;
    if (A.pos_out && leader) {
      A.pos_out[((size_t)k * n + e) * 2] = s.posx;
      A.pos_out[((size_t)k * n + e) * 2 + 1] = s.posy;
    }
    if (terminal) {
      int ep = s.episodes + 1;
      make_template(s, dx);
      s.post = true;
      s.episodes = ep;
      if (COUNT) ecnt[EV_RESETS]++;
    }
    if (leader) {
      if (A.obs_out) {
        get_obs(s, obs);
#pragma unroll
        for (int i = 0; i < 12; i++) A.obs_out[((size_t)k * n + e) * 12 + i] = obs[i];
      }
      if (A.rew_out) A.rew_out[(size_t)k * n + e] = reward;
      if (A.done_out) A.done_out[(size_t)k * n + e] = terminal ? 1 : 0;
      if (RECORD) {
        const size_t idx = (size_t)(A.t0 + k) * n + e;
        A.traj_r[idx] = reward;
        A.traj_d[idx] = terminal ? 1 : 0;
      }
    }
    t++;
  }
  if (leader) {
    store_state(s, A.st, e, n);
    A.rng_t[e] = t;
    if (A.fault_out) A.fault_out[e] |= fault;
  }
  if constexpr (COUNT) {  // wave sums, one 64-bit atomic per counter and wave
#pragma unroll
    for (int i = 0; i < NEV; i++) {
      uint32_t v = ecnt[i];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
      if ((threadIdx.x & 63) == 0 && v) atomicAdd(A.counts + i, (unsigned long long)v);
    }
  }
}

// ---------------- side-split mapping: a lane pair per walker (L = 2) ----------------
// Lane `side` of the pair (0 = left leg, 1 = right leg) owns that leg's two segments; the
// torso is held replicated by both.  Inside StepObjects (Environment.cs:130-142) the
// RigidBody.Step calls run in list order LLL, LLU, BODY, RLL, RLU and every candidate
// pair is either inside one leg or against the static floor (Walker.cs:212-234), so the
// left and right collision chains touch disjoint bodies: both run at once, one per lane,
// and the torso's own step + floor pair runs replicated (bit-identical in both lanes).
// Joints 0 and 1 (Walker.cs:182-187) both move the torso, so they run one lane at a time
// with the torso copied across the pair after each; joints 2 and 3 run at once.  Every
// per-body operation is the same op sequence as the one-lane mapping, so trajectories
// stay bit-identical to the oracle.
struct SideState {
  Poly<6> lo, up;  // this side's lower / upper leg segment
  Poly<5> body;
  Dyn dlo, dup, dbody;
  bool clo, cup, cbody;
  float tq_up, tq_lo;  // joint torques [side] (body-upper) and [2 + side] (upper-lower)
  float posx, posy, prevx, prevy;
  int steps, episodes;
  bool post, terminal;
};

// the legs' 24 vertex coordinates (NR = 6 records; NR = 4: the first 16 of them) to / from a
// lane's float4 column (stride FS); see k_env_side
template <int FS, int NR = 6>
DEV void park_legs(const SideState& s, float4* r) {
  r[0 * FS] = make_float4(s.lo.x[0], s.lo.x[1], s.lo.x[2], s.lo.x[3]);
  r[1 * FS] = make_float4(s.lo.x[4], s.lo.x[5], s.lo.y[0], s.lo.y[1]);
  r[2 * FS] = make_float4(s.lo.y[2], s.lo.y[3], s.lo.y[4], s.lo.y[5]);
  r[3 * FS] = make_float4(s.up.x[0], s.up.x[1], s.up.x[2], s.up.x[3]);
  if constexpr (NR == 6) {
    r[4 * FS] = make_float4(s.up.x[4], s.up.x[5], s.up.y[0], s.up.y[1]);
    r[5 * FS] = make_float4(s.up.y[2], s.up.y[3], s.up.y[4], s.up.y[5]);
  }
}
template <int FS, int NR = 6>
DEV void unpark_legs(SideState& s, const float4* r) {
  float4 a = r[0 * FS], b = r[1 * FS], c = r[2 * FS];
  s.lo.x[0] = a.x; s.lo.x[1] = a.y; s.lo.x[2] = a.z; s.lo.x[3] = a.w;
  s.lo.x[4] = b.x; s.lo.x[5] = b.y; s.lo.y[0] = b.z; s.lo.y[1] = b.w;
  s.lo.y[2] = c.x; s.lo.y[3] = c.y; s.lo.y[4] = c.z; s.lo.y[5] = c.w;
  a = r[3 * FS];
  s.up.x[0] = a.x; s.up.x[1] = a.y; s.up.x[2] = a.z; s.up.x[3] = a.w;
  if constexpr (NR == 6) {
    b = r[4 * FS]; c = r[5 * FS];
    s.up.x[4] = b.x; s.up.x[5] = b.y; s.up.y[0] = b.z; s.up.y[1] = b.w;
    s.up.y[2] = c.x; s.up.y[3] = c.y; s.up.y[4] = c.z; s.up.y[5] = c.w;
  }
}

template <int CTRL>
DEV float dppc(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
DEV float pswap(float v) { return dppc<0xB1>(v); }  // quad_perm [1,0,3,2]: the partner lane

// copy the torso from the even (CTRL = quad_perm [0,0,2,2]) or odd ([1,1,3,3]) lane
template <int CTRL>
DEV void bcast_torso(Poly<5>& b, Dyn& d) {
#pragma unroll
  for (int i = 0; i < 5; i++) { b.x[i] = dppc<CTRL>(b.x[i]); b.y[i] = dppc<CTRL>(b.y[i]); }
  b.cx = dppc<CTRL>(b.cx); b.cy = dppc<CTRL>(b.cy);
  d.vx = dppc<CTRL>(d.vx); d.vy = dppc<CTRL>(d.vy); d.w = dppc<CTRL>(d.w);
}

DEV void load_side(SideState& s, const float* __restrict__ st, int e, int side) {
  const int blo = side ? RLL : LLL, bup = side ? RLU : LLU;
  load_poly(s.lo, st, blo, e, 0);
  load_poly(s.up, st, bup, e, 0);
  load_poly(s.body, st, BODY, e, 0);
  load_dyn(s.dlo, s.clo, st, blo, e, 0);
  load_dyn(s.dup, s.cup, st, bup, e, 0);
  load_dyn(s.dbody, s.cbody, st, BODY, e, 0);
  const float* r = st + (size_t)e * NSTATE;
  s.tq_up = r[S_TORQUE + side];
  s.tq_lo = r[S_TORQUE + 2 + side];
  s.posx = r[S_POS]; s.posy = r[S_POS + 1];
  s.prevx = r[S_PREV]; s.prevy = r[S_PREV + 1];
  s.steps = (int)r[S_STEPS];
  s.post = r[S_POSTRESET] != 0.0f;
  s.terminal = r[S_TERMINAL] != 0.0f;
  s.episodes = (int)r[S_EPISODES];
}

DEV void store_side(const SideState& s, float* __restrict__ st, int e, int side) {
  store_body(s.lo, s.dlo, s.clo, st, side ? RLL : LLL, e, 0);
  store_body(s.up, s.dup, s.cup, st, side ? RLU : LLU, e, 0);
  float* r = st + (size_t)e * NSTATE;
  r[S_TORQUE + side] = s.tq_up;
  r[S_TORQUE + 2 + side] = s.tq_lo;
  if (side == 0) {
    store_body(s.body, s.dbody, s.cbody, st, BODY, e, 0);
    r[S_POS] = s.posx; r[S_POS + 1] = s.posy;
    r[S_PREV] = s.prevx; r[S_PREV + 1] = s.prevy;
    r[S_STEPS] = (float)s.steps;
    r[S_POSTRESET] = s.post ? 1.0f : 0.0f;
    r[S_TERMINAL] = s.terminal ? 1.0f : 0.0f;
    r[S_EPISODES] = (float)s.episodes;
  }
}

// Walker.CreateCreature / Reset (both legs are the same two poles) -- cf. make_template
DEV void make_template_side(SideState& s, float dx) {
  float px = 125.0f + dx, py = 800.0f;
  s.body.x[0] = px + 20; s.body.y[0] = py + 20;
  s.body.x[1] = px;      s.body.y[1] = py + 20;
  s.body.x[2] = px - 20; s.body.y[2] = py + 20;
  s.body.x[3] = px - 20; s.body.y[3] = py - 20;
  s.body.x[4] = px + 20; s.body.y[4] = py - 20;
  find_centroid(s.body);
  make_pole(s.up, px + 0.0f, py + 30.0f);
  make_pole(s.lo, px + 0.0f, py + 60.0f);
  zero_dyn(s.dlo); zero_dyn(s.dup); zero_dyn(s.dbody);
  s.clo = s.cup = s.cbody = false;
  s.tq_up = 0.0f; s.tq_lo = 0.0f;
  s.steps = 0;
  s.terminal = false;
  s.prevx = px; s.prevy = py;
  s.posx = s.body.cx; s.posy = s.body.cy;
}

// Walker.GetState (Walker.cs:132-152) assembled from both lanes of the pair
DEV void get_obs_side(const SideState& s, int side, float o[12]) {
  const float ux = s.up.x[2], uy = s.up.y[2], tlo = s.dlo.th, tup = s.dup.th;
  const float oux = pswap(ux), ouy = pswap(uy), otlo = pswap(tlo), otup = pswap(tup);
  const bool left = side == 0;
  o[0] = s.body.x[1] / 900.0f;
  o[1] = s.body.y[1] / 500.0f;
  o[2] = (left ? ux : oux) / 900.0f;
  o[3] = (left ? uy : ouy) / 500.0f;
  o[4] = (left ? oux : ux) / 900.0f;
  o[5] = (left ? ouy : uy) / 500.0f;
  o[6] = s.dbody.vx / 60.0f;
  o[7] = s.dbody.vy / 60.0f;
  o[8] = left ? tlo : otlo;
  o[9] = left ? tup : otup;
  o[10] = left ? otlo : tlo;
  o[11] = left ? otup : tup;
}

// The torso's RigidBody.Step (RigidBody.cs:54-96), replicated in every lane of the walker (traced
// by the left lane): integrate, then its only candidate, the floor.  It reads and writes the torso
// alone (its leg pairs are associated bodies, Walker.cs:202-209), and no leg step reads the torso,
// so it commutes with the legs' steps that precede it in the list [LLL, LLU, Body, RLL, RLU]:
// substep_side runs it right after the joints, in the lower leg's integrate's basic
// block, where the two independent integrate chains interleave (bit-identical either way; round 5,
// within noise).
template <bool TRACE, bool ROUGH, int TS>
DEV void torso_step(SideState& s, const Mat& mb, float dt, float adx, float ady, PairTraceDev* tr,
                    int side, RegionProf* rp, const float* ter) {
  integrate(s.body, s.dbody, dt, adx, ady);
  rp_mark(rp, RP_INTEG, s.body.x[0], s.body.y[3], s.dbody.th);
  if constexpr (ROUGH) {
    floor_pairs<5, TRACE, 1, true, TS>(s.body, s.dbody, mb, s.cbody, side == 0 ? tr : nullptr, 4, 0, ter);
  } else {
    Poly<4> fl;
    floor_poly(fl);
    Dyn dfl;
    zero_dyn(dfl);
    const Mat mf{0.0f, 0.0f, 0.3f, 1.0f};
    resolve_pair<5, 4, true, TRACE, 1>(s.body, s.dbody, mb, fl, dfl, mf, s.cbody,
                                       side == 0 ? tr : nullptr, 4, 0, rp);
  }
}

// ROUGH: the floor candidates are CreateRoughFloor's 10 segments (floor_pairs, general SAT /
// contacts, replicated in both halves of the quad mapping; ter: this walker's terrain column in
// LDS with stride TS); the leg-leg pairs keep their split
template <bool TRACE, int Q, bool ROUGH = false, int TS = 1, int FS = 0>
DEV void substep_side(SideState& s, const Mat& mp, const Mat& mb, float dt, float adx, float ady,
                      PairTraceDev* tr, int side, int half, RegionProf* rp, const float* ter = nullptr,
                      float4* frec = nullptr) {
  rp_mark(rp, RP_OTHER);
  Poly<4> fl;
  floor_poly(fl);
  Dyn dfl;
  zero_dyn(dfl);
  const Mat mf{0.0f, 0.0f, 0.3f, 1.0f};
  // joints [bodyJointLeft, bodyJointRight, leftJoint, rightJoint] (Walker.cs:182-187)
  if (side == 0) joint_step<5, 6, 1, 4, TRACE>(s.body, s.dbody, mb, s.up, s.dup, mp, tr, 0);
  bcast_torso<0xA0>(s.body, s.dbody);
  if (side == 1) joint_step<5, 6, 1, 4, TRACE>(s.body, s.dbody, mb, s.up, s.dup, mp, tr, 1);
  bcast_torso<0xF5>(s.body, s.dbody);
  joint_step<6, 6, 2, 3, TRACE>(s.up, s.dup, mp, s.lo, s.dlo, mp, tr, 2 + side);
  rp_mark(rp, RP_JOINT, s.dup.w, s.dlo.w, s.up.x[0], s.lo.x[0], s.dbody.w, s.body.x[0]);
  // this leg's RigidBody.Step calls (lower then upper); a segment's two candidates run
  // floor-first after a reset, floor-last in episode 0: three slots keep a wave with
  // both kinds of walkers at three pair evaluations instead of four
  const int pb = side ? 5 : 0;
  torso_step<TRACE, ROUGH, TS>(s, mb, dt, adx, ady, tr, side, rp, ter);
  integrate(s.lo, s.dlo, dt, adx, ady);
  rp_mark(rp, RP_INTEG, s.lo.x[0], s.lo.y[3], s.lo.x[5], s.dlo.th);
#pragma unroll
  for (int q = 0; q < 3; q++) {  // [floor if post], other segment, [floor if episode 0]
    if (q == 1) resolve_pair<6, 6, false, TRACE, 1, false, Q, FS>(s.lo, s.dlo, mp, s.up, s.dup, mp, s.clo, tr, pb + 0, half, rp, nullptr, frec);
    else if ((q == 0) == s.post) {
      if constexpr (ROUGH) floor_pairs<6, TRACE, 1, true, TS>(s.lo, s.dlo, mp, s.clo, tr, pb + 1, 0, ter);
      else resolve_pair<6, 4, true, TRACE, 1, false, Q, FS>(s.lo, s.dlo, mp, fl, dfl, mf, s.clo, tr, pb + 1, half, rp, nullptr, frec);
    }
    rp_mark(rp, RP_OTHER);
  }
  integrate(s.up, s.dup, dt, adx, ady);
  rp_mark(rp, RP_INTEG, s.up.x[0], s.up.y[3], s.up.x[5], s.dup.th);
#pragma unroll
  for (int q = 0; q < 3; q++) {
    if (q == 1) resolve_pair<6, 6, false, TRACE, 1, false, Q, FS>(s.up, s.dup, mp, s.lo, s.dlo, mp, s.cup, tr, pb + 2, half, rp, nullptr, frec);
    else if ((q == 0) == s.post) {
      if constexpr (ROUGH) floor_pairs<6, TRACE, 1, true, TS>(s.up, s.dup, mp, s.cup, tr, pb + 3, 0, ter);
      else resolve_pair<6, 4, true, TRACE, 1, false, Q, FS>(s.up, s.dup, mp, fl, dfl, mf, s.cup, tr, pb + 3, half, rp, nullptr, frec);
    }
    rp_mark(rp, RP_OTHER);
  }
  rp_mark(rp, RP_OTHER);
}

DEV bool side_finite(const SideState& s) {  // this side's legs and the torso (see state_finite)
  const float acc = nonfinite_acc(s.lo, s.dlo) + nonfinite_acc(s.up, s.dup) + nonfinite_acc(s.body, s.dbody);
  return acc == 0.0f;
}

// PPOAgent.SampleActions / GetValueEstimate forward passes (NeuralNetwork.FeedForward,
// DenseLayer.cs:82-98) for the 32 walkers of a wave on the matrix cores, with the layouts
// of wk_ppo_mfma.hip: observations staged through LDS into v_mfma_f32_16x16x4_f32 B
// operands (walkers on n, two 16-walker tiles), W1 / W2 A operands streamed from the
// operand-order image (wk_mfma_layout.h, L2-resident), layer 2 chained on layer 1's D
// registers, and the 64-long output rows (actor W3, critic Wc2) on the VALU summed over
// the four lane groups.  fp32 throughout; only the association of the k-sums differs
// from the sequential reference (parity tests: rtol 1e-5).
typedef float pf4 __attribute__((ext_vector_type(4)));
// an opaque copy of a lane value: the address arithmetic built on it is redone where it is used
// instead of being strength-reduced into per-lane 64-bit pointers that live across a loop
DEV uint32_t lane_opaque(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
// the trajectory rows as plain stores.  Written bytes per rollout launch at 65,536 walkers
// (rollouts only, profiles/r05_write_probe.txt): non-temporal 439 MiB, plain 403 MiB against 384
// MiB algorithmic (385 MiB with the identity lane order): a walker the lane order moved into
// another wave writes into lines that wave fills, and plain stores let the L2 merge those parts
// before the line is written back; the one-byte done rows likewise (their 32 bytes per wave share
// a 128-byte line with three other waves).  Time unchanged.
template <typename T>
DEV void st_row(T v, T* p) { *p = v; }
DEV void st_row4(float* p, float a, float b, float c, float d) {
  const pf4 v = {a, b, c, d};
  st_row(v, (pf4*)p);
}
DEV pf4 pmfma(float a, float b, pf4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
DEV float plrelu(float z) { return z < 0.0f ? 0.2f * z : z; }  // == Math.Max(0.2 z, z), see mf_lrelu

// Q = 2 (quad mapping): 16 walkers per wave, one N tile
template <int Q>
DEV void policy_mfma(const float* __restrict__ Wz, const float obs[12], bool writer,
                     float* __restrict__ pl, float z3[4], float& value, int tx) {
  using namespace mf;
  constexpr int NT = 2 / Q;  // 16-walker tiles per wave
  const int lane = tx & 63, n = lane & 15, g = lane >> 4, wl = lane >> (Q == 2 ? 2 : 1);
  float* tile = pl;          // [32 walkers][16]: 12 observations
  float* outs = pl + 512;    // [32 walkers][8]: z3[0..3], critic output (disjoint from tile)
  if (writer) {
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const pf4 v = {obs[4 * q], obs[4 * q + 1], obs[4 * q + 2], obs[4 * q + 3]};
      *(pf4*)(tile + wl * 16 + 4 * q) = v;
    }
  }
  wave_lds_sync();
  // one 16-walker tile at a time (not unrolled): a tile's layer-1 activations (16 VGPRs) are
  // the only large live set, so the physics state around the call stays in registers
  // (two tiles at once spilled ~56 VGPRs of the walker state per env-step at 65,536 walkers)
  const pf4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 1
  for (int nt = 0; nt < NT; nt++) {
    float sB[3];
#pragma unroll
    for (int t = 0; t < 3; t++) sB[t] = tile[(16 * nt + n) * 16 + 4 * t + g];
    pf4 h1[4];
    float pv = 0.0f;
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++) {
      float wa[3], wc[3];
#pragma unroll
      for (int t = 0; t < 3; t++) {
        wa[t] = Wz[AW1F + (Mt * 3 + t) * 64 + lane];
        wc[t] = Wz[CW1F + (Mt * 3 + t) * 64 + lane];
      }
      const pf4 ba = *(const pf4*)(Wz + BA1 + 16 * Mt + 4 * g);
      const pf4 bc = *(const pf4*)(Wz + BC1 + 16 * Mt + 4 * g);
      const pf4 w2c = *(const pf4*)(Wz + WC2 + 16 * Mt + 4 * g);
      pf4 acc = z4, accc = z4;
#pragma unroll
      for (int t = 0; t < 3; t++) {
        acc = pmfma(wa[t], sB[t], acc);
        accc = pmfma(wc[t], sB[t], accc);
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        h1[Mt][r] = plrelu(acc[r] + ba[r]);
        pv = pv + w2c[r] * plrelu(accc[r] + bc[r]);
      }
    }
    float p3[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 1
    for (int Mt = 0; Mt < 4; Mt++) {  // not unrolled: keeps one Mt's weights in flight
      pf4 acc = z4;
#pragma unroll
      for (int Mp = 0; Mp < 4; Mp++) {
        const pf4 w = *(const pf4*)(Wz + W2F + ((Mt * 4 + Mp) * 64 + lane) * 4);
#pragma unroll
        for (int r = 0; r < 4; r++) acc = pmfma(w[r], h1[Mp][r], acc);
      }
      const pf4 b2 = *(const pf4*)(Wz + BA2 + 16 * Mt + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int k = 16 * Mt + 4 * g + r;
        const float h2 = plrelu(acc[r] + b2[r]);
#pragma unroll
        for (int d = 0; d < 4; d++) p3[d] = p3[d] + Wz[W3 + d * 64 + k] * h2;
      }
    }
    // the sums over the four lane groups (wk_mfma_layout.h: permlane swaps, the whole wave
    // active); lane (n, g) holds dim g's
    const float z3g = rows_rsum4(p3);
    pv = rows_sum4(pv);
    outs[(16 * nt + n) * 8 + g] = z3g;
    if (g == 0) outs[(16 * nt + n) * 8 + 4] = pv;
  }
  wave_lds_sync();  // the outputs are written before any lane reads its walker's
  const pf4 b3 = *(const pf4*)(Wz + BA3);
  const pf4 o = *(const pf4*)(outs + wl * 8);
#pragma unroll
  for (int d = 0; d < 4; d++) z3[d] = o[d] + b3[d];
  value = outs[wl * 8 + 4] + Wz[BC2];
  wave_lds_sync();  // outputs read before the next env-step rewrites the tile
}

constexpr int SIDE_BLOCK = SIDE_BLOCK_THREADS;  // 4 waves: the policy's weight image is staged once per block
// Q = 1: a lane pair per walker (L = 2); Q = 2: a lane quad (L = 4, side = lane bit 0, half =
// lane bit 1), for shards of at most one wave per SIMD, where the split shortens each wave's
// dependent chain -- with room for every register (one wave per SIMD: no spills)
template <bool POLICY, bool RECORD, bool TRACE, int Q, bool ROUGH = false>
__global__ __launch_bounds__(SIDE_BLOCK)
__attribute__((amdgpu_waves_per_eu(Q == 2 ? 1 : 2, Q == 2 ? 1 : 2)))  // (quad: one wave per SIMD)
void k_env_side(EnvParams P, StepArgs A) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int side = tid & 1;
  const int half = Q == 2 ? (tid >> 1) & 1 : 0;
  constexpr int SH = Q == 2 ? 2 : 1;  // log2 lanes per walker
  const int n = P.n_env;
  // sparse quad mapping (P.wpw < 16 walkers per wave, chosen so that one wave per SIMD still
  // holds every walker): the wave's first 4 wpw lanes hold wpw walkers, the other lanes replay
  // them (same walker, same branches, never store), so a wave's divergent branches are the
  // union over wpw walkers instead of sixteen
  const int wpw = Q == 2 ? P.wpw : 64 >> SH;  // (a power of two)
  const int eraw = ((tid >> 6) * wpw) + ((tid & ((wpw << SH) - 1)) >> SH);
  // a partial last wave keeps every lane (the policy's MFMAs need the whole wave):
  // out-of-range lanes replay walker n-1 and never store
  const bool active = eraw < n && (tid & 63) < (wpw << SH);
  // lane slot -> walker (wk_order.hip: episode-0 walkers first, so each wave's walkers visit
  // their floor pairs in one list order); every index below is the walker's own
  const int slot = eraw < n ? eraw : n - 1;
  const int e = A.order ? A.order[slot] : slot;
  const bool leader = side == 0 && half == 0 && active;
  __shared__ float pol_lds[POLICY ? (SIDE_BLOCK / 64) * 768 : 1];
  __shared__ float wz_lds[POLICY ? mf::WEND : 1];  // operand-order weights (41 KB, 2 blocks/CU)
  // RoughFloor: the walker's terrain heights 800 + Random.Next(0, 100) (Environment.cs:242-250),
  // [draw][walker of block]; the walker's lanes write the same values and read only its column
  constexpr int WPB = SIDE_BLOCK >> SH;
  __shared__ float ter_lds[ROUGH ? 11 * WPB : 1];
  // the pair mapping's contact faces (significant_face_lds): 6 float4 records per lane,
  // [record][lane of block] (24 KB per block; 2 blocks of 77 KB fit a CU's 160 KB -- not with the
  // rough floor's terrain as well, which would leave one block per CU).  The quad mapping keeps
  // the select chains (its LDS build: bit-exact, 1 % slower, profiles/r04_face_lds_ab.txt)
  constexpr int FS = (Q == 1 && !ROUGH) ? SIDE_BLOCK : 0;
  __shared__ float4 face_lds[FS ? 6 * SIDE_BLOCK : 1];
  // the rough floor's pair kernel has no face column (its terrain would push two blocks past the
  // CU's LDS); a 4-record column (16 KB per block, 2 x 75 KB fit) parks 16 of the legs' 24
  // vertex coordinates over the policy instead of leaving them to the spill
  constexpr int RS = (Q == 1 && ROUGH) ? SIDE_BLOCK : 0;
  __shared__ float4 rstash_lds[RS ? 4 * SIDE_BLOCK : 1];
  // the legs' stash across the policy section: the face column
  constexpr int SS = FS;
  const int wib = ((threadIdx.x >> 6) * wpw) + ((threadIdx.x & ((wpw << SH) - 1)) >> SH);
  const float* const ter = ter_lds + wib;
  if constexpr (ROUGH) {
#pragma unroll 1
    for (int i = 0; i < 11; i++)
      ter_lds[i * WPB + wib] = 800.0f + (float)terrain_draw(P.seed, (uint32_t)(P.env_offset + e), i);
  }
  if (POLICY) {
    for (int i = threadIdx.x; i < mf::WEND / 4; i += SIDE_BLOCK)
      ((pf4*)wz_lds)[i] = ((const pf4*)A.Wz)[i];
    __syncthreads();
  }
  SideState s;
  load_side(s, A.st, e, side);
  const MatConst mc = material(A.mat[e]);
  const Mat mp{mc.inv_mass, 0.001f * mc.inv_mass, mc.restitution, mc.friction};
  const Mat mb{mc.inv_mass, 0.0003f, mc.restitution, mc.friction};  // Walker.cs:168
  const float dt = P.dt_sub;
  const float adx = 0.0f * dt, ady = 980.0f * dt;
  uint32_t t = A.rng_t[e];
  uint32_t fault = 0;
  RP_KERNEL_BEGIN(SIDE_BLOCK / 64);  // (probe builds only, wk_region_prof.h)

#pragma unroll 1
  for (int k = 0; k < A.k_steps; k++) {
    float a[4], lp[4], obs[12];
    if (Q == 1 && A.pace) pace_partner(A.pace, A.pace_seq, k);
    rp_mark(rp, RP_OTHER);
    // every LDS address of the env-step derived from the thread index afresh (an opaque copy
    // made inside the loop): hoisted out of the loop they were ten loop-invariant VGPRs that
    // the register allocator kept in scratch
    const int tx = (int)lane_opaque(threadIdx.x);
    float4* const frec = face_lds + (FS ? tx : 0);
    float4* const stash = frec;
    float* const wave_pol = pol_lds + (POLICY ? (tx >> 6) * 768 : 0);
    if (POLICY) {
      get_obs_side(s, side, obs);
      // The policy's matrix-core section needs the most registers of the loop, while the legs'
      // 24 vertex coordinates wait unused until the substeps: park them in this lane's contact-
      // face column (free outside the contact clipping) rather than leave them to the spill; the
      // empty asm with a memory clobber keeps the compiler from forwarding the parked values in
      // registers across the section.  Pure data movement: bit-identical.
      if constexpr (SS != 0) {
        park_legs<SS>(s, stash);
        asm volatile("" ::: "memory");
      } else if constexpr (RS != 0) {
        park_legs<RS, 4>(s, rstash_lds + tx);
        asm volatile("" ::: "memory");
      }
      float z3[4], mean[4], v;
      policy_mfma<Q>(wz_lds, obs, side == 0 && half == 0, wave_pol, z3, v, tx);
#pragma unroll
      for (int d = 0; d < 4; d++) mean[d] = tanhf(z3[d]);
      // (the walker's Philox counter word through an opaque copy: the first round's per-lane
      // products are recomputed per env-step rather than hoisted into seven spilled VGPRs)
      sample_actions(P, A.lp_const, (uint32_t)P.env_offset + lane_opaque((uint32_t)e), t, mean, a, lp);
      if (RECORD && leader) {  // the rows: 16-byte plain stores (st_row)
        // row base (uniform, SGPRs) + the lane's 32-bit offset (global_store saddr form): no
        // per-lane 64-bit pointer per array stays live across the env-step loop (they spilled)
        const size_t row = (size_t)(A.t0 + k) * n;
        const uint32_t eo = lane_opaque((uint32_t)e);
#pragma unroll
        for (int q = 0; q < 3; q++)
          st_row4(A.traj_s + row * 12 + (eo * 12u + 4u * q), obs[4 * q], obs[4 * q + 1], obs[4 * q + 2],
                  obs[4 * q + 3]);
        st_row4(A.traj_a + row * 4 + eo * 4u, a[0], a[1], a[2], a[3]);
        st_row4(A.traj_lp + row * 4 + eo * 4u, lp[0], lp[1], lp[2], lp[3]);
        st_row(v, A.traj_v + row + eo);
      }
      if constexpr (SS != 0) {
        asm volatile("" ::: "memory");
        unpark_legs<SS>(s, stash);
      } else if constexpr (RS != 0) {
        asm volatile("" ::: "memory");
        unpark_legs<RS, 4>(s, rstash_lds + tx);
      }
    } else {
#pragma unroll
      for (int d = 0; d < 4; d++) a[d] = A.actions[((size_t)k * n + e) * 4 + d];
    }
    rp_mark(rp, RP_POLICY);
    s.steps++;
    // Clip + Joint.SetTorque: joint `side` drives this upper leg, joint 2+side the lower
    {
      const float au = clip1(side ? a[1] : a[0]), al = clip1(side ? a[3] : a[2]);
      float c = au - s.tq_up; s.tq_up = au; s.dup.w = s.dup.w + c * 5.0f;
      c = al - s.tq_lo; s.tq_lo = al; s.dlo.w = s.dlo.w + c * 5.0f;
    }
#pragma unroll 1
    for (int it = 0; it < P.iterations; it++) {
      PairTraceDev* tr = (TRACE && active && half == 0) ? A.trace + ((size_t)e * P.iterations + it) : nullptr;
      substep_side<TRACE, Q, ROUGH, WPB, FS>(s, mp, mb, dt, adx, ady, tr, side, half, rp, ter, frec);
    }
    // Walker.Update + terminal flags (both upper legs and the torso)
    s.prevx = s.posx; s.prevy = s.posy;
    s.posx = s.body.cx; s.posy = s.body.cy;
    const bool other_cup = pswap(s.cup ? 1.0f : 0.0f) != 0.0f;
    if (s.cbody || s.cup || other_cup) s.terminal = true;
    float reward = 0.0f;
    float dX = s.posx - s.prevx;
    float yb = s.body.y[1];
    reward = reward + ((dX > 0.0f && ((yb / 500.0f) < 1.6f)) ? dX : 0.0f);
    reward = reward - (((yb / 500.0f) > 1.65f) ? -0.1f : 0.0f);
    bool terminal = false;
    if (s.terminal || s.steps > P.max_timesteps) {
      if (s.terminal) reward -= 40.0f;
      terminal = true;
    }
    if (s.posx > 900.0f) {
      reward += 80.0f;
      terminal = true;
    }
    if (!side_finite(s)) fault |= 1u;
    const size_t krow = (size_t)k * n;  // (uniform) + the lane's 32-bit offset, as above
    const uint32_t eo = lane_opaque((uint32_t)e);
    if (A.pos_out && leader) {
      A.pos_out[krow * 2 + eo * 2u] = s.posx;
      A.pos_out[krow * 2 + (eo * 2u + 1u)] = s.posy;
    }
    if (terminal) {
      int ep = s.episodes + 1;
      // (the start offset re-read here: a loop-invariant dx or the template's vertices from it
      // would otherwise stay live, i.e. in scratch, across the whole loop)
      make_template_side(s, A.dxoff[lane_opaque((uint32_t)e)]);
      s.post = true;
      s.episodes = ep;
    }
    if (A.obs_out) {
      get_obs_side(s, side, obs);
      if (leader) {
#pragma unroll
        for (int i = 0; i < 12; i++) A.obs_out[krow * 12 + (eo * 12u + i)] = obs[i];
      }
    }
    if (leader) {
      if (A.rew_out) A.rew_out[krow + eo] = reward;
      if (A.done_out) A.done_out[krow + eo] = terminal ? 1 : 0;
      if (RECORD) {
        const size_t row = (size_t)(A.t0 + k) * n;
        st_row(reward, A.traj_r + row + eo);
        st_row((uint8_t)(terminal ? 1 : 0), A.traj_d + row + eo);
      }
    }
    t++;
  }
  // (the side and its record offsets formed here again: kept from the loads they stayed in scratch)
  if (active && half == 0) store_side(s, A.st, lane_opaque((uint32_t)e), (int)(lane_opaque(threadIdx.x) & 1u));
  RP_KERNEL_END();
  fault |= (uint32_t)pswap((float)fault);
  if (leader) {
    const uint32_t eo = lane_opaque((uint32_t)e);  // (addresses formed here, not kept from the loads)
    A.rng_t[eo] = t;
    if (A.fault_out) A.fault_out[eo] |= fault;
  }
}

// env initialisation: Environment ctor (Environment.cs:39-51) -- episode-0 body order
#if WK_PART(3)
__global__ void k_env_init(EnvParams P, float* st, const float* dxoff, const uint8_t* mask,
                           int post) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.n_env) return;
  if (mask && !mask[e]) return;
  EnvState s;
  int episodes = post ? (int)st[(size_t)e * NSTATE + S_EPISODES] : 0;
  make_template(s, dxoff[e]);
  s.post = post != 0;
  s.episodes = episodes;
  store_state(s, st, e, P.n_env);
}

__global__ void k_get_obs(EnvParams P, const float* st, float* obs) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.n_env) return;
  EnvState s;
  load_state(s, st, e, P.n_env);
  float o[12];
  get_obs(s, o);
  for (int i = 0; i < 12; i++) obs[(size_t)e * 12 + i] = o[i];
}

// standalone policy evaluation (wk_policy_sample / wk_value)
__global__ void k_policy(EnvParams P, const float* __restrict__ W, float lp_const, int n,
                         const float* obs, const int32_t* env_ids, const uint32_t* steps,
                         float* mean_out, float* act_out, float* logp_out, float* v_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s[12];
  for (int k = 0; k < 12; k++) s[k] = obs[(size_t)i * 12 + k];
  if (v_out) {
    v_out[i] = critic_value(W, s);
    return;
  }
  float mean[4], a[4], lp[4];
  actor_mean(W, s, mean);
  uint32_t gid = env_ids ? (uint32_t)env_ids[i] : (uint32_t)(P.env_offset + i);
  uint32_t t = steps ? steps[i] : 0u;
  sample_actions(P, lp_const, gid, t, mean, a, lp);
  for (int d = 0; d < 4; d++) {
    if (mean_out) mean_out[(size_t)i * 4 + d] = mean[d];
    if (act_out) act_out[(size_t)i * 4 + d] = a[d];
    if (logp_out) logp_out[(size_t)i * 4 + d] = lp[d];
  }
}

// returns / advantages (PPOAgent.cs:175-189, 414-498), one lane per env, reverse scan
// over the horizon; done[t] ends an episode at t.
__global__ void k_returns(int n, int T, int use_gae, float gamma, float lambda,
                          const float* __restrict__ r, const float* __restrict__ v,
                          const uint8_t* __restrict__ done, float* ret, float* adv) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  if (!use_gae) {
    float disc = 0.0f;
    for (int t = T - 1; t >= 0; t--) {
      size_t i = (size_t)t * n + e;
      if (done[i]) disc = 0.0f;
      disc = r[i] + (disc * gamma);
      ret[i] = disc;
      adv[i] = disc - v[i];
    }
  } else {
    float nextGae = 0.0f, nextValue = 0.0f;
    for (int t = T - 1; t >= 0; t--) {
      size_t i = (size_t)t * n + e;
      if (done[i]) nextValue = 0.0f;
      float cur = v[i];
      float delta = r[i] + (gamma * nextValue) - cur;
      nextValue = cur;
      float gae = delta + (gamma * lambda * nextGae);  // reference quirk: nextGae stays 0
      adv[i] = gae;
      ret[i] = gae + cur;
    }
  }
}

#endif  // WK_PART(3)
}  // namespace wk

#if WK_PART(2) || WK_PART(4) || WK_PART(6) || WK_PART(7)
namespace wk {
#include "wk_scene.inc"
}  // namespace wk
#endif

// host-side launch shims (C++ linkage, used by wk_api.cpp)
namespace wk {
template <int L, bool ROUGH>
static void launch_lanes_floor(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s) {
  dim3 blk(64), grd((unsigned)(((size_t)P.n_env * L + 63) / 64));
  switch (mode) {
    case 0: hipLaunchKernelGGL((k_env_step<false, false, false, L, ROUGH>), grd, blk, 0, s, P, A); break;
    case 1: hipLaunchKernelGGL((k_env_step<false, false, true, L, ROUGH>), grd, blk, 0, s, P, A); break;
    case 2: hipLaunchKernelGGL((k_env_step<true, false, false, L, ROUGH>), grd, blk, 0, s, P, A); break;
    default: hipLaunchKernelGGL((k_env_step<true, true, false, L, ROUGH>), grd, blk, 0, s, P, A); break;
  }
}
template <int L>
static void launch_lanes(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s) {
  if (P.rough) launch_lanes_floor<L, true>(mode, P, A, s);
  else launch_lanes_floor<L, false>(mode, P, A, s);
}
#if WK_PART(1) || WK_PART(5) || WK_PART(8)
template <int Q, bool ROUGH>
static void launch_side(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s) {
  const size_t lanes = Q == 2 ? ((size_t)P.n_env + P.wpw - 1) / P.wpw * 64 : (size_t)P.n_env * 2;
  dim3 blk(SIDE_BLOCK), grd((unsigned)((lanes + SIDE_BLOCK - 1) / SIDE_BLOCK));
  switch (mode) {
    case 0: hipLaunchKernelGGL((k_env_side<false, false, false, Q, ROUGH>), grd, blk, 0, s, P, A); break;
    case 1: hipLaunchKernelGGL((k_env_side<false, false, true, Q, ROUGH>), grd, blk, 0, s, P, A); break;
    case 2: hipLaunchKernelGGL((k_env_side<true, false, false, Q, ROUGH>), grd, blk, 0, s, P, A); break;
    default: hipLaunchKernelGGL((k_env_side<true, true, false, Q, ROUGH>), grd, blk, 0, s, P, A); break;
  }
}
#endif
#if WK_PART(1)
void launch_side_pair(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s) { launch_side<1, false>(mode, P, A, s); }
#endif
#if WK_PART(8)  // the quad mapping: its own part, built with the default scheduler (Makefile)
void launch_side_quad(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s) { launch_side<2, false>(mode, P, A, s); }
#endif
#if WK_PART(5)  // RoughFloor on the pair / quad mappings (their own build part: compile time)
void launch_side_pair_rough(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s) { launch_side<1, true>(mode, P, A, s); }
void launch_side_quad_rough(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s) { launch_side<2, true>(mode, P, A, s); }
#endif
#if WK_PART(2) || WK_PART(6)
template <bool ROUGH>
static void scene_given(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S, hipStream_t s) {
  dim3 blk(64), grd((unsigned)((P.n_env + 63) / 64));
  if (mode == 0) hipLaunchKernelGGL((k_env_scene<false, false, false, ROUGH>), grd, blk, 0, s, P, A, S);
  else hipLaunchKernelGGL((k_env_scene<false, false, true, ROUGH>), grd, blk, 0, s, P, A, S);
}
#endif
#if WK_PART(4) || WK_PART(7)
template <bool ROUGH>
static void scene_policy(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S, hipStream_t s) {
  dim3 blk(64), grd((unsigned)((P.n_env + 63) / 64));
  if (mode == 2) hipLaunchKernelGGL((k_env_scene<true, false, false, ROUGH>), grd, blk, 0, s, P, A, S);
  else hipLaunchKernelGGL((k_env_scene<true, true, false, ROUGH>), grd, blk, 0, s, P, A, S);
}
#endif
#if WK_PART(2)
void launch_env_scene_given(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                            hipStream_t s) { scene_given<false>(mode, P, A, S, s); }
#endif
#if WK_PART(6)  // scene props on the rough floor (own build parts: compile time)
void launch_env_scene_given_rough(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                                  hipStream_t s) { scene_given<true>(mode, P, A, S, s); }
#endif
#if WK_PART(4)
void launch_env_scene_policy(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                             hipStream_t s) { scene_policy<false>(mode, P, A, S, s); }
#endif
#if WK_PART(7)
void launch_env_scene_policy_rough(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                                   hipStream_t s) { scene_policy<true>(mode, P, A, S, s); }
#endif
#if WK_PART(3)
void launch_side_pair(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s);
void launch_side_quad(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s);
void launch_side_pair_rough(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s);
void launch_side_quad_rough(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s);
void launch_env_scene_given(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                            hipStream_t s);
void launch_env_scene_policy(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                             hipStream_t s);
void launch_env_scene_given_rough(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                                  hipStream_t s);
void launch_env_scene_policy_rough(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                                   hipStream_t s);
hipError_t launch_env_scene(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                            hipStream_t s) {
  if (mode <= 1) (P.rough ? launch_env_scene_given_rough : launch_env_scene_given)(mode, P, A, S, s);
  else (P.rough ? launch_env_scene_policy_rough : launch_env_scene_policy)(mode, P, A, S, s);
  return hipGetLastError();
}
hipError_t launch_env_step(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s) {
  if (mode == 4) {  // counting replay: one lane per walker, given actions (flat or rough floor)
    if (!A.counts || !A.actions) return hipErrorInvalidValue;
    dim3 blk(64), grd((unsigned)((P.n_env + 63) / 64));
    if (P.rough) hipLaunchKernelGGL((k_env_step<false, false, false, 1, true, true>), grd, blk, 0, s, P, A);
    else hipLaunchKernelGGL((k_env_step<false, false, false, 1, false, true>), grd, blk, 0, s, P, A);
    return hipGetLastError();
  }
  if (P.lanes == 2) (P.rough ? launch_side_pair_rough : launch_side_pair)(mode, P, A, s);
  else if (P.lanes == 4) (P.rough ? launch_side_quad_rough : launch_side_quad)(mode, P, A, s);
  else if (P.lanes == 16) launch_lanes<16>(mode, P, A, s);
  else launch_lanes<1>(mode, P, A, s);
  return hipGetLastError();
}
#endif  // WK_PART(3)
#if WK_PART(3)
hipError_t launch_env_init(const EnvParams& P, float* st, const float* dx, const uint8_t* mask,
                           int post, hipStream_t s) {
  hipLaunchKernelGGL(k_env_init, dim3((P.n_env + 255) / 256), dim3(256), 0, s, P, st, dx, mask, post);
  return hipGetLastError();
}
hipError_t launch_get_obs(const EnvParams& P, const float* st, float* obs, hipStream_t s) {
  hipLaunchKernelGGL(k_get_obs, dim3((P.n_env + 255) / 256), dim3(256), 0, s, P, st, obs);
  return hipGetLastError();
}
hipError_t launch_policy(const EnvParams& P, const float* W, float lp_const, int n,
                         const float* obs, const int32_t* env_ids, const uint32_t* steps,
                         float* mean, float* act, float* logp, float* v, hipStream_t s) {
  hipLaunchKernelGGL(k_policy, dim3((n + 63) / 64), dim3(64), 0, s, P, W, lp_const, n, obs,
                     env_ids, steps, mean, act, logp, v);
  return hipGetLastError();
}
hipError_t launch_returns(int n, int T, int use_gae, float gamma, float lambda, const float* r,
                          const float* v, const uint8_t* d, float* ret, float* adv,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_returns, dim3((n + 255) / 256), dim3(256), 0, s, n, T, use_gae, gamma,
                     lambda, r, v, d, ret, adv);
  return hipGetLastError();
}
#endif  // WK_PART(3)
}  // namespace wk
#if WK_PART(1)
RP_HOST_READER  // (probe builds only)
#endif
