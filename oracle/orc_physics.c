/*
 * orc_physics.c -- CPU restatement of the reference's physics step and environment.
 * TEST INFRASTRUCTURE ONLY (see wk_oracle.h).  PARITY UNPINNED (no C# toolchain; the
 * reference has no tests) -- pinned by the hand-derived KATs in tests/.
 *
 * Follows, line by line:
 *   Bodies/RigidBody.cs            (Step :54-61, ResolveCollisions :66-96, MoveObjects
 *                                   :99-113, StepLinear/AngularVelocity :116-129, Wrap :132-140)
 *   Bodies/Physics/SATCollision.cs (IsColliding :15-35, AxisChecks :39-59, Project :63-76,
 *                                   IsOverlapping :100-104)
 *   Bodies/Physics/ContactPoints.cs(GetContactPoints :13-53, ClipVectors :56-76,
 *                                   GetSignificantFace :79-94, GetSignificantVertex :97-113,
 *                                   Mod :131-134)
 *   Bodies/Physics/Impulses.cs     (ResolveCollisions :12-28, ResolveJoint :31-40,
 *                                   ApplyImpulses :57-82, CalculateImpulse :86-115)
 *   Objects/RigidBodies/Skeleton.cs(Move :76-85, Rotate :89-97, FindCentroid :100-113,
 *                                   BoundingBox :117-176)
 *   Objects/RigidBodies/Joint.cs   (Step :31-41, SetTorque :56-61)
 *   Objects/RigidBodies/Pole.cs:18-34, Hull.cs:23-29, Materials/<Name>.cs
 *   Walker/Walker.cs               (Update :49-54, TakeActions :66-75, GetState :132-152,
 *                                   CreateBodies :155-177, CreateJoints :180-188,
 *                                   AddAssociatedBodies :202-209, Reset :212-234)
 *   Environment.cs                 (Update :64-92, Step :96-122, StepObjects :126-143,
 *                                   CalculateReward :148-154, Reset :167-180, CreateFloor :211-226,
 *                                   CreateRoughFloor :230-261)
 */
#include "wk_oracle.h"
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------- MonoGame Vector2 (numeric contract) ---------------- */
typedef struct { float x, y; } v2;
static inline v2 V(float x, float y) { v2 r; r.x = x; r.y = y; return r; }
static inline v2 vadd(v2 a, v2 b) { return V(a.x + b.x, a.y + b.y); }
static inline v2 vsub(v2 a, v2 b) { return V(a.x - b.x, a.y - b.y); }
static inline v2 vmul(v2 a, float s) { return V(a.x * s, a.y * s); }
static inline v2 vdiv(v2 a, float d) { float f = 1.0f / d; return V(a.x * f, a.y * f); }
static inline v2 vneg(v2 a) { return V(-a.x, -a.y); }
static inline float vdot(v2 a, v2 b) { return a.x * b.x + a.y * b.y; }
static inline float vlen(v2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
static inline v2 vnormalize(v2 a) {
  float val = 1.0f / sqrtf(a.x * a.x + a.y * a.y);
  return V(a.x * val, a.y * val);
}
static inline int veq(v2 a, v2 b) { return a.x == b.x && a.y == b.y; }

/* System.Math.Min/Max(float,float), IEEE 754:2019 minimum/maximum (.NET Core 3.0+) */
static inline float net_minf(float x, float y) {
  if (x != y) { if (!isnan(x)) return x < y ? x : y; return x; }
  return signbit(x) ? x : y;
}
static inline float net_maxf(float x, float y) {
  if (x != y) { if (!isnan(x)) return y < x ? x : y; return x; }
  return signbit(y) ? x : y;
}

/* ---------------- materials (Materials/<Name>.cs) ---------------- */
typedef struct { float inv_mass, restitution, friction; } material;
static const material MATS[ORC_NMAT] = {
  {5.0f, 0.3f, 0.8f},     /* Carpet.cs:7-9 */
  {11.0f, 0.3f, 0.0f},    /* Ice.cs:7-9 */
  {11.0f, 0.7f, 0.5f},    /* Rubber.cs:7-9 */
  {15.0f, 0.3f, 1.0f},    /* Metal.cs:7-9 */
  {20.0f, 0.3f, 0.01f},   /* Wood.cs:7-9 */
  {1.0f, 0.3f, 0.1f},     /* Paper.cs:7-9 */
  {0.01f, 0.1f, 0.2f},    /* Titanium.cs:7-9 */
  {11.0f, 1.0f, 1.0f},    /* SuperRubber.cs:7-9 */
};

/* ---------------- rigid bodies ---------------- */
typedef struct {
  int nv;
  v2 v[ORC_PROP_MAXV];
  v2 centroid;
  int is_static, is_floor, collided;
  float inv_mass, inv_inertia, restitution, friction;
  v2 accel, lin_vel;
  float ang_vel, angle;
  int assoc[6], n_assoc;
} body;

typedef struct { int a, b, ia, ib; float torque; } joint;

enum { MAXB = 5 + ORC_ROUGH_SEGMENTS + ORC_MAX_PROPS };
struct orc_env {
  orc_hyper h;
  body bodies[MAXB];   /* ORC_LLL..ORC_RLU, the floor body / rough-floor segments, props */
  int order[MAXB];     /* List<RigidBody> order */
  int nbodies;         /* 6, or 15 with the rough floor, + props */
  int nprops;
  int rough;
  joint joints[4];
  v2 position, prev_position;
  v2 step_position;    /* position after the last Step, before any Reset (Environment.cs:119) */
  int terminal;
  int steps, episodes, post_reset;
  int material;
  float dx;
};

/* Skeleton.FindCentroid (Skeleton.cs:100-113): sum from Vector2.Zero, then sum /= count */
static v2 find_centroid(const v2* v, int n) {
  v2 s = V(0.0f, 0.0f);
  for (int i = 0; i < n; i++) s = vadd(s, v[i]);
  return vdiv(s, (float)n);
}

/* RigidBody ctor (RigidBody.cs:36-50) + Skeleton.AddVectors (Skeleton.cs:56-61) */
static void body_init(body* b, int mat, const v2* verts, int nv, int is_static, int is_floor) {
  memset(b, 0, sizeof(*b));
  b->nv = nv;
  for (int i = 0; i < nv; i++) b->v[i] = verts[i];
  b->centroid = find_centroid(b->v, nv);
  b->is_static = is_static;
  b->is_floor = is_floor;
  b->collided = 0;
  b->restitution = MATS[mat].restitution;
  b->friction = MATS[mat].friction;
  b->inv_mass = is_static ? 0.0f : MATS[mat].inv_mass;
  b->inv_inertia = is_static ? 0.0f : 0.001f * MATS[mat].inv_mass;
  b->accel = V(0.0f, 0.0f);
  b->lin_vel = V(0.0f, 0.0f);
  b->ang_vel = 0.0f;
  b->angle = 0.0f;
}

/* Pole.FromSize (Pole.cs:18-34) */
static void make_pole(body* b, int mat, v2 c, float size) {
  float adjustment = 0.1f * size;
  float h = adjustment * 3.5f;
  v2 vs[6] = {
    V(c.x + adjustment, c.y + h), V(c.x, c.y + h), V(c.x - adjustment, c.y + h),
    V(c.x - adjustment, c.y - h), V(c.x, c.y - h), V(c.x + adjustment, c.y - h)};
  body_init(b, mat, vs, 6, 0, 0);
}

/* Skeleton.Move (Skeleton.cs:76-85); the AABB is a pure function of the vertices and
 * is evaluated where it is read (BoundingBox.Update :127-130). */
static void sk_move(body* b, v2 d) {
  for (int i = 0; i < b->nv; i++) b->v[i] = vadd(b->v[i], d);
  b->centroid = vadd(b->centroid, d);
}

/* Skeleton.Rotate (Skeleton.cs:89-97) with XNA CreateRotationZ / Vector2.Transform */
static void sk_rotate(body* b, float angle) {
  float c = (float)cos((double)angle);
  float s = (float)sin((double)angle);
  float m11 = c, m12 = s, m21 = -s, m22 = c;
  for (int i = 0; i < b->nv; i++) {
    v2 p = vsub(b->v[i], b->centroid);
    v2 t = V((p.x * m11) + (p.y * m21) + 0.0f, (p.x * m12) + (p.y * m22) + 0.0f);
    b->v[i] = vadd(t, b->centroid);
  }
}

/* BoundingBox.FindSignificantCorners (Skeleton.cs:144-176) */
static void aabb(const body* b, v2* mn, v2* mx) {
  float maxX = -FLT_MAX, maxY = -FLT_MAX, minX = FLT_MAX, minY = FLT_MAX;
  for (int i = 0; i < b->nv; i++) {
    v2 p = b->v[i];
    if (p.x > maxX) maxX = p.x;
    if (p.y > maxY) maxY = p.y;
    if (p.x < minX) minX = p.x;
    if (p.y < minY) minY = p.y;
  }
  *mn = V(minX - 0.0f, minY - 0.0f);
  *mx = V(maxX + 0.0f, maxY + 0.0f);
}

/* BoundingBox.IsColliding (Skeleton.cs:133-140) */
static int aabb_overlap(const body* a, const body* b) {
  v2 a0, a1, b0, b1;
  aabb(a, &a0, &a1);
  aabb(b, &b0, &b1);
  return a0.x < b1.x && a1.x > b0.x && a0.y < b1.y && a1.y > b0.y;
}

/* ---------------- SAT (SATCollision.cs) ---------------- */
static void project(v2 axis, const v2* vs, int n, float* mn, float* mx) {
  float lo = FLT_MAX, hi = -FLT_MAX;
  for (int i = 0; i < n; i++) {
    float p = vdot(axis, vs[i]);
    if (p < lo) lo = p;
    if (p > hi) hi = p;
  }
  *mn = lo;
  *mx = hi;
}

static int axis_checks(const v2* a, int na, const v2* b, int nb, v2* normal, float* depth) {
  for (int i = 0; i < na; i++) {
    v2 edge = vsub(a[(i + 1) % na], a[i]);
    v2 axis = V(-edge.y, edge.x);
    if (axis.x == 0.0f && axis.y == 0.0f) continue;
    axis = vnormalize(axis);
    float amin, amax, bmin, bmax;
    project(axis, a, na, &amin, &amax);
    project(axis, b, nb, &bmin, &bmax);
    float temp = net_minf(bmax - amin, amax - bmin);
    int overlapping = (amin < bmax) && (bmin < amax);
    if (!overlapping) return 0;
    if (temp >= *depth) continue;
    *depth = temp;
    *normal = axis;
  }
  return 1;
}

static int sat(const v2* a, int na, const v2* b, int nb, v2 ca, v2 cb, v2* normal, float* depth) {
  *normal = V(0.0f, 0.0f);
  *depth = FLT_MAX;
  int result = axis_checks(a, na, b, nb, normal, depth) && axis_checks(b, nb, a, na, normal, depth);
  v2 direction = vsub(cb, ca);
  if (vdot(direction, *normal) > 0.0f) *normal = vmul(*normal, -1.0f);
  return result;
}

/* ---------------- contact points (ContactPoints.cs, dyn4j clipping) ---------------- */
typedef struct { v2 A, B, Max; } face;

static int mod_ref(float a, float b) {
  double r = (double)a - (double)b * floor((double)(a / b));
  return (int)nearbyint(r);
}

static v2 significant_vertex(const v2* vs, int n, v2 normal, int* index) {
  v2 sig = V(0.0f, 0.0f);
  *index = -1;
  float mind = FLT_MAX;
  for (int i = 0; i < n; i++) {
    float p = vdot(vs[i], normal);
    if (!(p < mind)) continue;
    sig = vs[i];
    *index = i;
    mind = p;
  }
  return sig;
}

static face significant_face(const v2* vs, int n, v2 normal) {
  int index;
  v2 sig = significant_vertex(vs, n, normal, &index);
  v2 after = vnormalize(vsub(sig, vs[(index + 1) % n]));
  int bi = mod_ref((float)(index - 1), (float)n);
  v2 before = vnormalize(vsub(sig, vs[bi]));
  face f;
  if (vdot(normal, before) >= vdot(normal, after)) {
    f.A = sig; f.B = vs[bi]; f.Max = sig;
  } else {
    f.A = vs[(index + 1) % n]; f.B = sig; f.Max = sig;
  }
  return f;
}

static int clip(v2 a, v2 b, v2 n, float offset, v2* out) {
  int cnt = 0;
  float da = vdot(a, n) - offset;
  float db = vdot(b, n) - offset;
  if (da >= 0.0f) out[cnt++] = a;
  if (db >= 0.0f) out[cnt++] = b;
  if (da * db < 0.0f) {
    v2 edge = vsub(b, a);
    float location = da / (da - db);
    edge = vmul(edge, location);
    edge = vadd(edge, a);
    out[cnt++] = edge;
  }
  return cnt;
}

/* List<Vector2>.Remove(item): removes the first element equal (==) to item */
static int list_remove(v2* l, int n, v2 item) {
  for (int i = 0; i < n; i++) {
    if (veq(l[i], item)) {
      for (int j = i; j < n - 1; j++) l[j] = l[j + 1];
      return n - 1;
    }
  }
  return n;
}

static int contact_points(const v2* a, int na, const v2* b, int nb, v2 normal, v2* out) {
  face ref = significant_face(a, na, normal);
  v2 rf = vsub(ref.B, ref.A);
  face inc = significant_face(b, nb, vneg(normal));
  v2 iv = vsub(inc.B, inc.A);
  if (fabsf(vdot(rf, normal)) > fabsf(vdot(iv, normal))) {
    face t = ref; ref = inc; inc = t;
    rf = vsub(ref.B, ref.A);
  }
  rf = vnormalize(rf);
  float offset = vdot(rf, ref.A);
  v2 c1[3];
  int n1 = clip(inc.A, inc.B, rf, offset, c1);
  if (n1 < 2) return 0;
  offset = vdot(rf, ref.B);
  v2 c2[3];
  int n2 = clip(c1[0], c1[1], vneg(rf), -offset, c2);
  if (n2 < 2) return 0;
  v2 refn = V(rf.y, -rf.x);
  float maximum = vdot(refn, ref.Max);
  if (vdot(refn, c2[0]) - maximum < 0.0f) n2 = list_remove(c2, n2, c2[0]);
  if (vdot(refn, c2[n2 - 1]) - maximum < 0.0f) n2 = list_remove(c2, n2, c2[n2 - 1]);
  for (int i = 0; i < n2; i++) out[i] = c2[i];
  return n2;
}

/* ---------------- impulses (Impulses.cs) ---------------- */
static void calc_impulse(const body* A, const body* B, v2 contact, float force, v2 normal,
                         v2* rA, v2* rB, float* impulse) {
  *rA = vsub(contact, A->centroid);
  v2 pA = V(-rA->y, rA->x);
  float ctcA = vdot(normal, pA);
  *rB = vsub(contact, B->centroid);
  v2 pB = V(-rB->y, rB->x);
  float ctcB = vdot(normal, pB);
  v2 aVel = vadd(A->lin_vel, vmul(pA, A->ang_vel));
  v2 bVel = vadd(B->lin_vel, vmul(pB, B->ang_vel));
  v2 vel = vsub(bVel, aVel);
  float vdn = vdot(vel, normal);
  float j = -force * vdn;
  float denom = (A->inv_mass + B->inv_mass) + ((ctcA * ctcA) * A->inv_inertia) +
                ((ctcB * ctcB) * B->inv_inertia);
  j /= denom;
  *impulse = j;
}

static void apply_impulses(body* A, body* B, v2 normal, float impulse, v2 rA, v2 rB) {
  v2 J = vmul(normal, impulse);
  v2 va = vsub(A->lin_vel, vmul(J, A->inv_mass));
  v2 vb = vadd(B->lin_vel, vmul(J, B->inv_mass));
  A->lin_vel = va;
  B->lin_vel = vb;
  v2 pA = V(-rA.y, rA.x);
  float wa = A->ang_vel - (vdot(pA, J) * A->inv_inertia);
  v2 pB = V(-rB.y, rB.x);
  float wb = B->ang_vel + (vdot(pB, J) * B->inv_inertia);
  A->ang_vel = wa;
  B->ang_vel = wb;
}

static void resolve_collision(body* A, body* B, const v2* cps, int ncp, v2 normal, float* jout) {
  if (ncp == 0) return;
  float e = net_maxf(A->restitution, B->restitution);
  float mu = net_minf(A->friction, B->friction);
  v2 contact = ncp == 2 ? vdiv(vadd(cps[0], cps[1]), 2.0f) : cps[0];
  v2 rA, rB, rAF, rBF;
  float j, jf;
  calc_impulse(A, B, contact, 1.0f + e, normal, &rA, &rB, &j);
  v2 tangent = V(-normal.y, normal.x);
  calc_impulse(A, B, contact, mu, tangent, &rAF, &rBF, &jf);
  if (jout) { jout[0] = j; jout[1] = jf; }
  apply_impulses(A, B, normal, j, rA, rB);
  apply_impulses(A, B, tangent, jf, rAF, rBF);
}

static float resolve_joint(body* A, body* B, v2 p0, v2 p1, v2 normal) {
  v2 contact = vdiv(vadd(p0, p1), 2.0f);
  v2 rA, rB;
  float j;
  calc_impulse(A, B, contact, 1.0f + 1.0f, normal, &rA, &rB, &j);
  apply_impulses(A, B, normal, j, rA, rB);
  return j;
}

/* ---------------- RigidBody.Step / ResolveCollisions ---------------- */
static const int PAIR_IDX[6][6] = {
  /* LLL */ {-1, 0, -1, -1, -1, 1},
  /* LLU */ {2, -1, -1, -1, -1, 3},
  /* BODY*/ {-1, -1, -1, -1, -1, 4},
  /* RLL */ {-1, -1, -1, -1, 5, 6},
  /* RLU */ {-1, -1, -1, 7, -1, 8},
  /* FLR */ {-1, -1, -1, -1, -1, -1},
};

static void move_objects(body* A, body* B, v2 normal, float depth) {
  if (A->is_static) {
    sk_move(B, vmul(vneg(normal), depth));
  } else if (B->is_static) {
    sk_move(A, vmul(normal, depth));
  } else {
    sk_move(A, vdiv(vmul(normal, depth), 2.0f));
    sk_move(B, vdiv(vmul(vneg(normal), depth), 2.0f));
  }
}

static int is_assoc(const body* b, int other) {
  for (int i = 0; i < b->n_assoc; i++)
    if (b->assoc[i] == other) return 1;
  return 0;
}

static void resolve_collisions(orc_env* e, int self, orc_pair_trace* tr) {
  body* A = &e->bodies[self];
  for (int k = 0; k < e->nbodies; k++) {
    int o = e->order[k];
    if (o == self) continue;
    if (is_assoc(A, o)) continue;
    body* B = &e->bodies[o];
    if (!aabb_overlap(A, B)) continue;
    /* traced pairs: the walker's own 9 candidates (the flat floor's, not a segment's or a prop's) */
    int pi = (self < ORC_FLOOR && o < ORC_FLOOR + (e->rough ? 0 : 1)) ? PAIR_IDX[self][o] : -1;
    if (tr && pi >= 0) tr->aabb_hit[pi] = 1;
    if (B->is_floor) A->collided = 1;
    if (A->is_floor) B->collided = 1;
    v2 normal;
    float depth;
    if (sat(A->v, A->nv, B->v, B->nv, A->centroid, B->centroid, &normal, &depth)) {
      v2 cps[3];
      int ncp = contact_points(A->v, A->nv, B->v, B->nv, normal, cps);
      if (tr && pi >= 0) {
        tr->sat_hit[pi] = 1;
        tr->n_contacts[pi] = (uint8_t)ncp;
        tr->normal[pi][0] = normal.x;
        tr->normal[pi][1] = normal.y;
        tr->depth[pi] = depth;
        for (int q = 0; q < ncp && q < 2; q++) {
          tr->contact[pi][q][0] = cps[q].x;
          tr->contact[pi][q][1] = cps[q].y;
        }
      }
      move_objects(A, B, normal, depth);
      resolve_collision(A, B, cps, ncp, normal, (tr && pi >= 0) ? tr->impulse[pi] : NULL);
    }
  }
}

static float wrap_angle(float angle) {
  const float PI_F = 3.14159265358979323846f, TAU_F = 6.28318530717958647692f;
  if (angle > PI_F) return angle - TAU_F;
  if (angle < -PI_F) return angle + TAU_F;
  return angle;
}

static void body_step(orc_env* e, int self, float dt, orc_pair_trace* tr) {
  body* b = &e->bodies[self];
  /* StepLinearVelocity (RigidBody.cs:116-120) */
  b->lin_vel = vadd(b->lin_vel, vmul(b->accel, dt));
  sk_move(b, vmul(b->lin_vel, dt));
  if (b->is_static) return;
  /* StepAngularVelocity (RigidBody.cs:123-129) */
  b->angle = b->angle + b->ang_vel * dt;
  b->angle = wrap_angle(b->angle);
  sk_rotate(b, b->ang_vel * dt);
  resolve_collisions(e, self, tr);
}

/* Joint.Step (Joint.cs:31-41) */
static void joint_step(orc_env* e, joint* jn, float* jd, float* jj) {
  body* A = &e->bodies[jn->a];
  body* B = &e->bodies[jn->b];
  v2 ab = vsub(B->v[jn->ib], A->v[jn->ia]);
  float depth = vlen(ab);
  if (depth < 0.1f) return;
  ab = vnormalize(ab);
  sk_move(A, vdiv(vmul(ab, depth), 2.0f));
  sk_move(B, vdiv(vmul(vneg(ab), depth), 2.0f));
  float j = resolve_joint(B, A, A->v[jn->ia], B->v[jn->ib], ab);
  if (jd) *jd = depth;
  if (jj) *jj = j;
}

void orc_env_joint_step(orc_env* e, int j) { joint_step(e, &e->joints[j], NULL, NULL); }

void orc_env_step_objects(orc_env* e, float deltaTime, orc_pair_trace* trace) {
  deltaTime = deltaTime / (float)e->h.Iterations;
  for (int i = 0; i < e->h.Iterations; i++) {
    orc_pair_trace* tr = trace ? &trace[i] : NULL;
    if (tr) memset(tr, 0, sizeof(*tr));
    for (int j = 0; j < 4; j++)
      joint_step(e, &e->joints[j], tr ? &tr->joint_depth[j] : NULL, tr ? &tr->joint_impulse[j] : NULL);
    for (int k = 0; k < e->nbodies; k++) body_step(e, e->order[k], deltaTime, tr);
  }
}

/* ---------------- Walker ---------------- */
static void create_creature(orc_env* e) {
  v2 pos = e->position;
  int mat = e->material;
  v2 bv[5] = {V(pos.x + 20, pos.y + 20), V(pos.x, pos.y + 20), V(pos.x - 20, pos.y + 20),
              V(pos.x - 20, pos.y - 20), V(pos.x + 20, pos.y - 20)};
  body_init(&e->bodies[ORC_BODY], mat, bv, 5, 0, 0);
  e->bodies[ORC_BODY].inv_inertia = 0.0003f;
  make_pole(&e->bodies[ORC_LLU], mat, vadd(pos, V(0, 30)), 75);
  make_pole(&e->bodies[ORC_LLL], mat, vadd(pos, V(0, 60.0f)), 75);
  make_pole(&e->bodies[ORC_RLU], mat, vadd(pos, V(0, 30)), 75);
  make_pole(&e->bodies[ORC_RLL], mat, vadd(pos, V(0, 60.0f)), 75);
  /* CreateJoints (Walker.cs:180-188) */
  joint js[4] = {{ORC_BODY, ORC_LLU, 1, 4, 0.0f}, {ORC_BODY, ORC_RLU, 1, 4, 0.0f},
                 {ORC_LLU, ORC_LLL, 2, 3, 0.0f}, {ORC_RLU, ORC_RLL, 2, 3, 0.0f}};
  memcpy(e->joints, js, sizeof(js));
  /* AddAssociatedBodies (Walker.cs:202-209) */
  int al[3] = {ORC_RLU, ORC_RLL, ORC_BODY}, ar[3] = {ORC_LLU, ORC_LLL, ORC_BODY};
  int ab[4] = {ORC_LLU, ORC_RLU, ORC_LLL, ORC_RLL};
  memcpy(e->bodies[ORC_LLU].assoc, al, sizeof(al)); e->bodies[ORC_LLU].n_assoc = 3;
  memcpy(e->bodies[ORC_LLL].assoc, al, sizeof(al)); e->bodies[ORC_LLL].n_assoc = 3;
  memcpy(e->bodies[ORC_RLU].assoc, ar, sizeof(ar)); e->bodies[ORC_RLU].n_assoc = 3;
  memcpy(e->bodies[ORC_RLL].assoc, ar, sizeof(ar)); e->bodies[ORC_RLL].n_assoc = 3;
  memcpy(e->bodies[ORC_BODY].assoc, ab, sizeof(ab)); e->bodies[ORC_BODY].n_assoc = 4;
  /* AddAcceleration((0, 980)) (Walker.cs:45,191-198) */
  for (int b = 0; b < 5; b++) e->bodies[b].accel = vadd(e->bodies[b].accel, V(0, 980));
}

/* Walker.Update (Walker.cs:49-54) */
static void walker_update(orc_env* e) {
  e->prev_position = e->position;
  e->position = e->bodies[ORC_BODY].centroid;
  if (e->bodies[ORC_BODY].collided || e->bodies[ORC_LLU].collided || e->bodies[ORC_RLU].collided)
    e->terminal = 1;
}

/* Walker.GetState (Walker.cs:132-152) */
void orc_env_get_obs(const orc_env* e, float s[12]) {
  const body* bd = &e->bodies[ORC_BODY];
  v2 j0 = bd->v[1], j2 = e->bodies[ORC_LLU].v[2], j3 = e->bodies[ORC_RLU].v[2];
  s[0] = j0.x / 900.0f;
  s[1] = j0.y / 500.0f;
  s[2] = j2.x / 900.0f;
  s[3] = j2.y / 500.0f;
  s[4] = j3.x / 900.0f;
  s[5] = j3.y / 500.0f;
  s[6] = bd->lin_vel.x / 60.0f;
  s[7] = bd->lin_vel.y / 60.0f;
  s[8] = e->bodies[ORC_LLL].angle;
  s[9] = e->bodies[ORC_LLU].angle;
  s[10] = e->bodies[ORC_RLL].angle;
  s[11] = e->bodies[ORC_RLU].angle;
}

static void initial_state(orc_env* e) { walker_update(e); }

/* List<RigidBody> order.  Episode 0: the walker (CreateCreature), then the floor body /
 * segments (CreateFloor), then the scene props in the order they were added.  After a
 * reset the walker's five bodies are removed and re-appended (Walker.Reset / RemoveRigidObjects,
 * Walker.cs:212-234): the floor bodies and props keep their relative order in front. */
static void build_order(orc_env* e) {
  const int nf = e->nbodies - 5;
  const int w0 = e->post_reset ? nf : 0, f0 = e->post_reset ? 0 : 5;
  e->order[w0 + 0] = ORC_LLL; e->order[w0 + 1] = ORC_LLU; e->order[w0 + 2] = ORC_BODY;
  e->order[w0 + 3] = ORC_RLL; e->order[w0 + 4] = ORC_RLU;
  for (int k = 0; k < nf; k++) e->order[f0 + k] = ORC_FLOOR + k;
}

void orc_env_reset(orc_env* e) {
  /* Environment.Reset (:167-173) -> Walker.Reset (Walker.cs:212-223): the walker's
   * bodies are removed and re-appended AFTER the floor. */
  e->steps = 0;
  e->terminal = 0;
  e->position = V(125.0f + e->dx, 800.0f);
  e->prev_position = e->position;
  create_creature(e);
  e->post_reset = 1;
  build_order(e);
  initial_state(e);
}

void orc_hyper_defaults(orc_hyper* h) {
  h->Iterations = 50;
  h->MaxTimesteps = 1000;
  h->Epochs = 5;
  h->BatchSize = 64;
  h->UseGAE = 0;
  h->NormalizeAdvantages = 0;
  h->Gamma = 0.9f;
  h->Lambda = 0.95f;
  h->Epsilon = 0.3f;
  h->LogStandardDeviation = -1.0f;
  h->Alpha = 0.001f;
  h->Beta1 = 0.9f;
  h->Beta2 = 0.999f;
  h->AdamEpsilon = 1e-8f;
  h->DeltaTime = (float)(166667.0 / 10000000.0);
}

/* CreateRoughFloor (Environment.cs:230-261), segments = 10, roughness = 100: draws[0] is
 * the first previousVector's Random.Next(0, 100), draws[1..10] the segments' */
static void create_rough_floor(orc_env* e, const int* draws) {
  const int initialY = 800, initialX = -50, movement = 1200 / ORC_ROUGH_SEGMENTS;
  v2 prev = V((float)initialX, (float)(initialY + draws[0]));
  for (int i = 0; i < ORC_ROUGH_SEGMENTS; i++) {
    int x = initialX + i * movement;
    int y = 800 + draws[i + 1];
    v2 pos[4] = {V((float)x, 1050.0f), prev, V((float)x, (float)y), V((float)(x + movement), 1050.0f)};
    body_init(&e->bodies[ORC_FLOOR + i], ORC_MAT_METAL, pos, 4, 1, 1);
    prev = V((float)x, (float)y);
  }
}

orc_env* orc_env_create_floor(const orc_hyper* h, float dx, int material, const int* rough_draws) {
  orc_env* e = (orc_env*)calloc(1, sizeof(orc_env));
  e->h = *h;
  e->dx = dx;
  e->material = material;
  e->rough = rough_draws != NULL;
  e->nbodies = e->rough ? 5 + ORC_ROUGH_SEGMENTS : 6;
  /* Environment ctor (Environment.cs:39-51): walker first, then the floor (CreateFloor :211-226) */
  e->position = V(125.0f + dx, 800.0f);
  e->prev_position = e->position;
  create_creature(e);
  if (e->rough) {
    create_rough_floor(e, rough_draws);
  } else {
    v2 fl[4] = {V(-50, 1050), V(-50, 900), V(1050, 900), V(1050, 1050)};
    body_init(&e->bodies[ORC_FLOOR], ORC_MAT_METAL, fl, 4, 1, 1);
  }
  e->post_reset = 0;
  build_order(e);
  initial_state(e);
  return e;
}

/* ---------------- scene props (Objects/RigidBodies/{Square,Triangle,Hexagon}.cs) ----------------
 * FromSize(material, centroid, size, isStatic): adjustment = (float)0.5 * size, vertices in
 * the listed order; RigidBody ctor (RigidBody.cs:36-50); then, as a caller would,
 * SmoothCorners(count) (Skeleton.cs:33-53: the vertex list is replaced, the centroid is NOT
 * recomputed), SetLinearVelocity / SetAngularVelocity / AddAcceleration (:143-183). */
int orc_prop_vertices(const orc_prop* p, float* xy) {
  const v2 c = V(p->cx, p->cy);
  const float adj = (float)0.5 * p->size;
  v2 vs[ORC_PROP_MAXV];
  int n;
  if (p->shape == ORC_SHAPE_SQUARE) {        /* Square.cs:18-31 */
    vs[0] = V(c.x + adj, c.y + adj); vs[1] = V(c.x - adj, c.y + adj);
    vs[2] = V(c.x - adj, c.y - adj); vs[3] = V(c.x + adj, c.y - adj);
    n = 4;
  } else if (p->shape == ORC_SHAPE_TRIANGLE) {  /* Triangle.cs:18-30 */
    vs[0] = V(c.x, c.y + adj); vs[1] = V(c.x - adj, c.y - adj); vs[2] = V(c.x + adj, c.y - adj);
    n = 3;
  } else if (p->shape == ORC_SHAPE_HEXAGON) {   /* Hexagon.cs:18-33 */
    vs[0] = V(c.x + (adj * 0.5f), c.y + adj); vs[1] = V(c.x - (adj * 0.5f), c.y + adj);
    vs[2] = V(c.x - adj, c.y);                 vs[3] = V(c.x - (adj * 0.5f), c.y - adj);
    vs[4] = V(c.x + (adj * 0.5f), c.y - adj); vs[5] = V(c.x + adj, c.y);
    n = 6;
  } else {
    return -1;
  }
  if (p->smooth < 0) return -1;
  for (int it = 0; it < p->smooth; it++) {   /* SmoothCorners(count) */
    if (2 * n > ORC_PROP_MAXV) return -1;
    v2 nv[ORC_PROP_MAXV];
    for (int j = 0; j < n; j++) {
      v2 faceAB = vsub(vs[(j + 1) % n], vs[j]);
      faceAB = vmul(faceAB, 0.2f);
      v2 faceAC = vsub(vs[mod_ref((float)(j - 1), (float)n)], vs[j]);
      faceAC = vmul(faceAC, 0.2f);
      nv[2 * j] = vadd(vs[j], faceAC);
      nv[2 * j + 1] = vadd(vs[j], faceAB);
    }
    n *= 2;
    memcpy(vs, nv, sizeof(v2) * (size_t)n);
  }
  if (xy)
    for (int i = 0; i < n; i++) { xy[2 * i] = vs[i].x; xy[2 * i + 1] = vs[i].y; }
  return n;
}

int orc_env_add_prop(orc_env* e, const orc_prop* p) {
  if (e->nprops >= ORC_MAX_PROPS || p->material < 0 || p->material >= ORC_NMAT) return -1;
  float xy[2 * ORC_PROP_MAXV];
  const int n = orc_prop_vertices(p, xy);
  if (n < 3) return -1;
  /* the centroid of FromSize's vertices (AddVectors), before SmoothCorners */
  orc_prop base = *p;
  base.smooth = 0;
  float bxy[2 * ORC_PROP_MAXV];
  const int nb = orc_prop_vertices(&base, bxy);
  v2 bv[ORC_PROP_MAXV];
  for (int i = 0; i < nb; i++) bv[i] = V(bxy[2 * i], bxy[2 * i + 1]);
  body* b = &e->bodies[e->nbodies];
  body_init(b, p->material, bv, nb, p->is_static != 0, 0);
  b->nv = n;
  for (int i = 0; i < n; i++) b->v[i] = V(xy[2 * i], xy[2 * i + 1]);
  b->lin_vel = V(p->vx, p->vy);
  b->ang_vel = p->w;
  b->accel = vadd(b->accel, V(p->ax, p->ay));
  e->nbodies++;
  e->nprops++;
  build_order(e);
  return e->nprops - 1;
}

/* prop k: vertices (x0, y0, ...) and {cx, cy, vx, vy, w, angle}; returns the vertex count */
int orc_env_prop(const orc_env* e, int k, float* xy, float st[6]) {
  if (k < 0 || k >= e->nprops) return 0;
  const body* b = &e->bodies[e->nbodies - e->nprops + k];
  if (xy)
    for (int i = 0; i < b->nv; i++) { xy[2 * i] = b->v[i].x; xy[2 * i + 1] = b->v[i].y; }
  if (st) {
    st[0] = b->centroid.x; st[1] = b->centroid.y; st[2] = b->lin_vel.x; st[3] = b->lin_vel.y;
    st[4] = b->ang_vel; st[5] = b->angle;
  }
  return b->nv;
}

orc_env* orc_env_create(const orc_hyper* h, float dx, int material) {
  return orc_env_create_floor(h, dx, material, NULL);
}

/* floor body k's vertices (x0, y0, x1, y1, ...); returns the vertex count */
int orc_env_floor_body(const orc_env* e, int k, float* xy) {
  if (k < 0 || k >= e->nbodies - 5 - e->nprops) return 0;
  const body* b = &e->bodies[ORC_FLOOR + k];
  for (int i = 0; i < b->nv; i++) { xy[2 * i] = b->v[i].x; xy[2 * i + 1] = b->v[i].y; }
  return b->nv;
}

void orc_env_destroy(orc_env* e) { free(e); }

/* Joint.SetTorque (Joint.cs:56-61) via Walker.TakeActions (Walker.cs:66-75) */
void orc_env_set_torques(orc_env* e, const float a[4]) {
  for (int i = 0; i < 4; i++) {
    joint* j = &e->joints[i];
    float change = a[i] - j->torque;
    j->torque = a[i];
    e->bodies[j->b].ang_vel = e->bodies[j->b].ang_vel + change * 5.0f;
  }
}

/* Matrix.Clip(m, 1, -1) (Matrix.cs:377-405) */
static float clip1(float x) {
  if (x >= 1.0f) return 1.0f;
  if (x <= -1.0f) return -1.0f;
  return x;
}

/* Environment.Update (:64-92) minus the policy (the caller supplies the action) */
void orc_env_step(orc_env* e, const float action[4], float obs[12], float* reward_out,
                  int* done_out, orc_pair_trace* trace) {
  e->steps++;
  float ac[4];
  for (int i = 0; i < 4; i++) ac[i] = clip1(action[i]);
  orc_env_set_torques(e, ac);
  /* Environment.Step (:96-122) */
  int terminal = 0;
  orc_env_step_objects(e, e->h.DeltaTime, trace);
  walker_update(e);
  /* CalculateReward (:148-154) */
  float reward = 0.0f;
  float dX = e->position.x - e->prev_position.x;
  float yb = e->bodies[ORC_BODY].v[1].y;
  reward = reward + ((dX > 0.0f && ((yb / 500.0f) < 1.6f)) ? dX : 0.0f);
  reward = reward - (((yb / 500.0f) > 1.65f) ? -0.1f : 0.0f);
  if (e->terminal || e->steps > e->h.MaxTimesteps) {
    if (e->terminal) reward -= 40.0f;
    terminal = 1;
  }
  if (e->position.x > 900.0f) {
    reward += 80.0f;
    terminal = 1;
  }
  orc_env_get_obs(e, obs);
  e->step_position = e->position;  /* _bestDistance reads it here (Environment.cs:119) */
  if (terminal) {
    e->episodes++;
    orc_env_reset(e);
    orc_env_get_obs(e, obs);
  }
  *reward_out = reward;
  *done_out = terminal;
}

void orc_env_step_position(const orc_env* e, float out[2]) {
  out[0] = e->step_position.x;
  out[1] = e->step_position.y;
}

void orc_env_dump(const orc_env* e, float out[ORC_STATE_FLOATS]) {
  memset(out, 0, sizeof(float) * ORC_STATE_FLOATS);
  for (int b = 0; b < ORC_NB; b++) {
    const body* bd = &e->bodies[b];
    float* o = out + b * ORC_BODY_STRIDE;
    for (int i = 0; i < bd->nv; i++) {
      o[2 * i] = bd->v[i].x;
      o[2 * i + 1] = bd->v[i].y;
    }
    o[12] = bd->centroid.x;
    o[13] = bd->centroid.y;
    o[14] = bd->lin_vel.x;
    o[15] = bd->lin_vel.y;
    o[16] = bd->ang_vel;
    o[17] = bd->angle;
    o[18] = (float)bd->collided;
  }
  for (int j = 0; j < 4; j++) out[ORC_ST_TORQUE + j] = e->joints[j].torque;
  out[ORC_ST_POS] = e->position.x;
  out[ORC_ST_POS + 1] = e->position.y;
  out[ORC_ST_PREV] = e->prev_position.x;
  out[ORC_ST_PREV + 1] = e->prev_position.y;
  out[ORC_ST_STEPS] = (float)e->steps;
  out[ORC_ST_POSTRESET] = (float)e->post_reset;
  out[ORC_ST_TERMINAL] = (float)e->terminal;
  out[ORC_ST_EPISODES] = (float)e->episodes;
}

/* the inverse of orc_env_dump for the walker (flat-floor or rough env): vertices,
 * centroids, velocities, angles, Collided, torques, positions, counters and the body order
 * (materials / inertia stay the env's).  Test infrastructure: lets a test start the oracle
 * from a state the GPU context was given (wk_set_state). */
void orc_env_load(orc_env* e, const float in[ORC_STATE_FLOATS]) {
  for (int b = 0; b < ORC_NB; b++) {
    body* bd = &e->bodies[b];
    const float* o = in + b * ORC_BODY_STRIDE;
    for (int i = 0; i < bd->nv; i++) bd->v[i] = V(o[2 * i], o[2 * i + 1]);
    bd->centroid = V(o[12], o[13]);
    bd->lin_vel = V(o[14], o[15]);
    bd->ang_vel = o[16];
    bd->angle = o[17];
    bd->collided = o[18] != 0.0f;
  }
  for (int j = 0; j < 4; j++) e->joints[j].torque = in[ORC_ST_TORQUE + j];
  e->position = V(in[ORC_ST_POS], in[ORC_ST_POS + 1]);
  e->prev_position = V(in[ORC_ST_PREV], in[ORC_ST_PREV + 1]);
  e->steps = (int)in[ORC_ST_STEPS];
  e->post_reset = in[ORC_ST_POSTRESET] != 0.0f;
  e->terminal = in[ORC_ST_TERMINAL] != 0.0f;
  e->episodes = (int)in[ORC_ST_EPISODES];
  build_order(e);
}

/* K3: an axis-aligned Carpet pole centred at (125, 874.75) -- bottom edge
 * 1 px into the flat Metal floor -- moving with velocity (0, vy), resolved against the
 * floor exactly as RigidBody.ResolveCollisions does.  out: v.x, v.y, w, c.x, c.y,
 * n_contacts, normal.x, normal.y, depth */
void orc_kat_pole_floor(float vy, float out[9]) {
  body p, f;
  make_pole(&p, ORC_MAT_CARPET, V(125.0f, 874.75f), 75.0f);
  p.lin_vel = V(0.0f, vy);
  v2 fl[4] = {V(-50, 1050), V(-50, 900), V(1050, 900), V(1050, 1050)};
  body_init(&f, ORC_MAT_METAL, fl, 4, 1, 1);
  v2 normal;
  float depth;
  int hit = sat(p.v, 6, f.v, 4, p.centroid, f.centroid, &normal, &depth);
  int ncp = 0;
  if (hit) {
    v2 cps[3];
    ncp = contact_points(p.v, 6, f.v, 4, normal, cps);
    move_objects(&p, &f, normal, depth);
    resolve_collision(&p, &f, cps, ncp, normal, NULL);
  }
  out[0] = p.lin_vel.x; out[1] = p.lin_vel.y; out[2] = p.ang_vel;
  out[3] = p.centroid.x; out[4] = p.centroid.y; out[5] = (float)ncp;
  out[6] = normal.x; out[7] = normal.y; out[8] = depth;
}

/* exported geometry primitives for KATs */
int orc_sat(const float* va, int na, const float* vb, int nb, const float ca[2], const float cb[2],
            float normal[2], float* depth) {
  v2 a[16], b[16];
  for (int i = 0; i < na; i++) a[i] = V(va[2 * i], va[2 * i + 1]);
  for (int i = 0; i < nb; i++) b[i] = V(vb[2 * i], vb[2 * i + 1]);
  v2 n;
  int r = sat(a, na, b, nb, V(ca[0], ca[1]), V(cb[0], cb[1]), &n, depth);
  normal[0] = n.x;
  normal[1] = n.y;
  return r;
}

int orc_contacts(const float* va, int na, const float* vb, int nb, const float normal[2],
                 float out[4]) {
  v2 a[16], b[16], c[3];
  for (int i = 0; i < na; i++) a[i] = V(va[2 * i], va[2 * i + 1]);
  for (int i = 0; i < nb; i++) b[i] = V(vb[2 * i], vb[2 * i + 1]);
  int n = contact_points(a, na, b, nb, V(normal[0], normal[1]), c);
  for (int i = 0; i < n; i++) {
    out[2 * i] = c[i].x;
    out[2 * i + 1] = c[i].y;
  }
  return n;
}
