/*
 * wk_oracle.h -- CPU restatement ("oracle") of the De-Rosa/PPO-BipedalWalker hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline -- never as the product path.  The product (libwk.so) never links it.
 *
 * PARITY UNPINNED: the reference is C# (.NET >= 6 + MonoGame, no project file); no
 * C# toolchain exists in this container or on the GPU box, and the reference ships no
 * tests, fixtures or golden vectors.  This restatement is therefore pinned only by the
 * hand-derived known-answer tests in tests/test_oracle_kat.py (constants read straight
 * from the reference source), not by outputs of the
 * reference itself.
 *
 * Numeric contract restated: fp32 IEEE, no FMA contraction
 * (-ffp-contract=off), no fast-math; MonoGame Vector2 semantics (v / f == v * (1/f),
 * Normalize == v * (1/sqrt(x*x+y*y))); XNA CreateRotationZ uses (float)Math.Cos/Sin
 * on the double-promoted angle; System.Random replaced by seeded Philox4x32-10.
 */
#ifndef WK_ORACLE_H
#define WK_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- canonical per-env state dump (shared layout with include/wk_api.h) ---- */
enum {
  ORC_NB = 5,          /* walker bodies, canonical order below */
  ORC_LLL = 0, ORC_LLU = 1, ORC_BODY = 2, ORC_RLL = 3, ORC_RLU = 4, ORC_FLOOR = 5,
  ORC_BODY_STRIDE = 20, /* verts[12], cx, cy, vx, vy, w, angle, collided, pad */
  ORC_ST_TORQUE = 100,  /* 4 previous joint torques */
  ORC_ST_POS = 104,     /* walker position (x,y) */
  ORC_ST_PREV = 106,    /* walker previous position (x,y) */
  ORC_ST_STEPS = 108,   /* Environment._steps */
  ORC_ST_POSTRESET = 109, /* 1 once the env has been reset (floor first in body list) */
  ORC_ST_TERMINAL = 110,  /* Walker.Terminal */
  ORC_ST_EPISODES = 111,  /* completed episodes */
  ORC_STATE_FLOATS = 112,
  ORC_ROUGH_SEGMENTS = 10, /* CreateRoughFloor(segments = 10) */
  ORC_MAX_PROPS = 4,       /* scene props (extension: Square / Triangle / Hexagon bodies) */
  ORC_PROP_MAXV = 24       /* vertices of one prop after SmoothCorners */
};

/* candidate pair checks per substep, canonical index (this, other):
 * 0 (LLL,LLU) 1 (LLL,FLOOR) 2 (LLU,LLL) 3 (LLU,FLOOR) 4 (BODY,FLOOR)
 * 5 (RLL,RLU) 6 (RLL,FLOOR) 7 (RLU,RLL) 8 (RLU,FLOOR)                       */
enum { ORC_NPAIRS = 9 };
typedef struct {
  uint8_t aabb_hit[ORC_NPAIRS];
  uint8_t sat_hit[ORC_NPAIRS];
  uint8_t n_contacts[ORC_NPAIRS];
  uint8_t pad[5];
  float normal[ORC_NPAIRS][2];
  float depth[ORC_NPAIRS];
  float contact[ORC_NPAIRS][2][2];
  float impulse[ORC_NPAIRS][2];
  float joint_depth[4];
  float joint_impulse[4];
} orc_pair_trace;

/* materials (Materials/<Name>.cs) */
enum { ORC_MAT_CARPET = 0, ORC_MAT_ICE = 1, ORC_MAT_RUBBER = 2, ORC_MAT_METAL = 3,
       ORC_MAT_WOOD = 4, ORC_MAT_PAPER = 5, ORC_MAT_TITANIUM = 6, ORC_MAT_SUPERRUBBER = 7,
       ORC_NMAT = 8 };

/* Hyperparameters (Walker/PPO/Hyperparameters.cs:80-121), same names and defaults */
typedef struct {
  int Iterations;          /* 50 */
  int MaxTimesteps;        /* 1000 */
  int Epochs;              /* 5 */
  int BatchSize;           /* 64 */
  int UseGAE;              /* 0 */
  int NormalizeAdvantages; /* 0 */
  float Gamma;             /* 0.9 */
  float Lambda;            /* 0.95 */
  float Epsilon;           /* 0.3 */
  float LogStandardDeviation; /* -1 */
  float Alpha, Beta1, Beta2, AdamEpsilon; /* 1e-3 0.9 0.999 1e-8 */
  float DeltaTime;         /* MonoGame fixed step: (float)(166667 ticks / 1e7) */
} orc_hyper;

void orc_hyper_defaults(orc_hyper* h);

/* ---------------- physics / environment ---------------- */
typedef struct orc_env orc_env;
orc_env* orc_env_create(const orc_hyper* h, float dx, int material);
/* rough_draws: NULL = the flat floor; else the 11 Random.Next(0, 100) draws of
 * CreateRoughFloor (Environment.cs:230-261), e.g. orc_terrain_draw(seed, env, 0..10) */
orc_env* orc_env_create_floor(const orc_hyper* h, float dx, int material, const int* rough_draws);
int orc_env_floor_body(const orc_env* e, int k, float* xy);
int orc_terrain_draw(uint64_t seed, int env, int i);
void orc_env_destroy(orc_env* e);
/* scene props: Square / Triangle / Hexagon.FromSize (+ SmoothCorners, velocities,
 * acceleration) appended to the body list after the floor; same layout as wk_prop */
enum { ORC_SHAPE_SQUARE = 0, ORC_SHAPE_TRIANGLE = 1, ORC_SHAPE_HEXAGON = 2 };
typedef struct {
  int32_t shape, smooth, material, is_static;
  float cx, cy, size, vx, vy, w, ax, ay;
} orc_prop;
int orc_prop_vertices(const orc_prop* p, float* xy);
int orc_env_add_prop(orc_env* e, const orc_prop* p);
int orc_env_prop(const orc_env* e, int k, float* xy, float st[6]);
/* one Environment.Update with a given (unclipped) action; clip as Environment.cs:78.
 * obs: 12 floats after the step (after auto-reset if done). trace: per-substep pair
 * trace array of h->Iterations entries (may be NULL). */
void orc_env_step(orc_env* e, const float action[4], float obs[12], float* reward,
                  int* done, orc_pair_trace* trace);
void orc_env_get_obs(const orc_env* e, float obs[12]);
/* torso position after the last orc_env_step, before its auto-reset (Environment.cs:119) */
void orc_env_step_position(const orc_env* e, float out[2]);
/* inverse of orc_env_dump (walker bodies, counters, body order) */
void orc_env_load(orc_env* e, const float in[ORC_STATE_FLOATS]);
void orc_env_dump(const orc_env* e, float out[ORC_STATE_FLOATS]);
void orc_env_reset(orc_env* e);
/* substep-level hooks for unit tests */
void orc_env_set_torques(orc_env* e, const float clipped[4]);
void orc_env_step_objects(orc_env* e, float deltaTime, orc_pair_trace* trace);
void orc_env_joint_step(orc_env* e, int j);

/* geometry primitives exposed for KATs */
int orc_sat(const float* va, int na, const float* vb, int nb, const float ca[2],
            const float cb[2], float normal[2], float* depth);
int orc_contacts(const float* va, int na, const float* vb, int nb, const float normal[2],
                 float out[4]);

void orc_kat_pole_floor(float vy, float out[9]);

/* ---------------- RNG (Philox4x32-10) ---------------- */
void orc_philox(uint64_t key, const uint32_t ctr[4], uint32_t out[4]);
float orc_uniform_f(uint64_t key, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, int which);
float orc_env_offset(uint64_t seed, int env);     /* 200 * u */
int orc_env_material(uint64_t seed, int env);     /* Ice/Rubber/Carpet */
void orc_synth_action(uint64_t seed, int env, uint32_t t, float a[4]);
void orc_noise_uniforms(uint64_t seed, int env, uint32_t t, int d, float* u1, float* u2);
void orc_xavier_uniforms(uint64_t seed, int layer, int k, float* u1, float* u2);
uint32_t orc_perm(uint32_t i, uint32_t n, const uint32_t key[4]);
void orc_perm_key(uint64_t seed, uint32_t update, uint32_t epoch, uint32_t key[4]);

/* ---------------- PPO ---------------- */
enum { ORC_NPARAM_CRITIC = 897, ORC_NPARAM_ACTOR = 5252, ORC_NPARAM = 6149 };
typedef struct orc_agent orc_agent;
orc_agent* orc_agent_create(const orc_hyper* h, uint64_t seed);
void orc_agent_destroy(orc_agent* a);
void orc_agent_get_params(const orc_agent* a, float* p);   /* ORC_NPARAM floats */
void orc_agent_set_params(orc_agent* a, const float* p);
void orc_agent_get_adam(const orc_agent* a, float* m, float* v, int* t);
void orc_agent_set_adam(orc_agent* a, const float* m, const float* v, int t);
void orc_actor_mean(orc_agent* a, const float s[12], float mean[4]);
float orc_critic_value(orc_agent* a, const float s[12]);
/* SampleActions with Philox noise (env e, global step t) */
void orc_sample_actions(orc_agent* a, const float s[12], uint64_t seed, int env, uint32_t t,
                        float act[4], float logp[4]);
float orc_log_density(float mean, float std, float action);
/* Train(Batch) (PPOAgent.cs:218-346) on B samples, then Adam.  grads_out (optional):
 * the accumulated gradient (ORC_NPARAM, critic then actor) before Adam.
 * Returns number of skipped samples. B_div is the divisor used for dV/dmu (the
 * reference uses BatchSize). */
int orc_train_batch(orc_agent* a, int B, float B_div, const float* states, const float* actions,
                    const float* logp_old, const float* returns, const float* adv,
                    float* critic_diag, float* actor_diag, float* grads_out, int apply_adam);
void orc_returns_mc(int T, const float* r, const float* v, const uint8_t* done, float gamma,
                    float* ret, float* adv);
void orc_returns_gae(int T, const float* r, const float* v, const uint8_t* done, float gamma,
                     float lambda, float* ret, float* adv);
void orc_normalize(int n, float* x, float eps_clip);

/* single-walker reference loop (Game1.Update x n_steps, Train at each terminal):
 * the CPU baseline workload.  Returns episodes completed. */
int orc_reference_loop(const orc_hyper* h, uint64_t seed, int n_steps, double* train_seconds);
int orc_reference_loop_env(const orc_hyper* h, uint64_t seed, int env_id, int n_steps,
                           double* train_seconds);
void orc_train_trajectory(orc_agent* ag, const orc_hyper* h, uint64_t seed, uint32_t update, int T,
                          const float* S, const float* Ac, const float* Lp, const float* R);
int orc_physics_loop(const orc_hyper* h, uint64_t seed, int env_id, int n_steps);
double orc_train_episode_seconds(const orc_hyper* h, uint64_t seed, int T);

/* batched drivers (orc_batch.c, OpenMP over independent walkers) */
int orc_replay_batch(const orc_hyper* h, int n, int T, const float* dx, const int* mat,
                     const float* actions, float* obs_before, float* reward, uint8_t* done,
                     float* dump);
void orc_perm_batch(uint32_t count, uint32_t n, const uint32_t key[4], uint32_t* out);
void orc_env_setup_batch(uint64_t seed, int first, int n, float* dx, int* mat);

#ifdef __cplusplus
}
#endif
#endif
