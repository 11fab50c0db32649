/*
 * wk_api.h -- C ABI of the MI355X-native batched bipedal-walker physics + PPO engine.
 *
 * Drop-in boundary for the reference's hot path (De-Rosa/PPO-BipedalWalker, C#).  The
 * reference has no FFI of its own; these entry points replace the managed calls that
 * sit on the path (citations are /root/reference file:line):
 *
 *   wk_create / wk_destroy     Environment ctor (Environment.cs:39-51), Walker ctor
 *                              (Walker/Walker.cs:25-46), PPOAgent ctor (PPOAgent.cs:23-37),
 *                              CreateFloor (Environment.cs:211-226)
 *   wk_step, wk_step_sampled   Environment.Update (Environment.cs:64-92): SampleActions
 *                              (PPOAgent.cs:381-398) or caller actions, Clip (:78),
 *                              Walker.TakeActions/Joint.SetTorque (Walker.cs:66-75,
 *                              Joint.cs:56-61), StepObjects (Environment.cs:126-143:
 *                              Joint.Step Joint.cs:31-41 + IObject.Update Objects/IObject.cs:9
 *                              -> RigidBody.Step Bodies/RigidBody.cs:54-61), Walker.Update
 *                              (Walker.cs:49-54), CalculateReward (Environment.cs:148-154),
 *                              terminal (:106-117), GetState (Walker.cs:132-152),
 *                              auto Reset (Environment.cs:167-180)
 *   wk_reset                   Environment.Reset / Walker.Reset (Environment.cs:167-173,
 *                              Walker.cs:212-223)
 *   wk_set_materials           Walker._material : IMaterial (Walker.cs:17,30; Materials/<Name>.cs)
 *   wk_get_body_view           RigidBody.GetVectors/GetCentroid/... for Renderer and
 *                              ConsoleRenderer (Bodies/RigidBody.cs:191-261)
 *   wk_policy_sample           PPOAgent.SampleActions (PPOAgent.cs:381-398)
 *   wk_value                   PPOAgent.GetValueEstimate (PPOAgent.cs:350-364)
 *   wk_rollout                 Environment.Update x horizon with Trajectory recording
 *                              (Environment.cs:71-89, Trajectory.cs:7-50) + CalculateValues
 *                              (PPOAgent.cs:175-189)
 *   wk_ppo_update              PPOAgent.Train(Trajectory) (PPOAgent.cs:147-172): CreateBatches
 *                              (:501-540), Train(Batch) (:218-346), NeuralNetwork.Optimise /
 *                              DenseLayer.Adam (NeuralNetwork.cs:85-91, DenseLayer.cs:125-159)
 *   wk_train_batch             PPOAgent.Train(Batch) on caller data (parity entry)
 *   wk_get/set_weights         NeuralNetwork.Save/Load (NeuralNetwork.cs:94-115,159-176),
 *                              flat fp32, critic layers then actor layers, each W (out x in,
 *                              row-major) then B -- the .weights order (DenseLayer.cs:73-79)
 *   wk_comm_*                  (new) RCCL all-reduce of policy gradients across GPUs
 *
 * Conventions: every call returns 0 on success or a negative wk_status; the text is
 * in wk_last_error(ctx).  The C# side forwards it to ErrorLogger.LogError and
 * continues (the reference's log-and-continue convention, Rendering/ErrorLogger.cs:42-78).
 * Per-env soft faults (non-finite state, skipped PPO samples) are reported as bitmasks,
 * never as errors.  Host arrays are caller-owned, borrowed for the call and copied;
 * *_device variants take device pointers on the context's stream.  A context is not
 * thread-safe: one host thread per context / GPU.
 */
#ifndef WK_API_H
#define WK_API_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wk_ctx wk_ctx;

enum wk_status {
  WK_OK = 0,
  WK_ERR_ARG = -1,       /* invalid argument */
  WK_ERR_HIP = -2,       /* HIP runtime error */
  WK_ERR_CONFIG = -3,    /* unsupported configuration (e.g. non-default network DSL) */
  WK_ERR_COMM = -4,      /* RCCL error */
  WK_ERR_STATE = -5      /* call order (e.g. ppo_update before rollout) */
};

/* per-env fault bits (wk_step fault[] / wk_rollout) */
enum wk_fault { WK_FAULT_NONFINITE = 1u, WK_FAULT_SKIPPED_SAMPLE = 2u };

/* materials: Materials/<Name>.cs */
enum wk_material {
  WK_MAT_CARPET = 0, WK_MAT_ICE = 1, WK_MAT_RUBBER = 2, WK_MAT_METAL = 3, WK_MAT_WOOD = 4,
  WK_MAT_PAPER = 5, WK_MAT_TITANIUM = 6, WK_MAT_SUPERRUBBER = 7
};

/* Hyperparameters (Walker/PPO/Hyperparameters.cs:80-121): same names and defaults.
 * Batched extensions are marked (new). */
typedef struct wk_config {
  int GameSpeed;            /* 1 (UI only; ignored) */
  int Iterations;           /* 50 physics substeps per env-step */
  int MaxTimesteps;         /* 1000 */
  int RoughFloor;           /* 0; 1: CreateRoughFloor's 10 static segments with a per-walker
                               Philox terrain (every mapping) */
  int Epochs;               /* 5 */
  int BatchSize;            /* 64 */
  int UseGAE;               /* 0 */
  int NormalizeAdvantages;  /* 0 */
  float Gamma;              /* 0.9 */
  float Lambda;             /* 0.95 */
  float Epsilon;            /* 0.3 */
  float LogStandardDeviation; /* -1 */
  float Alpha;              /* 1e-3 */
  float Beta1;              /* 0.9 */
  float Beta2;              /* 0.999 */
  float AdamEpsilon;        /* 1e-8 */
  const char* CriticNeuralNetwork; /* NULL or "Input |64| (LeakyReLU) |1| Output" */
  const char* ActorNeuralNetwork;  /* NULL or "Input |64| (LeakyReLU) |64| (LeakyReLU) |4| (TanH) Output" */
  float DeltaTime;          /* MonoGame fixed step, (float)(166667 ticks / 1e7) */
  /* (new) batched extensions */
  int Horizon;              /* rollout horizon T_h of the device trajectory buffer (64) */
  int Minibatch;            /* local minibatch M for wk_ppo_update (0 -> BatchSize) */
  int MinibatchGlobal;      /* divisor of dV/dmu = global minibatch (0 -> Minibatch * nranks) */
  int EnvOffset;            /* global id of this context's env 0 (Philox streams) */
  int RandomizeStart;       /* 1: env e starts at x + 200*u_e (BASELINE config 2) */
  int RandomizeMaterial;    /* 1: env material in {Ice, Rubber, Carpet} (config 5) */
  int LanesPerWalker;       /* physics kernel mapping (all bit-exact): 2 = a lane pair per
                               walker, left / right leg chains in parallel; 4 = two lanes per
                               leg (SAT axes and contact faces split; for shards of at most
                               one wave per SIMD); 16 = SAT axes over a 16-lane row; 1 = one
                               walker per lane; 0 = auto (4 up to 16,384 walkers, else 2) */
} wk_config;

/* The host-only fields of the reference's JSON configuration (SerializableHyperparameters,
 * Hyperparameters.cs:11-77), plus storage for the network DSL strings that
 * wk_config_from_json points wk_config at.  Not used by the kernels. */
typedef struct wk_host_settings {
  int CollectData;                /* 1 */
  int SaveWeights;                /* 1 */
  char CriticNeuralNetwork[256];  /* "Input |64| (LeakyReLU) |1| Output" */
  char ActorNeuralNetwork[256];   /* "Input |64| (LeakyReLU) |64| (LeakyReLU) |4| (TanH) Output" */
  char CriticWeightFileName[256]; /* "critic" */
  char ActorWeightFileName[256];  /* "actor" */
  char FilePath[1024];            /* AppDomain BaseDirectory: the executable's directory + "/" */
} wk_host_settings;

/* canonical per-env state dump: WK_STATE_FLOATS floats per env (identical layout to
 * the oracle's orc_env_dump).  Body b in {LLL, LLU, BODY, RLL, RLU} at b*20:
 * verts x0,y0..x5,y5 (BODY uses 5), centroid x,y, v x,y, w, angle, collided, pad. */
enum {
  WK_STATE_FLOATS = 112, WK_ST_TORQUE = 100, WK_ST_POS = 104, WK_ST_PREV = 106,
  WK_ST_STEPS = 108, WK_ST_POSTRESET = 109, WK_ST_TERMINAL = 110, WK_ST_EPISODES = 111,
  WK_NPARAM_CRITIC = 897, WK_NPARAM_ACTOR = 5252, WK_NPARAM = 6149, WK_OBS = 12, WK_ACT = 4,
  WK_NPAIRS = 9
};

/* per-substep pair bookkeeping (bit-exact parity outputs).  Canonical
 * pair index: 0 (LLL,LLU) 1 (LLL,FLOOR) 2 (LLU,LLL) 3 (LLU,FLOOR) 4 (BODY,FLOOR)
 * 5 (RLL,RLU) 6 (RLL,FLOOR) 7 (RLU,RLL) 8 (RLU,FLOOR). */
typedef struct wk_pair_trace {
  uint8_t aabb_hit[WK_NPAIRS];
  uint8_t sat_hit[WK_NPAIRS];
  uint8_t n_contacts[WK_NPAIRS];
  uint8_t pad[5];
  float normal[WK_NPAIRS][2];
  float depth[WK_NPAIRS];
  float contact[WK_NPAIRS][2][2]; /* contact points (n_contacts valid) */
  float impulse[WK_NPAIRS][2];    /* normal and friction impulse */
  float joint_depth[4];           /* Joint.Step gap per joint (0 if < 0.1) */
  float joint_impulse[4];
} wk_pair_trace;

/* one body of one env, for Renderer.RenderRigidObject / ConsoleRenderer */
typedef struct wk_body_view {
  int n_vertices;
  float vertices[6][2];
  float centroid[2];
  float linear_velocity[2];
  float angular_velocity;
  float angle;
  int collided;
  int is_static;
} wk_body_view;

/* Scene prop (extension of SURVEY 8(f) next-3): a Square / Triangle / Hexagon body built by
 * <Shape>.FromSize(material, (cx, cy), size, isStatic) (Objects/RigidBodies/Square.cs:18-31,
 * Triangle.cs:18-30, Hexagon.cs:18-33), then SmoothCorners(smooth) (Skeleton.cs:33-53; the
 * centroid keeps its FromSize value), SetLinearVelocity((vx, vy)), SetAngularVelocity(w) and
 * AddAcceleration((ax, ay)) (RigidBody.cs:143-183; gravity would be (0, 980)).  Every walker
 * gets its own copy, listed after the floor: the line a maintainer adds after CreateFloor()
 * in the Environment constructor (Environment.cs:39-51).  Walker resets keep the props. */
enum { WK_SHAPE_SQUARE = 0, WK_SHAPE_TRIANGLE = 1, WK_SHAPE_HEXAGON = 2 };
enum { WK_MAX_PROPS = 4, WK_PROP_MAXV = 24, WK_SCENE_MAX_VERTS = 32 };
typedef struct wk_prop {
  int32_t shape;      /* WK_SHAPE_* */
  int32_t smooth;     /* SmoothCorners count: vertices = 4 / 3 / 6 times 2^smooth, <= 24 */
  int32_t material;   /* 0 Carpet, 1 Ice, 2 Rubber, 3 Metal, 4 Wood, 5 Paper, 6 Titanium,
                         7 SuperRubber (Materials/<Name>.cs) */
  int32_t is_static;
  float cx, cy, size;
  float vx, vy, w;    /* initial linear / angular velocity */
  float ax, ay;       /* acceleration */
} wk_prop;

/* one scene prop of one env (Renderer.RenderRigidObject) */
typedef struct wk_prop_view {
  int n_vertices;
  float vertices[WK_PROP_MAXV][2];
  float centroid[2];
  float linear_velocity[2];
  float angular_velocity;
  float angle;
  int is_static;
} wk_prop_view;

typedef struct wk_ppo_args {
  int epochs;          /* 0 -> config Epochs */
  int minibatch;       /* 0 -> config Minibatch */
  int minibatch_global;/* 0 -> config MinibatchGlobal */
  uint32_t update_index; /* permutation key: minibatch sampling of update #k */
} wk_ppo_args;

typedef struct wk_rollout_stats {
  double reward_sum;     /* sum of rewards over the horizon, this context */
  int64_t episodes;      /* terminal steps in the horizon */
  int64_t env_steps;     /* n_env * horizon */
  uint32_t fault_or;     /* OR of per-env fault bits */
  int32_t pad;
} wk_rollout_stats;

/* one finished episode (data collection) */
typedef struct wk_episode_rec {
  float total_reward;  /* (float) of the double sum of its rewards, like Enumerable.Sum */
  int32_t env;         /* global walker id (EnvOffset + index) */
  int32_t length;      /* env-steps in the episode */
  uint32_t step;       /* env-step it finished at, counted over this context's wk_rollout
                          calls (equal across ranks stepping in lockstep) */
} wk_episode_rec;

/* kernel timing (HIP events on the context's stream), cumulative since last reset */
typedef struct wk_profile {
  double physics_ms;   int64_t physics_launches;  int64_t physics_env_steps;
  double grad_ms;      int64_t grad_launches;
  double reduce_ms;    int64_t reduce_launches;
  double adam_ms;      int64_t adam_launches;
  double allreduce_ms; int64_t allreduce_calls;
  double returns_ms;   int64_t returns_launches;
  double update_ms;    int64_t update_calls;     /* whole wk_ppo_update calls */
} wk_profile;

void wk_config_defaults(wk_config* cfg);
const char* wk_version(void);

int wk_create(const wk_config* cfg, int device, int n_env, uint64_t seed, wk_ctx** out);
int wk_destroy(wk_ctx* ctx);
const char* wk_last_error(const wk_ctx* ctx); /* ctx may be NULL (create errors) */
int wk_sync(wk_ctx* ctx);
int wk_num_envs(const wk_ctx* ctx);

/* environment */
int wk_reset(wk_ctx* ctx, const uint8_t* mask /* n_env or NULL = all */);
int wk_set_materials(wk_ctx* ctx, const int32_t* mat_id /* n_env */);
/* start offsets (applied at each walker's next reset); on the rough floor the split mappings'
   lane order (walkers sorted by offset, results unaffected) is rebuilt from them */
int wk_set_offsets(wk_ctx* ctx, const float* dx /* n_env; start x = 125 + dx */);
int wk_step(wk_ctx* ctx, const float* actions_or_null /* k*n_env*4, unclipped */, int k_steps,
            float* obs /* k*n_env*12 or NULL */, float* reward /* k*n_env or NULL */,
            uint8_t* done /* k*n_env or NULL */, uint32_t* fault /* n_env or NULL */);
/* Environment.Update with the agent's own sampling, returning what Environment.cs:70-89
 * records in the Trajectory: for each of k env-steps and walkers, the state observed before
 * the step (_trajectory.States, :73), the sampled UNCLIPPED action (Walker.GetActions ->
 * PPOAgent.SampleActions, :74 / PPOAgent.cs:381-398; recorded at :86), its per-dimension
 * log-probability (:74, :87), the reward (:88) and terminal flag, the critic value of the
 * state (GetValueEstimate, PPOAgent.cs:447-456), the next state (post-reset after a
 * terminal step) and the torso position after the step, BEFORE any auto-reset
 * (Walker.GetPosition as Step reads it for _bestDistance, Environment.cs:113-119).  Any
 * output may be NULL.  Layouts [k][n_env][...]. */
int wk_step_sampled(wk_ctx* ctx, int k_steps, float* states /* k*n*12 */,
                    float* actions /* k*n*4 */, float* logp /* k*n*4 */,
                    float* values /* k*n */, float* reward /* k*n */, uint8_t* done /* k*n */,
                    float* next_obs /* k*n*12 */, uint32_t* fault /* n */,
                    float* position /* k*n*2 */);
int wk_step_device(wk_ctx* ctx, const float* d_actions_or_null, int k_steps, float* d_obs,
                   float* d_reward, uint8_t* d_done, uint32_t* d_fault);
/* one env-step with per-substep pair bookkeeping: trace[n_env * Iterations] */
int wk_step_traced(wk_ctx* ctx, const float* actions /* n_env*4 */, wk_pair_trace* trace);
int wk_get_obs(wk_ctx* ctx, float* obs /* n_env*12 */);
int wk_get_state(wk_ctx* ctx, float* state /* n_env*WK_STATE_FLOATS */);
/* wk_set_state (and wk_checkpoint_load's walker records) refuse, with WK_ERR_ARG and the walker
 * and body in wk_last_error, a state whose leg segments are not rigid walker poles: the kernels
 * project a pole onto its own edge axes over fixed vertex groups (exact for Pole.FromSize's
 * shape, Pole.cs:18-34, moved and rotated rigidly), so every vertex must stay >= 3.5 px outside
 * the groups it is left out of (the template has 7.5 px).  Non-finite poles are not checked.
 * wk_check_state runs the same check on host memory (no context, no device): WK_OK, or
 * WK_ERR_ARG with the first failing walker and body (record body index) in *bad_env / *bad_body. */
int wk_set_state(wk_ctx* ctx, const float* state /* n_env*WK_STATE_FLOATS */);
int wk_check_state(const float* state, int n_env, int* bad_env, int* bad_body);
/* The reference's per-body call shape (new entry points for a host that keeps
 * Environment.StepObjects, Environment.cs:126-143): per substep it calls Joint.Step on the 4 joints
 * (Joint.cs:31-41) and IObject.Update (Objects/IObject.cs:9) on every body of its list, after
 * Walker.TakeActions (Walker.cs:66-75).  The GPU resolves a whole env-step (every substep, joint
 * and body of every walker of the context) in one launch, so:
 *   wk_take_actions   stores walker env's 4 torques (unclipped; clipped in-kernel) for the next
 *                     frame; a walker given none keeps its current torques (no kick)
 *   wk_object_update  the frame's FIRST call runs one env-step of every walker with those torques
 *                     (returns 1); the other list_count * Iterations - 1 calls of the frame are
 *                     counted and return 0 (deltaTime: the caller's substep; the context's
 *                     DeltaTime is used)
 *   wk_joint_step     resolved inside the step: a no-op (returns 0)
 *   wk_body_order     walker env's body list now: part ids (0 LLL, 1 LLU, 2 Body, 3 RLL, 4 RLU,
 *                     5 floor / 5..14 rough-floor segments) floor last in episode 0 and first after
 *                     a reset (Walker.cs:191-234) -- at most 15 */
int wk_take_actions(wk_ctx* ctx, int env, const float* actions /* 4 */);
int wk_object_update(wk_ctx* ctx, int list_count, float delta_time);
int wk_joint_step(wk_ctx* ctx);
int wk_body_order(wk_ctx* ctx, int env, int* parts /* 15 */, int* count);
int wk_get_body_view(wk_ctx* ctx, int env, int body /* 0..4 walker, 5 floor (5..14 rough-floor segments) */,
                     wk_body_view* out);

/* policy / value */
/* Scene props for every walker (n_props <= WK_MAX_PROPS, at most WK_SCENE_MAX_VERTS vertices
 * in total; 0 removes them), each initialised as described at wk_prop.  With props the
 * env-step runs the one-lane scene kernel (LanesPerWalker 0 or 1), on either floor: with
 * RoughFloor the list is [walker, 10 segments, props] (after a reset [segments, props,
 * walker]), and props resolve against every segment. */
int wk_set_scene(wk_ctx* ctx, const wk_prop* props, int n_props);
int wk_get_prop_view(wk_ctx* ctx, int env, int prop, wk_prop_view* out);
int wk_get_weights(wk_ctx* ctx, float* params /* WK_NPARAM */);
int wk_set_weights(wk_ctx* ctx, const float* params);
int wk_get_adam(wk_ctx* ctx, float* m, float* v, int* t);
int wk_set_adam(wk_ctx* ctx, const float* m, const float* v, int t);

/* JSON configuration files (replaces Hyperparameters.SerializeJson / DeserializeJson,
 * Hyperparameters.cs:124-187, System.Text.Json default options, WriteIndented on save).
 * wk_config_to_json: NULL cfg / host = defaults; returns -(bytes needed) when cap is too
 * small.  wk_config_from_json: the document updates *cfg and *host in place (missing
 * properties keep their values); a malformed document or a value outside
 * ValidateHyperparameterValues (:189-217) returns WK_ERR_CONFIG and changes nothing;
 * otherwise returns the number of ValidateVariables (:240-290) corrections (invalid file
 * path / weights file names / network strings reset to defaults), their messages (one per
 * line) in wk_last_error(NULL).  cfg's network-string pointers are set to host's buffers.
 * No device is touched. */
void wk_host_settings_defaults(wk_host_settings* host);
int wk_config_to_json(const wk_config* cfg, const wk_host_settings* host, char* out, size_t cap);
int wk_config_from_json(const char* json, wk_config* cfg, wk_host_settings* host);
int wk_config_save_json(const char* path, const wk_config* cfg, const wk_host_settings* host);
int wk_config_load_json(const char* path, wk_config* cfg, wk_host_settings* host);

/* Weights files in the reference's text format (replaces PPOAgent.Save / Load,
 * PPOAgent.cs:192-213, over NeuralNetwork.Save / Load NeuralNetwork.cs:94-176,
 * DenseLayer.Save / Load DenseLayer.cs:55-79, Matrix.Save / Load Matrix.cs:109-153):
 * line 0 the network DSL string, then per dense layer "W <out*in row-major> B <out>",
 * floats written as .NET Core's float.ToString() (shortest round-trip, "1E-05" style).
 * Unlike the reference (which silently keeps its weights), a mismatching DSL line or a
 * malformed token is an error (WK_ERR_CONFIG / WK_ERR_ARG) and nothing is changed. */
int wk_save_weights(wk_ctx* ctx, const char* critic_path, const char* actor_path);
int wk_load_weights(wk_ctx* ctx, const char* critic_path, const char* actor_path);
/* context-free text conversion of a WK_NPARAM vector (no GPU).  wk_format_weights returns
 * -(bytes needed) when a buffer is too small. */
int wk_format_weights(const float* params, char* critic_text, size_t critic_cap,
                      char* actor_text, size_t actor_cap);
int wk_parse_weights(const char* critic_text, const char* actor_text, float* params);

/* Binary checkpoint for bit-exact resume (new; the reference persists only weights):
 * weights, Adam m / v / t, every walker record, Philox step counters, start offsets,
 * materials, running episode rewards / lengths, the episode-log clock and the scene props
 * (descriptions and every walker's prop state; loading replaces the context's scene) (the episode and
 * loss logs are not included: drain them first).  Loading requires the same n_env, seed and EnvOffset; it invalidates the
 * trajectory buffer (roll out again before wk_ppo_update). */
int wk_checkpoint_save(wk_ctx* ctx, const char* path);
int wk_checkpoint_load(wk_ctx* ctx, const char* path);
int wk_policy_sample(wk_ctx* ctx, int n, const float* obs /* n*12 */, const int32_t* env_ids,
                     const uint32_t* steps, float* mean, float* act, float* logp);
int wk_value(wk_ctx* ctx, int n, const float* obs, float* v);

/* rollout + PPO (device-resident trajectory buffer [Horizon][n_env]) */
int wk_rollout(wk_ctx* ctx, int horizon /* <= config Horizon; 0 = Horizon */);
int wk_rollout_stats_get(wk_ctx* ctx, wk_rollout_stats* out);
int wk_get_trajectory(wk_ctx* ctx, float* states, float* actions, float* logp, float* rewards,
                      uint8_t* dones, float* values, float* returns, float* advantages);
int wk_set_trajectory(wk_ctx* ctx, int horizon, const float* states, const float* actions,
                      const float* logp, const float* rewards, const uint8_t* dones,
                      const float* values);
int wk_compute_returns(wk_ctx* ctx);
int wk_ppo_update(wk_ctx* ctx, const wk_ppo_args* args, float* critic_diag, float* actor_diag);
/* Train(Batch) on caller data: B samples, divisor b_div; grads_out (optional, WK_NPARAM)
 * receives the accumulated gradient before Adam. Returns skipped-sample count in *skipped. */
int wk_train_batch(wk_ctx* ctx, int B, float b_div, const float* states, const float* actions,
                   const float* logp_old, const float* returns, const float* adv,
                   float* critic_diag, float* actor_diag, float* grads_out, int apply_adam,
                   int* skipped);
/* The same minibatch gradient as computed inside wk_ppo_update (matrix-core kernel,
 * samples summed in 16-sample MFMA blocks -- a different fp32 association than
 * Train(Batch)'s sequential loop, PPOAgent.cs:228-335); no Adam step. */
int wk_minibatch_gradient(wk_ctx* ctx, int B, float b_div, const float* states,
                          const float* actions, const float* logp_old, const float* returns,
                          const float* adv, float* critic_diag, float* actor_diag,
                          float* grads_out, int* skipped);

/* Data collection (replaces ConsoleRenderer.AddTotalEpisodeReward / AddCriticLoss /
 * AddActorLoss, ConsoleRenderer.cs:79-95, fed by PPOAgent.Train PPOAgent.cs:151,165-166,
 * and CreateDataFile :124-135).  On by default (Hyperparameters.CollectData = true): every
 * wk_rollout appends each finished episode to a device log in completion order
 * (env-step, walker) -- wk_step does not feed it -- and every wk_ppo_update appends its last minibatch's
 * (critic, actor) diagnostics.  The episode log holds n_env * Horizon records and the loss
 * log 65,536 updates; drain them at least that often (the overflow is counted in
 * *dropped).  Drains clear the logs; a cap smaller than the held count is WK_ERR_ARG. */
int wk_collect_data(wk_ctx* ctx, int on);
int wk_episode_log_count(wk_ctx* ctx, int64_t* episodes, int64_t* updates);
int wk_episode_log_drain(wk_ctx* ctx, wk_episode_rec* out, int64_t cap, int64_t* n_out,
                         int64_t* dropped);
int wk_loss_log_drain(wk_ctx* ctx, float* critic, float* actor, int64_t cap, int64_t* n_out,
                      int64_t* dropped);
/* the reference's data file: rewards / critic losses / actor losses lists, no device */
int wk_write_data_file(const char* path, const float* total_rewards, int64_t n_rewards,
                       const float* critic_losses, int64_t n_critic, const float* actor_losses,
                       int64_t n_actor);

/* multi-GPU: RCCL communicator over the ranks' contexts (one per GPU) */
int wk_comm_unique_id(uint8_t* id /* 128 bytes */);
int wk_comm_init(wk_ctx* ctx, int rank, int nranks, const uint8_t* unique_id);
/* sum of host_buf over the ranks, in place, through the context's exchange: RCCL, or with
 * wk_comm_init_ipc one round of the IPC exchange (n <= 6,152 floats; ranks summed in rank order;
 * WK_ERR_COMM when a peer never publishes) -- tests, and bench.py's check of a fresh IPC mapping */
int wk_allreduce_test(wk_ctx* ctx, float* host_buf, int n);
/* The same minibatch sequence with a caller-supplied all-reduce instead of RCCL: after the
 * ordered reduction each minibatch's slab (gradient + diagnostics, n floats) is copied to the
 * host, fn must replace it in place with the sum over ranks (return 0), and it is copied back
 * before Adam.  For hosts without RCCL (MPI, a CPU control plane) and for testing the
 * multi-rank path of several processes sharing one GPU (RCCL refuses duplicate devices).
 * fn is kept for the context's lifetime (a managed caller must keep its delegate alive).  A
 * non-zero return fails this rank's wk_ppo_update with WK_ERR_COMM mid-update (no Adam step
 * for that minibatch) while the peers wait in their own all-reduce: it is fatal for the
 * whole job -- abort every rank. */
typedef int (*wk_host_allreduce_fn)(float* buf, int n, void* user);
int wk_comm_init_host(wk_ctx* ctx, int rank, int nranks, wk_host_allreduce_fn fn, void* user);
/* The one-shot exchange over peer-mapped memory instead of RCCL (ranks on one node, at most 8):
 * wk_comm_ipc_handle allocates this rank's exchange region and returns its record (the IPC
 * handle, then the PCI bus id of the rank's GPU); the caller all-gathers the records (any
 * control plane) and passes all of them, in rank order, to wk_comm_init_ipc, which maps the
 * peers' regions (WK_ERR_ARG if more than 4 ranks share one GPU: they would stall).  Per
 * minibatch one kernel publishes this rank's ordered block sum, waits (bounded: 30 s of the
 * GPU's constant clock by default; WK_XCH_TIMEOUT_S in the environment at wk_comm_init_ipc, or
 * wk_comm_set_timeout, changes it -- the ranks must stay within it of each other: a rank busy
 * elsewhere longer than that while its peers have an update queued kills the job) for every
 * peer's, sums the ranks' slabs in rank order and applies Adam -- no collective library, no host
 * round trip.  A peer that never publishes (or gave up first) fails wk_ppo_update /
 * wk_train_batch / wk_minibatch_gradient / wk_allreduce_test with WK_ERR_COMM, fatal for the
 * job as a failed all-reduce: from the failed minibatch on this rank applies no Adam step and
 * marks its flags aborted, so a late peer fails that same minibatch instead of applying it, and
 * wk_get_adam reports the steps actually applied.  The replicas may still differ after a
 * failure (a peer that read this rank's flag just before the abort, or blocks straddling the
 * bound), and the failed context stays failed (its error word and aborted flags are not cleared
 * by wk_checkpoint_load): stop the job, or on every rank destroy the context, create a new one,
 * map the exchange again (wk_comm_ipc_handle / wk_comm_init_ipc) and load a checkpoint.
 * wk_minibatch_gradient and
 * wk_train_batch(apply_adam = 0) run the exchange as well (collective calls: every rank must
 * make them), returning the sum over the ranks as on an RCCL context. */
enum { WK_IPC_HANDLE_BYTES = 128 };
int wk_comm_ipc_handle(wk_ctx* ctx, uint8_t* handle /* WK_IPC_HANDLE_BYTES */);
int wk_comm_init_ipc(wk_ctx* ctx, int rank, int nranks, const uint8_t* handles /* nranks * 128 */);
/* the IPC exchange's bounded peer wait, in seconds (0 < seconds <= 1e6) */
int wk_comm_set_timeout(wk_ctx* ctx, double seconds);
/* the context's minibatch exchange: *kind 0 none, 1 RCCL, 2 host callback, 3 IPC; *flags bit 0:
 * the IPC exchange region is uncached device memory (else coarse-grained hipMalloc memory) */
int wk_comm_info(wk_ctx* ctx, int* kind, int* flags);
/* IPC exchange timing (new; the exchange replaces the all-reduce before PPOAgent.cs:344-345's
 * Optimise): with minibatches > 0 every exchange launch of the context stamps the GPU's 100 MHz
 * constant clock per block at four points -- entry, its slab published (flag released), every
 * peer's flag seen, exit (peer slabs read, Adam stored) -- into a device ring of `minibatches`
 * launches; 0 frees the ring.  wk_comm_xch_stamps copies the last min(stamped, max_launches)
 * launches, oldest first, as stamps[(launch * blocks + block) * 4 + point] (ticks of 10 ns). */
int wk_comm_xch_profile(wk_ctx* ctx, int minibatches);
int wk_comm_xch_stamps(wk_ctx* ctx, uint64_t* stamps, int max_launches, int* launches, int* blocks);

/* profiling */
/* level 0 off; 1: HIP events around each rollout / returns pass / whole PPO update (cheap
 * enough inside a timed loop); 2: also around every gradient / reduce / all-reduce / Adam
 * launch of the update */
int wk_profile_enable(wk_ctx* ctx, int on);
int wk_profile_get(wk_ctx* ctx, wk_profile* out);
int wk_profile_reset(wk_ctx* ctx);

/* Counting replay (the flop model priced on the physics events that actually
 * happen, RigidBody.cs:66-96 / Joint.cs:31-41): steps the walkers k env-steps with the
 * actions recorded in the device trajectory (rows 0..k-1 of the last rollout; k <= its
 * horizon) through the one-lane kernel with per-lane event counters -- the same physics bit
 * for bit as the rollout when the state is the rollout's starting state (see wk_snapshot).
 * counts[WK_NEV] (added to, not cleared) receives, in order: joints past the 0.1 early-out;
 * bounding-box hits leg-leg / leg-floor / torso-floor (each runs SAT); SAT collisions
 * (contacts + MoveObjects) in the same three classes; contact resolutions with >= 1 point
 * (the impulse pair) in the same three classes; contact points; walker-substeps; env-steps;
 * auto-resets; walker env-steps with >= 1 leg-floor bounding-box hit; walker env-steps with
 * >= 1 leg-leg SAT collision. */
#define WK_NEV 16
int wk_count_events(wk_ctx* ctx, int k, uint64_t* counts);

/* Device-side snapshot of the training state: walker records, Philox step counters, weights,
 * Adam m / v / t, episode bookkeeping and scene props (not the trajectory buffer, which keeps
 * the last rollout).  op 0 saves, op 1 restores (stream-ordered device copies, no host sync); bench.py restores one before every timed iteration so
 * each measures the same regime (the throughput no longer drifts with training). */
int wk_snapshot(wk_ctx* ctx, int op);

/* The update's gradient kernel alone: `reps` back-to-back launches on minibatch 0 (update 0,
 * epoch 0 of the keyed sequence; minibatch 0 = config Minibatch) of the current trajectory,
 * timed by one HIP-event pair on the context's stream -- the kernel's mean duration without
 * per-launch event overhead (bench.py's update roofline).  Writes only scratch slabs. */
int wk_time_gradient(wk_ctx* ctx, int minibatch, int reps, double* ms_per_launch);
/* The same with flags: bit 0 puts an event pair around EVERY launch (the elapsed times summed),
 * as profile level 2 times each launch of the update.  bench.py prices the update roofline on
 * the gradient kernel's in-update duration: the level-2 per-launch mean inside a real update
 * minus the per-launch event overhead (this burst with bit 0 minus the plain burst). */
int wk_time_gradient_ex(wk_ctx* ctx, int minibatch, int reps, int flags, double* ms_per_launch);

/* The rollout kernel's mapping as launched: lanes per walker (1, 2, 4 or 16), walkers per
 * wave (fewer than 64 / lanes for the sparse quad mapping), the waves that hold walkers and
 * (waves_launched, nullable) the waves the grid launches -- the split kernels launch whole
 * 4-wave blocks whose idle waves replay the last walker.  bench.py's VALU ceiling is priced on
 * the launched grid (one wave per SIMD below 1,024 waves). */
int wk_rollout_mapping(wk_ctx* ctx, int* lanes_per_walker, int* walkers_per_wave, int64_t* waves,
                       int64_t* waves_launched);

/* Which matrix-core gradient kernel the update launches for a per-GPU minibatch of `minibatch`
 * samples (0 = config Minibatch): 0 producer / consumer waves (k_ppo_grad_ws), 1 tile-parallel
 * teams (k_ppo_grad_tp, two per block), 2 the same with one team per block, 3 one wave per chunk
 * (k_ppo_grad_mfma).  By size (tp1 up to 4,096 samples, tp below 32,768, ws from there) unless
 * WK_GRAD_IMPL = ws / tp / tp1 / mf was set at wk_create. */
int wk_grad_kernel(wk_ctx* ctx, int minibatch);

#ifdef __cplusplus
}
#endif
#endif
