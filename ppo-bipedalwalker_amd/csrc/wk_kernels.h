// wk_kernels.h -- kernel argument blocks and host launch shims shared by
// wk_physics.hip, wk_ppo.hip and wk_api.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "wk_common.h"

namespace wk {

// per-substep pair bookkeeping; layout == wk_pair_trace (include/wk_api.h)
struct PairTraceDev {
  uint8_t aabb_hit[9];
  uint8_t sat_hit[9];
  uint8_t n_contacts[9];
  uint8_t pad[5];
  float normal[9][2];
  float depth[9];
  float contact[9][2][2];
  float impulse[9][2];
  float joint_depth[4];
  float joint_impulse[4];
};

// physics event counters of the counting replay (wk_count_events; SURVEY 8(d) F_counted)
enum : int {
  EV_JOINT = 0,                            // Joint.Step past the 0.1 gap early-out
  EV_AABB_LL, EV_AABB_LF, EV_AABB_BF,      // bounding boxes overlap -> SAT runs
  EV_SAT_LL, EV_SAT_LF, EV_SAT_BF,         // SAT reports a collision -> contacts + MoveObjects
  EV_IMP_LL, EV_IMP_LF, EV_IMP_BF,         // >= 1 contact point -> the impulse pair
  EV_CONTACTS,                             // contact points found
  EV_SUBSTEPS,                             // walker-substeps
  EV_ENV_STEPS, EV_RESETS,                 // env-steps, auto-resets
  EV_STEPS_LF, EV_STEPS_SATLL,             // walker env-steps with >= 1 leg-floor AABB hit /
                                           // >= 1 leg-leg SAT hit (how concentrated they are)
  NEV = 16                                 // (LL leg-leg, LF leg-floor, BF torso-floor)
};

struct StepArgs {
  float* st;                 // walker state records [n][NSTATE]
  const float* dxoff;        // [n] start offset (x = 125 + dx)
  const int32_t* mat;        // [n] material id
  uint32_t* rng_t;           // [n] per-env env-step counter (Philox counter)
  const float* actions;      // [k][n][4] or null (policy)
  float* obs_out;            // [k][n][12] or null
  float* pos_out;            // [k][n][2] torso centroid after the step, before any auto-reset
                             // (Walker.GetPosition at Environment.cs:119) or null
  float* rew_out;            // [k][n] or null
  uint8_t* done_out;         // [k][n] or null
  uint32_t* fault_out;       // [n] or null (OR-accumulated)
  const float* W;            // params (policy)
  const float* Wz;           // params in the matrix-core operand order (wk_mfma_layout.h)
  float lp_const;            // -ln(std) - ln(sqrt(2 pi))
  // trajectory buffer (RECORD), index t*n + e
  float* traj_s; float* traj_a; float* traj_lp; float* traj_r; uint8_t* traj_d; float* traj_v;
  int t0;
  PairTraceDev* trace;       // [n][iterations] (TRACE)
  int k_steps;
  float* props;              // scene props [n][SceneDev::pstride] (k_env_scene) or null
  unsigned long long* counts;  // [NEV] event totals (counting replay, mode 4) or null
  const int32_t* order;      // k_env_side: walker of lane slot s (wk_order.hip) or null (identity)
  // k_env_side pair mapping / k_env_step: per-SIMD progress tags of the co-resident waves
  // ([PACE_SLOTS], zeroed at creation; null: no pacing) and this launch's sequence number
  unsigned long long* pace;
  uint32_t pace_seq;
};
enum : int { PACE_SLOTS = 8 * 8 * 2 * 16 * 4 };  // XCC x SE x SH x CU x SIMD (HW_ID fields)

// scene props (wk_scene.inc): Square / Triangle / Hexagon bodies after the floor, the same
// shapes for every walker; per walker and prop k the state x[nv], y[nv], cx, cy, vx, vy, w,
// angle starts at float off[k] of the walker's prop record
enum : int {
  SCENE_MAX_PROPS = 4, SCENE_PROP_MAXV = 24, SCENE_MAX_VERTS = 32,
  SCENE_FIELDS = 2 * SCENE_MAX_VERTS + 6 * SCENE_MAX_PROPS
};
struct SceneDev {
  int n_props, pstride;
  int nv[SCENE_MAX_PROPS], off[SCENE_MAX_PROPS], stat[SCENE_MAX_PROPS];
  float im[SCENE_MAX_PROPS], ii[SCENE_MAX_PROPS], e[SCENE_MAX_PROPS], mu[SCENE_MAX_PROPS];
  float adx[SCENE_MAX_PROPS], ady[SCENE_MAX_PROPS];  // acceleration * deltaTime
};

struct AdamArgs {
  float* W; float* m; float* v; const float* grad;
  float* Wz;  // operand-order image kept in step with W (or null)
  float c1, c2, beta1, beta2, bc1, bc2, alpha, eps;
};

struct GradArgs {
  const float* W;        // params
  const float* Wz;       // the same params in the matrix-core operand order (wk_mfma_layout.h)
  const float* states;   // [P][12]
  const float* actions;  // [P][4]
  const float* logp_old; // [P][4]
  const float* returns;  // [P]
  const float* adv;      // [P]
  uint32_t pool;         // P
  uint32_t base;         // first permuted position of this minibatch
  int use_perm;
  PermKey pk;
  int samples;           // samples in this minibatch (local)
  int spw;               // samples per wave
  float b_div;           // divisor of dV / dmu (BatchSize / global minibatch)
  float std_;            // MathF.Exp(LogStandardDeviation)
  float lp_const;        // -ln(std) - ln(sqrt(2 pi))
  float upper, lower;    // 1 + eps, 1 - eps
  float* partial;        // [nblocks][SLAB]
};

// gradient + critic diag, actor diag, skipped, then zero pads to a multiple of 4 floats (16-byte
// rows: the matrix-core kernel's block fold and slab stores are f4-wide)
enum : int { SLAB = (NPARAM + 3 + 3) / 4 * 4 };
static_assert(SLAB % 4 == 0 && SLAB >= NPARAM + 3, "slab layout");

hipError_t launch_env_step(int mode, const EnvParams& P, const StepArgs& A, hipStream_t s);
hipError_t launch_env_scene(int mode, const EnvParams& P, const StepArgs& A, const SceneDev& S,
                            hipStream_t s);
hipError_t launch_env_init(const EnvParams& P, float* st, const float* dx, const uint8_t* mask,
                           int post, hipStream_t s);
hipError_t launch_get_obs(const EnvParams& P, const float* st, float* obs, hipStream_t s);
hipError_t launch_policy(const EnvParams& P, const float* W, float lp_const, int n,
                         const float* obs, const int32_t* env_ids, const uint32_t* steps,
                         float* mean, float* act, float* logp, float* v, hipStream_t s);
hipError_t launch_returns(int n, int T, int use_gae, float gamma, float lambda, const float* r,
                          const float* v, const uint8_t* d, float* ret, float* adv, hipStream_t s);
hipError_t launch_ppo_grad(const GradArgs& g, int wpb, int nblocks, hipStream_t s);
hipError_t configure_device_kernels();  // dynamic-LDS attributes, current device (wk_create)
hipError_t configure_mfma_kernels();
// matrix-core gradient kernels: producer / consumer pairs (ws), tile-parallel teams of four
// waves, two (tp) or one (tp1) per block, one wave per chunk (mf); GI_AUTO picks by size
enum : int { GI_AUTO = -1, GI_WS = 0, GI_TP2 = 1, GI_TP1 = 2, GI_MF = 3 };
int grad_impl_env();                       // WK_GRAD_IMPL = ws / tp / tp1 / mf, else GI_AUTO
int grad_impl_for(int impl, int samples);  // resolves GI_AUTO
hipError_t launch_ppo_grad_mfma(const GradArgs& g, int nblocks, int impl, hipStream_t s);
hipError_t launch_swizzle(const float* W, float* Wz, hipStream_t s);
int mfma_image_floats();
int ppo_grad_mfma_blocks(int samples, int impl);
hipError_t launch_grad_reduce(const float* partial, int nblocks, float* part2, float* grad,
                              hipStream_t s);
int grad_reduce_groups(int nblocks);
hipError_t launch_grad_reduce_adam(const float* partial, int nblocks, float* part2, float* grad,
                                   const AdamArgs& a, hipStream_t s);
hipError_t launch_adam(const AdamArgs& a, hipStream_t s);

// One-shot gradient exchange over peer-mapped (IPC) memory, fused with the ordered block
// reduction and Adam (wk_comm_init_ipc): rank r's exchange region is [2][SLAB] floats
// (double-buffered by minibatch parity) then XCH_FLAGS uint64 sequence flags, one per block of
// the fused kernel (each block owns a span of parameter quads).
// XCH_TIMEOUT_S_DEFAULT: the bounded wait for a peer's flag (s_memrealtime ticks of the 100 MHz
// constant clock, XCH_TICKS_PER_S); a context takes WK_XCH_TIMEOUT_S from the environment at
// wk_comm_init_ipc or wk_comm_set_timeout.  XCH_ABORT: the flag value of a rank whose exchange
// timed out (or that saw an earlier timeout): a peer that reads it fails the same minibatch
// instead of applying it.  XCH_MAX_RANKS_PER_DEVICE: more ranks sharing one GPU stall (their
// waiting exchange blocks hold the CUs a peer's gradient kernel needs), so wk_comm_init_ipc
// refuses them.
// threads per block of the split (pair / quad) rollout kernels; wk_rollout_mapping reports the
// launched grid from it
#ifndef WK_SIDE_BLOCK
#define WK_SIDE_BLOCK 256
#endif
constexpr int SIDE_BLOCK_THREADS = WK_SIDE_BLOCK;
enum : int { XCH_FLAGS = 128, XCH_MAX_RANKS = 8, XCH_MAX_RANKS_PER_DEVICE = 4 };
constexpr double XCH_TIMEOUT_S_DEFAULT = 30.0;
constexpr double XCH_TICKS_PER_S = 1.0e8;
constexpr uint64_t XCH_ABORT = ~0ull;
struct XchArgs {
  const float* partial;                // this rank's gradient-kernel block slabs [nblocks][SLAB]
  int nblocks;
  float* grad_out;                     // the rank-order sum over ranks [SLAB]
  float* slab[XCH_MAX_RANKS];          // every rank's exchange region (own + peer-mapped)
  uint64_t* flag[XCH_MAX_RANKS];       // every rank's XCH_BLOCKS flags
  int rank, nranks;
  uint64_t seq;                        // this minibatch's sequence number (from 1)
  uint32_t* err;                       // [0] set to 1 if a peer never published (bounded wait) or
                                       // aborted; once set, every later exchange is a no-op (no
                                       // Adam); [1] the Adam step t block 0 last applied
  uint64_t timeout_ticks;              // the bounded wait (s_memrealtime ticks)
  uint32_t t;                          // this minibatch's Adam step (with a.W)
  AdamArgs a;                          // a.W == null: exchange only (gradient-only calls)
  uint64_t* stamps;                    // null, or this launch's [blocks][XCH_POINTS] clock stamps
};
// exchange timing (wk_comm_xch_profile): per block, the 100 MHz constant clock at entry, slab
// published, every peer's flag seen, exit
enum : int { XCH_POINTS = 4 };
int xch_blocks();
size_t xch_region_bytes();
hipError_t launch_reduce_xch_adam(const XchArgs& x, hipStream_t s);
hipError_t launch_normalize(float* x, int n, float eps, hipStream_t s);
hipError_t launch_xavier(float* W, uint64_t seed, hipStream_t s);

// data collection: per-episode totals of a recorded rollout appended to the device log;
// layout == wk_episode_rec (include/wk_api.h)
struct EpisodeRecDev {
  float total_reward;
  int32_t env;
  int32_t length;
  uint32_t step;
};
struct EpisodeArgs {
  int n, T, env_offset;
  uint32_t step0;             // rollout env-steps taken before this one
  const float* rewards;      // [T][n]
  const uint8_t* dones;      // [T][n]
  double* acc;               // [n] running episode reward (carried across rollouts)
  int32_t* len;              // [n] running episode length
  float2* scratch;           // [T][n] (total, length bits), written where done
  uint32_t* row_cnt;         // [episode_count_cells(n, T)], zero on entry and exit
  uint64_t* log_count;       // records appended so far (may exceed cap: dropped)
  uint64_t cap;
  EpisodeRecDev* log;
};
hipError_t launch_episode_log(const EpisodeArgs& a, hipStream_t s);
// lane order for k_env_side: episode-0 walkers first, then the post-reset ones (wk_order.hip)
int order_cells(int n);  // counters: one per tile of 1,024 slots + the swap count
hipError_t launch_walker_order(const float* st, int n, uint32_t* cnt, int32_t* order,
                               int32_t* scratch /* [2 n] */, hipStream_t s);
int episode_count_cells(int n, int T);
hipError_t launch_episode_reset(int n, const uint8_t* mask, double* acc, int32_t* len,
                                hipStream_t s);

}  // namespace wk
