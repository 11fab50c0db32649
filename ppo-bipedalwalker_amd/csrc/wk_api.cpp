// wk_api.cpp -- C-ABI implementation (include/wk_api.h): context, device memory,
// launches on the context's HIP stream, RCCL gradient all-reduce, kernel timing.
//
// Host responsibilities only: argument validation (Hyperparameters validation,
// Walker/PPO/Hyperparameters.cs:189-217), buffer management, the per-minibatch launch
// sequence of PPOAgent.Train(Trajectory) (PPOAgent.cs:147-172) and the double-precision
// Adam bias corrections (DenseLayer.cs:142-145: (float)(1 - Math.Pow(beta, t))).
// Every compute step runs in a HIP kernel; there is no CPU fallback.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/wk_api.h"
#include "wk_common.h"
#include "wk_kernels.h"
#include "wk_text.h"


static const char* kCriticDefault = "Input |64| (LeakyReLU) |1| Output";
static const char* kActorDefault = "Input |64| (LeakyReLU) |64| (LeakyReLU) |4| (TanH) Output";
static thread_local std::string g_create_error;
namespace wk {
void set_last_error(const std::string& msg) { g_create_error = msg; }
}  // namespace wk

// level 1: one event pair per rollout / returns / whole PPO update (cheap enough for a
// timed loop); level 2 adds one per gradient / reduce / all-reduce / Adam launch
enum ProfKind { PK_PHYS = 0, PK_GRAD, PK_REDUCE, PK_ADAM, PK_ALLRED, PK_RET, PK_UPDATE, PK_N };

struct wk_ctx {
  wk_config cfg;
  int grad_impl = -1;  // matrix-core gradient kernel (wk::GI_*; -1 = by minibatch size)
  int device = 0;
  int n = 0;
  uint64_t seed = 0;
  hipStream_t stream = nullptr;
  std::string err;
  wk::EnvParams P{};
  float lp_const = 0.0f;
  // env
  float* st = nullptr;        // walker records [n][NSTATE]
  float* dxoff = nullptr;     // [n]
  int32_t* mat = nullptr;     // [n]
  uint32_t* rng_t = nullptr;  // [n]
  // params
  float* W = nullptr; float* m = nullptr; float* v = nullptr; float* grad = nullptr;
  float* Wz = nullptr;        // W in the matrix-core operand order (wk_mfma_layout.h)
  int adam_t = 0;
  // trajectory [T][n]
  int T = 0, T_valid = 0;
  float *ts = nullptr, *ta = nullptr, *tlp = nullptr, *tr = nullptr, *tv = nullptr, *tret = nullptr, *tadv = nullptr;
  uint8_t* td = nullptr;
  bool returns_valid = false;
  // data collection (ConsoleRenderer.AddTotalEpisodeReward / AddCriticLoss / AddActorLoss)
  int collect = 1;
  uint32_t rollout_steps = 0;  // env-steps taken by wk_rollout so far (episode log clock)
  double* ep_acc = nullptr;       // [n] running episode reward
  int32_t* ep_len = nullptr;      // [n]
  void* ep_scratch = nullptr;     // [T][n] float2
  uint32_t* ep_rowcnt = nullptr;  // [T][tiles] episode counts per (row, 4,096-walker tile)
  uint64_t* ep_count = nullptr;   // device: records appended since the last drain
  wk::EpisodeRecDev* ep_log = nullptr;
  uint64_t ep_cap = 0;
  float* loss_log = nullptr;      // [loss_cap][2] (critic, actor) per PPO update
  uint64_t loss_count = 0, loss_cap = 0;
  // scratch
  float* partial = nullptr; size_t partial_floats = 0;
  void* scratch = nullptr; size_t scratch_bytes = 0;
  void* scratch2 = nullptr; size_t scratch2_bytes = 0;
  // scene props (wk_set_scene): descriptions, kernel constants, [n][pstride] state
  std::vector<wk_prop> scene_desc;
  wk::SceneDev scene{};
  float* props = nullptr;
  // wk_snapshot: one device block holding every snapshotted buffer, plus the host counters
  void* snap = nullptr; size_t snap_bytes = 0;
  int snap_adam_t = 0; uint32_t snap_rollout_steps = 0; uint64_t snap_loss_count = 0;
  bool snap_valid = false;
  unsigned long long* counts = nullptr;  // [WK_NEV] device (wk_count_events)
  int32_t* order = nullptr;       // [n] lane order of the split physics kernels (null: identity)
  uint32_t* order_cnt = nullptr;  // [order_cells(n)] episode-0 walkers per tile + swap count
  unsigned long long* pace = nullptr;  // [PACE_SLOTS] per-SIMD progress tags of the env-step kernels
  uint32_t pace_seq = 0;
  // comm
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  wk_host_allreduce_fn host_ar = nullptr;  // wk_comm_init_host: a caller-supplied all-reduce
  void* host_ar_user = nullptr;
  std::vector<float> host_ar_buf;
  // wk_comm_init_ipc: the one-shot exchange over peer-mapped memory (k_reduce_xch_adam)
  void* xch = nullptr;                 // this rank's exchange region (exported by IPC handle)
  std::vector<void*> xch_peers;        // peers' regions, opened from their handles
  wk::XchArgs xa{};                    // slab / flag pointers of every rank
  bool ipc = false;
  uint64_t xch_seq = 0;
  uint32_t* xch_err = nullptr;         // device word: a peer never published
  bool xch_uncached = false;           // the region is uncached device memory (else hipMalloc)
  uint64_t xch_timeout_ticks = 0;      // bounded peer wait (WK_XCH_TIMEOUT_S / wk_comm_set_timeout)
  uint64_t* xch_stamps = nullptr;      // wk_comm_xch_profile: [cap][blocks][XCH_POINTS] clock ring
  int xch_stamp_cap = 0;
  int64_t xch_stamp_launches = 0;      // launches stamped since the ring was (re)armed
  // the reference's per-body call shape (wk_take_actions / wk_object_update)
  std::vector<float> pend;             // [n][4] torques wk_take_actions stored for the next frame
  std::vector<uint8_t> pend_set;       // [n] walker given torques since the last frame
  int64_t frame_calls = 0, frame_len = 0;
  // profiling
  int prof = 0;  // profile level
  struct Ev { int kind; hipEvent_t a, b; int64_t units; };
  std::vector<Ev> pending;
  std::vector<hipEvent_t> pool;
  double prof_ms[PK_N] = {0};
  int64_t prof_cnt[PK_N] = {0};
  int64_t prof_units = 0;
};

// Every entry point binds the context's device for its duration: buffers are
// allocated and copied on c->device whatever the calling thread's current device is, and the
// caller's current device is restored afterwards.
struct DevGuard {
  int prev = -1;
  bool switched = false;
  explicit DevGuard(const wk_ctx* c) {
    if (c && hipGetDevice(&prev) == hipSuccess && prev != c->device)
      switched = hipSetDevice(c->device) == hipSuccess;
  }
  ~DevGuard() {
    if (switched) (void)hipSetDevice(prev);
  }
  DevGuard(const DevGuard&) = delete;
  DevGuard& operator=(const DevGuard&) = delete;
};

#define SETERR(ctx, ...)                                           \
  do {                                                             \
    char _b[512];                                                  \
    snprintf(_b, sizeof(_b), __VA_ARGS__);                         \
    (ctx)->err = _b;                                               \
  } while (0)

#define HIPCHK(ctx, call)                                                               \
  do {                                                                                  \
    hipError_t _e = (call);                                                             \
    if (_e != hipSuccess) {                                                             \
      SETERR(ctx, "%s failed: %s (%s:%d)", #call, hipGetErrorString(_e), __FILE__, __LINE__); \
      return WK_ERR_HIP;                                                                \
    }                                                                                   \
  } while (0)

static hipEvent_t ev_get(wk_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

struct ProfScope {
  wk_ctx* c; int kind; int64_t units; hipEvent_t a = nullptr, b = nullptr;
  bool on;
  ProfScope(wk_ctx* c_, int k, int64_t u = 0, int level = 1)
      : c(c_), kind(k), units(u), on(c_->prof >= level) {
    if (on) {
      a = ev_get(c); b = ev_get(c);
      if (a) (void)hipEventRecord(a, c->stream);
    }
  }
  ~ProfScope() {
    if (on && a && b) {
      (void)hipEventRecord(b, c->stream);
      c->pending.push_back({kind, a, b, units});
    }
  }
};

static void prof_drain(wk_ctx* c) {
  for (auto& e : c->pending) {
    float ms = 0.0f;
    if (hipEventSynchronize(e.b) == hipSuccess && hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
      c->prof_ms[e.kind] += ms;
      c->prof_cnt[e.kind] += 1;
      if (e.kind == PK_PHYS) c->prof_units += e.units;
    }
    c->pool.push_back(e.a);
    c->pool.push_back(e.b);
  }
  c->pending.clear();
}

static int ensure(wk_ctx* c, void** p, size_t* have, size_t need) {
  if (*have >= need) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *have = 0;
  HIPCHK(c, hipMalloc(p, need));
  *have = need;
  return 0;
}

extern "C" {

void wk_config_defaults(wk_config* c) {
  if (!c) return;
  memset(c, 0, sizeof(*c));
  c->GameSpeed = 1;
  c->Iterations = 50;
  c->MaxTimesteps = 1000;
  c->RoughFloor = 0;
  c->Epochs = 5;
  c->BatchSize = 64;
  c->UseGAE = 0;
  c->NormalizeAdvantages = 0;
  c->Gamma = 0.9f;
  c->Lambda = 0.95f;
  c->Epsilon = 0.3f;
  c->LogStandardDeviation = -1.0f;
  c->Alpha = 0.001f;
  c->Beta1 = 0.9f;
  c->Beta2 = 0.999f;
  c->AdamEpsilon = 1e-8f;
  c->CriticNeuralNetwork = nullptr;
  c->ActorNeuralNetwork = nullptr;
  c->DeltaTime = (float)(166667.0 / 10000000.0);
  c->Horizon = 64;
  c->Minibatch = 0;
  c->MinibatchGlobal = 0;
  c->EnvOffset = 0;
  c->RandomizeStart = 0;
  c->RandomizeMaterial = 0;
}

const char* wk_version(void) { return "wk 0.1 (gfx950)"; }

const char* wk_last_error(const wk_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

// ValidateHyperparameterValues (Hyperparameters.cs:189-217) + the kernel's fixed shapes
static int validate(const wk_config* c, std::string& why) {
  char b[256];
  auto bad = [&](const char* m) { why = m; return WK_ERR_CONFIG; };
  if (c->GameSpeed <= 0 || c->GameSpeed >= 10) return bad("Invalid game speed, should be in range 0<x<10");
  if (c->Iterations <= 0 || c->Iterations >= 200) return bad("Invalid iterations count, should be in range 0<x<200");
  if (c->MaxTimesteps <= 0) return bad("Invalid maximum time steps amount, should be in range x>0");
  if (c->Alpha <= 0 || c->Alpha >= 10) return bad("Invalid alpha value, should be in range 0<x<10");
  if (c->Beta1 <= 0 || c->Beta1 > 1) return bad("Invalid beta1 value, should be in range 0<x<1");
  if (c->Beta2 <= 0 || c->Beta2 > 1) return bad("Invalid beta2 value, should be in range 0<x<1");
  if (c->AdamEpsilon <= 0 || c->AdamEpsilon >= 1) return bad("Invalid Adam epsilon value, should be in range 0<x<1");
  if (c->Epochs <= 0 || c->Epochs >= 50) return bad("Invalid epochs value, should be in range 0<x<50");
  if (c->BatchSize <= 0 || c->BatchSize >= 1000) return bad("Invalid batch size value, should be in range 0<x<1000");
  if (c->Gamma <= 0 || c->Gamma > 1) return bad("Invalid gamma value, should be in range 0<x<1");
  if (c->Lambda <= 0 || c->Lambda > 1) return bad("Invalid lambda value, should be in range 0<x<1");
  if (c->Epsilon <= 0 || c->Epsilon > 1) return bad("Invalid epsilon value, should be in range 0<x<1");
  if (c->LogStandardDeviation <= -5 || c->LogStandardDeviation >= 5) return bad("Invalid log standard deviation value, should be in range -5<x<5");
  if (c->CriticNeuralNetwork && strcmp(c->CriticNeuralNetwork, kCriticDefault) != 0) {
    snprintf(b, sizeof(b), "critic network '%s' unsupported: the kernels implement '%s'", c->CriticNeuralNetwork, kCriticDefault);
    why = b;
    return WK_ERR_CONFIG;
  }
  if (c->ActorNeuralNetwork && strcmp(c->ActorNeuralNetwork, kActorDefault) != 0) {
    snprintf(b, sizeof(b), "actor network '%s' unsupported: the kernels implement '%s'", c->ActorNeuralNetwork, kActorDefault);
    why = b;
    return WK_ERR_CONFIG;
  }
  if (c->Horizon <= 0) return bad("Horizon must be > 0");
  if (c->Minibatch < 0) return bad("Minibatch must be >= 0");
  if (c->LanesPerWalker != 0 && c->LanesPerWalker != 1 && c->LanesPerWalker != 2 &&
      c->LanesPerWalker != 4 && c->LanesPerWalker != 16)
    return bad("LanesPerWalker must be 0 (auto), 1, 2, 4 or 16");
  return WK_OK;
}

// The rough floor's lane order (split mappings): the walkers sorted by start offset, so that a
// wave's walkers stand over the same stretch of terrain and its floor-segment loop resolves the
// union of fewer segments (Environment.cs:230-261: segments 240 px wide every 120 px; the
// offsets span 200 px).  Static -- a walker keeps its offset, and rough-floor episodes end
// within a few steps, so the flat floor's episode-0 partition has nothing to gather -- and
// recomputed whenever the offsets change (wk_create, wk_set_offsets, wk_checkpoint_load).
// Measured with the offsets themselves sorted by walker id (scripts/rough_dx_sort.py): rollout
// 110 -> 87.6 ms at 65,536 walkers (pair), 63.9 -> 50.4 ms at 8,192 (quad).  Bit-identical:
// every walker's arithmetic is keyed by its id (tests/test_gpu_order.py).
static hipError_t rough_order_upload(wk_ctx* c, const float* dx_host) {
  if (!c->order || !c->P.rough || !(c->P.lanes == 2 || c->P.lanes == 4)) return hipSuccess;
  std::vector<int32_t> ord(c->n);
  for (size_t e = 0; e < c->n; e++) ord[e] = (int32_t)e;
  std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) {
    return dx_host[a] < dx_host[b];  // (a NaN offset compares false: it keeps its relative place)
  });
  return hipMemcpy(c->order, ord.data(), sizeof(int32_t) * c->n, hipMemcpyHostToDevice);
}

int wk_create(const wk_config* cfg, int device, int n_env, uint64_t seed, wk_ctx** out) {
  if (!out) { g_create_error = "out is NULL"; return WK_ERR_ARG; }
  *out = nullptr;
  wk_config c;
  if (cfg) c = *cfg; else wk_config_defaults(&c);
  if (n_env <= 0) { g_create_error = "n_env must be > 0"; return WK_ERR_ARG; }
  std::string why;
  int vs = validate(&c, why);
  if (vs != WK_OK) { g_create_error = why; return vs; }
  int ndev = 0;
  hipError_t he = hipGetDeviceCount(&ndev);
  if (he != hipSuccess || ndev == 0) {
    g_create_error = std::string("no HIP device available: ") + hipGetErrorString(he);
    return WK_ERR_HIP;
  }
  if (device < 0 || device >= ndev) { g_create_error = "device index out of range"; return WK_ERR_ARG; }
  struct Restore {  // the caller's current device, as every other entry point leaves it
    int prev = -1;
    Restore() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~Restore() { if (prev >= 0) (void)hipSetDevice(prev); }
  } restore;
  wk_ctx* x = new wk_ctx();
  x->cfg = c;
  x->cfg.CriticNeuralNetwork = nullptr;
  x->cfg.ActorNeuralNetwork = nullptr;
  if (x->cfg.Minibatch == 0) x->cfg.Minibatch = x->cfg.BatchSize;
  x->device = device;
  x->n = n_env;
  x->seed = seed;
  x->T = c.Horizon;
  auto fail = [&](int code) {
    g_create_error = x->err;
    wk_destroy(x);
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) { x->err = "hipSetDevice failed"; return fail(WK_ERR_HIP); }
  // > 64 KiB dynamic LDS for the gradient kernels, set on this device (the attribute is
  // per device; wk_create is the only place, so launches never race on it)
  if (wk::configure_device_kernels() != hipSuccess) { x->err = "hipFuncSetAttribute failed"; return fail(WK_ERR_HIP); }
  x->grad_impl = wk::grad_impl_env();
  if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) {
    x->err = "hipStreamCreate failed";
    return fail(WK_ERR_HIP);
  }
  auto& P = x->P;
  P.n_env = n_env;
  P.iterations = c.Iterations;
  P.max_timesteps = c.MaxTimesteps;
  P.dt_frame = c.DeltaTime;
  P.dt_sub = c.DeltaTime / (float)c.Iterations;
  P.log_std = c.LogStandardDeviation;
  P.std_ = expf(c.LogStandardDeviation);
  P.seed = seed;
  P.env_offset = c.EnvOffset;
  // auto on the flat floor: the side-split pair mapping from 16,385 walkers up, the quad
  // mapping (two lanes per leg) below -- measured on one MI355X (scripts/side_times.sh,
  // rollout T = 16): 5.94 vs 7.56 ms at 8,192 and 16,384 walkers (one wave per SIMD at most,
  // where the split shortens each wave's chain), 11.7 vs 7.6 ms at 32,768 (two waves per
  // SIMD: issue-bound, the split's extra selects and exchanges cost more than they save).
  // Round 1: the pair mapping 32.1 ms at 8,192 walkers vs 83.2 ms for the 16-lane rows and
  // 104 ms one lane per walker (T = 64).  The rough floor takes the same choice: its segment
  // pairs run unsplit in every mapping, the leg-leg pairs keep the pair / quad split.
  P.lanes = c.LanesPerWalker ? c.LanesPerWalker : (n_env <= 16384 ? 4 : 2);
  P.rough = c.RoughFloor ? 1 : 0;
  // the quad mapping with fewer walkers per wave (the other lanes replay them) while one wave
  // per SIMD still holds every walker (1,024 SIMDs): each wave's divergent branches are the
  // union over fewer walkers -- rollout 5.72 -> 5.52 ms per 16 env-steps at 8,192 walkers
  // (eight per wave), physics only 5.95 -> 5.62.  Test hook (tests/test_gpu_parity.py, the
  // sparse mapping against the dense one): WK_QUAD_SPARSE=0 at wk_create, always sixteen
  {
    const char* sp = getenv("WK_QUAD_SPARSE");
    int wpw = 16;
    if (!(sp && sp[0] == '0'))
      while (wpw > 1 && (size_t)n_env <= (size_t)512 * wpw) wpw >>= 1;  // n / (wpw / 2) <= 1,024 waves
    P.wpw = wpw;
  }
  const float PI_F = 3.14159265358979323846f;
  x->lp_const = -logf(P.std_) - logf(sqrtf(2.0f * PI_F));

  const size_t n = (size_t)n_env, T = (size_t)x->T;
#define ALLOC(ptr, bytes)                                                   \
  if (hipMalloc((void**)&(ptr), (bytes)) != hipSuccess) {                  \
    x->err = "hipMalloc failed for " #ptr;                                  \
    return fail(WK_ERR_HIP);                                                \
  }
  ALLOC(x->st, sizeof(float) * wk::NSTATE * n);
  ALLOC(x->dxoff, sizeof(float) * n);
  ALLOC(x->mat, sizeof(int32_t) * n);
  ALLOC(x->rng_t, sizeof(uint32_t) * n);
  ALLOC(x->W, sizeof(float) * wk::NPARAM);
  ALLOC(x->Wz, sizeof(float) * wk::mfma_image_floats());
  ALLOC(x->m, sizeof(float) * wk::NPARAM);
  ALLOC(x->v, sizeof(float) * wk::NPARAM);
  ALLOC(x->grad, sizeof(float) * wk::SLAB);
  ALLOC(x->ts, sizeof(float) * 12 * n * T);
  ALLOC(x->ta, sizeof(float) * 4 * n * T);
  ALLOC(x->tlp, sizeof(float) * 4 * n * T);
  ALLOC(x->tr, sizeof(float) * n * T);
  ALLOC(x->tv, sizeof(float) * n * T);
  ALLOC(x->tret, sizeof(float) * n * T);
  ALLOC(x->tadv, sizeof(float) * n * T);
  ALLOC(x->td, n * T);
  x->ep_cap = (uint64_t)n * T;  // one rollout's worst case: every env-step ends an episode
  x->loss_cap = 1u << 16;
  ALLOC(x->ep_acc, sizeof(double) * n);
  ALLOC(x->ep_len, sizeof(int32_t) * n);
  ALLOC(x->ep_scratch, sizeof(float) * 2 * n * T);
  ALLOC(x->ep_rowcnt, sizeof(uint32_t) * wk::episode_count_cells((int)n, T));
  ALLOC(x->ep_count, sizeof(uint64_t));
  ALLOC(x->ep_log, sizeof(wk::EpisodeRecDev) * x->ep_cap);
  ALLOC(x->loss_log, sizeof(float) * 2 * x->loss_cap);
  // test hook (tests/test_gpu_order.py, the lane order against the identity order): WK_ORDER=0
  if (P.lanes == 2 || P.lanes == 4) {
    const char* o = getenv("WK_ORDER");
    if (!(o && o[0] == '0')) {
      ALLOC(x->order, sizeof(int32_t) * 3 * n);  // order, then the swap ranks' scratch
      ALLOC(x->order_cnt, sizeof(uint32_t) * wk::order_cells((int)n));
    }
  }
  // pacing of co-resident waves (k_env_side's pair mapping, k_env_step; the quad mapping runs one
  // wave per SIMD); test hook WK_PACE=0: without
  if (P.lanes != 4) {
    const char* o = getenv("WK_PACE");
    if (!(o && o[0] == '0')) {
      ALLOC(x->pace, sizeof(unsigned long long) * wk::PACE_SLOTS);
      if (hipMemset(x->pace, 0, sizeof(unsigned long long) * wk::PACE_SLOTS) != hipSuccess) {
        x->err = "pacing table clear failed";
        return fail(WK_ERR_HIP);
      }
    }
  }
#undef ALLOC
  // synthetic randomisation of the initial state (BASELINE.json config 2 / 5)
  std::vector<float> dx(n, 0.0f);
  std::vector<int32_t> mt(n, WK_MAT_CARPET);
  for (size_t e = 0; e < n; e++) {
    uint32_t gid = (uint32_t)(c.EnvOffset + (int)e);
    if (c.RandomizeStart) dx[e] = wk::env_offset(seed, gid);
    if (c.RandomizeMaterial) mt[e] = wk::env_material(seed, gid);
  }
  if (hipMemcpy(x->dxoff, dx.data(), sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(x->mat, mt.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(x->rng_t, 0, sizeof(uint32_t) * n) != hipSuccess ||
      hipMemset(x->m, 0, sizeof(float) * wk::NPARAM) != hipSuccess ||
      hipMemset(x->v, 0, sizeof(float) * wk::NPARAM) != hipSuccess ||
      hipMemset(x->td, 0, n * T) != hipSuccess ||
      hipMemset(x->ep_acc, 0, sizeof(double) * n) != hipSuccess ||
      hipMemset(x->ep_len, 0, sizeof(int32_t) * n) != hipSuccess ||
      hipMemset(x->ep_rowcnt, 0, sizeof(uint32_t) * wk::episode_count_cells((int)n, T)) != hipSuccess ||
      hipMemset(x->ep_count, 0, sizeof(uint64_t)) != hipSuccess) {
    x->err = "initial upload failed";
    return fail(WK_ERR_HIP);
  }
  if (rough_order_upload(x, dx.data()) != hipSuccess) {
    x->err = "lane order upload failed";
    return fail(WK_ERR_HIP);
  }
  if (wk::launch_env_init(P, x->st, x->dxoff, nullptr, 0, x->stream) != hipSuccess ||
      wk::launch_xavier(x->W, seed, x->stream) != hipSuccess ||
      wk::launch_swizzle(x->W, x->Wz, x->stream) != hipSuccess ||
      hipStreamSynchronize(x->stream) != hipSuccess) {
    x->err = "init kernels failed";
    return fail(WK_ERR_HIP);
  }
  *out = x;
  return WK_OK;
}

int wk_destroy(wk_ctx* c) {
  DevGuard dg_(c);
  if (!c) return WK_OK;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& e : c->pending) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
  for (auto e : c->pool) (void)hipEventDestroy(e);
  if (c->comm) ncclCommDestroy(c->comm);
  for (void* p : c->xch_peers)
    if (p) (void)hipIpcCloseMemHandle(p);
  if (c->xch) (void)hipFree(c->xch);
  if (c->xch_err) (void)hipFree(c->xch_err);
  if (c->xch_stamps) (void)hipFree(c->xch_stamps);
  void* bufs[] = {c->st, c->dxoff, c->mat, c->rng_t, c->W, c->Wz, c->m, c->v, c->grad, c->ts, c->ta,
                  c->tlp, c->tr, c->tv, c->tret, c->tadv, c->td, c->partial, c->scratch, c->scratch2,
                  c->ep_acc, c->ep_len, c->ep_scratch, c->ep_rowcnt, c->ep_count, c->ep_log,
                  c->loss_log, c->props, c->snap, c->counts, c->order, c->order_cnt, c->pace};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return WK_OK;
}

int wk_sync(wk_ctx* c) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}

int wk_num_envs(const wk_ctx* c) { return c ? c->n : 0; }

int wk_reset(wk_ctx* c, const uint8_t* mask) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  const uint8_t* dmask = nullptr;
  if (mask) {
    if (ensure(c, &c->scratch, &c->scratch_bytes, c->n)) return WK_ERR_HIP;
    HIPCHK(c, hipMemcpyAsync(c->scratch, mask, c->n, hipMemcpyHostToDevice, c->stream));
    dmask = (const uint8_t*)c->scratch;
  }
  // Environment.Reset re-creates the walker after the floor (post-reset body order)
  HIPCHK(c, wk::launch_env_init(c->P, c->st, c->dxoff, dmask, 1, c->stream));
  HIPCHK(c, wk::launch_episode_reset(c->n, dmask, c->ep_acc, c->ep_len, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}

int wk_set_materials(wk_ctx* c, const int32_t* mat_id) {
  DevGuard dg_(c);
  if (!c || !mat_id) return WK_ERR_ARG;
  for (int e = 0; e < c->n; e++)
    if (mat_id[e] < 0 || mat_id[e] > 7) { SETERR(c, "invalid material id %d at env %d", mat_id[e], e); return WK_ERR_ARG; }
  // the context's stream is non-blocking: queued rollouts read mat (also on auto-reset)
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(c->mat, mat_id, sizeof(int32_t) * c->n, hipMemcpyHostToDevice));
  return WK_OK;
}

int wk_set_offsets(wk_ctx* c, const float* dx) {
  DevGuard dg_(c);
  if (!c || !dx) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // queued kernels read dxoff on auto-reset
  HIPCHK(c, hipMemcpy(c->dxoff, dx, sizeof(float) * c->n, hipMemcpyHostToDevice));
  HIPCHK(c, rough_order_upload(c, dx));
  return WK_OK;
}

// the env-step kernel of the context's mapping; with scene props the one-lane scene kernel.
// The split mappings first order their lanes (WK_ORDER=0 keeps the identity order, for
// measurements).  Flat floor: episode-0 walkers in the last slots (wk_order.hip, before every
// launch; the quad mapping gains 2-3 %, the pair mapping 9.5 %).  Rough floor: the static order by
// start offset (rough_order_upload) -- not the episode-0 partition, which at one wave per SIMD
// gathered the few long-lived episode-0 walkers into one slowest wave (63 -> 74 ms per rollout
// at 8,192 walkers, scripts/r04_rough2.sh)
static hipError_t launch_physics(wk_ctx* c, int mode, wk::StepArgs& A) {
  if (c->scene.n_props > 0) {
    A.props = c->props;
    return wk::launch_env_scene(mode, c->P, A, c->scene, c->stream);
  }
  if (c->order && (c->P.lanes == 2 || c->P.lanes == 4)) {
    if (!c->P.rough) {
      const hipError_t e = wk::launch_walker_order(c->st, c->n, c->order_cnt, c->order, c->order + c->n,
                                                   c->stream);
      if (e != hipSuccess) return e;
    }
    A.order = c->order;
  }
  A.pace = c->pace;
  if (c->pace && ++c->pace_seq == 0) {  // (2^32 launches: the tags start over, so clear the slots)
    const hipError_t e = hipMemsetAsync(c->pace, 0, sizeof(unsigned long long) * wk::PACE_SLOTS, c->stream);
    if (e != hipSuccess) return e;
    c->pace_seq = 1;
  }
  A.pace_seq = c->pace_seq;
  return wk::launch_env_step(mode, c->P, A, c->stream);
}

static int step_impl(wk_ctx* c, const float* d_actions, int k, float* d_obs, float* d_rew,
                     uint8_t* d_done, uint32_t* d_fault, int mode, void* trace) {
  wk::StepArgs A{};
  A.st = c->st; A.dxoff = c->dxoff; A.mat = c->mat; A.rng_t = c->rng_t;
  A.actions = d_actions; A.obs_out = d_obs; A.rew_out = d_rew; A.done_out = d_done;
  A.fault_out = d_fault; A.W = c->W; A.Wz = c->Wz; A.lp_const = c->lp_const;
  A.traj_s = c->ts; A.traj_a = c->ta; A.traj_lp = c->tlp; A.traj_r = c->tr; A.traj_d = c->td;
  A.traj_v = c->tv; A.t0 = 0;
  A.trace = (wk::PairTraceDev*)trace;
  A.k_steps = k;
  ProfScope ps(c, PK_PHYS, (int64_t)k * c->n);
  HIPCHK(c, launch_physics(c, mode, A));
  return WK_OK;
}

int wk_step_device(wk_ctx* c, const float* d_actions, int k, float* d_obs, float* d_rew,
                   uint8_t* d_done, uint32_t* d_fault) {
  DevGuard dg_(c);
  if (!c || k <= 0) return WK_ERR_ARG;
  return step_impl(c, d_actions, k, d_obs, d_rew, d_done, d_fault, d_actions ? 0 : 2, nullptr);
}

int wk_step(wk_ctx* c, const float* actions, int k, float* obs, float* reward, uint8_t* done,
            uint32_t* fault) {
  DevGuard dg_(c);
  if (!c || k <= 0) return WK_ERR_ARG;
  const size_t n = c->n;
  const size_t b_act = actions ? sizeof(float) * 4 * n * k : 0;
  const size_t b_obs = sizeof(float) * 12 * n * k, b_rew = sizeof(float) * n * k, b_done = n * k;
  const size_t b_fault = sizeof(uint32_t) * n;
  const size_t total = b_act + b_obs + b_rew + b_done + b_fault + 64;
  if (ensure(c, &c->scratch2, &c->scratch2_bytes, total)) return WK_ERR_HIP;
  char* base = (char*)c->scratch2;
  float* d_act = actions ? (float*)base : nullptr;
  float* d_obs = (float*)(base + b_act);
  float* d_rew = (float*)(base + b_act + b_obs);
  uint32_t* d_fault = (uint32_t*)(base + b_act + b_obs + b_rew);
  uint8_t* d_done = (uint8_t*)(base + b_act + b_obs + b_rew + b_fault);
  if (actions) HIPCHK(c, hipMemcpyAsync(d_act, actions, b_act, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(d_fault, 0, b_fault, c->stream));
  int r = step_impl(c, d_act, k, obs ? d_obs : nullptr, reward ? d_rew : nullptr,
                    done ? d_done : nullptr, d_fault, actions ? 0 : 2, nullptr);
  if (r) return r;
  if (obs) HIPCHK(c, hipMemcpyAsync(obs, d_obs, b_obs, hipMemcpyDeviceToHost, c->stream));
  if (reward) HIPCHK(c, hipMemcpyAsync(reward, d_rew, b_rew, hipMemcpyDeviceToHost, c->stream));
  if (done) HIPCHK(c, hipMemcpyAsync(done, d_done, b_done, hipMemcpyDeviceToHost, c->stream));
  if (fault) HIPCHK(c, hipMemcpyAsync(fault, d_fault, b_fault, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}

// ---------------- the reference's per-body call shape ----------------
// Environment.StepObjects (Environment.cs:126-143) calls, per substep, Joint.Step on the 4 joints
// and IObject.Update (Objects/IObject.cs:9) on every body of the list: list_count * Iterations
// Update calls per frame.  The GPU resolves the whole frame in one launch, so the frame's FIRST
// Update call runs one env-step of every walker and the rest are counted no-ops; the torques are
// the ones Walker.TakeActions (Walker.cs:66-75) stored since the last frame, and a walker given
// none keeps its joints' current torques (Joint.SetTorque with the same value: no kick,
// Joint.cs:56-61) -- as in the reference, where nothing else changes them.
static int current_torques(wk_ctx* c, float* out /* [n][4] */) {
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy2D(out, sizeof(float) * 4, c->st + wk::S_TORQUE, sizeof(float) * wk::NSTATE,
                        sizeof(float) * 4, c->n, hipMemcpyDeviceToHost));
  return WK_OK;
}

int wk_take_actions(wk_ctx* c, int env, const float* actions) {
  if (!c || !actions || env < 0 || env >= c->n) return WK_ERR_ARG;
  if (c->pend_set.empty()) {
    c->pend.assign((size_t)c->n * 4, 0.0f);
    c->pend_set.assign((size_t)c->n, 0);
  }
  for (int j = 0; j < 4; j++) c->pend[(size_t)env * 4 + j] = actions[j];
  c->pend_set[env] = 1;
  return WK_OK;
}

int wk_object_update(wk_ctx* c, int list_count, float delta_time) {
  DevGuard dg_(c);
  if (!c || list_count <= 0 || !(delta_time >= 0.0f)) return WK_ERR_ARG;
  int stepped = 0;
  if (c->frame_calls == 0) {
    c->frame_len = (int64_t)list_count * c->cfg.Iterations;
    std::vector<float> a((size_t)c->n * 4);
    if (int r = current_torques(c, a.data())) return r;  // (the state as of this frame)
    for (size_t e = 0; e < c->pend_set.size(); e++)
      if (c->pend_set[e])
        for (int j = 0; j < 4; j++) a[e * 4 + j] = c->pend[e * 4 + j];
    std::fill(c->pend_set.begin(), c->pend_set.end(), (uint8_t)0);
    if (int r = wk_step(c, a.data(), 1, nullptr, nullptr, nullptr, nullptr)) return r;
    stepped = 1;
  }
  if (++c->frame_calls >= c->frame_len) c->frame_calls = 0;
  return stepped;
}

int wk_joint_step(wk_ctx* c) { return c ? WK_OK : WK_ERR_ARG; }

int wk_body_order(wk_ctx* c, int env, int* parts, int* count) {
  DevGuard dg_(c);
  if (!c || !parts || !count || env < 0 || env >= c->n) return WK_ERR_ARG;
  float post = 0.0f;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(&post, c->st + (size_t)env * wk::NSTATE + wk::S_POSTRESET, sizeof(float),
                      hipMemcpyDeviceToHost));
  const int nfloor = c->P.rough ? 10 : 1;  // the floor body ids are 5 .. 5 + nfloor - 1
  int k = 0;
  if (post != 0.0f)
    for (int f = 0; f < nfloor; f++) parts[k++] = 5 + f;
  for (int b = 0; b < 5; b++) parts[k++] = b;  // CreateBodies' order: LLL, LLU, Body, RLL, RLU
  if (post == 0.0f)
    for (int f = 0; f < nfloor; f++) parts[k++] = 5 + f;
  *count = k;
  return WK_OK;
}

int wk_step_sampled(wk_ctx* c, int k, float* states, float* actions, float* logp, float* values,
                    float* reward, uint8_t* done, float* next_obs, uint32_t* fault,
                    float* position) {
  DevGuard dg_(c);
  if (!c || k <= 0) return WK_ERR_ARG;
  const size_t n = c->n, kn = (size_t)k * n;
  // the policy-sampling kernel with RECORD rows pointed at scratch (the device trajectory
  // buffer of wk_rollout is not touched)
  const size_t b12 = sizeof(float) * 12 * kn, b4 = sizeof(float) * 4 * kn, b1 = sizeof(float) * kn;
  const size_t b_fault = sizeof(uint32_t) * n;
  const size_t b_pos = sizeof(float) * 2 * kn;
  const size_t total = 2 * b12 + 2 * b4 + 2 * b1 + kn + b_fault + b_pos + 9 * 64;
  if (ensure(c, &c->scratch2, &c->scratch2_bytes, total)) return WK_ERR_HIP;
  char* p = (char*)c->scratch2;
  auto take = [&](size_t bytes) { char* r = p; p += (bytes + 63) & ~(size_t)63; return r; };
  float* d_s = (float*)take(b12);
  float* d_a = (float*)take(b4);
  float* d_lp = (float*)take(b4);
  float* d_v = (float*)take(b1);
  float* d_r = (float*)take(b1);
  float* d_o = (float*)take(b12);
  uint32_t* d_f = (uint32_t*)take(b_fault);
  float* d_pos = (float*)take(b_pos);
  uint8_t* d_d = (uint8_t*)take(kn);
  HIPCHK(c, hipMemsetAsync(d_f, 0, b_fault, c->stream));
  wk::StepArgs A{};
  A.st = c->st; A.dxoff = c->dxoff; A.mat = c->mat; A.rng_t = c->rng_t;
  A.obs_out = next_obs ? d_o : nullptr; A.fault_out = d_f;
  A.pos_out = position ? d_pos : nullptr;
  A.W = c->W; A.Wz = c->Wz; A.lp_const = c->lp_const;
  A.traj_s = d_s; A.traj_a = d_a; A.traj_lp = d_lp; A.traj_r = d_r; A.traj_d = d_d; A.traj_v = d_v;
  A.t0 = 0; A.k_steps = k;
  {
    ProfScope ps(c, PK_PHYS, (int64_t)kn);
    HIPCHK(c, launch_physics(c, 3, A));
  }
  if (states) HIPCHK(c, hipMemcpyAsync(states, d_s, b12, hipMemcpyDeviceToHost, c->stream));
  if (actions) HIPCHK(c, hipMemcpyAsync(actions, d_a, b4, hipMemcpyDeviceToHost, c->stream));
  if (logp) HIPCHK(c, hipMemcpyAsync(logp, d_lp, b4, hipMemcpyDeviceToHost, c->stream));
  if (values) HIPCHK(c, hipMemcpyAsync(values, d_v, b1, hipMemcpyDeviceToHost, c->stream));
  if (reward) HIPCHK(c, hipMemcpyAsync(reward, d_r, b1, hipMemcpyDeviceToHost, c->stream));
  if (done) HIPCHK(c, hipMemcpyAsync(done, d_d, kn, hipMemcpyDeviceToHost, c->stream));
  if (next_obs) HIPCHK(c, hipMemcpyAsync(next_obs, d_o, b12, hipMemcpyDeviceToHost, c->stream));
  if (fault) HIPCHK(c, hipMemcpyAsync(fault, d_f, b_fault, hipMemcpyDeviceToHost, c->stream));
  if (position) HIPCHK(c, hipMemcpyAsync(position, d_pos, b_pos, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}

int wk_step_traced(wk_ctx* c, const float* actions, wk_pair_trace* trace) {
  DevGuard dg_(c);
  if (!c || !actions || !trace) return WK_ERR_ARG;
  static_assert(sizeof(wk_pair_trace) == sizeof(wk::PairTraceDev), "trace layout");
  const size_t n = c->n;
  const size_t b_act = sizeof(float) * 4 * n;
  const size_t b_tr = sizeof(wk_pair_trace) * n * c->cfg.Iterations;
  if (ensure(c, &c->scratch2, &c->scratch2_bytes, b_act + b_tr + 64)) return WK_ERR_HIP;
  float* d_act = (float*)c->scratch2;
  void* d_tr = (char*)c->scratch2 + ((b_act + 63) / 64) * 64;
  HIPCHK(c, hipMemcpyAsync(d_act, actions, b_act, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(d_tr, 0, b_tr, c->stream));
  int r = step_impl(c, d_act, 1, nullptr, nullptr, nullptr, nullptr, 1, d_tr);
  if (r) return r;
  HIPCHK(c, hipMemcpyAsync(trace, d_tr, b_tr, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}

int wk_get_obs(wk_ctx* c, float* obs) {
  DevGuard dg_(c);
  if (!c || !obs) return WK_ERR_ARG;
  if (ensure(c, &c->scratch, &c->scratch_bytes, sizeof(float) * 12 * c->n)) return WK_ERR_HIP;
  HIPCHK(c, wk::launch_get_obs(c->P, c->st, (float*)c->scratch, c->stream));
  HIPCHK(c, hipMemcpyAsync(obs, c->scratch, sizeof(float) * 12 * c->n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}

// the device state is [n_env][WK_STATE_FLOATS] (one 448-B record per walker), the same
// layout as the canonical dump, so these are plain copies
int wk_get_state(wk_ctx* c, float* state) {
  DevGuard dg_(c);
  if (!c || !state) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(state, c->st, sizeof(float) * wk::NSTATE * c->n, hipMemcpyDeviceToHost));
  return WK_OK;
}

// the rigid-pole shortcut (pole_own_minmax, csrc/wk_device.h) projects a walker
// pole onto its own edge axes with min / max over fixed vertex groups, which equals the reference's
// min / max over all six vertices (SATCollision.cs:63-76 ProjectPoints) only while the pole keeps
// its template shape (Pole.FromSize, Pole.cs:18-34): every vertex left out of a group lies >= 7.5
// px beyond the group's extreme.  A state from outside (wk_set_state, wk_checkpoint_load) must keep
// that margin; the kernel's own states do (rigid motion, << 1 px of rounding drift).
// Required margin: POLE_MARGIN_PX, above the worst-case drift bound (~3 px over 50,000 substeps).
// Poles with a non-finite coordinate are not checked (the NaN path is exact).
static constexpr double POLE_MARGIN_PX = 3.5;
static const int kPoleGroups[6][2][3] = {  // per own edge: {min group, max group}, -1 = unused
    {{0, 1, 2}, {3, 4, 5}}, {{0, 1, 2}, {3, 4, 5}}, {{2, 3, -1}, {5, 0, -1}},
    {{3, 4, 5}, {0, 1, 2}}, {{3, 4, 5}, {0, 1, 2}}, {{5, 0, -1}, {2, 3, -1}}};
// the smallest margin of one pole (record floats x0 y0 .. x5 y5), or +inf if non-finite
static double pole_margin(const float* v) {
  for (int i = 0; i < 12; i++)
    if (!std::isfinite(v[i])) return INFINITY;
  double worst = INFINITY;
  for (int e = 0; e < 6; e++) {
    const int e1 = (e + 1) % 6;
    const double ex = (double)v[2 * e1] - v[2 * e], ey = (double)v[2 * e1 + 1] - v[2 * e + 1];
    const double len = std::sqrt(ex * ex + ey * ey);
    if (!(len > 0.0)) return -INFINITY;  // a zero edge: not a rigid template pole
    const double ax = -ey / len, ay = ex / len;
    double p[6];
    for (int i = 0; i < 6; i++) p[i] = ax * v[2 * i] + ay * v[2 * i + 1];
    bool inmin[6] = {}, inmax[6] = {};
    double gmin = INFINITY, gmax = -INFINITY;
    for (int k = 0; k < 3; k++) {
      const int a = kPoleGroups[e][0][k], b = kPoleGroups[e][1][k];
      if (a >= 0) { inmin[a] = true; gmin = std::min(gmin, p[a]); }
      if (b >= 0) { inmax[b] = true; gmax = std::max(gmax, p[b]); }
    }
    for (int i = 0; i < 6; i++) {
      if (!inmin[i]) worst = std::min(worst, p[i] - gmin);
      if (!inmax[i]) worst = std::min(worst, gmax - p[i]);
    }
  }
  return worst;
}

int wk_check_state(const float* state, int n_env, int* bad_env, int* bad_body) {
  if (!state || n_env <= 0) return WK_ERR_ARG;
  static const int poles[4] = {wk::LLL, wk::LLU, wk::RLL, wk::RLU};
  for (int e = 0; e < n_env; e++)
    for (int b : poles)
      if (!(pole_margin(state + (size_t)e * wk::NSTATE + (size_t)b * wk::BSTRIDE) >= POLE_MARGIN_PX)) {
        if (bad_env) *bad_env = e;
        if (bad_body) *bad_body = b;
        return WK_ERR_ARG;
      }
  if (bad_env) *bad_env = -1;
  if (bad_body) *bad_body = -1;
  return WK_OK;
}

static int check_state_or_fail(wk_ctx* c, const float* state) {
  int e = -1, b = -1;
  if (wk_check_state(state, c->n, &e, &b) != WK_OK) {
    SETERR(c, "walker %d body %d is not a rigid walker pole (a vertex group closer than %.1f px to "
           "the excluded vertices on one of its own edge axes: deformed or reordered vertices); "
           "the state is refused", e, b, POLE_MARGIN_PX);
    return WK_ERR_ARG;
  }
  return WK_OK;
}

int wk_set_state(wk_ctx* c, const float* state) {
  DevGuard dg_(c);
  if (!c || !state) return WK_ERR_ARG;
  if (int r = check_state_or_fail(c, state)) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(c->st, state, sizeof(float) * wk::NSTATE * c->n, hipMemcpyHostToDevice));
  return WK_OK;
}

int wk_get_body_view(wk_ctx* c, int env, int body, wk_body_view* o) {
  DevGuard dg_(c);
  if (!c || !o || env < 0 || env >= c->n || body < 0 || body >= (c->P.rough ? 15 : 6)) return WK_ERR_ARG;
  memset(o, 0, sizeof(*o));
  if (c->P.rough && body >= 5) {  // rough-floor segment body - 5 (Environment.cs:230-261)
    const int k = body - 5;
    const uint32_t gid = (uint32_t)(c->cfg.EnvOffset + env);
    const float x = -50.0f + 120.0f * (float)k;
    const float yp = 800.0f + (float)wk::terrain_draw(c->seed, gid, k);
    const float y = 800.0f + (float)wk::terrain_draw(c->seed, gid, k + 1);
    const float v[4][2] = {{x, 1050.0f}, {k == 0 ? x : x - 120.0f, yp}, {x, y}, {x + 120.0f, 1050.0f}};
    float sx = 0.0f, sy = 0.0f;
    o->n_vertices = 4;
    for (int i = 0; i < 4; i++) {
      o->vertices[i][0] = v[i][0]; o->vertices[i][1] = v[i][1];
      sx += v[i][0]; sy += v[i][1];
    }
    o->centroid[0] = sx * 0.25f; o->centroid[1] = sy * 0.25f;  // FindCentroid: sum * (1/4)
    o->is_static = 1;
    return WK_OK;
  }
  if (body == 5) {  // the static Metal floor (Environment.cs:219-223)
    const float fl[4][2] = {{-50, 1050}, {-50, 900}, {1050, 900}, {1050, 1050}};
    o->n_vertices = 4;
    for (int i = 0; i < 4; i++) { o->vertices[i][0] = fl[i][0]; o->vertices[i][1] = fl[i][1]; }
    o->centroid[0] = 500.0f; o->centroid[1] = 975.0f;
    o->is_static = 1;
    return WK_OK;
  }
  float f[wk::BSTRIDE];
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(f, c->st + (size_t)env * wk::NSTATE + (size_t)body * wk::BSTRIDE,
                      sizeof(f), hipMemcpyDeviceToHost));
  o->n_vertices = body == wk::BODY ? 5 : 6;
  for (int i = 0; i < o->n_vertices; i++) { o->vertices[i][0] = f[2 * i]; o->vertices[i][1] = f[2 * i + 1]; }
  o->centroid[0] = f[wk::F_CX]; o->centroid[1] = f[wk::F_CY];
  o->linear_velocity[0] = f[wk::F_VX]; o->linear_velocity[1] = f[wk::F_VY];
  o->angular_velocity = f[wk::F_W];
  o->angle = f[wk::F_TH];
  o->collided = f[wk::F_COL] != 0.0f;
  return WK_OK;
}

// ---------------- scene props (wk_scene.inc) ----------------
// <Shape>.FromSize (Square.cs:18-31, Triangle.cs:18-30, Hexagon.cs:18-33) then
// Skeleton.SmoothCorners (Skeleton.cs:33-53) in host fp32 (built with -ffp-contract=off,
// the same IEEE ops as the oracle); returns the vertex count or -1
static int prop_vertices(const wk_prop& p, int smooth, float* xs, float* ys) {
  const float cx = p.cx, cy = p.cy, adj = (float)0.5 * p.size;
  int n;
  if (p.shape == WK_SHAPE_SQUARE) {
    const float vx[4] = {cx + adj, cx - adj, cx - adj, cx + adj};
    const float vy[4] = {cy + adj, cy + adj, cy - adj, cy - adj};
    n = 4;
    for (int i = 0; i < n; i++) { xs[i] = vx[i]; ys[i] = vy[i]; }
  } else if (p.shape == WK_SHAPE_TRIANGLE) {
    const float vx[3] = {cx, cx - adj, cx + adj};
    const float vy[3] = {cy + adj, cy - adj, cy - adj};
    n = 3;
    for (int i = 0; i < n; i++) { xs[i] = vx[i]; ys[i] = vy[i]; }
  } else if (p.shape == WK_SHAPE_HEXAGON) {
    const float h = adj * 0.5f;
    const float vx[6] = {cx + h, cx - h, cx - adj, cx - h, cx + h, cx + adj};
    const float vy[6] = {cy + adj, cy + adj, cy, cy - adj, cy - adj, cy};
    n = 6;
    for (int i = 0; i < n; i++) { xs[i] = vx[i]; ys[i] = vy[i]; }
  } else {
    return -1;
  }
  for (int it = 0; it < smooth; it++) {
    if (2 * n > WK_PROP_MAXV) return -1;
    float nx[WK_PROP_MAXV], ny[WK_PROP_MAXV];
    for (int j = 0; j < n; j++) {
      const int a = (j + 1) % n, b = (j + n - 1) % n;  // ContactPoints.Mod(j - 1, n)
      const float abx = (xs[a] - xs[j]) * 0.2f, aby = (ys[a] - ys[j]) * 0.2f;
      const float acx = (xs[b] - xs[j]) * 0.2f, acy = (ys[b] - ys[j]) * 0.2f;
      nx[2 * j] = xs[j] + acx; ny[2 * j] = ys[j] + acy;
      nx[2 * j + 1] = xs[j] + abx; ny[2 * j + 1] = ys[j] + aby;
    }
    n *= 2;
    for (int i = 0; i < n; i++) { xs[i] = nx[i]; ys[i] = ny[i]; }
  }
  return n;
}

static const float kMatProps[8][3] = {  // Materials/*.cs: inverse mass, restitution, friction
    {5.0f, 0.3f, 0.8f}, {11.0f, 0.3f, 0.0f}, {11.0f, 0.7f, 0.5f}, {15.0f, 0.3f, 1.0f},
    {20.0f, 0.3f, 0.01f}, {1.0f, 0.3f, 0.1f}, {0.01f, 0.1f, 0.2f}, {11.0f, 1.0f, 1.0f}};

int wk_set_scene(wk_ctx* c, const wk_prop* props, int n_props) {
  DevGuard dg_(c);
  if (!c || n_props < 0 || (n_props > 0 && !props)) return WK_ERR_ARG;
  if (n_props > WK_MAX_PROPS) { SETERR(c, "at most %d scene props", (int)WK_MAX_PROPS); return WK_ERR_ARG; }
  if (n_props > 0 && c->cfg.LanesPerWalker > 1) {
    SETERR(c, "scene props run on the one-lane mapping (LanesPerWalker 0 or 1)");
    return WK_ERR_CONFIG;
  }
  wk::SceneDev S{};
  std::vector<float> rec;
  for (int k = 0; k < n_props; k++) {
    const wk_prop& p = props[k];
    const float fin[8] = {p.cx, p.cy, p.size, p.vx, p.vy, p.w, p.ax, p.ay};
    for (float f : fin)
      if (!std::isfinite(f)) { SETERR(c, "prop %d: non-finite parameter", k); return WK_ERR_ARG; }
    if (p.material < 0 || p.material > 7 || p.smooth < 0 || !(p.size > 0.0f)) {
      SETERR(c, "prop %d: invalid material, smooth count or size", k);
      return WK_ERR_ARG;
    }
    float xs[WK_PROP_MAXV], ys[WK_PROP_MAXV], bx[WK_PROP_MAXV], by[WK_PROP_MAXV];
    const int nv = prop_vertices(p, p.smooth, xs, ys);
    if (nv < 0) { SETERR(c, "prop %d: unknown shape or more than %d vertices", k, (int)WK_PROP_MAXV); return WK_ERR_ARG; }
    if ((int)rec.size() + 2 * nv + 6 > wk::SCENE_FIELDS) {
      SETERR(c, "scene props exceed %d vertices in total", (int)WK_SCENE_MAX_VERTS);
      return WK_ERR_ARG;
    }
    int total = nv;
    for (int j = 0; j < k; j++) total += S.nv[j];
    if (total > WK_SCENE_MAX_VERTS) { SETERR(c, "scene props exceed %d vertices in total", (int)WK_SCENE_MAX_VERTS); return WK_ERR_ARG; }
    // Skeleton.AddVectors -> FindCentroid of the FromSize vertices (before SmoothCorners)
    const int nb = prop_vertices(p, 0, bx, by);
    float sx = 0.0f, sy = 0.0f;
    for (int i = 0; i < nb; i++) { sx = sx + bx[i]; sy = sy + by[i]; }
    const float inv = 1.0f / (float)nb;
    S.nv[k] = nv;
    S.off[k] = (int)rec.size();
    S.stat[k] = p.is_static ? 1 : 0;
    // RigidBody ctor (RigidBody.cs:36-50)
    S.im[k] = p.is_static ? 0.0f : kMatProps[p.material][0];
    S.ii[k] = p.is_static ? 0.0f : 0.001f * kMatProps[p.material][0];
    S.e[k] = kMatProps[p.material][1];
    S.mu[k] = kMatProps[p.material][2];
    S.adx[k] = p.ax * c->P.dt_sub;  // _acceleration * deltaTime (StepLinearVelocity)
    S.ady[k] = p.ay * c->P.dt_sub;
    for (int i = 0; i < nv; i++) rec.push_back(xs[i]);
    for (int i = 0; i < nv; i++) rec.push_back(ys[i]);
    const float tail[6] = {sx * inv, sy * inv, p.vx, p.vy, p.w, 0.0f};
    for (float f : tail) rec.push_back(f);
  }
  S.n_props = n_props;
  S.pstride = (int)rec.size();
  float* dev = nullptr;
  if (n_props > 0) {
    std::vector<float> all((size_t)c->n * rec.size());
    for (int e = 0; e < c->n; e++) memcpy(all.data() + (size_t)e * rec.size(), rec.data(), sizeof(float) * rec.size());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMalloc(&dev, sizeof(float) * all.size()));
    if (hipMemcpy(dev, all.data(), sizeof(float) * all.size(), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(dev);
      SETERR(c, "scene upload failed");
      return WK_ERR_HIP;
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->props) (void)hipFree(c->props);
  c->props = dev;
  c->scene = S;
  c->snap_valid = false;  // the snapshot's layout no longer matches
  c->scene_desc.assign(props, props + n_props);
  return WK_OK;
}

int wk_get_prop_view(wk_ctx* c, int env, int k, wk_prop_view* o) {
  DevGuard dg_(c);
  if (!c || !o || env < 0 || env >= c->n || k < 0 || k >= c->scene.n_props) return WK_ERR_ARG;
  memset(o, 0, sizeof(*o));
  const int nv = c->scene.nv[k];
  std::vector<float> f(2 * nv + 6);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(f.data(), c->props + (size_t)env * c->scene.pstride + c->scene.off[k],
                      sizeof(float) * f.size(), hipMemcpyDeviceToHost));
  o->n_vertices = nv;
  for (int i = 0; i < nv; i++) { o->vertices[i][0] = f[i]; o->vertices[i][1] = f[nv + i]; }
  o->centroid[0] = f[2 * nv]; o->centroid[1] = f[2 * nv + 1];
  o->linear_velocity[0] = f[2 * nv + 2]; o->linear_velocity[1] = f[2 * nv + 3];
  o->angular_velocity = f[2 * nv + 4];
  o->angle = f[2 * nv + 5];
  o->is_static = c->scene.stat[k];
  return WK_OK;
}

int wk_get_weights(wk_ctx* c, float* p) {
  DevGuard dg_(c);
  if (!c || !p) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(p, c->W, sizeof(float) * wk::NPARAM, hipMemcpyDeviceToHost));
  return WK_OK;
}
int wk_set_weights(wk_ctx* c, const float* p) {
  DevGuard dg_(c);
  if (!c || !p) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(c->W, p, sizeof(float) * wk::NPARAM, hipMemcpyHostToDevice));
  HIPCHK(c, wk::launch_swizzle(c->W, c->Wz, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}
int wk_get_adam(wk_ctx* c, float* m, float* v, int* t) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (m) HIPCHK(c, hipMemcpy(m, c->m, sizeof(float) * wk::NPARAM, hipMemcpyDeviceToHost));
  if (v) HIPCHK(c, hipMemcpy(v, c->v, sizeof(float) * wk::NPARAM, hipMemcpyDeviceToHost));
  if (t) *t = c->adam_t;
  return WK_OK;
}
int wk_set_adam(wk_ctx* c, const float* m, const float* v, int t) {
  DevGuard dg_(c);
  if (!c || t < 0) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (m) HIPCHK(c, hipMemcpy(c->m, m, sizeof(float) * wk::NPARAM, hipMemcpyHostToDevice));
  if (v) HIPCHK(c, hipMemcpy(c->v, v, sizeof(float) * wk::NPARAM, hipMemcpyHostToDevice));
  c->adam_t = t;
  return WK_OK;
}

static int policy_impl(wk_ctx* c, int n, const float* obs, const int32_t* ids, const uint32_t* steps,
                       float* mean, float* act, float* logp, float* v) {
  const size_t b_obs = sizeof(float) * 12 * n, b4 = sizeof(float) * 4 * n, b1 = sizeof(float) * n;
  const size_t total = b_obs + 3 * b4 + 2 * b1 + 2 * sizeof(int32_t) * n + 256;
  if (ensure(c, &c->scratch2, &c->scratch2_bytes, total)) return WK_ERR_HIP;
  char* p = (char*)c->scratch2;
  float* d_obs = (float*)p; p += b_obs;
  float* d_mean = (float*)p; p += b4;
  float* d_act = (float*)p; p += b4;
  float* d_lp = (float*)p; p += b4;
  float* d_v = (float*)p; p += b1;
  int32_t* d_ids = (int32_t*)p; p += sizeof(int32_t) * n;
  uint32_t* d_steps = (uint32_t*)p;
  HIPCHK(c, hipMemcpyAsync(d_obs, obs, b_obs, hipMemcpyHostToDevice, c->stream));
  if (ids) HIPCHK(c, hipMemcpyAsync(d_ids, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  if (steps) HIPCHK(c, hipMemcpyAsync(d_steps, steps, sizeof(uint32_t) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, wk::launch_policy(c->P, c->W, c->lp_const, n, d_obs, ids ? d_ids : nullptr,
                              steps ? d_steps : nullptr, v ? nullptr : d_mean, v ? nullptr : d_act,
                              v ? nullptr : d_lp, v ? d_v : nullptr, c->stream));
  if (v) {
    HIPCHK(c, hipMemcpyAsync(v, d_v, b1, hipMemcpyDeviceToHost, c->stream));
  } else {
    if (mean) HIPCHK(c, hipMemcpyAsync(mean, d_mean, b4, hipMemcpyDeviceToHost, c->stream));
    if (act) HIPCHK(c, hipMemcpyAsync(act, d_act, b4, hipMemcpyDeviceToHost, c->stream));
    if (logp) HIPCHK(c, hipMemcpyAsync(logp, d_lp, b4, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}

int wk_policy_sample(wk_ctx* c, int n, const float* obs, const int32_t* env_ids,
                     const uint32_t* steps, float* mean, float* act, float* logp) {
  DevGuard dg_(c);
  if (!c || n <= 0 || !obs) return WK_ERR_ARG;
  return policy_impl(c, n, obs, env_ids, steps, mean, act, logp, nullptr);
}

int wk_value(wk_ctx* c, int n, const float* obs, float* v) {
  DevGuard dg_(c);
  if (!c || n <= 0 || !obs || !v) return WK_ERR_ARG;
  return policy_impl(c, n, obs, nullptr, nullptr, nullptr, nullptr, nullptr, v);
}

static int returns_impl(wk_ctx* c) {
  {
    ProfScope ps(c, PK_RET);
    HIPCHK(c, wk::launch_returns(c->n, c->T_valid, c->cfg.UseGAE, c->cfg.Gamma, c->cfg.Lambda,
                                 c->tr, c->tv, c->td, c->tret, c->tadv, c->stream));
  }
  if (c->cfg.NormalizeAdvantages)
    HIPCHK(c, wk::launch_normalize(c->tadv, c->n * c->T_valid, c->cfg.Epsilon, c->stream));
  c->returns_valid = true;
  return WK_OK;
}

int wk_rollout(wk_ctx* c, int horizon) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  if (horizon <= 0) horizon = c->T;
  if (horizon > c->T) { SETERR(c, "horizon %d exceeds the configured Horizon %d", horizon, c->T); return WK_ERR_ARG; }
  wk::StepArgs A{};
  A.st = c->st; A.dxoff = c->dxoff; A.mat = c->mat; A.rng_t = c->rng_t;
  A.W = c->W; A.Wz = c->Wz; A.lp_const = c->lp_const;
  A.traj_s = c->ts; A.traj_a = c->ta; A.traj_lp = c->tlp; A.traj_r = c->tr; A.traj_d = c->td;
  A.traj_v = c->tv; A.t0 = 0; A.k_steps = horizon;
  {
    ProfScope ps(c, PK_PHYS, (int64_t)horizon * c->n);
    HIPCHK(c, launch_physics(c, 3, A));
  }
  c->T_valid = horizon;
  if (c->collect) {
    wk::EpisodeArgs e{c->n, horizon, c->cfg.EnvOffset, c->rollout_steps, c->tr, c->td, c->ep_acc,
                      c->ep_len, (float2*)c->ep_scratch, c->ep_rowcnt, c->ep_count, c->ep_cap,
                      c->ep_log};
    ProfScope ps(c, PK_RET);
    HIPCHK(c, wk::launch_episode_log(e, c->stream));
  }
  c->rollout_steps += (uint32_t)horizon;
  return returns_impl(c);
}

int wk_compute_returns(wk_ctx* c) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  if (c->T_valid <= 0) { SETERR(c, "no trajectory recorded"); return WK_ERR_STATE; }
  return returns_impl(c);
}

int wk_rollout_stats_get(wk_ctx* c, wk_rollout_stats* o) {
  DevGuard dg_(c);
  if (!c || !o) return WK_ERR_ARG;
  memset(o, 0, sizeof(*o));
  const size_t cnt = (size_t)c->n * c->T_valid;
  std::vector<float> r(cnt);
  std::vector<uint8_t> d(cnt);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (cnt) {
    HIPCHK(c, hipMemcpy(r.data(), c->tr, sizeof(float) * cnt, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(d.data(), c->td, cnt, hipMemcpyDeviceToHost));
  }
  for (size_t i = 0; i < cnt; i++) { o->reward_sum += r[i]; o->episodes += d[i]; }
  o->env_steps = (int64_t)cnt;
  return WK_OK;
}

int wk_get_trajectory(wk_ctx* c, float* s, float* a, float* lp, float* r, uint8_t* d, float* v,
                      float* ret, float* adv) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  const size_t cnt = (size_t)c->n * c->T_valid;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (s) HIPCHK(c, hipMemcpy(s, c->ts, sizeof(float) * 12 * cnt, hipMemcpyDeviceToHost));
  if (a) HIPCHK(c, hipMemcpy(a, c->ta, sizeof(float) * 4 * cnt, hipMemcpyDeviceToHost));
  if (lp) HIPCHK(c, hipMemcpy(lp, c->tlp, sizeof(float) * 4 * cnt, hipMemcpyDeviceToHost));
  if (r) HIPCHK(c, hipMemcpy(r, c->tr, sizeof(float) * cnt, hipMemcpyDeviceToHost));
  if (d) HIPCHK(c, hipMemcpy(d, c->td, cnt, hipMemcpyDeviceToHost));
  if (v) HIPCHK(c, hipMemcpy(v, c->tv, sizeof(float) * cnt, hipMemcpyDeviceToHost));
  if (ret) HIPCHK(c, hipMemcpy(ret, c->tret, sizeof(float) * cnt, hipMemcpyDeviceToHost));
  if (adv) HIPCHK(c, hipMemcpy(adv, c->tadv, sizeof(float) * cnt, hipMemcpyDeviceToHost));
  return WK_OK;
}

int wk_set_trajectory(wk_ctx* c, int horizon, const float* s, const float* a, const float* lp,
                      const float* r, const uint8_t* d, const float* v) {
  DevGuard dg_(c);
  if (!c || horizon <= 0 || horizon > c->T || !s || !a || !lp || !r || !d || !v) return WK_ERR_ARG;
  const size_t cnt = (size_t)c->n * horizon;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(c->ts, s, sizeof(float) * 12 * cnt, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->ta, a, sizeof(float) * 4 * cnt, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->tlp, lp, sizeof(float) * 4 * cnt, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->tr, r, sizeof(float) * cnt, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->td, d, cnt, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->tv, v, sizeof(float) * cnt, hipMemcpyHostToDevice));
  c->T_valid = horizon;
  c->returns_valid = false;
  return WK_OK;
}

// the ring slot of the next stamped exchange launch (wk_comm_xch_profile), or null
static uint64_t* xch_stamp_slot(wk_ctx* c) {
  if (!c->xch_stamps) return nullptr;
  const int64_t slot = c->xch_stamp_launches++ % c->xch_stamp_cap;
  return c->xch_stamps + (size_t)slot * wk::xch_blocks() * wk::XCH_POINTS;
}

// one minibatch: gradient kernel -> ordered block reduction -> [RCCL all-reduce] -> Adam
// wpb == 0: the matrix-core kernel (wk_ppo_mfma.hip); wpb >= 1: the lane-per-neuron
// kernel (wk_ppo.hip; wpb == 1 visits the samples in minibatch order)
static int minibatch(wk_ctx* c, wk::GradArgs g, int wpb, int apply_adam) {
  const int gi = wk::grad_impl_for(c->grad_impl, g.samples);
  const int nblocks = wpb == 0 ? wk::ppo_grad_mfma_blocks(g.samples, gi)
                               : (g.samples + wpb * g.spw - 1) / (wpb * g.spw);
  // block slabs followed by the stage-1 group sums of the ordered reduction
  const size_t need = ((size_t)nblocks + wk::grad_reduce_groups(nblocks)) * wk::SLAB;
  if (c->partial_floats < need) {
    if (c->partial) (void)hipFree(c->partial);
    c->partial = nullptr;
    c->partial_floats = 0;
    HIPCHK(c, hipMalloc((void**)&c->partial, sizeof(float) * need));
    c->partial_floats = need;
  }
  g.partial = c->partial;
  wk::AdamArgs a{};
  if (apply_adam) {
    c->adam_t += 1;
    const wk_config& k = c->cfg;
    a.W = c->W; a.m = c->m; a.v = c->v; a.grad = c->grad; a.Wz = c->Wz;
    a.c1 = 1.0f - k.Beta1;
    a.c2 = 1.0f - k.Beta2;
    a.beta1 = k.Beta1;
    a.beta2 = k.Beta2;
    a.bc1 = (float)(1.0 - pow((double)k.Beta1, (double)c->adam_t));
    a.bc2 = (float)(1.0 - pow((double)k.Beta2, (double)c->adam_t));
    a.alpha = k.Alpha;
    a.eps = k.AdamEpsilon;
  }
  float* part2 = c->partial + (size_t)nblocks * wk::SLAB;
  // with a communicator (any size, also one rank) the collective path runs: reduction,
  // RCCL all-reduce, Adam -- a single-GPU test then covers the multi-GPU sequence
  const bool multi = c->comm != nullptr || c->host_ar != nullptr || c->ipc;
  {
    ProfScope ps(c, PK_GRAD, 0, 2);
    HIPCHK(c, wpb == 0 ? wk::launch_ppo_grad_mfma(g, nblocks, gi, c->stream)
                       : wk::launch_ppo_grad(g, wpb, nblocks, c->stream));
  }
  // reduction, exchange and Adam in one launch (k_reduce_xch_adam); a gradient-only call
  // (apply_adam 0: a.W == null) runs the exchange alone, so on every kind of context the
  // returned gradient is the sum over the ranks
  if (c->ipc) {
    ProfScope ps(c, PK_ALLRED, 0, 2);
    wk::XchArgs x = c->xa;
    x.partial = c->partial;
    x.nblocks = nblocks;
    x.grad_out = c->grad;
    x.seq = ++c->xch_seq;
    x.err = c->xch_err;
    x.timeout_ticks = c->xch_timeout_ticks;
    x.t = (uint32_t)c->adam_t;
    x.a = a;
    x.stamps = xch_stamp_slot(c);
    HIPCHK(c, wk::launch_reduce_xch_adam(x, c->stream));
    return WK_OK;
  }
  if (apply_adam && !multi) {  // one GPU: the last reduction stage applies Adam
    ProfScope ps(c, PK_REDUCE, 0, 2);
    HIPCHK(c, wk::launch_grad_reduce_adam(c->partial, nblocks, part2, c->grad, a, c->stream));
    return WK_OK;
  }
  {
    ProfScope ps(c, PK_REDUCE, 0, 2);
    HIPCHK(c, wk::launch_grad_reduce(c->partial, nblocks, part2, c->grad, c->stream));
  }

  if (multi) {
    ProfScope ps(c, PK_ALLRED, 0, 2);
    if (c->comm) {
      ncclResult_t r = ncclAllReduce(c->grad, c->grad, wk::SLAB, ncclFloat, ncclSum,
                                     c->comm, c->stream);
      if (r != ncclSuccess) { SETERR(c, "ncclAllReduce: %s", ncclGetErrorString(r)); return WK_ERR_COMM; }
    } else {  // host all-reduce: the slab goes through the caller's function between two copies
      c->host_ar_buf.resize(wk::SLAB);
      HIPCHK(c, hipMemcpyAsync(c->host_ar_buf.data(), c->grad, sizeof(float) * wk::SLAB,
                               hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      if (c->host_ar(c->host_ar_buf.data(), wk::SLAB, c->host_ar_user) != 0) {
        SETERR(c, "host all-reduce callback failed");
        return WK_ERR_COMM;
      }
      HIPCHK(c, hipMemcpyAsync(c->grad, c->host_ar_buf.data(), sizeof(float) * wk::SLAB,
                               hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));  // the host buffer is reused next minibatch
    }
  }
  if (apply_adam) {
    ProfScope ps(c, PK_ADAM, 0, 2);
    HIPCHK(c, wk::launch_adam(a, c->stream));
  }
  return WK_OK;
}

// IPC contexts: WK_ERR_COMM once an exchange timed out or met a peer's abort (from then on every
// exchange is a no-op); the host's Adam step count rolls back to the last step block 0 applied
// (wk_get_adam and checkpoints report the steps actually taken)
static int xch_status(wk_ctx* c) {
  if (!c->ipc) return WK_OK;
  uint32_t err[2] = {0, 0};
  HIPCHK(c, hipMemcpyAsync(err, c->xch_err, sizeof err, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (err[0]) {
    c->adam_t = (int)err[1];
    SETERR(c, "IPC gradient exchange: a peer did not publish its minibatch slab within %.1f s or "
           "gave up on it (no Adam step applied since step %u; the replicas may differ and this "
           "context stays failed: stop the job, or on every rank destroy the context, create and "
           "map a new one and load a checkpoint)",
           (double)c->xch_timeout_ticks / wk::XCH_TICKS_PER_S, err[1]);
    return WK_ERR_COMM;
  }
  return WK_OK;
}

// the device's record of the last applied Adam step starts from the host's count (a checkpoint
// or wk_set_adam may have moved it since the last exchange)
static int xch_mark_t(wk_ctx* c) {
  if (!c->ipc) return WK_OK;
  HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)(c->xch_err + 1), (int)c->adam_t, 1, c->stream));
  return WK_OK;
}

static uint64_t xch_ticks_of(double seconds) {
  return (uint64_t)(seconds * wk::XCH_TICKS_PER_S);
}

int wk_comm_set_timeout(wk_ctx* c, double seconds) {
  if (!c || !(seconds > 0.0) || seconds > 1.0e6) return WK_ERR_ARG;
  c->xch_timeout_ticks = xch_ticks_of(seconds);
  return WK_OK;
}

static wk::GradArgs grad_base(wk_ctx* c) {
  wk::GradArgs g{};
  g.W = c->W;
  g.Wz = c->Wz;
  g.std_ = c->P.std_;
  g.lp_const = c->lp_const;
  g.upper = 1.0f + c->cfg.Epsilon;
  g.lower = 1.0f - c->cfg.Epsilon;
  return g;
}

static int ppo_update_impl(wk_ctx* c, const wk_ppo_args* args);
// The gradient kernel alone, `reps` back-to-back launches on minibatch 0 of the keyed sequence
// (update 0, epoch 0) of the current trajectory, between one HIP-event pair on the context's
// stream: the kernel's mean duration without per-launch event overhead (bench.py's update
// roofline; the launches write only the scratch slabs, no weights change)
int wk_grad_kernel(wk_ctx* c, int minibatch) {
  if (!c || minibatch < 0) return WK_ERR_ARG;
  return wk::grad_impl_for(c->grad_impl, minibatch > 0 ? minibatch : c->cfg.Minibatch);
}

int wk_rollout_mapping(wk_ctx* c, int* lanes_per_walker, int* walkers_per_wave, int64_t* waves,
                       int64_t* waves_launched) {
  if (!c || !lanes_per_walker || !walkers_per_wave || !waves) return WK_ERR_ARG;
  const int64_t n = c->n;
  int64_t launched;
  if (c->scene.n_props > 0) {  // the one-lane scene kernel (64-thread blocks)
    *lanes_per_walker = 1; *walkers_per_wave = 64; *waves = (n + 63) / 64;
    launched = *waves;
  } else {
    const int L = c->P.lanes;
    *lanes_per_walker = L;
    if (L == 4) {  // sparse quad: wpw walkers in the first 4 wpw lanes of each wave
      *walkers_per_wave = c->P.wpw;
      *waves = (n + c->P.wpw - 1) / c->P.wpw;
    } else {
      *walkers_per_wave = 64 / L;
      *waves = (n * L + 63) / 64;
    }
    launched = *waves;
    if (L == 2 || L == 4) {  // k_env_side launches whole SIDE_BLOCK blocks: the idle
      // waves of the last block still run the loop, replaying the last walker
      constexpr int64_t wpb = wk::SIDE_BLOCK_THREADS / 64;
      launched = (*waves + wpb - 1) / wpb * wpb;
    }
  }
  if (waves_launched) *waves_launched = launched;
  return WK_OK;
}

int wk_time_gradient(wk_ctx* c, int minibatch, int reps, double* ms_per_launch) {
  return wk_time_gradient_ex(c, minibatch, reps, 0, ms_per_launch);
}

int wk_time_gradient_ex(wk_ctx* c, int minibatch, int reps, int flags, double* ms_per_launch) {
  DevGuard dg_(c);
  if (!c || reps <= 0 || !ms_per_launch || (flags & ~1)) return WK_ERR_ARG;
  if (c->T_valid <= 0) { SETERR(c, "wk_time_gradient before wk_rollout / wk_set_trajectory"); return WK_ERR_STATE; }
  if (!c->returns_valid) {
    int r = returns_impl(c);
    if (r) return r;
  }
  const int M = minibatch > 0 ? minibatch : c->cfg.Minibatch;
  const uint32_t pool = (uint32_t)((size_t)c->n * c->T_valid);
  if ((uint32_t)M > pool) { SETERR(c, "minibatch %d larger than the pool %u", M, pool); return WK_ERR_ARG; }
  wk::GradArgs g = grad_base(c);
  g.states = c->ts; g.actions = c->ta; g.logp_old = c->tlp; g.returns = c->tret; g.adv = c->tadv;
  g.pool = pool;
  g.use_perm = 1;
  g.samples = M;
  g.b_div = (float)(c->cfg.MinibatchGlobal > 0 ? c->cfg.MinibatchGlobal : M);
  g.pk = wk::perm_key(c->seed, 0u, 0u, pool);
  g.base = 0;
  const int gi = wk::grad_impl_for(c->grad_impl, M);
  const int nblocks = wk::ppo_grad_mfma_blocks(M, gi);
  const size_t need = ((size_t)nblocks + wk::grad_reduce_groups(nblocks)) * wk::SLAB;
  if (c->partial_floats < need) {
    if (c->partial) (void)hipFree(c->partial);
    c->partial = nullptr;
    c->partial_floats = 0;
    HIPCHK(c, hipMalloc((void**)&c->partial, sizeof(float) * need));
    c->partial_floats = need;
  }
  g.partial = c->partial;
  HIPCHK(c, wk::launch_ppo_grad_mfma(g, nblocks, gi, c->stream));  // warm
  // flags & 1: an event pair around EVERY launch (as profile level 2 times the update's
  // launches), the elapsed times summed -- the burst's per-launch event overhead is the
  // difference to one pair around the whole burst
  const int npairs = (flags & 1) ? reps : 1;
  std::vector<hipEvent_t> ev(2 * (size_t)npairs, nullptr);
  for (auto& e : ev) HIPCHK(c, hipEventCreate(&e));
  for (int i = 0; i < reps; i++) {
    if ((flags & 1) || i == 0) HIPCHK(c, hipEventRecord(ev[2 * ((flags & 1) ? i : 0)], c->stream));
    HIPCHK(c, wk::launch_ppo_grad_mfma(g, nblocks, gi, c->stream));
    if ((flags & 1) || i == reps - 1) HIPCHK(c, hipEventRecord(ev[2 * ((flags & 1) ? i : 0) + 1], c->stream));
  }
  HIPCHK(c, hipEventSynchronize(ev.back()));
  double total = 0.0;
  for (int i = 0; i < npairs; i++) {
    float ms = 0.0f;
    HIPCHK(c, hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
    total += ms;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  *ms_per_launch = total / reps;
  return WK_OK;
}

int wk_ppo_update(wk_ctx* c, const wk_ppo_args* args, float* critic_diag, float* actor_diag) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  if (c->T_valid <= 0) { SETERR(c, "wk_ppo_update before wk_rollout / wk_set_trajectory"); return WK_ERR_STATE; }
  {
    ProfScope ps(c, PK_UPDATE);
    int r = ppo_update_impl(c, args);
    if (r) return r;
  }
  {  // a peer that never published is fatal for the job (like a failed all-reduce)
    int r = xch_status(c);
    if (r) return r;
  }
  if (c->collect) {  // the last minibatch's losses, as PPOAgent.Train hands them on (:165-166)
    if (c->loss_count < c->loss_cap)
      HIPCHK(c, hipMemcpyAsync(c->loss_log + 2 * c->loss_count, c->grad + wk::NPARAM,
                               2 * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
    c->loss_count++;
  }
  if (!critic_diag && !actor_diag) return WK_OK;  // stays asynchronous on the stream
  float diag[3] = {0, 0, 0};
  HIPCHK(c, hipMemcpyAsync(diag, c->grad + wk::NPARAM, sizeof(diag), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (critic_diag) *critic_diag = diag[0];
  if (actor_diag) *actor_diag = diag[1];
  return WK_OK;
}

static int ppo_update_impl(wk_ctx* c, const wk_ppo_args* args) {
  if (!c->returns_valid) {
    int r = returns_impl(c);
    if (r) return r;
  }
  if (int r = xch_mark_t(c)) return r;
  const int epochs = (args && args->epochs > 0) ? args->epochs : c->cfg.Epochs;
  const int M = (args && args->minibatch > 0) ? args->minibatch : c->cfg.Minibatch;
  int Mg = (args && args->minibatch_global > 0) ? args->minibatch_global : c->cfg.MinibatchGlobal;
  if (Mg <= 0) Mg = M * c->nranks;
  const uint32_t update = args ? args->update_index : 0u;
  const uint32_t pool = (uint32_t)((size_t)c->n * c->T_valid);
  const int nmb = (int)(pool / (uint32_t)M);  // remainder dropped (PPOAgent.cs:506)
  if (nmb <= 0) { SETERR(c, "minibatch %d larger than the pool %u", M, pool); return WK_ERR_ARG; }
  const int wpb = 0;  // matrix cores
  const int spw = 0;
  wk::GradArgs g = grad_base(c);
  g.states = c->ts; g.actions = c->ta; g.logp_old = c->tlp; g.returns = c->tret; g.adv = c->tadv;
  g.pool = pool;
  g.use_perm = 1;
  g.samples = M;
  g.spw = spw;
  g.b_div = (float)Mg;
  for (int e = 0; e < epochs; e++) {
    g.pk = wk::perm_key(c->seed, update, (uint32_t)e, pool);
    for (int j = 0; j < nmb; j++) {
      g.base = (uint32_t)j * (uint32_t)M;
      int r = minibatch(c, g, wpb, 1);
      if (r) return r;
    }
  }
  return WK_OK;
}

static int batch_impl(wk_ctx* c, int wpb, int B, float b_div, const float* s, const float* a,
                      const float* lpo, const float* ret, const float* adv, float* cd, float* ad,
                      float* grads_out, int apply_adam, int* skipped) {
  if (!c || B <= 0 || !s || !a || !lpo || !ret || !adv) return WK_ERR_ARG;
  const size_t bs = sizeof(float) * B;
  const size_t total = bs * (12 + 4 + 4 + 1 + 1) + 256;
  if (ensure(c, &c->scratch2, &c->scratch2_bytes, total)) return WK_ERR_HIP;
  char* p = (char*)c->scratch2;
  float* d_s = (float*)p; p += bs * 12;
  float* d_a = (float*)p; p += bs * 4;
  float* d_l = (float*)p; p += bs * 4;
  float* d_r = (float*)p; p += bs;
  float* d_v = (float*)p;
  HIPCHK(c, hipMemcpyAsync(d_s, s, bs * 12, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_a, a, bs * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_l, lpo, bs * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_r, ret, bs, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_v, adv, bs, hipMemcpyHostToDevice, c->stream));
  wk::GradArgs g = grad_base(c);
  g.states = d_s; g.actions = d_a; g.logp_old = d_l; g.returns = d_r; g.adv = d_v;
  g.pool = (uint32_t)B;
  g.base = 0;
  g.use_perm = 0;
  g.samples = B;
  g.spw = B;  // wpb 1: one wave, samples in order (the reference's sequential sums)
  g.b_div = b_div;
  int r = xch_mark_t(c);
  if (r) return r;
  r = minibatch(c, g, wpb, apply_adam);
  if (r) return r;
  std::vector<float> slab(wk::SLAB);
  HIPCHK(c, hipMemcpyAsync(slab.data(), c->grad, sizeof(float) * slab.size(), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  r = xch_status(c);  // (IPC: a timed-out exchange left grad stale and applied no Adam)
  if (r) return r;
  if (grads_out) memcpy(grads_out, slab.data(), sizeof(float) * wk::NPARAM);
  if (cd) *cd = slab[wk::NPARAM];
  if (ad) *ad = slab[wk::NPARAM + 1];
  if (skipped) *skipped = (int)slab[wk::NPARAM + 2];
  return WK_OK;
}

int wk_train_batch(wk_ctx* c, int B, float b_div, const float* s, const float* a, const float* lpo,
                   const float* ret, const float* adv, float* cd, float* ad, float* grads_out,
                   int apply_adam, int* skipped) {
  DevGuard dg_(c);
  return batch_impl(c, 1, B, b_div, s, a, lpo, ret, adv, cd, ad, grads_out, apply_adam, skipped);
}

int wk_minibatch_gradient(wk_ctx* c, int B, float b_div, const float* s, const float* a,
                          const float* lpo, const float* ret, const float* adv, float* cd,
                          float* ad, float* grads_out, int* skipped) {
  DevGuard dg_(c);
  return batch_impl(c, 0, B, b_div, s, a, lpo, ret, adv, cd, ad, grads_out, 0, skipped);
}

int wk_comm_unique_id(uint8_t* id) {
  if (!id) return WK_ERR_ARG;
  static_assert(sizeof(ncclUniqueId) == 128, "nccl id size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) { g_create_error = ncclGetErrorString(r); return WK_ERR_COMM; }
  memcpy(id, &u, sizeof(u));
  return WK_OK;
}

int wk_comm_init(wk_ctx* c, int rank, int nranks, const uint8_t* id) {
  DevGuard dg_(c);
  if (!c || !id || nranks <= 0 || rank < 0 || rank >= nranks) return WK_ERR_ARG;
  if (c->host_ar) { SETERR(c, "the context already has a host all-reduce"); return WK_ERR_STATE; }
  HIPCHK(c, hipSetDevice(c->device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) { SETERR(c, "ncclCommInitRank: %s", ncclGetErrorString(r)); c->comm = nullptr; return WK_ERR_COMM; }
  c->rank = rank;
  c->nranks = nranks;
  return WK_OK;
}

int wk_comm_init_host(wk_ctx* c, int rank, int nranks, wk_host_allreduce_fn fn, void* user) {
  DevGuard dg_(c);
  if (!c || !fn || nranks <= 0 || rank < 0 || rank >= nranks) return WK_ERR_ARG;
  if (c->comm) { SETERR(c, "the context already has an RCCL communicator"); return WK_ERR_STATE; }
  c->host_ar = fn;
  c->host_ar_user = user;
  c->rank = rank;
  c->nranks = nranks;
  return WK_OK;
}

// the exchange record of one rank: [0, 64) the region's hipIpcMemHandle_t, [64, 128) the PCI bus
// id of the rank's device (NUL-padded), so every rank can count the ranks sharing its GPU
static constexpr size_t kIpcDevOff = 64;
static_assert(sizeof(hipIpcMemHandle_t) == kIpcDevOff && WK_IPC_HANDLE_BYTES == 128, "IPC record");

int wk_comm_ipc_handle(wk_ctx* c, uint8_t* handle) {
  DevGuard dg_(c);
  if (!c || !handle) return WK_ERR_ARG;
  if (!c->xch) {
    // uncached (MTYPE UC) device memory: the peers read it over xGMI and this GPU writes it
    // through no cache; coarse-grained hipMalloc memory is the fallback where the driver cannot
    // export an uncached allocation (the system-scope release / acquire covers it as well)
    const size_t bytes = wk::xch_region_bytes();
    hipIpcMemHandle_t probe;
    if (hipExtMallocWithFlags(&c->xch, bytes, hipDeviceMallocUncached) != hipSuccess ||
        hipIpcGetMemHandle(&probe, c->xch) != hipSuccess) {
      if (c->xch) (void)hipFree(c->xch);
      c->xch = nullptr;
      (void)hipGetLastError();
      HIPCHK(c, hipMalloc(&c->xch, bytes));
      c->xch_uncached = false;
    } else {
      c->xch_uncached = true;
    }
    HIPCHK(c, hipMemset(c->xch, 0, bytes));
    HIPCHK(c, hipMalloc((void**)&c->xch_err, 2 * sizeof(uint32_t)));
    HIPCHK(c, hipMemset(c->xch_err, 0, 2 * sizeof(uint32_t)));
  }
  hipIpcMemHandle_t h;
  HIPCHK(c, hipIpcGetMemHandle(&h, c->xch));
  memset(handle, 0, WK_IPC_HANDLE_BYTES);
  memcpy(handle, &h, sizeof h);
  HIPCHK(c, hipDeviceGetPCIBusId((char*)handle + kIpcDevOff, (int)(WK_IPC_HANDLE_BYTES - kIpcDevOff) - 1,
                                 c->device));
  return WK_OK;
}

int wk_comm_init_ipc(wk_ctx* c, int rank, int nranks, const uint8_t* handles) {
  DevGuard dg_(c);
  if (!c || !handles || nranks <= 0 || rank < 0 || rank >= nranks) return WK_ERR_ARG;
  if (nranks > wk::XCH_MAX_RANKS) { SETERR(c, "the IPC exchange spans at most %d ranks", (int)wk::XCH_MAX_RANKS); return WK_ERR_ARG; }
  if (c->comm || c->host_ar || c->ipc) { SETERR(c, "the context already has an all-reduce"); return WK_ERR_STATE; }
  if (!c->xch) { SETERR(c, "wk_comm_ipc_handle first"); return WK_ERR_STATE; }
  {  // ranks sharing this rank's GPU (a rehearsal): more than four stall, see XCH_MAX_RANKS_PER_DEVICE
    const char* mine = (const char*)handles + (size_t)rank * WK_IPC_HANDLE_BYTES + kIpcDevOff;
    int same = 0;
    for (int r = 0; r < nranks; r++)
      same += strncmp(mine, (const char*)handles + (size_t)r * WK_IPC_HANDLE_BYTES + kIpcDevOff,
                      WK_IPC_HANDLE_BYTES - kIpcDevOff) == 0;
    if (same > wk::XCH_MAX_RANKS_PER_DEVICE) {
      SETERR(c, "the IPC exchange takes at most %d ranks per GPU (%d share %s): their waiting "
             "exchange blocks would hold the CUs a peer's gradient kernel needs",
             (int)wk::XCH_MAX_RANKS_PER_DEVICE, same, mine);
      return WK_ERR_ARG;
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  wk::XchArgs x{};
  std::vector<void*> opened;
  for (int r = 0; r < nranks; r++) {
    void* base = c->xch;
    if (r != rank) {
      hipIpcMemHandle_t h;
      memcpy(&h, handles + (size_t)r * WK_IPC_HANDLE_BYTES, sizeof h);
      const hipError_t e = hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) {
        for (void* p : opened) (void)hipIpcCloseMemHandle(p);
        SETERR(c, "hipIpcOpenMemHandle (rank %d): %s", r, hipGetErrorString(e));
        return WK_ERR_COMM;
      }
      opened.push_back(base);
    }
    x.slab[r] = (float*)base;
    x.flag[r] = (uint64_t*)((char*)base + sizeof(float) * 2 * wk::SLAB);
  }
  x.rank = rank;
  x.nranks = nranks;
  c->xa = x;
  if (c->xch_timeout_ticks == 0) {  // wk_comm_set_timeout before the mapping wins
    double sec = wk::XCH_TIMEOUT_S_DEFAULT;
    if (const char* e = getenv("WK_XCH_TIMEOUT_S")) {
      const double v = atof(e);
      if (v > 0.0 && v <= 1.0e6) sec = v;
    }
    c->xch_timeout_ticks = xch_ticks_of(sec);
  }
  c->xch_peers = opened;
  c->ipc = true;
  c->rank = rank;
  c->nranks = nranks;
  return WK_OK;
}

int wk_comm_info(wk_ctx* c, int* kind, int* flags) {
  if (!c || !kind || !flags) return WK_ERR_ARG;
  *kind = c->ipc ? 3 : c->host_ar ? 2 : c->comm ? 1 : 0;
  *flags = (c->xch && c->xch_uncached) ? 1 : 0;
  return WK_OK;
}

int wk_comm_xch_profile(wk_ctx* c, int minibatches) {
  DevGuard dg_(c);
  if (!c || minibatches < 0 || minibatches > (1 << 20)) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));  // (no launch still writes the old ring)
  if (c->xch_stamps) (void)hipFree(c->xch_stamps);
  c->xch_stamps = nullptr;
  c->xch_stamp_cap = 0;
  c->xch_stamp_launches = 0;
  if (minibatches == 0) return WK_OK;
  const size_t bytes = sizeof(uint64_t) * (size_t)minibatches * wk::xch_blocks() * wk::XCH_POINTS;
  HIPCHK(c, hipMalloc((void**)&c->xch_stamps, bytes));
  HIPCHK(c, hipMemset(c->xch_stamps, 0, bytes));
  c->xch_stamp_cap = minibatches;
  return WK_OK;
}

int wk_comm_xch_stamps(wk_ctx* c, uint64_t* stamps, int max_launches, int* launches, int* blocks) {
  DevGuard dg_(c);
  if (!c || !launches || !blocks || max_launches < 0 || (max_launches > 0 && !stamps)) return WK_ERR_ARG;
  *blocks = wk::xch_blocks();
  if (!c->xch_stamps) { *launches = 0; return WK_OK; }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int64_t have = std::min<int64_t>(c->xch_stamp_launches, c->xch_stamp_cap);
  const int n = (int)std::min<int64_t>(have, max_launches);
  const size_t per = (size_t)wk::xch_blocks() * wk::XCH_POINTS;
  // the last n launches, oldest first (the ring wraps at cap)
  for (int i = 0; i < n; i++) {
    const int64_t launch = c->xch_stamp_launches - n + i;
    const int64_t slot = launch % c->xch_stamp_cap;
    HIPCHK(c, hipMemcpy(stamps + (size_t)i * per, c->xch_stamps + (size_t)slot * per,
                        sizeof(uint64_t) * per, hipMemcpyDeviceToHost));
  }
  *launches = n;
  return WK_OK;
}

int wk_allreduce_test(wk_ctx* c, float* host_buf, int n) {
  DevGuard dg_(c);
  if (!c || !host_buf || n <= 0) return WK_ERR_ARG;
  if (c->ipc) {  // one round of the IPC exchange (k_reduce_xch_adam without Adam) on this slab
    if (n > wk::SLAB) { SETERR(c, "the IPC exchange test takes at most %d floats", (int)wk::SLAB); return WK_ERR_ARG; }
    if (ensure(c, &c->scratch, &c->scratch_bytes, sizeof(float) * 2 * wk::SLAB)) return WK_ERR_HIP;
    float* in = (float*)c->scratch;
    float* out = in + wk::SLAB;
    HIPCHK(c, hipMemsetAsync(in, 0, sizeof(float) * wk::SLAB, c->stream));
    HIPCHK(c, hipMemcpyAsync(in, host_buf, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
    wk::XchArgs x = c->xa;
    x.partial = in;
    x.nblocks = 1;
    x.grad_out = out;
    x.seq = ++c->xch_seq;
    x.err = c->xch_err;
    x.timeout_ticks = c->xch_timeout_ticks;
    x.a = wk::AdamArgs{};
    HIPCHK(c, wk::launch_reduce_xch_adam(x, c->stream));
    HIPCHK(c, hipMemcpyAsync(host_buf, out, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return xch_status(c);
  }
  if (ensure(c, &c->scratch, &c->scratch_bytes, sizeof(float) * n)) return WK_ERR_HIP;
  HIPCHK(c, hipMemcpyAsync(c->scratch, host_buf, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  if (c->comm && c->nranks > 1) {
    ncclResult_t r = ncclAllReduce(c->scratch, c->scratch, n, ncclFloat, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) { SETERR(c, "ncclAllReduce: %s", ncclGetErrorString(r)); return WK_ERR_COMM; }
  }
  HIPCHK(c, hipMemcpyAsync(host_buf, c->scratch, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}

int wk_count_events(wk_ctx* c, int k, uint64_t* counts) {
  DevGuard dg_(c);
  if (!c || !counts || k <= 0) return WK_ERR_ARG;
  if (k > c->T_valid) { SETERR(c, "count replay of %d env-steps, the trajectory holds %d", k, c->T_valid); return WK_ERR_STATE; }
  if (c->scene.n_props > 0) { SETERR(c, "the counting replay runs without scene props"); return WK_ERR_CONFIG; }
  static_assert(WK_NEV == wk::NEV, "event counters");
  if (!c->counts) HIPCHK(c, hipMalloc((void**)&c->counts, sizeof(unsigned long long) * wk::NEV));
  HIPCHK(c, hipMemsetAsync(c->counts, 0, sizeof(unsigned long long) * wk::NEV, c->stream));
  wk::StepArgs A{};
  A.st = c->st; A.dxoff = c->dxoff; A.mat = c->mat; A.rng_t = c->rng_t;
  A.actions = c->ta; A.k_steps = k; A.counts = c->counts;
  HIPCHK(c, wk::launch_env_step(4, c->P, A, c->stream));
  unsigned long long h[wk::NEV];
  HIPCHK(c, hipMemcpyAsync(h, c->counts, sizeof h, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int i = 0; i < wk::NEV; i++) counts[i] += (uint64_t)h[i];
  return WK_OK;
}

int wk_snapshot(wk_ctx* c, int op) {
  DevGuard dg_(c);
  if (!c || op < 0 || op > 1) return WK_ERR_ARG;
  const size_t n = c->n;
  struct Seg { void* p; size_t bytes; };
  const Seg segs[] = {
      {c->st, sizeof(float) * wk::NSTATE * n}, {c->rng_t, sizeof(uint32_t) * n},
      {c->W, sizeof(float) * wk::NPARAM}, {c->Wz, sizeof(float) * wk::mfma_image_floats()},
      {c->m, sizeof(float) * wk::NPARAM}, {c->v, sizeof(float) * wk::NPARAM},
      {c->ep_acc, sizeof(double) * n}, {c->ep_len, sizeof(int32_t) * n},
      {c->ep_count, sizeof(uint64_t)},
      {c->props, c->props ? sizeof(float) * n * c->scene.pstride : 0}};
  size_t total = 0;
  for (const Seg& g : segs) total += (g.bytes + 255) & ~(size_t)255;
  if (op == 0) {
    if (c->snap_bytes < total) {
      if (c->snap) (void)hipFree(c->snap);
      c->snap = nullptr; c->snap_bytes = 0;
      HIPCHK(c, hipMalloc(&c->snap, total));
      c->snap_bytes = total;
    }
    c->snap_adam_t = c->adam_t;
    c->snap_rollout_steps = c->rollout_steps;
    c->snap_loss_count = c->loss_count;
  } else if (!c->snap_valid || c->snap_bytes < total) {
    SETERR(c, "no snapshot of this configuration to restore");
    return WK_ERR_STATE;
  }
  char* q = (char*)c->snap;
  for (const Seg& g : segs) {
    if (g.bytes)
      HIPCHK(c, hipMemcpyAsync(op == 0 ? (void*)q : g.p, op == 0 ? g.p : (const void*)q, g.bytes,
                               hipMemcpyDeviceToDevice, c->stream));
    q += (g.bytes + 255) & ~(size_t)255;
  }
  if (op == 0) {
    c->snap_valid = true;
  } else {
    c->adam_t = c->snap_adam_t;
    c->rollout_steps = c->snap_rollout_steps;
    c->loss_count = c->snap_loss_count;
    // the trajectory buffer is not part of the snapshot: it keeps the last rollout (the
    // counting replay reads its actions after a restore)
  }
  return WK_OK;
}

int wk_profile_enable(wk_ctx* c, int on) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  c->prof = on < 0 ? 0 : (on > 2 ? 2 : on);
  return WK_OK;
}

int wk_profile_reset(wk_ctx* c) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  prof_drain(c);
  for (int i = 0; i < PK_N; i++) { c->prof_ms[i] = 0; c->prof_cnt[i] = 0; }
  c->prof_units = 0;
  return WK_OK;
}

int wk_profile_get(wk_ctx* c, wk_profile* o) {
  DevGuard dg_(c);
  if (!c || !o) return WK_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  prof_drain(c);
  o->physics_ms = c->prof_ms[PK_PHYS]; o->physics_launches = c->prof_cnt[PK_PHYS];
  o->physics_env_steps = c->prof_units;
  o->grad_ms = c->prof_ms[PK_GRAD]; o->grad_launches = c->prof_cnt[PK_GRAD];
  o->reduce_ms = c->prof_ms[PK_REDUCE]; o->reduce_launches = c->prof_cnt[PK_REDUCE];
  o->adam_ms = c->prof_ms[PK_ADAM]; o->adam_launches = c->prof_cnt[PK_ADAM];
  o->allreduce_ms = c->prof_ms[PK_ALLRED]; o->allreduce_calls = c->prof_cnt[PK_ALLRED];
  o->returns_ms = c->prof_ms[PK_RET]; o->returns_launches = c->prof_cnt[PK_RET];
  o->update_ms = c->prof_ms[PK_UPDATE]; o->update_calls = c->prof_cnt[PK_UPDATE];
  return WK_OK;
}

}  // extern "C"

// ---------------- weights text format + binary checkpoint ----------
// Reference format (PPOAgent.Save PPOAgent.cs:192-213 -> NeuralNetwork.Save
// NeuralNetwork.cs:159-176 -> DenseLayer.Save DenseLayer.cs:73-79 -> Matrix.Save
// Matrix.cs:133-153): one file per network, line 0 the network DSL string, then one line
// per dense layer "W w00 w01 ... B b0 b1 ..." (row-major out x in, values joined by one
// space).  Values are written as .NET Core 3.0+'s float.ToString() writes them under
// en-US: shortest round-trip digits, "E-05" / "E+09"-style exponents for |v| < 1e-4 or
// >= 1e9, "-0", "NaN", "∞".  Parsing accepts strtof syntax plus "∞" (a superset of the
// digit strings float.Parse reads; "Infinity" and "NaN" included).

namespace {
struct DenseSpec { int off_w, rows, cols, off_b; };
const DenseSpec kCriticLayers[] = {{wk::OFF_C_W1, 64, 12, wk::OFF_C_B1}, {wk::OFF_C_W2, 1, 64, wk::OFF_C_B2}};
const DenseSpec kActorLayers[] = {{wk::OFF_A_W1, 64, 12, wk::OFF_A_B1},
                                  {wk::OFF_A_W2, 64, 64, wk::OFF_A_B2},
                                  {wk::OFF_A_W3, 4, 64, wk::OFF_A_B3}};

std::string format_network(const float* p, const char* dsl, const DenseSpec* layers, int nl) {
  std::string text = std::string(dsl) + "\n";
  for (int l = 0; l < nl; l++) {
    const DenseSpec& d = layers[l];
    std::string line = "W";
    for (int i = 0; i < d.rows * d.cols; i++) line += " " + wk::dotnet_float(p[d.off_w + i]);
    line += " B";
    for (int i = 0; i < d.rows; i++) line += " " + wk::dotnet_float(p[d.off_b + i]);
    text += line + "\n";
  }
  return text;
}

// NeuralNetwork.Load / ValidateWeights / DenseLayer.Load semantics: the DSL line must
// match, every token must parse, and each layer needs rows*cols weights then rows biases.
int parse_network(const char* text, const char* dsl, const DenseSpec* layers, int nl, float* p,
                  std::string& why) {
  std::vector<std::string> lines;
  std::string cur;
  for (const char* q = text; *q; q++) {
    if (*q == '\n') { lines.push_back(cur); cur.clear(); }
    else if (*q != '\r') cur += *q;
  }
  if (!cur.empty()) lines.push_back(cur);
  if ((int)lines.size() < nl + 1) { why = "weights file too short"; return WK_ERR_ARG; }
  if (lines[0] != dsl) { why = "network string '" + lines[0] + "' does not match '" + dsl + "'"; return WK_ERR_CONFIG; }
  for (int l = 0; l < nl; l++) {
    const DenseSpec& d = layers[l];
    const std::string& s = lines[l + 1];
    const size_t w = s.find('W'), b = s.find('B');
    if (w == std::string::npos || b == std::string::npos || b < w) { why = "weights structure issue"; return WK_ERR_ARG; }
    // "W a b c B d e": tokens separated by single spaces (ValidateWeights splits with
    // string.Split(), so an empty token fails float.TryParse)
    auto parse_list = [&](const std::string& seg, float* dst, int count) -> bool {
      if (seg.size() < 2 || seg.front() != ' ') return false;
      size_t at = 1;
      for (int i = 0; i < count; i++) {
        const size_t sp = seg.find(' ', at);
        const std::string tok = seg.substr(at, sp == std::string::npos ? std::string::npos : sp - at);
        if (tok.empty()) return false;
        if (tok == "\xe2\x88\x9e") dst[i] = INFINITY;
        else if (tok == "-\xe2\x88\x9e") dst[i] = -INFINITY;
        else {
          char* end = nullptr;
          dst[i] = strtof(tok.c_str(), &end);
          if (*end) return false;
        }
        if (sp == std::string::npos) return i == count - 1;
        at = sp + 1;
      }
      return at == seg.size();  // the weights segment ends with the space before "B"
    };
    if (!parse_list(s.substr(w + 1, b - w - 1), p + d.off_w, d.rows * d.cols)) { why = "error in weights section"; return WK_ERR_ARG; }
    if (!parse_list(s.substr(b + 1), p + d.off_b, d.rows)) { why = "error in biases section"; return WK_ERR_ARG; }
  }
  return WK_OK;
}

bool read_file(const char* path, std::string& out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  char buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, k);
  fclose(f);
  return true;
}
bool write_file(const char* path, const void* data, size_t n) {
  FILE* f = fopen(path, "wb");
  if (!f) return false;
  const bool ok = fwrite(data, 1, n, f) == n;
  return fclose(f) == 0 && ok;
}

const uint32_t kCkptMagic = 0x4B434B57u;  // "WKCK"
struct CkptHeader {
  uint32_t magic, version, n_env, nstate, nparam, adam_t;
  uint64_t seed;
  int32_t env_offset, iterations, max_timesteps;
  uint32_t rollout_steps;
};
static_assert(sizeof(CkptHeader) == 48, "checkpoint header");
// version 4 adds this block right after the header: the configuration that changes the
// physics beyond the header's fields (RoughFloor) and the mapping the file was written with
struct CkptExt {
  int32_t rough_floor, lanes_per_walker, reserved0, reserved1;
};
static_assert(sizeof(CkptExt) == 16, "checkpoint extension");
// 3: + scene section (int32 n_props, wk_prop[n_props], [n][pstride]); 4: + CkptExt
const uint32_t kCkptVersion = 4;
size_t ckpt_bytes(size_t n) {
  return sizeof(CkptHeader) + sizeof(float) * (3 * wk::NPARAM + n * wk::NSTATE + 2 * n) +
         sizeof(int32_t) * n + sizeof(double) * n + sizeof(int32_t) * n;
}
}  // namespace

extern "C" {

int wk_format_weights(const float* params, char* critic, size_t critic_cap, char* actor,
                      size_t actor_cap) {
  if (!params) return WK_ERR_ARG;
  const std::string c = format_network(params, kCriticDefault, kCriticLayers, 2);
  const std::string a = format_network(params, kActorDefault, kActorLayers, 3);
  if (!critic || !actor || critic_cap < c.size() + 1 || actor_cap < a.size() + 1)
    return -(int)(c.size() > a.size() ? c.size() + 1 : a.size() + 1);  // needed capacity
  memcpy(critic, c.c_str(), c.size() + 1);
  memcpy(actor, a.c_str(), a.size() + 1);
  return WK_OK;
}

int wk_parse_weights(const char* critic, const char* actor, float* params) {
  if (!critic || !actor || !params) { g_create_error = "null argument"; return WK_ERR_ARG; }
  std::vector<float> p(wk::NPARAM, 0.0f);
  std::string why;
  int r = parse_network(critic, kCriticDefault, kCriticLayers, 2, p.data(), why);
  if (r == WK_OK) r = parse_network(actor, kActorDefault, kActorLayers, 3, p.data(), why);
  if (r != WK_OK) { g_create_error = why; return r; }
  memcpy(params, p.data(), sizeof(float) * wk::NPARAM);
  return WK_OK;
}

int wk_save_weights(wk_ctx* c, const char* critic_path, const char* actor_path) {
  DevGuard dg_(c);
  if (!c || !critic_path || !actor_path) return WK_ERR_ARG;
  std::vector<float> p(wk::NPARAM);
  int r = wk_get_weights(c, p.data());
  if (r) return r;
  const std::string ct = format_network(p.data(), kCriticDefault, kCriticLayers, 2);
  const std::string at = format_network(p.data(), kActorDefault, kActorLayers, 3);
  if (!write_file(critic_path, ct.data(), ct.size()) || !write_file(actor_path, at.data(), at.size())) {
    SETERR(c, "cannot write weights files '%s' / '%s'", critic_path, actor_path);
    return WK_ERR_ARG;
  }
  return WK_OK;
}

int wk_load_weights(wk_ctx* c, const char* critic_path, const char* actor_path) {
  DevGuard dg_(c);
  if (!c || !critic_path || !actor_path) return WK_ERR_ARG;
  std::string ct, at;
  if (!read_file(critic_path, ct) || !read_file(actor_path, at)) {
    SETERR(c, "cannot read weights files '%s' / '%s'", critic_path, actor_path);
    return WK_ERR_ARG;
  }
  std::vector<float> p(wk::NPARAM, 0.0f);
  std::string why;
  int r = parse_network(ct.c_str(), kCriticDefault, kCriticLayers, 2, p.data(), why);
  if (r == WK_OK) r = parse_network(at.c_str(), kActorDefault, kActorLayers, 3, p.data(), why);
  if (r != WK_OK) { c->err = why; return r; }
  return wk_set_weights(c, p.data());
}

// Binary checkpoint for exact resume: weights, Adam m / v / t, every walker record,
// Philox step counters, start offsets and materials.
int wk_checkpoint_save(wk_ctx* c, const char* path) {
  DevGuard dg_(c);
  if (!c || !path) return WK_ERR_ARG;
  const size_t n = c->n;
  CkptHeader h{kCkptMagic, kCkptVersion, (uint32_t)n, (uint32_t)wk::NSTATE, (uint32_t)wk::NPARAM,
               (uint32_t)c->adam_t, c->seed, c->cfg.EnvOffset, c->cfg.Iterations,
               c->cfg.MaxTimesteps, c->rollout_steps};
  const int np = c->scene.n_props;
  const size_t scene_bytes = sizeof(int32_t) + sizeof(wk_prop) * np + sizeof(float) * n * c->scene.pstride;
  const CkptExt ext{c->cfg.RoughFloor, c->P.lanes, 0, 0};
  std::vector<char> buf(ckpt_bytes(n) + sizeof ext + scene_bytes);
  char* q = buf.data();
  memcpy(q, &h, sizeof h); q += sizeof h;
  memcpy(q, &ext, sizeof ext); q += sizeof ext;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(q, c->W, sizeof(float) * wk::NPARAM, hipMemcpyDeviceToHost)); q += sizeof(float) * wk::NPARAM;
  HIPCHK(c, hipMemcpy(q, c->m, sizeof(float) * wk::NPARAM, hipMemcpyDeviceToHost)); q += sizeof(float) * wk::NPARAM;
  HIPCHK(c, hipMemcpy(q, c->v, sizeof(float) * wk::NPARAM, hipMemcpyDeviceToHost)); q += sizeof(float) * wk::NPARAM;
  HIPCHK(c, hipMemcpy(q, c->st, sizeof(float) * n * wk::NSTATE, hipMemcpyDeviceToHost)); q += sizeof(float) * n * wk::NSTATE;
  HIPCHK(c, hipMemcpy(q, c->rng_t, sizeof(uint32_t) * n, hipMemcpyDeviceToHost)); q += sizeof(uint32_t) * n;
  HIPCHK(c, hipMemcpy(q, c->dxoff, sizeof(float) * n, hipMemcpyDeviceToHost)); q += sizeof(float) * n;
  HIPCHK(c, hipMemcpy(q, c->mat, sizeof(int32_t) * n, hipMemcpyDeviceToHost)); q += sizeof(int32_t) * n;
  HIPCHK(c, hipMemcpy(q, c->ep_acc, sizeof(double) * n, hipMemcpyDeviceToHost)); q += sizeof(double) * n;
  HIPCHK(c, hipMemcpy(q, c->ep_len, sizeof(int32_t) * n, hipMemcpyDeviceToHost)); q += sizeof(int32_t) * n;
  const int32_t np32 = np;
  memcpy(q, &np32, sizeof np32); q += sizeof np32;
  if (np > 0) {
    memcpy(q, c->scene_desc.data(), sizeof(wk_prop) * np); q += sizeof(wk_prop) * np;
    HIPCHK(c, hipMemcpy(q, c->props, sizeof(float) * n * c->scene.pstride, hipMemcpyDeviceToHost));
  }
  if (!write_file(path, buf.data(), buf.size())) { SETERR(c, "cannot write checkpoint '%s'", path); return WK_ERR_ARG; }
  return WK_OK;
}

// Every check runs before the first device write, so a rejected file leaves the context
// exactly as it was: header, sizes, seed / EnvOffset (the Philox streams),
// Iterations / MaxTimesteps / RoughFloor (the physics), and the scene's acceptability.
int wk_checkpoint_load(wk_ctx* c, const char* path) {
  DevGuard dg_(c);
  if (!c || !path) return WK_ERR_ARG;
  std::string data;
  if (!read_file(path, data)) { SETERR(c, "cannot read checkpoint '%s'", path); return WK_ERR_ARG; }
  const size_t n = c->n;
  CkptHeader h;
  if (data.size() < sizeof h) { SETERR(c, "checkpoint '%s' truncated", path); return WK_ERR_ARG; }
  memcpy(&h, data.data(), sizeof h);
  if (h.magic != kCkptMagic || h.version < 2 || h.version > kCkptVersion) {
    SETERR(c, "'%s' is not a wk checkpoint", path);
    return WK_ERR_ARG;
  }
  // version 2 (before scene props) has no scene section, version 3 no CkptExt.  Neither
  // records RoughFloor (which already existed when they were written), and nothing in the
  // walker records tells the floors apart: loading one could run the wrong physics on the
  // saved walkers, so it is refused
  if (h.version < 4) {
    SETERR(c, "checkpoint '%s' is version %u: its floor type (RoughFloor) was not recorded "
              "before version 4, so it cannot be resumed safely", path, h.version);
    return WK_ERR_CONFIG;
  }
  const size_t ext_bytes = sizeof(CkptExt);
  CkptExt ext{0, 0, 0, 0};
  if (data.size() >= sizeof h + ext_bytes) memcpy(&ext, data.data() + sizeof h, sizeof ext);
  size_t need = ckpt_bytes(n) + ext_bytes + sizeof(int32_t);
  int32_t np = 0;
  std::vector<wk_prop> desc;
  if (data.size() >= need) {
    memcpy(&np, data.data() + need - sizeof(int32_t), sizeof np);
    if (np < 0 || np > WK_MAX_PROPS) { SETERR(c, "checkpoint '%s': invalid scene section", path); return WK_ERR_ARG; }
    if (np > 0 && data.size() >= need + sizeof(wk_prop) * np) {
      desc.resize(np);
      memcpy(desc.data(), data.data() + need, sizeof(wk_prop) * np);
      need += sizeof(wk_prop) * np;
      size_t pstride = 0;
      for (const wk_prop& p : desc) {
        float xs[WK_PROP_MAXV], ys[WK_PROP_MAXV];
        const int nv = p.smooth >= 0 ? prop_vertices(p, p.smooth, xs, ys) : -1;
        pstride += nv > 0 ? (size_t)(2 * nv + 6) : (size_t)1 << 40;  // a bad record fails the size check
      }
      need += sizeof(float) * n * pstride;
    }
  }
  if (h.n_env != n || h.nstate != (uint32_t)wk::NSTATE || h.nparam != (uint32_t)wk::NPARAM || data.size() != need) {
    SETERR(c, "checkpoint '%s' is for %u walkers (context has %zu)", path, h.n_env, n);
    return WK_ERR_ARG;
  }
  if (h.seed != c->seed || h.env_offset != c->cfg.EnvOffset) {  // the Philox streams differ
    SETERR(c, "checkpoint '%s' was written with seed %llu / EnvOffset %d (context: %llu / %d)",
           path, (unsigned long long)h.seed, h.env_offset, (unsigned long long)c->seed, c->cfg.EnvOffset);
    return WK_ERR_CONFIG;
  }
  if (h.iterations != c->cfg.Iterations || h.max_timesteps != c->cfg.MaxTimesteps ||
      ext.rough_floor != c->cfg.RoughFloor) {
    SETERR(c, "checkpoint '%s' was written with Iterations %d / MaxTimesteps %d / RoughFloor %d "
              "(context: %d / %d / %d)", path, h.iterations, h.max_timesteps, ext.rough_floor,
           c->cfg.Iterations, c->cfg.MaxTimesteps, c->cfg.RoughFloor);
    return WK_ERR_CONFIG;
  }
  if (np > 0 && c->cfg.LanesPerWalker > 1) {  // wk_set_scene would refuse it
    SETERR(c, "checkpoint '%s' has scene props, which need the one-lane mapping "
              "(LanesPerWalker 0 or 1)", path);
    return WK_ERR_CONFIG;
  }
  {  // the walker records keep rigid template poles, checked before any write
    std::vector<float> rec(n * wk::NSTATE);
    memcpy(rec.data(), data.data() + sizeof h + ext_bytes + sizeof(float) * 3 * wk::NPARAM,
           sizeof(float) * rec.size());
    if (int r = check_state_or_fail(c, rec.data())) return r;
  }
  // the scene first: wk_set_scene is all-or-nothing and is the last step that can fail on
  // anything but a device error
  if (int r = wk_set_scene(c, desc.data(), (int)desc.size()); r != WK_OK) return r;
  const char* q = data.data() + sizeof h + ext_bytes;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(c->W, q, sizeof(float) * wk::NPARAM, hipMemcpyHostToDevice)); q += sizeof(float) * wk::NPARAM;
  HIPCHK(c, hipMemcpy(c->m, q, sizeof(float) * wk::NPARAM, hipMemcpyHostToDevice)); q += sizeof(float) * wk::NPARAM;
  HIPCHK(c, hipMemcpy(c->v, q, sizeof(float) * wk::NPARAM, hipMemcpyHostToDevice)); q += sizeof(float) * wk::NPARAM;
  HIPCHK(c, hipMemcpy(c->st, q, sizeof(float) * n * wk::NSTATE, hipMemcpyHostToDevice)); q += sizeof(float) * n * wk::NSTATE;
  HIPCHK(c, hipMemcpy(c->rng_t, q, sizeof(uint32_t) * n, hipMemcpyHostToDevice)); q += sizeof(uint32_t) * n;
  HIPCHK(c, hipMemcpy(c->dxoff, q, sizeof(float) * n, hipMemcpyHostToDevice));
  {
    std::vector<float> dxh(n);
    std::memcpy(dxh.data(), q, sizeof(float) * n);
    HIPCHK(c, rough_order_upload(c, dxh.data()));
  }
  q += sizeof(float) * n;
  HIPCHK(c, hipMemcpy(c->mat, q, sizeof(int32_t) * n, hipMemcpyHostToDevice)); q += sizeof(int32_t) * n;
  HIPCHK(c, hipMemcpy(c->ep_acc, q, sizeof(double) * n, hipMemcpyHostToDevice)); q += sizeof(double) * n;
  HIPCHK(c, hipMemcpy(c->ep_len, q, sizeof(int32_t) * n, hipMemcpyHostToDevice)); q += sizeof(int32_t) * n;
  if (np > 0) {
    q += sizeof(int32_t) + sizeof(wk_prop) * np;
    HIPCHK(c, hipMemcpy(c->props, q, sizeof(float) * n * c->scene.pstride, hipMemcpyHostToDevice));
  }
  c->adam_t = (int)h.adam_t;
  c->rollout_steps = h.rollout_steps;
  c->T_valid = 0;
  c->returns_valid = 0;
  HIPCHK(c, wk::launch_swizzle(c->W, c->Wz, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return WK_OK;
}


// ---------------- data collection ----------------
static_assert(sizeof(wk_episode_rec) == sizeof(wk::EpisodeRecDev), "episode record layout");

int wk_collect_data(wk_ctx* c, int on) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  c->collect = on ? 1 : 0;
  return WK_OK;
}

int wk_episode_log_count(wk_ctx* c, int64_t* episodes, int64_t* updates) {
  DevGuard dg_(c);
  if (!c) return WK_ERR_ARG;
  uint64_t cnt = 0;
  HIPCHK(c, hipMemcpyAsync(&cnt, c->ep_count, sizeof cnt, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (episodes) *episodes = (int64_t)cnt;
  if (updates) *updates = (int64_t)c->loss_count;
  return WK_OK;
}

int wk_episode_log_drain(wk_ctx* c, wk_episode_rec* out, int64_t cap, int64_t* n_out,
                         int64_t* dropped) {
  DevGuard dg_(c);
  if (!c || cap < 0 || (cap > 0 && !out)) return WK_ERR_ARG;
  uint64_t cnt = 0;
  HIPCHK(c, hipMemcpyAsync(&cnt, c->ep_count, sizeof cnt, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t kept = cnt < c->ep_cap ? cnt : c->ep_cap;
  if ((uint64_t)cap < kept) {
    SETERR(c, "episode log holds %llu records, buffer has room for %lld", (unsigned long long)kept, (long long)cap);
    return WK_ERR_ARG;
  }
  if (kept) HIPCHK(c, hipMemcpy(out, c->ep_log, sizeof(wk_episode_rec) * kept, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemsetAsync(c->ep_count, 0, sizeof(uint64_t), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (n_out) *n_out = (int64_t)kept;
  if (dropped) *dropped = (int64_t)(cnt - kept);
  return WK_OK;
}

int wk_loss_log_drain(wk_ctx* c, float* critic, float* actor, int64_t cap, int64_t* n_out,
                      int64_t* dropped) {
  DevGuard dg_(c);
  if (!c || cap < 0 || (cap > 0 && (!critic || !actor))) return WK_ERR_ARG;
  const uint64_t kept = c->loss_count < c->loss_cap ? c->loss_count : c->loss_cap;
  if ((uint64_t)cap < kept) {
    SETERR(c, "loss log holds %llu updates, buffer has room for %lld", (unsigned long long)kept, (long long)cap);
    return WK_ERR_ARG;
  }
  std::vector<float> buf(2 * kept);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (kept) HIPCHK(c, hipMemcpy(buf.data(), c->loss_log, sizeof(float) * 2 * kept, hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < kept; i++) {
    critic[i] = buf[2 * i];
    actor[i] = buf[2 * i + 1];
  }
  if (n_out) *n_out = (int64_t)kept;
  if (dropped) *dropped = (int64_t)(c->loss_count - kept);
  c->loss_count = 0;
  return WK_OK;
}

// ConsoleRenderer.CreateDataFile (ConsoleRenderer.cs:124-135): three space-joined float
// lists (float.ToString(), en-US) each followed by a "length N, <name>" line and a blank line
int wk_write_data_file(const char* path, const float* total_rewards, int64_t n_rewards,
                       const float* critic_losses, int64_t n_critic, const float* actor_losses,
                       int64_t n_actor) {
  if (!path || n_rewards < 0 || n_critic < 0 || n_actor < 0 ||
      (n_rewards && !total_rewards) || (n_critic && !critic_losses) || (n_actor && !actor_losses)) {
    g_create_error = "invalid argument";
    return WK_ERR_ARG;
  }
  std::string data;
  auto list = [&](const float* v, int64_t k, const char* name) {
    for (int64_t i = 0; i < k; i++) {
      if (i) data += ' ';
      data += wk::dotnet_float(v[i]);
    }
    data += "\nlength " + std::to_string(k) + ", " + name + "\n\n";
  };
  list(total_rewards, n_rewards, "total rewards");
  list(critic_losses, n_critic, "critic losses");
  list(actor_losses, n_actor, "actor losses");
  if (!write_file(path, data.data(), data.size())) {
    g_create_error = std::string("cannot write '") + path + "'";
    return WK_ERR_ARG;
  }
  return WK_OK;
}

}  // extern "C"
