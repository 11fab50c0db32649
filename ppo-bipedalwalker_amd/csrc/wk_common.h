// wk_common.h -- host/device shared definitions for the MI355X walker engine.
//
// Counter-based RNG replacing the reference's unseeded System.Random
// (Walker/PPO/Matrix.cs:68,544; PPOAgent.cs:149): Philox4x32-10, keyed by the run
// seed and addressed by (global env id, env-step, dimension, stream), so every lane
// draws its own numbers with no state and results do not depend on the GPU count.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define WK_HD __host__ __device__ __forceinline__

namespace wk {

enum Stream : uint32_t { ST_OFFSET = 1, ST_MAT = 2, ST_ACT = 3, ST_SYNTH = 4, ST_XAVIER = 5, ST_PERM = 6, ST_TERRAIN = 7 };

// canonical state layout (include/wk_api.h WK_STATE_FLOATS)
enum : int {
  NB = 5, LLL = 0, LLU = 1, BODY = 2, RLL = 3, RLU = 4,
  BSTRIDE = 20, F_CX = 12, F_CY = 13, F_VX = 14, F_VY = 15, F_W = 16, F_TH = 17, F_COL = 18,
  S_TORQUE = 100, S_POS = 104, S_PREV = 106, S_STEPS = 108, S_POSTRESET = 109,
  S_TERMINAL = 110, S_EPISODES = 111, NSTATE = 112,
  NPARAM_CRITIC = 897, NPARAM_ACTOR = 5252, NPARAM = 6149
};

// flat parameter offsets (critic then actor; each dense layer W then B)
enum : int {
  OFF_C_W1 = 0, OFF_C_B1 = 768, OFF_C_W2 = 832, OFF_C_B2 = 896,
  OFF_A_W1 = 897, OFF_A_B1 = 897 + 768, OFF_A_W2 = 897 + 832, OFF_A_B2 = 897 + 832 + 4096,
  OFF_A_W3 = 897 + 832 + 4096 + 64, OFF_A_B3 = 897 + 832 + 4096 + 64 + 256
};
static_assert(OFF_A_B3 + 4 == NPARAM, "param layout");

struct U4 { uint32_t x, y, z, w; };

WK_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

WK_HD U4 philox(uint64_t key, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
  for (int r = 0; r < 10; r++) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return U4{c0, c1, c2, c3};
}

// (float)Random.NextDouble(): 53-bit double in [0,1) rounded to float
WK_HD float next_double_f(uint32_t a, uint32_t b) {
  double d = ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
  return (float)d;
}

WK_HD float env_offset(uint64_t seed, uint32_t env) {
  U4 o = philox(seed, env, 0, 0, ST_OFFSET);
  return 200.0f * next_double_f(o.x, o.y);
}

WK_HD int env_material(uint64_t seed, uint32_t env) {
  U4 o = philox(seed, env, 0, 0, ST_MAT);
  float u = next_double_f(o.x, o.y);
  int k = (int)(3.0f * u);
  if (k > 2) k = 2;
  return k == 0 ? 1 /*Ice*/ : (k == 1 ? 2 /*Rubber*/ : 0 /*Carpet*/);
}

// Random.Next(0, roughness = 100) of CreateRoughFloor (Environment.cs:230-261): System.Random
// returns (int)(Sample() * range) + min with a double Sample().  Draw 0 is the first
// previousVector's height, draws 1..10 the segments'; per-walker Philox terrain replaces
// the unseeded Random (:242).
WK_HD int terrain_draw(uint64_t seed, uint32_t env, int i) {
  U4 o = philox(seed, env, (uint32_t)i, 0, ST_TERRAIN);
  double d = ((double)(o.x >> 5) * 67108864.0 + (double)(o.y >> 6)) * (1.0 / 9007199254740992.0);
  return (int)(d * 100.0);
}

WK_HD float synth_u(uint32_t w) { return (float)(w >> 8) * (1.0f / 16777216.0f); }

// keyed random permutation of [0,n): 4-round Feistel + cycle walking (minibatch
// sampling without replacement, PPOAgent.cs:501-540)
WK_HD uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

struct PermKey { uint32_t k[4]; uint32_t h, mask, n; };

WK_HD PermKey perm_key(uint64_t seed, uint32_t update, uint32_t epoch, uint32_t n) {
  U4 o = philox(seed, update, epoch, 0, ST_PERM);
  PermKey p;
  p.k[0] = o.x; p.k[1] = o.y; p.k[2] = o.z; p.k[3] = o.w;
  uint32_t bits = 2;
  while ((1u << bits) < n) bits++;
  if (bits & 1) bits++;
  p.h = bits / 2;
  p.mask = (1u << p.h) - 1u;
  p.n = n;
  return p;
}

WK_HD uint32_t perm_apply(uint32_t i, const PermKey& p) {
  uint32_t x = i;
  do {
    uint32_t L = x >> p.h, R = x & p.mask;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      uint32_t nL = R;
      uint32_t nR = L ^ (mix32(R ^ p.k[r]) & p.mask);
      L = nL; R = nR;
    }
    x = (L << p.h) | R;
  } while (x >= p.n);
  return x;
}

// Materials/<Name>.cs: inverse mass, restitution, friction
struct MatConst { float inv_mass, restitution, friction; };
WK_HD MatConst material(int id) {
  switch (id) {
    case 1: return MatConst{11.0f, 0.3f, 0.0f};   // Ice
    case 2: return MatConst{11.0f, 0.7f, 0.5f};   // Rubber
    case 3: return MatConst{15.0f, 0.3f, 1.0f};   // Metal
    case 4: return MatConst{20.0f, 0.3f, 0.01f};  // Wood
    case 5: return MatConst{1.0f, 0.3f, 0.1f};    // Paper
    case 6: return MatConst{0.01f, 0.1f, 0.2f};   // Titanium
    case 7: return MatConst{11.0f, 1.0f, 1.0f};   // SuperRubber
    default: return MatConst{5.0f, 0.3f, 0.8f};   // Carpet
  }
}

// kernel parameter blocks
struct EnvParams {
  int n_env;
  int iterations;
  int max_timesteps;
  float dt_frame;       // DeltaTime
  float dt_sub;         // DeltaTime / Iterations (float division, Environment.cs:128)
  float log_std;
  float std_;           // MathF.Exp(LogStandardDeviation)
  uint64_t seed;
  int env_offset;
  int lanes;            // lanes per walker in the env-step kernel (1, 2 or 16)
  int rough;            // Hyperparameters.RoughFloor: 10 static floor segments
  int wpw;              // quad mapping: walkers per wave (16; fewer, down to 1, at small n)
};

}  // namespace wk
