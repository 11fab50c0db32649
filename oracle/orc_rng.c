/*
 * orc_rng.c -- seeded replacements for the reference's unseeded System.Random.
 * TEST INFRASTRUCTURE ONLY (see wk_oracle.h).
 *
 * The reference draws from `new Random()` (Matrix.cs:68,544, PPOAgent.cs:149,
 * Environment.cs:242).  Parity needs a seeded, counter-based generator that the GPU
 * path can evaluate per env without state: Philox4x32-10 (Salmon et al., SC'11).
 * (float)Random.NextDouble() (NormalDistribution.cs:14-15) is restated as a 53-bit
 * double in [0,1) rounded to float.
 */
#include "wk_oracle.h"
#include <math.h>

enum { ST_OFFSET = 1, ST_MAT = 2, ST_ACT = 3, ST_SYNTH = 4, ST_XAVIER = 5, ST_PERM = 6, ST_TERRAIN = 7 };

static inline uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

void orc_philox(uint64_t key, const uint32_t ctr[4], uint32_t out[4]) {
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  for (int r = 0; r < 10; r++) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c0, &hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, &hi1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* (float)NextDouble(): 53-bit double in [0,1), rounded to float (may round to 1.0f,
 * exactly like the reference's cast). */
static inline float next_double_f(uint32_t a, uint32_t b) {
  double d = ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
  return (float)d;
}

float orc_uniform_f(uint64_t key, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, int which) {
  uint32_t ctr[4] = {c0, c1, c2, c3}, o[4];
  orc_philox(key, ctr, o);
  return which ? next_double_f(o[2], o[3]) : next_double_f(o[0], o[1]);
}

float orc_env_offset(uint64_t seed, int env) {
  return 200.0f * orc_uniform_f(seed, (uint32_t)env, 0, 0, ST_OFFSET, 0);
}

/* Random.Next(0, roughness) (System.Random: (int)(Sample() * range) + min, in double) for
 * CreateRoughFloor (Environment.cs:230-261): draw i = 0 is the first previousVector, draws
 * 1..10 the segment heights.  Per-env Philox terrain replaces the unseeded Random (:242). */
int orc_terrain_draw(uint64_t seed, int env, int i) {
  uint32_t ctr[4] = {(uint32_t)env, (uint32_t)i, 0, ST_TERRAIN}, o[4];
  orc_philox(seed, ctr, o);
  double d = ((double)(o[0] >> 5) * 67108864.0 + (double)(o[1] >> 6)) * (1.0 / 9007199254740992.0);
  return (int)(d * 100.0);
}

int orc_env_material(uint64_t seed, int env) {
  float u = orc_uniform_f(seed, (uint32_t)env, 0, 0, ST_MAT, 0);
  int k = (int)(3.0f * u);
  if (k > 2) k = 2;
  static const int map[3] = {ORC_MAT_ICE, ORC_MAT_RUBBER, ORC_MAT_CARPET};
  return map[k];
}

void orc_synth_action(uint64_t seed, int env, uint32_t t, float a[4]) {
  uint32_t ctr[4] = {(uint32_t)env, t, 0, ST_SYNTH}, o[4];
  orc_philox(seed, ctr, o);
  for (int j = 0; j < 4; j++) {
    float u = (float)(o[j] >> 8) * (1.0f / 16777216.0f);
    a[j] = 2.0f * u - 1.0f;
  }
}

/* Box-Muller draw for dimension d of env-step (env, t): NormalDistribution.cs:12-19 */
void orc_noise_uniforms(uint64_t seed, int env, uint32_t t, int d, float* u1, float* u2) {
  uint32_t ctr[4] = {(uint32_t)env, t, (uint32_t)d, ST_ACT}, o[4];
  orc_philox(seed, ctr, o);
  *u1 = next_double_f(o[0], o[1]);
  *u2 = next_double_f(o[2], o[3]);
}

void orc_xavier_uniforms(uint64_t seed, int layer, int k, float* u1, float* u2) {
  uint32_t ctr[4] = {(uint32_t)k, (uint32_t)layer, 0, ST_XAVIER}, o[4];
  orc_philox(seed, ctr, o);
  *u1 = next_double_f(o[0], o[1]);
  *u2 = next_double_f(o[2], o[3]);
}

/* ---- minibatch sampling without replacement (PPOAgent.cs:501-540) ----
 * The reference draws random.Next(0, remaining) and RemoveAt; restated as a keyed
 * random permutation of the pool (4-round Feistel network + cycle walking), so that
 * minibatch j of an epoch is {perm(j*B + k) : k < B} and the remainder beyond
 * floor(T/B)*B is dropped as in the reference. */
void orc_perm_key(uint64_t seed, uint32_t update, uint32_t epoch, uint32_t key[4]) {
  uint32_t ctr[4] = {update, epoch, 0, ST_PERM};
  orc_philox(seed, ctr, key);
}

static inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

uint32_t orc_perm(uint32_t i, uint32_t n, const uint32_t key[4]) {
  uint32_t bits = 2;
  while ((1u << bits) < n) bits++;
  if (bits & 1) bits++;
  uint32_t h = bits / 2, mask = (1u << h) - 1u;
  uint32_t x = i;
  do {
    uint32_t L = x >> h, R = x & mask;
    for (int r = 0; r < 4; r++) {
      uint32_t nL = R;
      uint32_t nR = L ^ (mix32(R ^ key[r]) & mask);
      L = nL; R = nR;
    }
    x = (L << h) | R;
  } while (x >= n);
  return x;
}
