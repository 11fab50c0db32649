/* orc_batch.c -- batched drivers over the single-walker oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The GPU parity tests at BASELINE's full shapes (8,192-walker shard, 4,096 walkers at
 * T_h = 64) replay tens of thousands of walkers for 64 env-steps each.  A ctypes call per
 * env-step costs more than the step, so these entry points loop in C, one independent
 * walker per OpenMP iteration (walkers never interact: Environment.cs:27,43-48).  Each
 * walker runs exactly orc_env_step (Environment.Update, Environment.cs:64-92) -- the same
 * code the per-step binding calls -- so the batch adds no arithmetic of its own. */
#include <stdlib.h>
#include <string.h>

#include "wk_oracle.h"

/* Replay n walkers for T env-steps with the given (unclipped) actions [T][n][4], starting
 * from the episode-0 template at offset dx[i] with material mat[i] (Environment ctor,
 * Environment.cs:39-51).  Outputs (each may be NULL): obs_before[T][n][12] (the state the
 * step's action was taken in, Environment.cs:73), reward[T][n], done[T][n], and the final
 * records dump[n][ORC_STATE_FLOATS].  Returns 0, or -1 on allocation failure. */
int orc_replay_batch(const orc_hyper* h, int n, int T, const float* dx, const int* mat,
                     const float* actions, float* obs_before, float* reward, uint8_t* done,
                     float* dump) {
  int fail = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(| : fail)
  for (int i = 0; i < n; i++) {
    orc_env* e = orc_env_create(h, dx ? dx[i] : 0.0f, mat ? mat[i] : 0);
    if (!e) { fail |= 1; continue; }
    for (int t = 0; t < T; t++) {
      const size_t r = (size_t)t * n + i;
      if (obs_before) orc_env_get_obs(e, obs_before + r * 12);
      float o[12], rw;
      int d;
      orc_env_step(e, actions + r * 4, o, &rw, &d, NULL);
      if (reward) reward[r] = rw;
      if (done) done[r] = (uint8_t)d;
    }
    if (dump) orc_env_dump(e, dump + (size_t)i * ORC_STATE_FLOATS);
    orc_env_destroy(e);
  }
  return fail ? -1 : 0;
}

/* orc_perm for i = 0..count-1 (CreateBatches' sampling order, PPOAgent.cs:501-540) */
void orc_perm_batch(uint32_t count, uint32_t n, const uint32_t key[4], uint32_t* out) {
#pragma omp parallel for schedule(static)
  for (uint32_t i = 0; i < count; i++) out[i] = orc_perm(i, n, key);
}

/* the per-walker offsets / materials of RandomizeStart / RandomizeMaterial for walkers
 * first .. first+n-1 */
void orc_env_setup_batch(uint64_t seed, int first, int n, float* dx, int* mat) {
  for (int i = 0; i < n; i++) {
    if (dx) dx[i] = orc_env_offset(seed, first + i);
    if (mat) mat[i] = orc_env_material(seed, first + i);
  }
}
