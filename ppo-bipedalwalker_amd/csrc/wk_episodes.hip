// wk_episodes.hip -- data collection: per-episode total rewards.
//
// The reference adds trajectory.Rewards.Sum() to ConsoleRenderer's list once per episode
// (PPOAgent.Train PPOAgent.cs:151 -> ConsoleRenderer.AddTotalEpisodeReward :79-82);
// Enumerable.Sum over float accumulates in double and rounds once.  Here every rollout's
// [T][n] reward / done rows are scanned after the physics kernel:
//   k_episode_scan    one lane per walker, t = 0..T-1: acc += (double) r; on done the
//                     (float) total and the length go to a sparse [T][n] scratch, and
//                     each wave adds its done count for row t to row_cnt[t]
//                     (ballot + popcount, one atomic per wave and row: integer, so the
//                     result is order-independent);
//   k_episode_compact one block per row t: the row's done walkers in env order are
//                     written to the log at log_count + sum(row_cnt[< t]) -- the log is in
//                     (env-step, env) order, i.e. completion order, deterministically;
//   k_episode_commit  one lane: log_count += sum(row_cnt), row_cnt = 0.
// Traffic: 5 B per env-step read (reward + done), ~16 B per finished episode written --
// ~5 % of the rollout's 112 B per env-step, in three launches of a few microseconds.
#include <hip/hip_runtime.h>

#include "wk_kernels.h"

namespace wk {

namespace {
constexpr int SCAN_BLOCK = 256;
constexpr int COMPACT_BLOCK = 1024;
}  // namespace

__global__ __launch_bounds__(SCAN_BLOCK) void k_episode_scan(
    int n, int T, const float* __restrict__ r, const uint8_t* __restrict__ d,
    double* __restrict__ acc, int32_t* __restrict__ len, float2* __restrict__ scratch,
    uint32_t* __restrict__ row_cnt) {
  const int e = blockIdx.x * SCAN_BLOCK + threadIdx.x;
  const bool live = e < n;
  double a = live ? acc[e] : 0.0;
  int l = live ? len[e] : 0;
  for (int t = 0; t < T; t++) {
    const size_t i = (size_t)t * n + e;
    const bool done = live && d[i] != 0;
    if (live) {
      a += (double)r[i];
      l++;
    }
    if (done) {
      scratch[i] = make_float2((float)a, __int_as_float(l));
      a = 0.0;
      l = 0;
    }
    const uint64_t b = __ballot(done);
    if (b && (threadIdx.x & 63) == 0) atomicAdd(&row_cnt[t], (uint32_t)__popcll(b));
  }
  if (live) {
    acc[e] = a;
    len[e] = l;
  }
}

__global__ __launch_bounds__(COMPACT_BLOCK) void k_episode_compact(
    int n, int T, int env_offset, uint32_t step0, const uint8_t* __restrict__ d,
    const float2* __restrict__ scratch, const uint32_t* __restrict__ row_cnt,
    const uint64_t* __restrict__ log_count, uint64_t cap, EpisodeRecDev* __restrict__ log) {
  __shared__ uint32_t wave_sum[COMPACT_BLOCK / 64];
  __shared__ uint64_t base_s;
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    uint64_t b = *log_count;
    for (int k = 0; k < t; k++) b += row_cnt[k];
    base_s = b;
  }
  __syncthreads();
  uint64_t base = base_s;
  for (int e0 = 0; e0 < n; e0 += COMPACT_BLOCK) {
    const int e = e0 + threadIdx.x;
    const size_t i = (size_t)t * n + e;
    const bool done = e < n && d[i] != 0;
    const uint64_t b = __ballot(done);
    if (lane == 0) wave_sum[wave] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (int w = 0; w < COMPACT_BLOCK / 64; w++) {
      before += w < wave ? wave_sum[w] : 0u;
      total += wave_sum[w];
    }
    const uint32_t in_wave = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
    if (done) {
      const uint64_t slot = base + before + in_wave;
      if (slot < cap) {
        const float2 s = scratch[i];
        EpisodeRecDev rec;
        rec.total_reward = s.x;
        rec.env = env_offset + e;
        rec.length = __float_as_int(s.y);
        rec.step = step0 + (uint32_t)t;
        log[slot] = rec;
      }
    }
    base += total;
    __syncthreads();  // wave_sum is rewritten by the next chunk
  }
}

__global__ void k_episode_commit(int T, uint32_t* __restrict__ row_cnt,
                                 uint64_t* __restrict__ log_count) {
  if (threadIdx.x != 0) return;
  uint64_t s = 0;
  for (int t = 0; t < T; t++) {
    s += row_cnt[t];
    row_cnt[t] = 0;
  }
  *log_count += s;
}

__global__ void k_episode_reset(int n, const uint8_t* __restrict__ mask, double* __restrict__ acc,
                                int32_t* __restrict__ len) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n && (!mask || mask[e])) {
    acc[e] = 0.0;
    len[e] = 0;
  }
}

hipError_t launch_episode_log(const EpisodeArgs& a, hipStream_t s) {
  if (a.n <= 0 || a.T <= 0) return hipSuccess;
  k_episode_scan<<<(a.n + SCAN_BLOCK - 1) / SCAN_BLOCK, SCAN_BLOCK, 0, s>>>(
      a.n, a.T, a.rewards, a.dones, a.acc, a.len, a.scratch, a.row_cnt);
  k_episode_compact<<<a.T, COMPACT_BLOCK, 0, s>>>(a.n, a.T, a.env_offset, a.step0, a.dones,
                                                  a.scratch, a.row_cnt, a.log_count, a.cap,
                                                  a.log);
  k_episode_commit<<<1, 64, 0, s>>>(a.T, a.row_cnt, a.log_count);
  return hipGetLastError();
}

hipError_t launch_episode_reset(int n, const uint8_t* mask, double* acc, int32_t* len,
                                hipStream_t s) {
  k_episode_reset<<<(n + 255) / 256, 256, 0, s>>>(n, mask, acc, len);
  return hipGetLastError();
}

}  // namespace wk
