// wk_episodes.hip -- data collection: per-episode total rewards.
//
// The reference adds trajectory.Rewards.Sum() to ConsoleRenderer's list once per episode
// (PPOAgent.Train PPOAgent.cs:151 -> ConsoleRenderer.AddTotalEpisodeReward :79-82);
// Enumerable.Sum over float accumulates in double and rounds once.  Here every rollout's
// [T][n] reward / done rows are scanned after the physics kernel:
//   k_episode_scan    one lane per walker, t = 0..T-1: acc += (double) r; on done the
//                     (float) total and the length go to a sparse [T][n] scratch, and
//                     each wave adds its done count to cnt[t][tile] (4,096-walker tiles;
//                     ballot + popcount, one atomic per wave and row: integer, so the
//                     result is order-independent);
//   k_episode_compact one block per (tile, row t): the cell's done walkers in env order
//                     are written to the log at log_count + (episodes of all earlier
//                     cells) -- the log is in (env-step, env) order, i.e. completion
//                     order, deterministically;
//   k_episode_commit  one block: log_count += sum(cnt), cnt = 0.
// Traffic: 5 B per env-step read (reward + done), ~16 B per finished episode written --
// ~5 % of the rollout's 112 B per env-step, in three launches of a few microseconds.
#include <hip/hip_runtime.h>

#include "wk_kernels.h"

namespace wk {

namespace {
constexpr int SCAN_BLOCK = 256;
constexpr int COMPACT_BLOCK = 1024;
constexpr int TILE = 4096;  // walkers per compaction tile (a multiple of the 64-lane wave)
__host__ __device__ inline int tiles_of(int n) { return (n + TILE - 1) / TILE; }

// exclusive-prefix helper: sum of cnt[0 .. upto) over the whole block
__device__ uint64_t block_prefix(const uint32_t* __restrict__ cnt, int upto, uint64_t* red) {
  uint64_t v = 0;
  for (int i = threadIdx.x; i < upto; i += COMPACT_BLOCK) v += cnt[i];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t s = 0;
  for (int w = 0; w < COMPACT_BLOCK / 64; w++) s += red[w];
  __syncthreads();
  return s;
}
}  // namespace

__global__ __launch_bounds__(SCAN_BLOCK) void k_episode_scan(
    int n, int T, const float* __restrict__ r, const uint8_t* __restrict__ d,
    double* __restrict__ acc, int32_t* __restrict__ len, float2* __restrict__ scratch,
    uint32_t* __restrict__ cnt) {
  const int e = blockIdx.x * SCAN_BLOCK + threadIdx.x;
  const bool live = e < n;
  const int tiles = tiles_of(n), tile = e / TILE;
  double a = live ? acc[e] : 0.0;
  int l = live ? len[e] : 0;
  constexpr int CH = 16;  // rows loaded ahead: the loads are independent of the scan
  for (int t0 = 0; t0 < T; t0 += CH) {
    float rv[CH];
    bool dv[CH];
#pragma unroll
    for (int k = 0; k < CH; k++) {
      const size_t i = (size_t)(t0 + k) * n + e;
      const bool in = live && t0 + k < T;
      rv[k] = in ? r[i] : 0.0f;
      dv[k] = in && d[i] != 0;
    }
#pragma unroll
    for (int k = 0; k < CH; k++) {
      const int t = t0 + k;
      if (t >= T) continue;  // uniform: T is the same for every lane
      if (live) {
        a += (double)rv[k];
        l++;
      }
      if (dv[k]) {
        scratch[(size_t)t * n + e] = make_float2((float)a, __int_as_float(l));
        a = 0.0;
        l = 0;
      }
      const uint64_t b = __ballot(dv[k]);
      if (b && (threadIdx.x & 63) == 0) atomicAdd(&cnt[t * tiles + tile], (uint32_t)__popcll(b));
    }
  }
  if (live) {
    acc[e] = a;
    len[e] = l;
  }
}

// block (tile, t): the done walkers of row t inside the tile, in walker order, go to
// log[count + (episodes of all earlier (row, tile) cells)]
__global__ __launch_bounds__(COMPACT_BLOCK) void k_episode_compact(
    int n, int env_offset, uint32_t step0, const uint8_t* __restrict__ d,
    const float2* __restrict__ scratch, const uint32_t* __restrict__ cnt,
    const uint64_t* __restrict__ log_count, uint64_t cap, EpisodeRecDev* __restrict__ log) {
  __shared__ uint32_t wave_sum[COMPACT_BLOCK / 64];
  __shared__ uint64_t red[COMPACT_BLOCK / 64];
  const int tile = blockIdx.x, t = blockIdx.y, tiles = gridDim.x;
  const int cell = t * tiles + tile;
  if (cnt[cell] == 0) return;  // uniform across the block
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t base = *log_count + block_prefix(cnt, cell, red);
  const int e_end = min(n, (tile + 1) * TILE);
  for (int e0 = tile * TILE; e0 < e_end; e0 += COMPACT_BLOCK) {
    const int e = e0 + threadIdx.x;
    const size_t i = (size_t)t * n + e;
    const bool done = e < e_end && d[i] != 0;
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

__global__ __launch_bounds__(COMPACT_BLOCK) void k_episode_commit(int cells, uint32_t* __restrict__ cnt,
                                                                  uint64_t* __restrict__ log_count) {
  __shared__ uint64_t red[COMPACT_BLOCK / 64];
  const uint64_t s = block_prefix(cnt, cells, red);
  for (int i = threadIdx.x; i < cells; i += COMPACT_BLOCK) cnt[i] = 0;
  if (threadIdx.x == 0) *log_count += s;
}

__global__ void k_episode_reset(int n, const uint8_t* __restrict__ mask, double* __restrict__ acc,
                                int32_t* __restrict__ len) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n && (!mask || mask[e])) {
    acc[e] = 0.0;
    len[e] = 0;
  }
}

int episode_count_cells(int n, int T) { return T * tiles_of(n); }

hipError_t launch_episode_log(const EpisodeArgs& a, hipStream_t s) {
  if (a.n <= 0 || a.T <= 0) return hipSuccess;
  const int tiles = tiles_of(a.n);
  k_episode_scan<<<(a.n + SCAN_BLOCK - 1) / SCAN_BLOCK, SCAN_BLOCK, 0, s>>>(
      a.n, a.T, a.rewards, a.dones, a.acc, a.len, a.scratch, a.row_cnt);
  k_episode_compact<<<dim3(tiles, a.T), COMPACT_BLOCK, 0, s>>>(
      a.n, a.env_offset, a.step0, a.dones, a.scratch, a.row_cnt, a.log_count, a.cap, a.log);
  k_episode_commit<<<1, COMPACT_BLOCK, 0, s>>>(a.T * tiles, a.row_cnt, a.log_count);
  return hipGetLastError();
}

hipError_t launch_episode_reset(int n, const uint8_t* mask, double* acc, int32_t* len,
                                hipStream_t s) {
  k_episode_reset<<<(n + 255) / 256, 256, 0, s>>>(n, mask, acc, len);
  return hipGetLastError();
}

}  // namespace wk
