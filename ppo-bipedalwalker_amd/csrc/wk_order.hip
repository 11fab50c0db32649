// wk_order.hip -- lane order of the walkers for the split physics kernels (k_env_side).
//
// A walker's RigidBody.Step calls visit a leg segment's two candidate pairs in list order
// (Bodies/RigidBody.cs:66-96): the floor LAST in episode 0 (the floor is created after the
// walker, Environment.cs:43-48) and FIRST after any reset (Walker.RemoveRigidObjects /
// CreateCreature re-append the walker behind the floor, Walker.cs:212-234).  The kernel runs
// three pair slots per segment -- [floor if post-reset], other segment, [floor if episode 0] --
// so a wave that holds both kinds of walker runs the leg-floor resolution (SAT, contact
// clipping, impulses) twice per segment, each time for a few of its lanes.  In the bench's
// regime ~2.5 % of the walkers are still in their first episode, which leaves about half of the
// 32-walker waves mixed.  Before every launch the lanes are reordered so that the m episode-0
// walkers occupy the LAST m lane slots: every episode-0 walker found in the head (slots
// [0, n - m)) trades places with a post-reset walker found in the tail, in rank order, and every
// other walker keeps its own slot.  So all but one wave at the boundary are uniform, and a wave
// still stores its walkers' trajectory rows as aligned contiguous runs (a full stable partition
// shifted every wave off the 128-B lines: +32 % written bytes).  The 65,536-walker rollout went
// from 48.9 to 44.2 ms.  Every walker's arithmetic is unchanged (its Philox stream, record and
// trajectory rows are keyed by its walker id; the policy's matrix-core sums run per walker), so
// the results are bit-identical to the identity order (tests/test_gpu_order.py).  Not used for
// the quad mapping on the rough floor (wk_api.cpp launch_physics: there the launch is as long as
// its slowest wave, and gathering the few long-lived episode-0 walkers into one wave made it the
// slowest).
//
//   k_order_count  one 1,024-lane block per tile of 1,024 slots: episode-0 walkers per tile
//   k_order_ranks  the same tiles: order[s] = s; the head's episode-0 slots go to hpos[rank],
//                  the tail's post-reset slots to tpos[rank] (ranks from tile counts + ballots)
//   k_order_swap   rank r: order[hpos[r]] = tpos[r], order[tpos[r]] = hpos[r]
#include <hip/hip_runtime.h>

#include "wk_kernels.h"

namespace wk {

namespace {
constexpr int OB = 1024, NW = OB / 64;
__device__ inline bool episode0(const float* __restrict__ st, int e) {
  return st[(size_t)e * NSTATE + S_POSTRESET] == 0.0f;
}
// episode-0 walkers among the tile's slots below `upto` (block-wide; every thread returns it)
__device__ uint32_t tile_count_below(const float* __restrict__ st, int n, int tile, int upto,
                                     uint32_t* ws) {
  const int e = tile * OB + threadIdx.x;
  const uint64_t b = __ballot(e < n && e < upto && episode0(st, e));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = (uint32_t)__popcll(b);
  __syncthreads();
  uint32_t s = 0;
  for (int w = 0; w < NW; w++) s += ws[w];
  return s;
}
}  // namespace

__global__ __launch_bounds__(OB) void k_order_count(const float* __restrict__ st, int n,
                                                   uint32_t* __restrict__ cnt) {
  __shared__ uint32_t ws[NW];
  const uint32_t s = tile_count_below(st, n, blockIdx.x, n, ws);
  if (threadIdx.x == 0) cnt[blockIdx.x] = s;
}

__global__ __launch_bounds__(OB) void k_order_ranks(const float* __restrict__ st, int n,
                                                   uint32_t* __restrict__ cnt, int tiles,
                                                   int32_t* __restrict__ order,
                                                   int32_t* __restrict__ hpos,
                                                   int32_t* __restrict__ tpos) {
  __shared__ uint32_t ws[NW];
  __shared__ uint32_t before_s, total_s, bt_before_s;
  if (threadIdx.x < 64) {  // episode-0 walkers in earlier tiles / all tiles / tiles before b's
    uint32_t a = 0, t = 0;
    for (int i = threadIdx.x; i < tiles; i += 64) {
      const uint32_t c = cnt[i];
      t += c;
      a += i < (int)blockIdx.x ? c : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) {
      a += (uint32_t)__shfl_xor((int)a, o);
      t += (uint32_t)__shfl_xor((int)t, o);
    }
    uint32_t bb = 0;  // (second pass: needs the total for b)
    const int btile = (n - (int)t) / OB;
    for (int i = threadIdx.x; i < btile; i += 64) bb += cnt[i];
    for (int o = 32; o > 0; o >>= 1) bb += (uint32_t)__shfl_xor((int)bb, o);
    if (threadIdx.x == 0) { before_s = a; total_s = t; bt_before_s = bb; }
  }
  __syncthreads();
  const int m = (int)total_s, b = n - m;  // tail = the last m slots
  // episode-0 walkers in slots [0, b): the tiles before b's tile plus b's tile below b
  const uint32_t head0 = bt_before_s + tile_count_below(st, n, b / OB, b, ws);
  const int s = blockIdx.x * OB + threadIdx.x;
  const bool z = s < n && episode0(st, s);
  const uint64_t bal = __ballot(z);
  const uint64_t lt = (threadIdx.x & 63) ? (~0ull >> (64 - (threadIdx.x & 63))) : 0ull;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = (uint32_t)__popcll(bal);
  __syncthreads();
  uint32_t r = (uint32_t)__popcll(bal & lt);
  for (int w = 0; w < (int)(threadIdx.x >> 6); w++) r += ws[w];
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[tiles] = head0;  // the swap count (k_order_swap)
  if (s >= n) return;
  order[s] = s;
  const uint32_t ep0_before = before_s + r;  // episode-0 walkers in slots [0, s)
  if (s < b && z) hpos[ep0_before] = s;
  if (s >= b && !z) tpos[(uint32_t)(s - b) - (ep0_before - head0)] = s;
}

__global__ void k_order_swap(const uint32_t* __restrict__ cnt, int tiles, int32_t* __restrict__ order,
                             const int32_t* __restrict__ hpos, const int32_t* __restrict__ tpos) {
  const uint32_t k = cnt[tiles];  // episode-0 walkers in the head = post-reset ones in the tail
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < k; r += gridDim.x * blockDim.x) {
    const int h = hpos[r], t = tpos[r];
    order[h] = t;
    order[t] = h;
  }
}

int order_tiles(int n) { return (n + OB - 1) / OB; }
int order_cells(int n) { return order_tiles(n) + 1; }

hipError_t launch_walker_order(const float* st, int n, uint32_t* cnt, int32_t* order,
                               int32_t* scratch, hipStream_t s) {
  const int tiles = order_tiles(n);
  int32_t* hpos = scratch;
  int32_t* tpos = scratch + n;
  hipLaunchKernelGGL(k_order_count, dim3(tiles), dim3(OB), 0, s, st, n, cnt);
  hipLaunchKernelGGL(k_order_ranks, dim3(tiles), dim3(OB), 0, s, st, n, cnt, tiles, order, hpos, tpos);
  hipLaunchKernelGGL(k_order_swap, dim3(16), dim3(256), 0, s, cnt, tiles, order, hpos, tpos);
  return hipGetLastError();
}

}  // namespace wk
