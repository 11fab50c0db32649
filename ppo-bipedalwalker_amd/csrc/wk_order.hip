// wk_order.hip -- lane order of the walkers for the split physics kernels (k_env_side).
//
// A walker's RigidBody.Step calls visit a leg segment's two candidate pairs in list order
// (Bodies/RigidBody.cs:66-96): the floor LAST in episode 0 (the floor is created after the
// walker, Environment.cs:43-48) and FIRST after any reset (Walker.RemoveRigidObjects /
// CreateCreature re-append the walker behind the floor, Walker.cs:212-234).  The kernel runs
// three pair slots per segment -- [floor if post-reset], other segment, [floor if episode 0] --
// so a wave that holds both kinds of walker runs the leg-floor resolution (SAT, contact
// clipping, impulses) twice per segment, each time for a few of its lanes.  With the bench's
// regime about one walker in ten is still in its first episode, so nearly every 32-walker wave
// is mixed.  Ordering the lanes so that the episode-0 walkers come first (a stable partition
// on the post-reset flag, recomputed before every launch) makes all but a few waves uniform.
// Every walker's arithmetic is unchanged (its Philox stream, record and trajectory rows are
// keyed by its walker id; the policy's matrix-core sums run per walker), so the results are
// bit-identical to the identity order.
//
//   k_order_count    one 1,024-lane block per tile of 1,024 walkers: episode-0 walkers per tile
//   k_order_scatter  the same tiles: order[slot] = walker, episode-0 walkers first, each group
//                    in walker order (tile offsets from the counts, in-tile ballot prefixes)
#include <hip/hip_runtime.h>

#include "wk_kernels.h"

namespace wk {

namespace {
constexpr int OB = 1024;
__device__ inline bool episode0(const float* __restrict__ st, int e) {
  return st[(size_t)e * NSTATE + S_POSTRESET] == 0.0f;
}
}  // namespace

__global__ __launch_bounds__(OB) void k_order_count(const float* __restrict__ st, int n,
                                                   uint32_t* __restrict__ cnt) {
  __shared__ uint32_t ws[OB / 64];
  const int e = blockIdx.x * OB + threadIdx.x;
  const uint64_t b = __ballot(e < n && episode0(st, e));
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = (uint32_t)__popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < OB / 64; w++) s += ws[w];
    cnt[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(OB) void k_order_scatter(const float* __restrict__ st, int n,
                                                     const uint32_t* __restrict__ cnt, int tiles,
                                                     int32_t* __restrict__ order) {
  __shared__ uint32_t ws[OB / 64];
  __shared__ uint32_t before0, total0;
  if (threadIdx.x < 64) {  // episode-0 walkers in earlier tiles and in all tiles (wave 0)
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
    if (threadIdx.x == 0) { before0 = a; total0 = t; }
  }
  const int e = blockIdx.x * OB + threadIdx.x;
  const bool live = e < n;
  const bool z = live && episode0(st, e);
  const uint64_t b = __ballot(z);
  const uint64_t lt = (threadIdx.x & 63) ? (~0ull >> (64 - (threadIdx.x & 63))) : 0ull;
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = (uint32_t)__popcll(b);
  __syncthreads();
  uint32_t wave0 = 0;  // episode-0 walkers of earlier waves of this tile
  for (int w = 0; w < (int)(threadIdx.x >> 6); w++) wave0 += ws[w];
  const uint32_t r0 = wave0 + (uint32_t)__popcll(b & lt);  // rank among the tile's episode-0
  if (!live) return;
  const uint32_t tile0 = (uint32_t)blockIdx.x * OB;
  // post-reset walkers before this one: the walkers before it minus the episode-0 ones
  const uint32_t slot = z ? before0 + r0
                          : total0 + (tile0 - before0) + ((uint32_t)threadIdx.x - r0);
  order[slot] = e;
}

int order_tiles(int n) { return (n + OB - 1) / OB; }

hipError_t launch_walker_order(const float* st, int n, uint32_t* cnt, int32_t* order,
                               hipStream_t s) {
  const int tiles = order_tiles(n);
  hipLaunchKernelGGL(k_order_count, dim3(tiles), dim3(OB), 0, s, st, n, cnt);
  hipLaunchKernelGGL(k_order_scatter, dim3(tiles), dim3(OB), 0, s, st, n, cnt, tiles, order);
  return hipGetLastError();
}

}  // namespace wk
