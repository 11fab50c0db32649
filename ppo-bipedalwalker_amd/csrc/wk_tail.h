// wk_tail.h -- the minibatch tail shared by the reduction kernels (wk_ppo.hip) and the fused tail
// of the matrix-core gradient kernels (wk_ppo_mfma.hip): the ordered two-level sum of the block
// slabs and DenseLayer.Adam (DenseLayer.cs:125-159).
//
// Ordered reduction (fixed association, no atomics on values): RG consecutive slabs in order,
// then the groups in order.  A "job" is k_grad_reduce_fused's block: QB parameter quads x RG
// groups on 256 threads; JOBS jobs cover the slab.
#ifndef WK_TAIL_H
#define WK_TAIL_H
#include "wk_common.h"
#include "wk_kernels.h"
#include "wk_mfma_layout.h"

namespace wk {

#ifndef WK_REDUCE_QB
#define WK_REDUCE_QB 16
#endif
enum { RG = 16 };
enum { QB = WK_REDUCE_QB };  // parameter quads per job (RG x QB threads; 16 timed best of 4 / 8 / 16)
enum { TAIL_JOBS = (SLAB / 4 + QB - 1) / QB };

// DenseLayer.Adam (DenseLayer.cs:125-159) for one parameter, from its current m, v, w
__device__ __forceinline__ void adam_apply(const AdamArgs& a, int p, float gr, float m0, float v0, float w0) {
  float m = (gr * a.c1) + (m0 * a.beta1);
  float v = (v0 * a.beta2) + ((gr * gr) * a.c2);
  a.m[p] = m;
  a.v[p] = v;
  float mh = m / a.bc1;
  float vh = v / a.bc2;
  float den = sqrtf(vh) + a.eps;
  const float w = w0 - ((mh / den) * a.alpha);
  a.W[p] = w;
  if (a.Wz) mf_scatter_param(a.Wz, p, w);
}

// One job of the one-launch reduction for nblocks <= RG * RG (thread t of 256: group gi = t / QB,
// quad qi = t % QB; gs: the job's [RG][QB] float4 LDS tile).  The caller's block meets the one
// barrier inside whether or not it has a job (job < 0: barrier only).  ADAM: also Adam (a.W set).
// SC1: the slab loads are sc1 buffer loads (the fused tail's hand-off without an acquire fence:
// MI355X_MICROARCH.md, inter-workgroup visibility, "valid forms": sc1 stores drained before the
// counter, sc1 loads after it)
__device__ __forceinline__ float4 slab_load_sc1(const float* slab, int q) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)slab, 0, SLAB * 4, 0x00020000);
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, q * 16, 0, 16);
  return __builtin_bit_cast(float4, v);
}
template <bool ADAM, bool SC1 = false>
__device__ __forceinline__ void reduce_job(int job, int t, const float* __restrict__ partial,
                                           int nblocks, float* grad, const AdamArgs& a, float4* gs) {
  const int qi = t % QB, gi = t / QB;
  const int q = job * QB + qi;  // parameters 4q .. 4q + 3
  const bool live = job >= 0 && q < SLAB / 4;
  const int ngroups = (nblocks + RG - 1) / RG;
  // the Adam operands do not depend on the reduction: their loads go out with the slab loads
  // (one memory latency per minibatch tail instead of two)
  const int pa = 4 * q + gi;
  const bool adam_lane = ADAM && live && gi < 4 && pa < NPARAM;
  float m0 = 0.0f, v0 = 0.0f, w0 = 0.0f;
  if (adam_lane) { m0 = a.m[pa]; v0 = a.v[pa]; w0 = a.W[pa]; }
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (live && gi < ngroups) {
    const int b0 = gi * RG;
    float4 v[RG];
#pragma unroll
    for (int j = 0; j < RG; j++)
      v[j] = (b0 + j < nblocks)
                 ? (SC1 ? slab_load_sc1(partial + (size_t)(b0 + j) * SLAB, q)
                        : ((const float4*)(partial + (size_t)(b0 + j) * SLAB))[q])
                 : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int j = 0; j < RG; j++)
      if (b0 + j < nblocks) {
        acc.x = acc.x + v[j].x; acc.y = acc.y + v[j].y;
        acc.z = acc.z + v[j].z; acc.w = acc.w + v[j].w;
      }
  }
  gs[gi * QB + qi] = acc;
  __syncthreads();
  if (live && gi < 4) {  // one parameter per thread: component gi of quad qi
    const float* gf = (const float*)gs;
    const int p = 4 * q + gi;
    float gv[RG], s = 0.0f;  // (all RG reads issued before the ordered adds)
#pragma unroll
    for (int g = 0; g < RG; g++) gv[g] = gf[(g * QB + qi) * 4 + gi];
#pragma unroll
    for (int g = 0; g < RG; g++)
      if (g < ngroups) s = s + gv[g];
    grad[p] = s;
    if (adam_lane) adam_apply(a, p, s, m0, v0, w0);
  }
}

// The fused minibatch tail of a gradient kernel (round 5): called by every
// thread of every block after the block's slab stores.  Each block drains its stores and bumps the
// launch's arrival counter; the LAST min(nblocks, JOBS / jobs-per-block) blocks to arrive become
// the tail: they wait (bounded) until every block of the launch has arrived and run the reduction
// jobs -- the same association as k_grad_reduce_fused, so the same bits -- with Adam.  No grid
// barrier: only the last arrivers wait, and only for blocks already running (the launch is at most
// one block per CU).  Hand-off (T.on): 1 -- agent-scope release on the counter, acquire after the
// wait; 2 -- the slabs' sc1 (write-through) stores drained before a relaxed counter, relaxed polls,
// sc1 loads of the slabs (no fences).  NT: threads per block (multiple of 256); gs: >= NT / 256 *
// RG * QB float4 of LDS the block no longer needs.
template <int NT>
__device__ __forceinline__ void grad_tail(const GradTail& T, const float* __restrict__ partial,
                                          int nblocks, float4* gs) {
  static_assert(NT % 256 == 0, "256-thread jobs");
  constexpr int JPB = NT / 256;
  __shared__ int s_rank;
  const bool sc1 = T.on == 2 || T.on == 4;  // (3 / 4: probes -- the counter / counter + wait only,
                                            // the host still launches the separate reduction)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores have left
  __syncthreads();
  if (threadIdx.x == 0) {
    if (!sc1) {  // (MI355X_MICROARCH.md, valid forms: release, then a wait the compiler cannot drop)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint32_t t = __hip_atomic_fetch_add(T.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_rank = (int)(t - (T.target - (uint32_t)nblocks));  // 1 .. nblocks: this block's arrival
  }
  __syncthreads();
  if (T.on == 3) return;
  const int ntail = nblocks < (TAIL_JOBS + JPB - 1) / JPB ? nblocks : (TAIL_JOBS + JPB - 1) / JPB;
  const int ti = s_rank - 1 - (nblocks - ntail);
  if (ti < 0) return;  // (block-uniform) an early arriver: done
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int ok = 1;
    while ((int)(__hip_atomic_load(T.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - T.target) < 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s: never in a sound launch
        atomicOr(T.err, 1u);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!sc1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate completes before the barrier
    }
    s_ok = ok;
  }
  __syncthreads();
  if (!s_ok || T.on == 4) return;
  const int grp = threadIdx.x >> 8;
  for (int j0 = ti * JPB; j0 < TAIL_JOBS; j0 += ntail * JPB) {  // (block-uniform trip count)
    const int job = j0 + grp < TAIL_JOBS ? j0 + grp : -1;
    if (sc1) reduce_job<true, true>(job, threadIdx.x & 255, partial, nblocks, T.grad, T.a, gs + grp * RG * QB);
    else reduce_job<true, false>(job, threadIdx.x & 255, partial, nblocks, T.grad, T.a, gs + grp * RG * QB);
    __syncthreads();  // the job tile is free for the next round
  }
}

}  // namespace wk
#endif
