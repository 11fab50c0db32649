// wk_tail.h -- the minibatch tail of the reduction kernels (wk_ppo.hip): the ordered two-level
// sum of the gradient kernels' block slabs and DenseLayer.Adam (DenseLayer.cs:125-159).  (Round 5
// also fused it into the gradient kernels' last-arriving blocks: bit-identical, +4.5 us per
// minibatch, profiles/r05_tail_ab.txt -- removed in round 6; the launch boundary is cheaper.)
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

enum { RG = 16 };
enum { QB = 16 };  // parameter quads per job (RG x QB threads; 16 timed best of 4 / 8 / 16)

// DenseLayer.Adam (DenseLayer.cs:125-159) for one parameter, from its current m, v, w
// (WT: the stores written through, see st_f)
template <bool WT = false>
__device__ __forceinline__ void adam_apply(const AdamArgs& a, int p, float gr, float m0, float v0, float w0) {
  float m = (gr * a.c1) + (m0 * a.beta1);
  float v = (v0 * a.beta2) + ((gr * gr) * a.c2);
  st_f<WT>(&a.m[p], m);
  st_f<WT>(&a.v[p], v);
  float mh = m / a.bc1;
  float vh = v / a.bc2;
  float den = sqrtf(vh) + a.eps;
  const float w = w0 - ((mh / den) * a.alpha);
  st_f<WT>(&a.W[p], w);
  if (a.Wz) mf_scatter_param<WT>(a.Wz, p, w);
}

// One job of the one-launch reduction for nblocks <= RG * RG (thread t of 256: group gi = t / QB,
// quad qi = t % QB; gs: the job's [RG][QB] float4 LDS tile).  The caller's block meets the one
// barrier inside whether or not it has a job (job < 0: barrier only).  ADAM: also Adam (a.W set).
template <bool ADAM>
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
      v[j] = (b0 + j < nblocks) ? ((const float4*)(partial + (size_t)(b0 + j) * SLAB))[q]
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

}  // namespace wk
#endif
