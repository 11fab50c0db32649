// wk_ppo.hip -- PPO clipped-surrogate gradient, deterministic reduction and Adam (gfx950).
//
// k_ppo_grad restates PPOAgent.Train(Batch) (Walker/PPO/PPOAgent.cs:218-346) for a
// minibatch: per sample the critic and actor forward passes with cache
// (NeuralNetwork.FeedForward, NeuralNetwork.cs:52-64), the per-dimension clipped ratio
// gradient (PPOAgent.cs:248-326), and NeuralNetwork.FeedBack (NeuralNetwork.cs:67-82,
// DenseLayer.FeedBack DenseLayer.cs:103-120, ActivationLayer.FeedBack
// ActivationLayer.cs:18-21) accumulating dW/db.  Mapping: one wave per sample stream,
// lane j = neuron j of every 64-wide layer; weights staged once per block in LDS in the
// two orientations the forward and backward passes read (both conflict-free); per-wave
// accumulators stay in VGPRs; waves fold into one LDS slab in wave order, blocks write
// partial slabs that k_grad_reduce sums in block order (no atomics: bit-reproducible).
// Within a wave the samples are visited in minibatch order, so a single-wave launch
// reproduces the reference's sequential accumulation exactly.
#include "wk_common.h"
#include "wk_kernels.h"
#include "wk_mfma_layout.h"
#include "wk_tail.h"

namespace wk {

#define DEV __device__ __forceinline__

DEV float net_maxf_(float x, float y) {
  if (x != y) { if (!__builtin_isnan(x)) return y < x ? x : y; return x; }
  return __builtin_signbit(y) ? x : y;
}
DEV float lrelu(float z) { return z < 0.0f ? 0.2f * z : z; }  // == Math.Max(0.2 z, z) incl. -0, NaN
DEV float dlrelu(float z) { return z < 0.0f ? 0.2f : 1.0f; }

// LDS weight image (floats)
enum : int {
  L_AW1 = 0,                  // [64][13] actor W1 (row j padded)
  L_CW1 = L_AW1 + 64 * 13,    // [64][13] critic W1
  L_AW2T = L_CW1 + 64 * 13,   // [64 k][64 j] actor W2 transposed (forward)
  L_AW2 = L_AW2T + 4096,      // [64 j][64 k] actor W2 (backward)
  L_AW3 = L_AW2 + 4096,       // [4][65]
  L_CW2 = L_AW3 + 4 * 65,     // [64]
  L_AB1 = L_CW2 + 64, L_AB2 = L_AB1 + 64, L_CB1 = L_AB2 + 64, L_AB3 = L_CB1 + 64,
  L_CB2 = L_AB3 + 4,
  L_WEND = L_CB2 + 4
};

template <int WPB>
__global__ __launch_bounds__(64 * WPB) void k_ppo_grad(GradArgs g) {
  extern __shared__ float lds[];
  float* wl = lds;                         // weights
  float* slab = lds + L_WEND;              // [SLAB] block accumulation
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* wv = slab + SLAB + wave * (64 * 4 + 24);  // per-wave scratch
  float* h1s = wv;
  float* h2s = wv + 64;
  float* hc1s = wv + 128;
  float* gz2s = wv + 192;
  float* smp = wv + 256;                   // 12 s + 4 a + 4 lpo + G + A (+pad)

  // ---- stage weights ----
  for (int i = threadIdx.x; i < 64 * 12; i += 64 * WPB) {
    int j = i / 12, k = i % 12;
    wl[L_AW1 + j * 13 + k] = g.W[OFF_A_W1 + i];
    wl[L_CW1 + j * 13 + k] = g.W[OFF_C_W1 + i];
  }
  for (int i = threadIdx.x; i < 4096; i += 64 * WPB) {
    int j = i >> 6, k = i & 63;
    float w = g.W[OFF_A_W2 + i];
    wl[L_AW2 + i] = w;
    wl[L_AW2T + k * 64 + j] = w;
  }
  for (int i = threadIdx.x; i < 256; i += 64 * WPB) wl[L_AW3 + (i >> 6) * 65 + (i & 63)] = g.W[OFF_A_W3 + i];
  for (int i = threadIdx.x; i < 64; i += 64 * WPB) {
    wl[L_CW2 + i] = g.W[OFF_C_W2 + i];
    wl[L_AB1 + i] = g.W[OFF_A_B1 + i];
    wl[L_AB2 + i] = g.W[OFF_A_B2 + i];
    wl[L_CB1 + i] = g.W[OFF_C_B1 + i];
  }
  if (threadIdx.x < 4) wl[L_AB3 + threadIdx.x] = g.W[OFF_A_B3 + threadIdx.x];
  if (threadIdx.x == 0) wl[L_CB2] = g.W[OFF_C_B2];
  for (int i = threadIdx.x; i < SLAB; i += 64 * WPB) slab[i] = 0.0f;
  __syncthreads();

  // ---- per-lane accumulators (lane = neuron) ----
  float dW2[64];
#pragma unroll
  for (int k = 0; k < 64; k++) dW2[k] = 0.0f;
  float dW1[12], dWc1[12];
#pragma unroll
  for (int i = 0; i < 12; i++) { dW1[i] = 0.0f; dWc1[i] = 0.0f; }
  float dW3[4] = {0.0f, 0.0f, 0.0f, 0.0f}, db3[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float db1 = 0.0f, db2 = 0.0f, dbc1 = 0.0f, dWc2 = 0.0f, dbc2 = 0.0f;
  float diagC = 0.0f, diagA = 0.0f, skipped = 0.0f;

  const float aw1_b = wl[L_AB1 + lane], aw2_b = wl[L_AB2 + lane], cw1_b = wl[L_CB1 + lane];
  const float cw2_l = wl[L_CW2 + lane];
  const float cb2 = wl[L_CB2];
  const int first = (blockIdx.x * WPB + wave) * g.spw;

#pragma unroll 1
  for (int q = 0; q < g.spw; q++) {
    const int pos = first + q;
    if (pos >= g.samples) break;  // wave-uniform
    // ---- gather the sample (CreateBatches, PPOAgent.cs:512-533) ----
    uint32_t idx = g.base + (uint32_t)pos;
    if (g.use_perm) idx = perm_apply(idx, g.pk);
    if (lane < 12) smp[lane] = g.states[(size_t)idx * 12 + lane];
    else if (lane < 16) smp[lane] = g.actions[(size_t)idx * 4 + lane - 12];
    else if (lane < 20) smp[lane] = g.logp_old[(size_t)idx * 4 + lane - 16];
    else if (lane == 20) smp[20] = g.returns[idx];
    else if (lane == 21) smp[21] = g.adv[idx];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float s[12];
#pragma unroll
    for (int i = 0; i < 12; i++) s[i] = smp[i];

    // ---- layer 1 (actor and critic): z_j = (sum_k W[j][k] s_k) + b_j ----
    float z1 = 0.0f, zc1 = 0.0f;
#pragma unroll
    for (int k = 0; k < 12; k++) {
      z1 = z1 + wl[L_AW1 + lane * 13 + k] * s[k];
      zc1 = zc1 + wl[L_CW1 + lane * 13 + k] * s[k];
    }
    z1 = z1 + aw1_b;
    zc1 = zc1 + cw1_b;
    const float h1 = lrelu(z1), hc1 = lrelu(zc1);
    h1s[lane] = h1;
    hc1s[lane] = hc1;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // ---- actor layer 2 ----
    float z2 = 0.0f;
#pragma unroll
    for (int k = 0; k < 64; k++) z2 = z2 + wl[L_AW2T + k * 64 + lane] * h1s[k];
    z2 = z2 + aw2_b;
    const float h2 = lrelu(z2);
    h2s[lane] = h2;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // ---- output layers, one row per lane: lanes 0..3 the actor's 4 outputs (W3 row d
    // on h2), lane 4 the critic's single output (Wc2 on hc1); sequential over k ----
    const int d = lane & 3;
    const bool vlane = lane == 4;
    const float* wrow = vlane ? (wl + L_CW2) : (wl + L_AW3 + d * 65);
    const float* xin = vlane ? hc1s : h2s;
    float zo = 0.0f;
#pragma unroll
    for (int k = 0; k < 64; k++) zo = zo + wrow[k] * xin[k];
    zo = zo + (vlane ? cb2 : wl[L_AB3 + d]);
    const float V = __shfl(zo, 4);
    const float z3 = zo;
    const float mean = tanhf(z3);
    // ---- PPO derivative (PPOAgent.cs:234-326), per dimension ----
    const float A = smp[21];
    float criticLoss = 2.0f * (V - smp[20]);
    const float act = smp[12 + d], lpo = smp[16 + d];
    float fr = (act - mean) / g.std_;
    fr *= fr;
    fr /= 2.0f;
    const float lp = g.lp_const - fr;
    const float r = expf(lp - lpo);
    const float cr = r >= g.upper ? g.upper : (r <= g.lower ? g.lower : r);
    const float cra = cr * A, ra = r * A;
    const float partA = (ra <= cra ? 1.0f : 0.0f) * A;
    const float partB = (cra < ra ? 1.0f : 0.0f) * A;
    const float partC = (r >= g.lower && r <= g.upper) ? 1.0f : 0.0f;
    float l = partA + (partB * partC);
    l = l * -1.0f;
    const float eo = expf(lpo);
    const bool zero_div = (lane < 4) && (eo == 0.0f);
    const float lcd = l / eo;
    const float prob = expf(lp);
    const float frac = (act - mean) / (g.std_ * g.std_);
    float actorLoss = (prob * frac) * lcd;
    const bool skip = __any(zero_div);  // Matrix.HadamardDivision throws -> continue
    if (skip) {
      skipped += 1.0f;
      continue;
    }
    criticLoss /= g.b_div;
    actorLoss = actorLoss / g.b_div;
    // broadcast the 4 per-dimension values
    const float al0 = __shfl(actorLoss, 0), al1 = __shfl(actorLoss, 1);
    const float al2 = __shfl(actorLoss, 2), al3 = __shfl(actorLoss, 3);
    diagC += criticLoss;
    diagA += ((((0.0f + al0) + al1) + al2) + al3) / 4.0f;
    // ---- actor backward ----
    const float th = tanhf(z3);
    const float gz3 = actorLoss * (1.0f - (th * th));
    float gz3v[4];
    gz3v[0] = __shfl(gz3, 0); gz3v[1] = __shfl(gz3, 1);
    gz3v[2] = __shfl(gz3, 2); gz3v[3] = __shfl(gz3, 3);
#pragma unroll
    for (int dd = 0; dd < 4; dd++) {
      dW3[dd] = dW3[dd] + gz3v[dd] * h2;   // lane = column k of W3
      db3[dd] = db3[dd] + gz3v[dd];
    }
    float gh2 = 0.0f;
#pragma unroll
    for (int dd = 0; dd < 4; dd++) gh2 = gh2 + wl[L_AW3 + dd * 65 + lane] * gz3v[dd];
    const float gz2 = gh2 * dlrelu(z2);
    gz2s[lane] = gz2;
    db2 = db2 + gz2;
#pragma unroll
    for (int k = 0; k < 64; k++) dW2[k] = dW2[k] + gz2 * h1s[k];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float gh1 = 0.0f;
#pragma unroll
    for (int j = 0; j < 64; j++) gh1 = gh1 + wl[L_AW2 + j * 64 + lane] * gz2s[j];
    const float gz1 = gh1 * dlrelu(z1);
    db1 = db1 + gz1;
#pragma unroll
    for (int i = 0; i < 12; i++) dW1[i] = dW1[i] + gz1 * s[i];
    // ---- critic backward ----
    dWc2 = dWc2 + criticLoss * hc1;
    dbc2 = dbc2 + criticLoss;
    const float ghc1 = 0.0f + cw2_l * criticLoss;
    const float gzc1 = ghc1 * dlrelu(zc1);
    dbc1 = dbc1 + gzc1;
#pragma unroll
    for (int i = 0; i < 12; i++) dWc1[i] = dWc1[i] + gzc1 * s[i];
  }

  // ---- fold waves into the block slab in wave order ----
#pragma unroll 1
  for (int w = 0; w < WPB; w++) {
    if (w == wave) {
      const int j = lane;
#pragma unroll
      for (int i = 0; i < 12; i++) {
        slab[OFF_C_W1 + j * 12 + i] += dWc1[i];
        slab[OFF_A_W1 + j * 12 + i] += dW1[i];
      }
      slab[OFF_C_B1 + j] += dbc1;
      slab[OFF_C_W2 + j] += dWc2;
      slab[OFF_A_B1 + j] += db1;
#pragma unroll
      for (int k = 0; k < 64; k++) slab[OFF_A_W2 + j * 64 + k] += dW2[k];
      slab[OFF_A_B2 + j] += db2;
#pragma unroll
      for (int dd = 0; dd < 4; dd++) slab[OFF_A_W3 + dd * 64 + j] += dW3[dd];
      if (lane == 0) {
        slab[OFF_C_B2] += dbc2;
#pragma unroll
        for (int dd = 0; dd < 4; dd++) slab[OFF_A_B3 + dd] += db3[dd];
        slab[NPARAM] += diagC;
        slab[NPARAM + 1] += diagA;
        slab[NPARAM + 2] += skipped;
      }
    }
    __syncthreads();
  }
  float* out = g.partial + (size_t)blockIdx.x * SLAB;
  for (int i = threadIdx.x; i < SLAB; i += 64 * WPB) out[i] = slab[i];
}

// Deterministic two-level sum of the block slabs (fixed association, no atomics):
// stage 1 folds groups of RG consecutive slabs (all RG loads issued before the ordered
// adds, so the chain is one memory latency, not RG); stage 2 folds the groups in order.
// (RG, QB, adam_apply and the one-launch job: wk_tail.h)
__global__ void k_grad_reduce1(const float* __restrict__ partial, int nblocks, float* part2) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (p >= SLAB) return;
  const int b0 = g * RG;
  float v[RG];
#pragma unroll
  for (int j = 0; j < RG; j++) v[j] = (b0 + j < nblocks) ? partial[(size_t)(b0 + j) * SLAB + p] : 0.0f;
  float acc = 0.0f;
#pragma unroll
  for (int j = 0; j < RG; j++)
    if (b0 + j < nblocks) acc = acc + v[j];
  part2[(size_t)g * SLAB + p] = acc;
}

// stage 2: the groups in order; up to RG groups are loaded at once (one latency), more
// fall back to a loop -- same association either way
DEV float sum_groups(const float* __restrict__ part2, int ngroups, int p) {
  if (ngroups <= RG) {
    float v[RG];
#pragma unroll
    for (int g = 0; g < RG; g++) v[g] = g < ngroups ? part2[(size_t)g * SLAB + p] : 0.0f;
    float acc = 0.0f;
#pragma unroll
    for (int g = 0; g < RG; g++)
      if (g < ngroups) acc = acc + v[g];
    return acc;
  }
  float acc = 0.0f;
  for (int g = 0; g < ngroups; g++) acc = acc + part2[(size_t)g * SLAB + p];
  return acc;
}
__global__ void k_grad_reduce2(const float* __restrict__ part2, int ngroups, float* grad) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= SLAB) return;
  grad[p] = sum_groups(part2, ngroups, p);
}

DEV void adam_param(const AdamArgs& a, int p, float gr) { adam_apply(a, p, gr, a.m[p], a.v[p], a.W[p]); }

// elementwise over all 6149 parameters
__global__ void k_adam(AdamArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < NPARAM) adam_param(a, p, a.grad[p]);
}

// single-GPU minibatch tail: the second reduction stage and Adam in one launch
__global__ void k_grad_reduce2_adam(const float* __restrict__ part2, int ngroups, float* grad,
                                    AdamArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= SLAB) return;
  const float acc = sum_groups(part2, ngroups, p);
  grad[p] = acc;
  if (p < NPARAM) adam_param(a, p, acc);
}

// One-launch form of the two stages for nblocks <= RG * RG, bit-identical association
// (RG consecutive slabs in order, then the groups in order): a block is one job of wk_tail.h's
// reduce_job (QB parameter quads; thread (group gi, quad qi) folds its group's RG slabs with
// 16-byte loads, all issued before the ordered adds, and the 16 group sums are folded in order
// through LDS).  ADAM: the single-GPU tail applies Adam as well.
template <bool ADAM>
__global__ __launch_bounds__(RG * QB) void k_grad_reduce_fused(const float* __restrict__ partial,
                                                              int nblocks, float* grad, AdamArgs a) {
  static_assert(SLAB % 4 == 0 && RG * QB == 256, "16-byte slab rows, 256-thread jobs");
  __shared__ float4 gs[RG * QB];
  reduce_job<ADAM>(blockIdx.x, threadIdx.x, partial, nblocks, grad, a, gs);
}

// Normalize (PPOAgent.cs:461-472): LINQ Average/Sum accumulate in double
__global__ void k_normalize(float* x, int n, float eps_clip) {
  __shared__ double red[1024];
  __shared__ float mean_s, std_s;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += (double)x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) mean_s = (float)(red[0] / (double)n);
  __syncthreads();
  const float mean = mean_s;
  double ss = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    double dv = (double)(x[i] - mean);
    ss += dv * dv;
  }
  __syncthreads();
  red[threadIdx.x] = ss;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) std_s = (float)sqrt(red[0] / (double)n);
  __syncthreads();
  const float sd = std_s;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float v = x[i] - mean;
    x[i] = v / (sd + eps_clip);
  }
}

// Xavier-normal init (Matrix.FromXavier, Matrix.cs:59-80) on the device
__global__ void k_xavier(float* W, uint64_t seed) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= NPARAM) return;
  // (offset, rows, cols, global dense-layer index) of the five dense layers
  const int offs[5] = {OFF_C_W1, OFF_C_W2, OFF_A_W1, OFF_A_W2, OFF_A_W3};
  const int rows[5] = {64, 1, 64, 64, 4}, cols[5] = {12, 64, 12, 64, 64};
  float v = 0.0f;
#pragma unroll
  for (int l = 0; l < 5; l++) {
    const int n = rows[l] * cols[l];
    if (p >= offs[l] && p < offs[l] + n) {
      const int k = p - offs[l];
      U4 o = philox(seed, (uint32_t)k, (uint32_t)l, 0, ST_XAVIER);
      float u1 = next_double_f(o.x, o.y), u2 = next_double_f(o.z, o.w);
      if (u1 == 0.0f) u1 = 1.0f;
      const float PI_F = 3.14159265358979323846f;
      float std_ = sqrtf(2.0f / (float)(rows[l] + cols[l]));
      float z = sqrtf(-2.0f * logf(u1)) * sinf(2.0f * PI_F * u2);
      v = 0.0f + (std_ * z);
    }
  }
  W[p] = v;
}

// > 64 KiB of dynamic LDS (a gfx950 CU has 160 KiB) for every gradient kernel, on the
// current device (called by wk_create after hipSetDevice)
hipError_t configure_device_kernels() {
  hipError_t e = hipFuncSetAttribute((const void*)k_ppo_grad<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_ppo_grad<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e == hipSuccess) e = configure_mfma_kernels();
  return e;
}

hipError_t launch_ppo_grad(const GradArgs& g, int wpb, int nblocks, hipStream_t s) {
  const size_t lds = sizeof(float) * (L_WEND + SLAB + wpb * (64 * 4 + 24));
  if (wpb == 1) {
    hipLaunchKernelGGL((k_ppo_grad<1>), dim3(nblocks), dim3(64), lds, s, g);
  } else {
    hipLaunchKernelGGL((k_ppo_grad<4>), dim3(nblocks), dim3(256), lds, s, g);
  }
  return hipGetLastError();
}
hipError_t launch_grad_reduce(const float* partial, int nblocks, float* part2, float* grad,
                              hipStream_t s) {
  if (nblocks <= RG * RG) {
    hipLaunchKernelGGL(k_grad_reduce_fused<false>, dim3((SLAB / 4 + QB - 1) / QB), dim3(RG * QB), 0, s,
                       partial, nblocks, grad, AdamArgs{});
    return hipGetLastError();
  }
  const int ng = (nblocks + RG - 1) / RG;
  hipLaunchKernelGGL(k_grad_reduce1, dim3((SLAB + 255) / 256, ng), dim3(256), 0, s, partial,
                     nblocks, part2);
  hipLaunchKernelGGL(k_grad_reduce2, dim3((SLAB + 255) / 256), dim3(256), 0, s, part2, ng, grad);
  return hipGetLastError();
}
int grad_reduce_groups(int nblocks) { return (nblocks + RG - 1) / RG; }
hipError_t launch_grad_reduce_adam(const float* partial, int nblocks, float* part2, float* grad,
                                   const AdamArgs& a, hipStream_t s) {
  if (nblocks <= RG * RG) {
    hipLaunchKernelGGL(k_grad_reduce_fused<true>, dim3((SLAB / 4 + QB - 1) / QB), dim3(RG * QB), 0, s,
                       partial, nblocks, grad, a);
    return hipGetLastError();
  }
  const int ng = (nblocks + RG - 1) / RG;
  hipLaunchKernelGGL(k_grad_reduce1, dim3((SLAB + 255) / 256, ng), dim3(256), 0, s, partial,
                     nblocks, part2);
  hipLaunchKernelGGL(k_grad_reduce2_adam, dim3((SLAB + 255) / 256), dim3(256), 0, s, part2, ng,
                     grad, a);
  return hipGetLastError();
}
// One-shot exchange (wk_comm_init_ipc): the minibatch's gradient all-reduce without a
// collective library, fused with the ordered block reduction and Adam -- one launch per
// minibatch after the gradient kernel, as on one GPU.  Block b (the grid of k_grad_reduce_fused)
// first forms this rank's ordered sum of its parameter quads exactly as k_grad_reduce_fused
// does, publishes it into this rank's exchange region (slab buffer seq & 1) and releases its
// sequence flag at system scope; it then waits (bounded) until every peer's flag b reaches
// seq, reads the peers' values directly through the IPC mappings and sums the ranks in rank
// order (rank 0's value first: for two ranks exactly the RCCL / host all-reduce's a + b), and
// applies Adam.  A buffer is reused two minibatches later only: a rank publishes seq + 2 after
// its exchange of seq + 1 saw every peer's seq + 1 flag, which a peer sets only once its own
// exchange of seq -- the last read of the seq buffers -- has completed (stream order).
// Failure: the wait is bounded by x.timeout_ticks of the constant 100 MHz clock (30 s unless
// WK_XCH_TIMEOUT_S / wk_comm_set_timeout say otherwise; ranks must stay within it of each other).
// A block whose wait times out, or that finds a peer's flag at XCH_ABORT, sets err[0], overwrites
// its own flag with XCH_ABORT and returns without writing grad_out or applying Adam; every later
// exchange sees err[0] at entry, writes XCH_ABORT into its flag and returns, so a late peer fails
// at once on that minibatch (it reads the abort value instead of this rank's sequence number)
// rather than applying it.  Block 0 records the last Adam step it applied in err[1], so the host
// rolls its step count back.  Not a consensus protocol: a peer that read this rank's sequence
// number before the abort overwrote it (a wait that ended within the same few microseconds), or
// blocks of one rank that straddle the timeout, leave the replicas' W / m / v differing -- after
// WK_ERR_COMM the job must stop or reload a checkpoint on every rank.
// Hand-off (round 6, MI355X_MICROARCH.md's valid forms at system scope): producer -- every wave's
// slab stores drained (s_waitcnt vmcnt(0)), block barrier, one lane's release store of the flag;
// consumer -- relaxed polls of the peers' flags by the polling wave, ONE acquire by that wave,
// s_waitcnt, block barrier, then the peer loads.  Adam's and grad_out's stores are written through
// (st_f<true>), so the next minibatch's release finds no dirty lines of them to write back.
// Measured uncontended at the 8-GPU shard's minibatch (scripts/r06_xch_own.py, 2 ranks on one
// GPU): 19.0 -> 8.2 us per launch (kernel trace), own work 13.9 -> 4.8 us per block (stamps),
// against 4.9 us for k_grad_reduce_fused<true> on the same slabs; before, every poll was an
// acquire load and every thread fenced.
// Timing (x.stamps, wk_comm_xch_profile): thread 0 reads the constant clock at entry, after its
// flag store, after the block's wait and after the block's last Adam store, and writes the four
// values with vector stores to the launch's ring slot -- wait time versus own work per minibatch.
__global__ __launch_bounds__(RG * QB) void k_reduce_xch_adam(XchArgs x) {
  __shared__ float4 gs[RG][QB];
  __shared__ int live;  // no exchange has timed out (entry), and this block's wait completed
  uint64_t ts[XCH_POINTS] = {0, 0, 0, 0};
  const bool stamp = x.stamps != nullptr && threadIdx.x == 0;
  if (stamp) ts[0] = __builtin_amdgcn_s_memrealtime();
  auto flush = [&]() {
    if (stamp)
      for (int k = 0; k < XCH_POINTS; k++) x.stamps[blockIdx.x * XCH_POINTS + k] = ts[k];
  };
  if (threadIdx.x == 0)
    live = __hip_atomic_load(x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u ? 1 : 0;
  const int qi = threadIdx.x % QB, gi = threadIdx.x / QB;
  const int q = blockIdx.x * QB + qi;
  const int ngroups = (x.nblocks + RG - 1) / RG;
  const int p = 4 * q + gi;  // (gi < 4) this thread's parameter
  const bool adam_lane = gi < 4 && p < NPARAM && x.a.W != nullptr;  // (no W: exchange only)
  float m0 = 0.0f, v0 = 0.0f, w0 = 0.0f;
  if (adam_lane) { m0 = x.a.m[p]; v0 = x.a.v[p]; w0 = x.a.W[p]; }
  float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (q < SLAB / 4 && gi < ngroups) {  // stage 1, as k_grad_reduce_fused
    const int b0 = gi * RG;
    float4 v[RG];
#pragma unroll
    for (int j = 0; j < RG; j++)
      v[j] = (b0 + j < x.nblocks) ? ((const float4*)(x.partial + (size_t)(b0 + j) * SLAB))[q]
                                  : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int j = 0; j < RG; j++)
      if (b0 + j < x.nblocks) {
        acc.x = acc.x + v[j].x; acc.y = acc.y + v[j].y;
        acc.z = acc.z + v[j].z; acc.w = acc.w + v[j].w;
      }
  }
  gs[gi][qi] = acc;
  __syncthreads();
  const int t = threadIdx.x;
  if (!live) {  // an earlier exchange failed (block-uniform: read after the barrier)
    if (t == 0)
      __hip_atomic_store(x.flag[x.rank] + blockIdx.x, XCH_ABORT, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    flush();
    return;
  }
  const int buf = (int)(x.seq & 1u);
  float mine = 0.0f;
  if (gi < 4 && q < SLAB / 4) {  // stage 2: this rank's ordered sum, published
    const float* gf = (const float*)gs;
    float gv[RG];
#pragma unroll
    for (int g = 0; g < RG; g++) gv[g] = gf[(g * QB + qi) * 4 + gi];
#pragma unroll
    for (int g = 0; g < RG; g++)
      if (g < ngroups) mine = mine + gv[g];
    x.slab[x.rank][(size_t)buf * SLAB + p] = mine;
  }
  // every storing wave drains its slab stores before the barrier: the flag's system-scope
  // release below (buffer_wbl2 in thread 0's wave) writes back only what has reached the L2 by
  // then, and a peer GPU reads this HBM over xGMI (MI355X_MICROARCH.md, inter-workgroup
  // visibility: the workgroup barrier alone does not wait for other waves' stores)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0)
    __hip_atomic_store(x.flag[x.rank] + blockIdx.x, x.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (stamp) ts[1] = __builtin_amdgcn_s_memrealtime();
  if (t < x.nranks && t != x.rank) {
    const uint64_t* f = x.flag[t] + blockIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t seen;
    while ((seen = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) < x.seq) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > x.timeout_ticks) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (seen < x.seq || seen == XCH_ABORT) {  // a peer is gone or gave up: report, never hang
      atomicOr(x.err, 1u);
      live = 0;
    }
  }
  if (t < 64) {  // ONE acquire (system scope), by the polling wave, before the barrier
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (stamp) ts[2] = __builtin_amdgcn_s_memrealtime();
  if (!live) {  // no grad_out, no Adam; a late peer reading this flag fails this minibatch too
    if (t == 0)
      __hip_atomic_store(x.flag[x.rank] + blockIdx.x, XCH_ABORT, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    flush();
    return;
  }
  if (gi < 4 && q < SLAB / 4) {
    float sum = x.rank == 0 ? mine : x.slab[0][(size_t)buf * SLAB + p];
    for (int r = 1; r < x.nranks; r++)
      sum = sum + (r == x.rank ? mine : x.slab[r][(size_t)buf * SLAB + p]);
    st_f<true>(&x.grad_out[p], sum);  // (written through: see below)
    if (adam_lane) adam_apply<true>(x.a, p, sum, m0, v0, w0);
  }
  if (blockIdx.x == 0 && t == 0 && x.a.W != nullptr)
    __hip_atomic_store(x.err + 1, x.t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (x.stamps != nullptr) {  // (block-uniform) the exit stamp after every thread's stores issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (stamp) ts[3] = __builtin_amdgcn_s_memrealtime();
    flush();
  }
}
int xch_blocks() { return (SLAB / 4 + QB - 1) / QB; }
size_t xch_region_bytes() { return sizeof(float) * 2 * SLAB + sizeof(uint64_t) * XCH_FLAGS; }
hipError_t launch_reduce_xch_adam(const XchArgs& x, hipStream_t s) {
  static_assert((SLAB / 4 + QB - 1) / QB <= XCH_FLAGS, "one flag per block");
  if (x.nblocks > RG * RG) return hipErrorInvalidValue;  // (the gradient kernel caps at 256)
  hipLaunchKernelGGL(k_reduce_xch_adam, dim3((SLAB / 4 + QB - 1) / QB), dim3(RG * QB), 0, s, x);
  return hipGetLastError();
}

hipError_t launch_adam(const AdamArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_adam, dim3((NPARAM + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_normalize(float* x, int n, float eps, hipStream_t s) {
  hipLaunchKernelGGL(k_normalize, dim3(1), dim3(1024), 0, s, x, n, eps);
  return hipGetLastError();
}
hipError_t launch_xavier(float* W, uint64_t seed, hipStream_t s) {
  hipLaunchKernelGGL(k_xavier, dim3((NPARAM + 255) / 256), dim3(256), 0, s, W, seed);
  return hipGetLastError();
}

}  // namespace wk
