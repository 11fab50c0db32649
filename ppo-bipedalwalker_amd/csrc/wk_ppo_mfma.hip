// wk_ppo_mfma.hip -- the PPO minibatch gradient on the CDNA4 matrix cores (gfx950).
//
// Same math as k_ppo_grad (PPOAgent.Train(Batch), Walker/PPO/PPOAgent.cs:218-346 with
// NeuralNetwork.FeedForward / FeedBack, NeuralNetwork.cs:52-82, DenseLayer.cs:82-120,
// ActivationLayer.cs:18-21), restated as batched GEMMs over chunks of 16 samples with
// v_mfma_f32_16x16x4_f32 (exact fp32 products and sums; only the association of each
// sum over k / over samples differs from the sequential reference, which the parity
// tests bound).  Per wave and chunk:
//
//   forward   Z1^T = W1 S^T, Zc1^T = Wc1 S^T      (M 64, K 12, N 16)
//             Z2^T = W2 H1^T                      (M 64, K 64, N 16; B = Z1's D registers)
//             z3, V: 64-long dots on the VALU, summed over the 4 lane groups
//   loss      per (sample, action dim) in lane (n, g = d): ratio, clip, dmu, dV
//   backward  gh2 = W3^T gz3 (VALU), dW3|dWc2 += [gz3; dV]^T [H2 | Hc1]  (M 16, K 16, N 128)
//             dW2 += gz2^T H1                     (M 64, K 16 samples, N 64)
//             gh1^T = W2^T gz2^T                  (chained, B = gz2's registers)
//             dW1|db1 += gz1^T [S | 1], dWc1|dbc1 likewise (M 64, K 16, N 16)
//
// Operand layouts of v_mfma_f32_16x16x4_f32 (probed, scripts/probe/mfma_layout.hip):
// lane l = 16 g + n holds A[n][g], B[g][n] and D[4 g + r][n] (r = 0..3).  With samples
// on n and neurons 16 Mt + 4 g + r on (g, r), a layer's D registers are directly the
// B operand of the next layer when its K steps are ordered (Mt, r) -- the weights are
// pre-swizzled into LDS in that order.  Weight-gradient GEMMs need samples on K, so
// activations / gradients pass through small per-wave [16][80] LDS tiles (row stride
// 80 = 16 mod 64 banks: conflict-free operand reads).  Accumulators stay in registers
// across chunks; waves fold into the block slab in wave order and blocks write partial
// slabs for the ordered reduction (bit-reproducible, no atomics).
#include <cstdlib>
#include <cstring>

#include "wk_common.h"
#include "wk_kernels.h"
#include "wk_mfma_layout.h"

namespace wk {

#define DEV __device__ __forceinline__
typedef float f4 __attribute__((ext_vector_type(4)));

namespace mf {
enum : int {
  RS = 80,               // row stride of a [16 samples][64] tile
  C_H1 = 0, C_HC1 = C_H1 + 16 * RS, C_H2 = C_HC1 + 16 * RS, C_G2 = C_H2 + 16 * RS,
  C_SX = C_G2 + 16 * RS,  // [16][16]: 12 features, 1.0 (bias column), 0, 0, 0
  C_G3 = C_SX + 256,      // [16][16]: gz3 (4 dims), dV, zeros
  CHUNK = C_G3 + 256,
  C_G1 = C_H2, C_GC1 = C_HC1,  // backward tiles reuse the forward ones
  WAVES = 4,
  LDS_FLOATS = WEND + WAVES * CHUNK
};
static_assert(LDS_FLOATS >= WAVES * SLAB, "the epilogue's per-wave slabs fit");
}  // namespace mf

// ActivationLayer LeakyReLU(0.2) = Math.Max(0.2 z, z): z for z >= 0 (and -0: Max keeps
// the equal-valued 0.2 * -0 = -0), 0.2 z below, NaN through.  As v_max_f32(0.2 z, z) it is the
// same value for every input (0.2 z is NaN exactly when z is, has z's sign, and is the larger
// one exactly when z < 0): two instructions instead of multiply, compare and select.
DEV float mf_lrelu(float z) { return __builtin_fmaxf(0.2f * z, z); }
DEV float mf_dlrelu(float z) { return z < 0.0f ? 0.2f : 1.0f; }
DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// [16 samples][RS] tile addressing, bank-conflict-free both ways (MI355X_MICROARCH §LDS):
// column groups of 4 are XOR-swizzled by row bits 1..2.  A lane (n, g) stores an f4 at
// [row n][cols c..c+3] (ds_write_b128: 8-lane groups, banks mod 32 -> the 8 rows of a group
// land on 8 distinct 16-B slots); a lane (n, g) reads [row 4t + g][col 16i + n]
// (ds_read_b32: 32-lane halves; the swizzle is uniform over a half, so RS = 80 keeps the two
// rows of a half on opposite 16-bank halves).
DEV int tw(int row, int col4) { return row * mf::RS + (col4 ^ (((row >> 1) & 3) << 2)); }
DEV int tr(int row, int col) { return row * mf::RS + (col ^ (((row >> 1) & 3) << 2)); }
// [16][16] tiles (SX, G3): columns XOR-swizzled by 2 (row >> 1), read as [row n][col 4t + g]
// and [row 4t + g][col n] without conflicts; the f4 store of SX moves its group and swaps
// its element pairs accordingly
DEV int sx(int row, int col) { return row * 16 + (col ^ ((row >> 1) << 1)); }
DEV f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
// sum over the 16 lanes of a DPP row (all lanes get the total)
DEV float row_sum16(float v) {
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

// Block slabs of the ordered reduction, written through to memory (sc1 buffer stores): the
// kernel-end release then has no dirty slab lines to write back out of the L2, and the
// reduction reads them from other XCDs anyway (tile-parallel kernel 12.9 -> 12.2 us per launch
// at 8,192 samples, the reduction unchanged).
struct SlabOut {
  __amdgpu_buffer_rsrc_t r;
  DEV explicit SlabOut(float* base) : r(__builtin_amdgcn_make_buffer_rsrc(base, 0, SLAB * 4, 0x00020000)) {}
  DEV void put(int i, f4 v) const {  // 16-byte element i
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, i * 16, 0, 16);
  }
};

__global__ __launch_bounds__(64 * mf::WAVES) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_ppo_grad_mfma(GradArgs ga) {
  using namespace mf;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 15, g = lane >> 4;

  const int nchunks = (ga.samples + 15) / 16;
  const int nw = gridDim.x * WAVES;
  // gather (CreateBatches, PPOAgent.cs:512-533), one chunk ahead of the math
  struct Smp { f4 sv; float act, lpo, ret, adv; };
  auto gather = [&](int c) {
    Smp m;
    const int pos = c * 16 + n;
    uint32_t idx = ga.base + (uint32_t)(pos < ga.samples ? pos : 0);
    if (ga.use_perm) idx = perm_apply(idx, ga.pk);
    m.sv = f4{1.0f, 0.0f, 0.0f, 0.0f};  // lane group 3: the bias column
    if (g < 3) m.sv = *(const f4*)(ga.states + (size_t)idx * 12 + 4 * g);
    m.act = ga.actions[(size_t)idx * 4 + g];
    m.lpo = ga.logp_old[(size_t)idx * 4 + g];
    m.ret = ga.returns[idx];
    m.adv = ga.adv[idx];
    return m;
  };
  int c = blockIdx.x * WAVES + wave;
  // the first chunk's gather is in flight while the weights are staged
  Smp nxt = gather(c < nchunks ? c : 0);

  // ---- stage the weight image (already in operand order, wk_mfma_layout.h): every
  // thread's loads are issued before its first LDS write, so the copy costs one L2
  // round trip instead of one per 4 KB ----
  {
    constexpr int NV = WEND / 4, PER = (NV + 64 * WAVES - 1) / (64 * WAVES);
    f4 wv[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) {
      const int e = tid + i * 64 * WAVES;
      if (e < NV) wv[i] = ((const f4*)ga.Wz)[e];
    }
#pragma unroll
    for (int i = 0; i < PER; i++) {
      const int e = tid + i * 64 * WAVES;
      if (e < NV) ((f4*)lds)[e] = wv[i];
    }
  }
  float* cb = lds + WEND + wave * CHUNK;
  for (int e = lane; e < 256; e += 64) cb[C_G3 + e] = 0.0f;
  __syncthreads();

  // ---- accumulators (registers, across chunks) ----
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
  f4 a2[4][4], a1[4], a1c[4], a3[8];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    a1[i] = z4; a1c[i] = z4;
#pragma unroll
    for (int j = 0; j < 4; j++) a2[i][j] = z4;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) a3[i] = z4;
  float db2[16];
#pragma unroll
  for (int i = 0; i < 16; i++) db2[i] = 0.0f;
  float db3 = 0.0f, dbc2 = 0.0f, diagC = 0.0f, diagA = 0.0f, skipped = 0.0f;

  const float b3g = lds[BA3 + g], bc2 = lds[BC2];
  // per-lane constants: this lane's rows of W1 / Wc1 (A operands), biases, W3 and Wc2
  // entries of its 16 neurons 16 Mt + 4 g + r
  float wa1[4][3], wc1[4][3];
  f4 ba1[4], bc1[4], ba2[4], wc2[4], w3[4][4];
#pragma unroll
  for (int Mt = 0; Mt < 4; Mt++) {
#pragma unroll
    for (int t = 0; t < 3; t++) {
      wa1[Mt][t] = lds[AW1F + (Mt * 3 + t) * 64 + lane];
      wc1[Mt][t] = lds[CW1F + (Mt * 3 + t) * 64 + lane];
    }
    ba1[Mt] = *(const f4*)(lds + BA1 + 16 * Mt + 4 * g);
    bc1[Mt] = *(const f4*)(lds + BC1 + 16 * Mt + 4 * g);
    ba2[Mt] = *(const f4*)(lds + BA2 + 16 * Mt + 4 * g);
    wc2[Mt] = *(const f4*)(lds + WC2 + 16 * Mt + 4 * g);
#pragma unroll
    for (int d = 0; d < 4; d++) w3[d][Mt] = *(const f4*)(lds + W3 + d * 64 + 16 * Mt + 4 * g);
  }
#pragma unroll 1
  for (; c < nchunks; c += nw) {
    const Smp cur = nxt;
    if (c + nw < nchunks) nxt = gather(c + nw);
    const bool valid = c * 16 + n < ga.samples;
    const float act = cur.act, lpo = cur.lpo, ret = cur.ret, adv = cur.adv;
    {
      const int h = (n >> 1) << 1;
      const f4 v = (h & 2) ? f4{cur.sv[2], cur.sv[3], cur.sv[0], cur.sv[1]} : cur.sv;
      *(f4*)(cb + C_SX + n * 16 + ((4 * g) ^ (h & 12))) = v;
    }
    wave_sync();

    // ---- layer 1, actor and critic ----
    float sB[3];
#pragma unroll
    for (int t = 0; t < 3; t++) sB[t] = cb[C_SX + sx(n, 4 * t + g)];
    // (the 8 accumulators' MFMAs interleaved: a dependent v_mfma_f32_16x16x4_f32 waits 40
    // cycles, an independent one issues after 32; the bias / activation VALU after the last)
    f4 z1[4], zc1[4], h1[4], hc1[4];
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++) { z1[Mt] = z4; zc1[Mt] = z4; }
#pragma unroll
    for (int t = 0; t < 3; t++)
#pragma unroll
      for (int Mt = 0; Mt < 4; Mt++) {
        z1[Mt] = mfma(wa1[Mt][t], sB[t], z1[Mt]);
        zc1[Mt] = mfma(wc1[Mt][t], sB[t], zc1[Mt]);
      }
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        z1[Mt][r] = z1[Mt][r] + ba1[Mt][r];
        zc1[Mt][r] = zc1[Mt][r] + bc1[Mt][r];
        h1[Mt][r] = mf_lrelu(z1[Mt][r]);
        hc1[Mt][r] = mf_lrelu(zc1[Mt][r]);
      }
      *(f4*)(cb + C_H1 + tw(n, 16 * Mt + 4 * g)) = h1[Mt];
      *(f4*)(cb + C_HC1 + tw(n, 16 * Mt + 4 * g)) = hc1[Mt];
    }
    // ---- layer 2 (B operand = layer 1's D registers) ----
    f4 w2[4][4];
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++)
#pragma unroll
      for (int Mp = 0; Mp < 4; Mp++) w2[Mt][Mp] = *(const f4*)(lds + W2F + ((Mt * 4 + Mp) * 64 + lane) * 4);
    // (four chains interleaved, each accumulator's k order (Mp, r) unchanged)
    f4 z2[4], h2[4];
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++) z2[Mt] = z4;
#pragma unroll
    for (int Mp = 0; Mp < 4; Mp++)
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int Mt = 0; Mt < 4; Mt++) z2[Mt] = mfma(w2[Mt][Mp][r], h1[Mp][r], z2[Mt]);
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        z2[Mt][r] = z2[Mt][r] + ba2[Mt][r];
        h2[Mt][r] = mf_lrelu(z2[Mt][r]);
      }
      *(f4*)(cb + C_H2 + tw(n, 16 * Mt + 4 * g)) = h2[Mt];
    }
    // ---- output rows: actor z3[0..3] on h2, critic V on hc1 ----
    float p3[4] = {0.0f, 0.0f, 0.0f, 0.0f}, pv = 0.0f;
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int d = 0; d < 4; d++) p3[d] = p3[d] + w3[d][Mt][r] * h2[Mt][r];
        pv = pv + wc2[Mt][r] * hc1[Mt][r];
      }
    }
    pv = rows_sum4(pv);
    const float z3 = rows_rsum4(p3) + b3g;  // (lane (n, g): dim g)
    const float V = pv + bc2;

    // ---- PPO derivative for action dimension d = g (PPOAgent.cs:234-326) ----
    const float mean = tanhf(z3);
    float criticLoss = 2.0f * (V - ret);
    float fr = (act - mean) / ga.std_;
    fr *= fr;
    fr /= 2.0f;
    const float lp = ga.lp_const - fr;
    const float rr = expf(lp - lpo);
    const float cr = rr >= ga.upper ? ga.upper : (rr <= ga.lower ? ga.lower : rr);
    const float cra = cr * adv, ra = rr * adv;
    const float partA = (ra <= cra ? 1.0f : 0.0f) * adv;
    const float partB = (cra < ra ? 1.0f : 0.0f) * adv;
    const float partC = (rr >= ga.lower && rr <= ga.upper) ? 1.0f : 0.0f;
    float l = partA + (partB * partC);
    l = l * -1.0f;
    const float eo = expf(lpo);
    float zd = eo == 0.0f ? 1.0f : 0.0f;  // Matrix.HadamardDivision throws -> sample skipped
    zd = rows_max4(zd);
    const bool use = valid && zd == 0.0f;
    const float lcd = l / eo;
    const float prob = expf(lp);
    const float frac = (act - mean) / (ga.std_ * ga.std_);
    float actorLoss = (prob * frac) * lcd;
    criticLoss = use ? criticLoss / ga.b_div : 0.0f;
    actorLoss = use ? actorLoss / ga.b_div : 0.0f;
    const float th = mean;  // tanh(z3) again in the reference's backward pass
    const float gz3 = actorLoss * (1.0f - (th * th));
    float al[4], q[4];
    rows_bcast4(actorLoss, al);
    rows_bcast4(gz3, q);
    if (g == 0) {
      diagC += criticLoss;
      diagA += use ? ((((0.0f + al[0]) + al[1]) + al[2]) + al[3]) / 4.0f : 0.0f;
      skipped += (valid && !use) ? 1.0f : 0.0f;
      dbc2 += criticLoss;
      cb[C_G3 + sx(n, 4)] = criticLoss;
    }
    db3 += gz3;
    cb[C_G3 + sx(n, g)] = gz3;
    // ---- gh2 = W3^T gz3 -> gz2; critic gzc1 = (Wc2 dV) * lrelu'(zc1) ----
    f4 gz2[4], gzc1[4];
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float gh = 0.0f;
#pragma unroll
        for (int d = 0; d < 4; d++) gh = gh + w3[d][Mt][r] * q[d];
        gz2[Mt][r] = gh * mf_dlrelu(z2[Mt][r]);
        db2[Mt * 4 + r] += gz2[Mt][r];
        const float ghc1 = 0.0f + wc2[Mt][r] * criticLoss;  // same in the sample's 4 lanes
        gzc1[Mt][r] = ghc1 * mf_dlrelu(zc1[Mt][r]);
      }
      *(f4*)(cb + C_G2 + tw(n, 16 * Mt + 4 * g)) = gz2[Mt];
    }
    wave_sync();
    // ---- dW3 | dWc2 += [gz3; dV]^T [H2 | Hc1]; dW2 += gz2^T H1 (samples on K) ----
    {
      float av[4], bv[4][8], ag[4][4], bh[4][4];
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int s = 4 * t + g;
        av[t] = cb[C_G3 + sx(s, n)];
#pragma unroll
        for (int Nt = 0; Nt < 4; Nt++) {
          bv[t][Nt] = cb[C_H2 + tr(s, 16 * Nt + n)];
          bv[t][Nt + 4] = cb[C_HC1 + tr(s, 16 * Nt + n)];
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
          ag[t][i] = cb[C_G2 + tr(s, 16 * i + n)];
          bh[t][i] = cb[C_H1 + tr(s, 16 * i + n)];
        }
      }
#pragma unroll
      for (int t = 0; t < 4; t++) {
#pragma unroll
        for (int Nt = 0; Nt < 8; Nt++) a3[Nt] = mfma(av[t], bv[t][Nt], a3[Nt]);
#pragma unroll
        for (int Mj = 0; Mj < 4; Mj++)
#pragma unroll
          for (int Nk = 0; Nk < 4; Nk++) a2[Mj][Nk] = mfma(ag[t][Mj], bh[t][Nk], a2[Mj][Nk]);
      }
    }
    wave_sync();  // H2 / Hc1 reads done before G1 / Gc1 overwrite them
    // ---- gh1^T = W2^T gz2^T (B = gz2 registers) -> gz1 ----
    {
#pragma unroll
    for (int Mk = 0; Mk < 4; Mk++)
#pragma unroll
      for (int Mj = 0; Mj < 4; Mj++) w2[Mk][Mj] = *(const f4*)(lds + W2B + ((Mk * 4 + Mj) * 64 + lane) * 4);
    f4 gh1[4];  // (four chains interleaved)
#pragma unroll
    for (int Mk = 0; Mk < 4; Mk++) gh1[Mk] = z4;
#pragma unroll
    for (int Mj = 0; Mj < 4; Mj++)
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int Mk = 0; Mk < 4; Mk++) gh1[Mk] = mfma(w2[Mk][Mj][r], gz2[Mj][r], gh1[Mk]);
#pragma unroll
    for (int Mk = 0; Mk < 4; Mk++) {
      f4 gz1;
#pragma unroll
      for (int r = 0; r < 4; r++) gz1[r] = gh1[Mk][r] * mf_dlrelu(z1[Mk][r]);
      *(f4*)(cb + C_G1 + tw(n, 16 * Mk + 4 * g)) = gz1;
      *(f4*)(cb + C_GC1 + tw(n, 16 * Mk + 4 * g)) = gzc1[Mk];
    }
    }
    wave_sync();
    // ---- dW1 | db1, dWc1 | dbc1 += gz1^T [S | 1] ----
    {
      float bx[4], a1v[4][4], a1cv[4][4];
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int s = 4 * t + g;
        bx[t] = cb[C_SX + sx(s, n)];
#pragma unroll
        for (int Mj = 0; Mj < 4; Mj++) {
          a1v[t][Mj] = cb[C_G1 + tr(s, 16 * Mj + n)];
          a1cv[t][Mj] = cb[C_GC1 + tr(s, 16 * Mj + n)];
        }
      }
#pragma unroll
      for (int t = 0; t < 4; t++)
#pragma unroll
        for (int Mj = 0; Mj < 4; Mj++) {
          a1[Mj] = mfma(a1v[t][Mj], bx[t], a1[Mj]);
          a1c[Mj] = mfma(a1cv[t][Mj], bx[t], a1c[Mj]);
        }
    }
    wave_sync();  // the next chunk rewrites every tile
  }

  // ---- per-lane sums over the 16 sample lanes of each row ----
#pragma unroll
  for (int i = 0; i < 16; i++) db2[i] = row_sum16(db2[i]);
  db3 = row_sum16(db3);
  dbc2 = row_sum16(dbc2);
  diagC = row_sum16(diagC);
  diagA = row_sum16(diagA);
  skipped = row_sum16(skipped);

  // ---- each wave writes its slab, then the block sums them in wave order ----
  __syncthreads();  // every wave is done with the weights and tiles
  float* slab = lds + wave * SLAB;  // every entry below is written exactly once
  if (lane < SLAB - (NPARAM + 3)) slab[NPARAM + 3 + lane] = 0.0f;  // (the pads)
#pragma unroll
  for (int Mj = 0; Mj < 4; Mj++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int j = 16 * Mj + 4 * g + r;
#pragma unroll
      for (int Nk = 0; Nk < 4; Nk++) slab[OFF_A_W2 + j * 64 + 16 * Nk + n] = a2[Mj][Nk][r];
      if (n < 12) {
        slab[OFF_A_W1 + j * 12 + n] = a1[Mj][r];
        slab[OFF_C_W1 + j * 12 + n] = a1c[Mj][r];
      } else if (n == 12) {
        slab[OFF_A_B1 + j] = a1[Mj][r];
        slab[OFF_C_B1 + j] = a1c[Mj][r];
      }
    }
#pragma unroll
  for (int Nt = 0; Nt < 4; Nt++) {
    if (g == 0) {
#pragma unroll
      for (int r = 0; r < 4; r++) slab[OFF_A_W3 + r * 64 + 16 * Nt + n] = a3[Nt][r];
    } else if (g == 1) {
      slab[OFF_C_W2 + 16 * Nt + n] = a3[Nt + 4][0];
    }
  }
  if (n == 0) {
#pragma unroll
    for (int Mt = 0; Mt < 4; Mt++)
#pragma unroll
      for (int r = 0; r < 4; r++) slab[OFF_A_B2 + 16 * Mt + 4 * g + r] = db2[Mt * 4 + r];
    slab[OFF_A_B3 + g] = db3;
    if (g == 0) {
      slab[OFF_C_B2] = dbc2;
      slab[NPARAM] = diagC;
      slab[NPARAM + 1] = diagA;
      slab[NPARAM + 2] = skipped;
    }
  }
  __syncthreads();
  // the block fold, 16 bytes per lane and step with every LDS read of a lane issued up front
  // (same element order: ((0 + w0) + w1) + w2) + w3)
  f4* out = (f4*)(ga.partial + (size_t)blockIdx.x * SLAB);
  constexpr int NV = SLAB / 4, PER = (NV + 64 * WAVES - 1) / (64 * WAVES);
  f4 sv[PER][WAVES];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int i = tid + k * 64 * WAVES;
#pragma unroll
    for (int w = 0; w < WAVES; w++) sv[k][w] = i < NV ? ((const f4*)(lds + w * SLAB))[i] : z4;
  }
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int i = tid + k * 64 * WAVES;
    f4 acc = z4;
#pragma unroll
    for (int w = 0; w < WAVES; w++) acc = acc + sv[k][w];
    if (i < NV) out[i] = acc;
  }
}

// ---------------------------------------------------------------------------------------
// k_ppo_grad_ws: the same minibatch gradient with two waves per SIMD in producer / consumer
// roles (8-wave blocks; waves p and p + 4 form pair p, one SIMD).  One wave per SIMD leaves
// the matrix core idle while the single wave runs its loss / activation VALU chain and waits
// on dependencies (k_ppo_grad_mfma: 40 % MFMA-busy, 40 % of wave cycles in dependency waits,
// profiles/r02_pmc_grad_sq_issue.csv).  Here the producer runs the forward pass, the loss and
// the VALU-side gradients of chunk k (layer 1 and 2: 88 MFMAs) while its partner runs the
// matrix-core backward of chunk k - 1 (dW2, gh1, dW1, dWc1: 160 MFMAs), so the SIMD always
// has independent work from the other wave; one block barrier per chunk step hands the
// chunk's tiles over (double-buffered).
//   producer: gather, Z1 / Zc1 / Z2 (N layout), z3, V, the loss, gz3, dV;
//             dW3 += gz3^T H2, dWc2 += dV^T Hc1 (VALU FMAs into per-lane partials),
//             db2 / db3 / dbc2 / diagnostics; tiles H1, G2 = gz2, GC1 = gzc1, SX = [S | 1]
//   consumer: gh1^T = W2^T gz2^T (B = gz2 read back in N layout), gz1 = gh1 * lrelu'(h1),
//             dW2 += gz2^T H1, then G1 (into the consumed H1 buffer), dW1 | db1 += gz1^T
//             [S | 1], dWc1 | dbc1 += gzc1^T [S | 1]
// Tiles [16 samples][68] (4 rows = 16 banks apart) and SX [16][20]: every access below is
// bank-conflict-free; the sample contractions take K step r = samples 4 g + r.  A pair's
// producer and consumer own disjoint parameters, so they write one slab and the block folds
// the four pair slabs in pair order (ordered reduction as before).
namespace ws {
enum : int {
  RT = 68, T68 = 16 * RT, RSX = 20, TSX = 16 * RSX,
  O_SX = 0, O_H1 = TSX, O_G2 = O_H1 + T68, O_GC1 = O_G2 + T68, TB = O_GC1 + T68,
  PAIRS = 4,
  LOOP_FLOATS = mf::WEND + PAIRS * 2 * TB,
  LDS_FLOATS = LOOP_FLOATS > PAIRS * SLAB ? LOOP_FLOATS : PAIRS * SLAB
};
static_assert(LOOP_FLOATS * 4 <= 160 * 1024, "fits the CU's LDS");
static_assert(TB % 4 == 0 && T68 % 4 == 0 && TSX % 4 == 0, "16-byte aligned tiles");
}  // namespace ws

__global__ __launch_bounds__(64 * 2 * ws::PAIRS) void k_ppo_grad_ws(GradArgs ga) {
  using namespace mf;
  using namespace ws;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;
  // Pairs by SIMD: the two waves that share a SIMD (HW_ID.SIMD_ID) become its producer and
  // consumer, so each SIMD holds one wave of each role whatever the wave placement; if the
  // eight waves do not sit two per SIMD, pair p = waves p and p + 4.  (The role is
  // wave-uniform in an SGPR: scalar branches, so each wave executes only its own path's
  // barriers -- both paths execute the same number.)
  // the weight image into LDS first, by the block's first four waves (the first launched): their
  // loads are in flight while the others launch, and the pairing barrier below publishes the image
  // with the SIMD ids (one block barrier and one L2 round trip fewer before the first chunk)
  if (tid < 256) {
    constexpr int NV = WEND / 4, PER = (NV + 256 - 1) / 256;
    f4 wv[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) {
      const int e = tid + i * 256;
      if (e < NV) wv[i] = ((const f4*)ga.Wz)[e];
    }
#pragma unroll
    for (int i = 0; i < PER; i++) {
      const int e = tid + i * 256;
      if (e < NV) ((f4*)lds)[e] = wv[i];
    }
  }
  __shared__ int simd_of[2 * PAIRS];
  if (lane == 0) simd_of[wave] = (int)((__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4) >> 0) & 3);
  __syncthreads();
  int pair = wave & 3;
  bool producer = wave < PAIRS;
  {
    int cnt[PAIRS] = {0, 0, 0, 0}, first[PAIRS] = {-1, -1, -1, -1};
#pragma unroll
    for (int w = 0; w < 2 * PAIRS; w++) {
      const int sm = simd_of[w];
#pragma unroll
      for (int q = 0; q < PAIRS; q++) {
        cnt[q] += sm == q ? 1 : 0;
        first[q] = (sm == q && first[q] < 0) ? w : first[q];
      }
    }
    bool two_each = true;
#pragma unroll
    for (int q = 0; q < PAIRS; q++) two_each = two_each && cnt[q] == 2;
    if (two_each) {
      pair = simd_of[wave];
      producer = first[pair] == wave;
    }
  }
  pair = __builtin_amdgcn_readfirstlane(pair);
  producer = __builtin_amdgcn_readfirstlane(producer ? 1 : 0) != 0;
  const int nchunks = (ga.samples + 15) / 16;
  const int nw = gridDim.x * PAIRS;
  const int c0 = blockIdx.x * PAIRS + pair;
  const int kp = c0 < nchunks ? (nchunks - 1 - c0) / nw + 1 : 0;         // this pair's chunks
  const int kmax = blockIdx.x * PAIRS < nchunks ? (nchunks - 1 - blockIdx.x * PAIRS) / nw + 1 : 0;

  struct Smp { f4 sv; float act, lpo, ret, adv; };
  auto gather = [&](int c) {
    Smp m;
    const int pos = c * 16 + n;
    uint32_t idx = ga.base + (uint32_t)(pos < ga.samples ? pos : 0);
    if (ga.use_perm) idx = perm_apply(idx, ga.pk);
    // (the lane group through an opaque copy: hoisted, `states + 4 g` was a per-lane 64-bit base
    // the allocator kept in scratch and reloaded before every chunk's gather)
    uint32_t go = (uint32_t)g;
    asm volatile("" : "+v"(go));
    m.sv = f4{1.0f, 0.0f, 0.0f, 0.0f};  // lane group 3: the bias column
    if (g < 3) m.sv = *(const f4*)(ga.states + ((size_t)idx * 12 + 4 * go));
    m.act = ga.actions[(size_t)idx * 4 + go];
    m.lpo = ga.logp_old[(size_t)idx * 4 + go];
    m.ret = ga.returns[idx];
    m.adv = ga.adv[idx];
    return m;
  };
  Smp nxt;
  if (producer) nxt = gather(c0 < nchunks ? c0 : 0);
  float* const pt = lds + WEND + pair * 2 * TB;  // this pair's two tile buffers
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};

  f4 a2[4][4], a1[4], a1c[4];  // the consumer's accumulators (written into its slab at the end)
  if (producer) {
    // ---------------- producer ----------------
    // (the producer's dependent chain sets the pace: the SIMD's arbiter serves it first, the
    // consumer's independent MFMAs fill the gaps)
    __builtin_amdgcn_s_setprio(2);
    f4 aw3[4][4], awc2[4], db2[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      awc2[i] = z4; db2[i] = z4;
#pragma unroll
      for (int j = 0; j < 4; j++) aw3[i][j] = z4;
    }
    float db3 = 0.0f, dbc2 = 0.0f, diagC = 0.0f, diagA = 0.0f, skipped = 0.0f;
    const float b3g = lds[BA3 + g], bc2 = lds[BC2];
    float wa1[4][3], wc1[4][3];
#pragma unroll
    for (int M = 0; M < 4; M++)
#pragma unroll
      for (int t = 0; t < 3; t++) {
        wa1[M][t] = lds[AW1F + (M * 3 + t) * 64 + lane];
        wc1[M][t] = lds[CW1F + (M * 3 + t) * 64 + lane];
      }
#pragma unroll 1
    for (int i = 0; i <= kmax; i++) {
      if (i < kp) {
        const int c = c0 + i * nw;
        float* const tb = pt + (i & 1) * TB;
        const Smp cur = nxt;
        if (i + 1 < kp) nxt = gather(c + nw);
        const bool valid = c * 16 + n < ga.samples;
        *(f4*)(tb + O_SX + n * RSX + 4 * g) = cur.sv;
        wave_sync();
        float sB[3];
#pragma unroll
        for (int t = 0; t < 3; t++) sB[t] = tb[O_SX + n * RSX + 4 * t + g];
        // ---- layer 1, actor and critic (N layout) ----
        f4 z1[4], zc1[4], h1[4], hc1[4];
#pragma unroll
        for (int M = 0; M < 4; M++) { z1[M] = z4; zc1[M] = z4; }
#pragma unroll
        for (int t = 0; t < 3; t++)
#pragma unroll
          for (int M = 0; M < 4; M++) {
            z1[M] = mfma(wa1[M][t], sB[t], z1[M]);
            zc1[M] = mfma(wc1[M][t], sB[t], zc1[M]);
          }
#pragma unroll
        for (int M = 0; M < 4; M++) {
          const f4 b1 = *(const f4*)(lds + BA1 + 16 * M + 4 * g);
          const f4 c1 = *(const f4*)(lds + BC1 + 16 * M + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; r++) {
            h1[M][r] = mf_lrelu(z1[M][r] + b1[r]);
            hc1[M][r] = mf_lrelu(zc1[M][r] + c1[r]);
          }
          *(f4*)(tb + O_H1 + n * RT + 16 * M + 4 * g) = h1[M];
        }
        // ---- layer 2 (B operand = layer 1's registers) ----
        f4 z2[4], h2[4];
#pragma unroll
        for (int M = 0; M < 4; M++) z2[M] = z4;
#pragma unroll
        for (int Mp = 0; Mp < 4; Mp++) {
          f4 w2[4];
#pragma unroll
          for (int M = 0; M < 4; M++) w2[M] = *(const f4*)(lds + W2F + ((M * 4 + Mp) * 64 + lane) * 4);
#pragma unroll
          for (int r = 0; r < 4; r++)
#pragma unroll
            for (int M = 0; M < 4; M++) z2[M] = mfma(w2[M][r], h1[Mp][r], z2[M]);
        }
#pragma unroll
        for (int M = 0; M < 4; M++) {
          const f4 b2 = *(const f4*)(lds + BA2 + 16 * M + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; r++) h2[M][r] = mf_lrelu(z2[M][r] + b2[r]);
        }
        // ---- output rows: actor z3[0..3] on h2, critic V on hc1 ----
        float p3[4] = {0.0f, 0.0f, 0.0f, 0.0f}, pv = 0.0f;
#pragma unroll
        for (int M = 0; M < 4; M++) {
          const f4 wc2 = *(const f4*)(lds + WC2 + 16 * M + 4 * g);
#pragma unroll
          for (int d = 0; d < 4; d++) {
            const f4 w3 = *(const f4*)(lds + W3 + d * 64 + 16 * M + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; r++) p3[d] = __builtin_fmaf(w3[r], h2[M][r], p3[d]);
          }
#pragma unroll
          for (int r = 0; r < 4; r++) pv = __builtin_fmaf(wc2[r], hc1[M][r], pv);
        }
        pv = rows_sum4(pv);
        const float z3 = rows_rsum4(p3) + b3g;  // (lane (n, g): dim g)
        const float V = pv + bc2;
        // ---- PPO derivative for action dimension d = g (PPOAgent.cs:234-326) ----
        const float act = cur.act, lpo = cur.lpo, ret = cur.ret, adv = cur.adv;
        const float mean = tanhf(z3);
        float criticLoss = 2.0f * (V - ret);
        float fr = (act - mean) / ga.std_;
        fr *= fr;
        fr /= 2.0f;
        const float lp = ga.lp_const - fr;
        const float rr = expf(lp - lpo);
        const float cr = rr >= ga.upper ? ga.upper : (rr <= ga.lower ? ga.lower : rr);
        const float cra = cr * adv, ra = rr * adv;
        const float partA = (ra <= cra ? 1.0f : 0.0f) * adv;
        const float partB = (cra < ra ? 1.0f : 0.0f) * adv;
        const float partC = (rr >= ga.lower && rr <= ga.upper) ? 1.0f : 0.0f;
        float l = partA + (partB * partC);
        l = l * -1.0f;
        const float eo = expf(lpo);
        float zd = eo == 0.0f ? 1.0f : 0.0f;  // Matrix.HadamardDivision throws -> sample skipped
        zd = rows_max4(zd);
        const bool use = valid && zd == 0.0f;
        const float lcd = l / eo;
        const float prob = expf(lp);
        const float frac = (act - mean) / (ga.std_ * ga.std_);
        float actorLoss = (prob * frac) * lcd;
        criticLoss = use ? criticLoss / ga.b_div : 0.0f;
        actorLoss = use ? actorLoss / ga.b_div : 0.0f;
        const float th = mean;  // tanh(z3) again in the reference's backward pass
        const float gz3 = actorLoss * (1.0f - (th * th));
        float al[4], q[4];
        rows_bcast4(actorLoss, al);
        rows_bcast4(gz3, q);
        if (g == 0) {
          diagC += criticLoss;
          diagA += use ? ((((0.0f + al[0]) + al[1]) + al[2]) + al[3]) / 4.0f : 0.0f;
          skipped += (valid && !use) ? 1.0f : 0.0f;
          dbc2 += criticLoss;
        }
        db3 += gz3;
        // ---- dW3 += gz3^T H2, dWc2 += dV^T Hc1 (per-lane partials over this lane's samples);
        // gz2 = (W3^T gz3) * lrelu'(z2), gzc1 = (Wc2 dV) * lrelu'(zc1) ----
#pragma unroll
        for (int M = 0; M < 4; M++) {
          const f4 wc2 = *(const f4*)(lds + WC2 + 16 * M + 4 * g);
          f4 w3[4];
#pragma unroll
          for (int d = 0; d < 4; d++) w3[d] = *(const f4*)(lds + W3 + d * 64 + 16 * M + 4 * g);
          f4 gz2, gzc1;
#pragma unroll
          for (int r = 0; r < 4; r++) {
#pragma unroll
            for (int d = 0; d < 4; d++) aw3[d][M][r] = __builtin_fmaf(q[d], h2[M][r], aw3[d][M][r]);
            awc2[M][r] = __builtin_fmaf(criticLoss, hc1[M][r], awc2[M][r]);
            float gh = 0.0f;
#pragma unroll
            for (int d = 0; d < 4; d++) gh = __builtin_fmaf(w3[d][r], q[d], gh);
            gz2[r] = gh * mf_dlrelu(h2[M][r]);
            gzc1[r] = (0.0f + wc2[r] * criticLoss) * mf_dlrelu(hc1[M][r]);
          }
          db2[M] = db2[M] + gz2;
          *(f4*)(tb + O_G2 + n * RT + 16 * M + 4 * g) = gz2;
          *(f4*)(tb + O_GC1 + n * RT + 16 * M + 4 * g) = gzc1;
        }
      }
      __syncthreads();  // chunk i's tiles to the consumer; its reads of buffer (i - 1) & 1 done
    }
    __syncthreads();  // every wave is done with the weights and tiles
    // ---- the producer's per-lane partials summed over the 16 sample lanes of each row, in
    // registers (row_tree16: the tree the former pass through LDS used, bit for bit), and the
    // row's first lane writes the sum into the pair slab (v order of the old pass: db2, dWc2,
    // dW3 by (d, M, r), db3; dbc2 and the three diagnostics from row 0 only) ----
    float* const slab = lds + pair * SLAB;
    const bool head = n == 0;
#pragma unroll
    for (int M = 0; M < 4; M++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const float sb = row_tree16(db2[M][r]), sc = row_tree16(awc2[M][r]);
        if (head) {
          slab[OFF_A_B2 + 16 * M + 4 * g + r] = sb;
          slab[OFF_C_W2 + 16 * M + 4 * g + r] = sc;
        }
#pragma unroll
        for (int d = 0; d < 4; d++) {
          const float sw = row_tree16(aw3[d][M][r]);
          if (head) slab[OFF_A_W3 + d * 64 + 16 * M + 4 * g + r] = sw;
        }
      }
    {
      const float s3 = row_tree16(db3), sv = row_tree16(dbc2), sC = row_tree16(diagC);
      const float sA = row_tree16(diagA), sk = row_tree16(skipped);
      if (head) slab[OFF_A_B3 + g] = s3;
      if (head && g == 0) {
        slab[OFF_C_B2] = sv;
        slab[NPARAM] = sC;
        slab[NPARAM + 1] = sA;
        slab[NPARAM + 2] = sk;
      }
    }
    if (lane < SLAB - (NPARAM + 3)) slab[NPARAM + 3 + lane] = 0.0f;  // (the pads)
  } else {
    // ---------------- consumer ----------------
#pragma unroll
    for (int i = 0; i < 4; i++) {
      a1[i] = z4; a1c[i] = z4;
#pragma unroll
      for (int j = 0; j < 4; j++) a2[i][j] = z4;
    }
#pragma unroll 1
    for (int i = 0; i <= kmax; i++) {
      if (i >= 1 && i <= kp) {
        float* const tb = pt + ((i - 1) & 1) * TB;
        // gz2 and h1 in N layout (the producer's own registers, read back)
        f4 gz2[4], dh1[4];
#pragma unroll
        for (int M = 0; M < 4; M++) {
          gz2[M] = *(const f4*)(tb + O_G2 + n * RT + 16 * M + 4 * g);
          const f4 h = *(const f4*)(tb + O_H1 + n * RT + 16 * M + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; r++) dh1[M][r] = mf_dlrelu(h[r]);  // lrelu(z) < 0 iff z < 0
        }
        // ---- dW2 += gz2^T H1 (samples on K: step r = samples 4 g + r) ----
        {
          float ag[4][4], bh[4][4];
#pragma unroll
          for (int r = 0; r < 4; r++)
#pragma unroll
            for (int M = 0; M < 4; M++) {
              ag[r][M] = tb[O_G2 + (4 * g + r) * RT + 16 * M + n];
              bh[r][M] = tb[O_H1 + (4 * g + r) * RT + 16 * M + n];
            }
#pragma unroll
          for (int r = 0; r < 4; r++)
#pragma unroll
            for (int Mj = 0; Mj < 4; Mj++)
#pragma unroll
              for (int Nk = 0; Nk < 4; Nk++) a2[Mj][Nk] = mfma(ag[r][Mj], bh[r][Nk], a2[Mj][Nk]);
        }
        // ---- gh1^T = W2^T gz2^T (B = gz2 registers) -> gz1 ----
        f4 gh1[4];
#pragma unroll
        for (int Mk = 0; Mk < 4; Mk++) gh1[Mk] = z4;
#pragma unroll
        for (int Mj = 0; Mj < 4; Mj++) {
          f4 w2[4];
#pragma unroll
          for (int Mk = 0; Mk < 4; Mk++) w2[Mk] = *(const f4*)(lds + W2B + ((Mk * 4 + Mj) * 64 + lane) * 4);
#pragma unroll
          for (int r = 0; r < 4; r++)
#pragma unroll
            for (int Mk = 0; Mk < 4; Mk++) gh1[Mk] = mfma(w2[Mk][r], gz2[Mj][r], gh1[Mk]);
        }
        wave_sync();  // the H1 reads are done: G1 goes into its buffer
#pragma unroll
        for (int Mk = 0; Mk < 4; Mk++) {
          f4 gz1;
#pragma unroll
          for (int r = 0; r < 4; r++) gz1[r] = gh1[Mk][r] * dh1[Mk][r];
          *(f4*)(tb + O_H1 + n * RT + 16 * Mk + 4 * g) = gz1;
        }
        wave_sync();
        // ---- dW1 | db1 += gz1^T [S | 1], dWc1 | dbc1 += gzc1^T [S | 1] ----
        {
          float bx[4], av[4][4], acv[4][4];
#pragma unroll
          for (int r = 0; r < 4; r++) {
            bx[r] = tb[O_SX + (4 * g + r) * RSX + n];
#pragma unroll
            for (int Mj = 0; Mj < 4; Mj++) {
              av[r][Mj] = tb[O_H1 + (4 * g + r) * RT + 16 * Mj + n];
              acv[r][Mj] = tb[O_GC1 + (4 * g + r) * RT + 16 * Mj + n];
            }
          }
#pragma unroll
          for (int r = 0; r < 4; r++)
#pragma unroll
            for (int Mj = 0; Mj < 4; Mj++) {
              a1[Mj] = mfma(av[r][Mj], bx[r], a1[Mj]);
              a1c[Mj] = mfma(acv[r][Mj], bx[r], a1c[Mj]);
            }
        }
      }
      __syncthreads();
    }
    __syncthreads();  // (matches the producer's: weights and tiles are free)
    float* const slab = lds + pair * SLAB;
#pragma unroll
    for (int Mj = 0; Mj < 4; Mj++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int j = 16 * Mj + 4 * g + r;
#pragma unroll
        for (int Nk = 0; Nk < 4; Nk++) slab[OFF_A_W2 + j * 64 + 16 * Nk + n] = a2[Mj][Nk][r];
        if (n < 12) {
          slab[OFF_A_W1 + j * 12 + n] = a1[Mj][r];
          slab[OFF_C_W1 + j * 12 + n] = a1c[Mj][r];
        } else if (n == 12) {
          slab[OFF_A_B1 + j] = a1[Mj][r];
          slab[OFF_C_B1 + j] = a1c[Mj][r];
        }
      }
  }
  __syncthreads();  // the pair slabs are complete
  // the block fold over the four pair slabs, in pair order
  const SlabOut out(ga.partial + (size_t)blockIdx.x * SLAB);
  constexpr int NV = SLAB / 4, PER = (NV + 512 - 1) / 512;
  // (the thread index through an opaque copy: otherwise the prologue's 16-byte offset of the
  // weight copy is reused here and kept in scratch across the chunk loop)
  int tf = tid;
  asm volatile("" : "+v"(tf));
  f4 sv[PER][PAIRS];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int i = tf + k * 512;
#pragma unroll
    for (int w = 0; w < PAIRS; w++) sv[k][w] = i < NV ? ((const f4*)(lds + w * SLAB))[i] : z4;
  }
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int i = tf + k * 512;
    f4 acc = z4;
#pragma unroll
    for (int w = 0; w < PAIRS; w++) acc = acc + sv[k][w];
    if (i < NV) out.put(i, acc);
  }
}

// ---------------------------------------------------------------------------------------
// k_ppo_grad_tp: the same minibatch gradient with the neurons of one chunk split over the four
// waves of a team ("tile-parallel").  k_ppo_grad_ws runs a chunk's 248 MFMAs and its loss chain
// on one SIMD, so a launch is at least one chunk's serial latency plus the weight staging: at a
// strong-scaling shard (8,192 samples = 512 chunks, one per SIMD pair) that is 15 us for 1.9 us
// of matrix work.  Here wave w of a team owns neuron tile w (neurons 16 w .. 16 w + 15 of every
// 64-wide layer) and with it a disjoint quarter of the parameters:
//   layer 1   z1 / zc1 of tile w                         (6 MFMAs, K 12)
//   layer 2   z2 of tile w = W2[tile w][:] H1            (16 MFMAs, B = H1 tile from LDS)
//   rows      z3 / V partial dots over the tile's 16 neurons, summed over the team in LDS
//   loss      every wave, redundantly (the same values in all four)
//   VALU      dW3 / dWc2 / db2 partials and gz2 / gzc1 of tile w
//   backward  dW2[tile w][:] += gz2^T H1                 (16 MFMAs)
//             gh1 of tile w = W2[:][tile w]^T gz2        (16 MFMAs, B = G2 tile from LDS)
//             dW1 | db1, dWc1 | dbc1 rows of tile w      (8 MFMAs)
// 62 MFMAs per wave and chunk, three block barriers per chunk (shared by the block's teams),
// weights in registers straight from the image (no LDS staging).  Every accumulator's k order
// is the one k_ppo_grad_ws uses; only the z3 / V dots are associated per tile.  A block holds
// TEAMS teams on separate chunks (two waves per SIMD).  At the end each wave writes its own
// parameters into its team's slab in LDS and the block writes the teams' sum (team order) as
// its partial slab.
namespace tp {
enum : int {
  RT = 68, T68 = 16 * RT, RSX = 20, TSX = 16 * RSX, RP = 80,  // P: [wave 4][d 5][16 samples]
  O_SX = 0, O_H1 = TSX, O_G2 = O_H1 + T68, O_GC1 = O_G2 + T68, O_G1 = O_GC1 + T68,
  O_P = O_G1 + T68, TB = O_P + 4 * RP
};
static_assert(TB % 4 == 0, "16-byte aligned tiles");
template <int TEAMS> struct L {
  enum : int { LOOP = TEAMS * 2 * TB, FLOATS = LOOP > TEAMS * SLAB ? LOOP : TEAMS * SLAB };
  static_assert(FLOATS * 4 <= 160 * 1024, "fits the CU's LDS");
};
}  // namespace tp

template <int TEAMS>
__global__ __launch_bounds__(256 * TEAMS) void k_ppo_grad_tp(GradArgs ga) {
  using namespace mf;
  using namespace tp;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int team = wv >> 2, w = wv & 3;
  const int n = lane & 15, g = lane >> 4;
  const int nchunks = (ga.samples + 15) / 16;
  const int nt = gridDim.x * TEAMS;
  const int c0 = blockIdx.x * TEAMS + team;
  const int kp = c0 < nchunks ? (nchunks - 1 - c0) / nt + 1 : 0;  // this team's chunks
  const int kmax = blockIdx.x * TEAMS < nchunks ? (nchunks - 1 - blockIdx.x * TEAMS) / nt + 1 : 0;
  const f4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};

  // gather (CreateBatches, PPOAgent.cs:512-533): lane (n, g) holds features g, 4 + g, 8 + g of
  // sample n (layer 1's B operand) and the sample's action dim g entries
  struct Smp { float s[3]; float act, lpo, ret, adv; };
  auto gather = [&](int c) {
    Smp m;
    const int pos = c * 16 + n;
    uint32_t idx = ga.base + (uint32_t)(pos < ga.samples ? pos : 0);
    if (ga.use_perm) idx = perm_apply(idx, ga.pk);
#pragma unroll
    for (int t = 0; t < 3; t++) m.s[t] = ga.states[(size_t)idx * 12 + 4 * t + g];
    m.act = ga.actions[(size_t)idx * 4 + g];
    m.lpo = ga.logp_old[(size_t)idx * 4 + g];
    m.ret = ga.returns[idx];
    m.adv = ga.adv[idx];
    return m;
  };
  Smp nxt = gather(c0 < nchunks ? c0 : 0);

  // this wave's weights (image order, wk_mfma_layout.h), loaded once into registers
  float wa1[3], wc1[3];
  f4 w2f[4], w2b[4], w3[4];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    wa1[t] = ga.Wz[AW1F + (w * 3 + t) * 64 + lane];
    wc1[t] = ga.Wz[CW1F + (w * 3 + t) * 64 + lane];
  }
#pragma unroll
  for (int M = 0; M < 4; M++) {
    w2f[M] = *(const f4*)(ga.Wz + W2F + ((w * 4 + M) * 64 + lane) * 4);
    w2b[M] = *(const f4*)(ga.Wz + W2B + ((w * 4 + M) * 64 + lane) * 4);
  }
#pragma unroll
  for (int d = 0; d < 4; d++) w3[d] = *(const f4*)(ga.Wz + W3 + d * 64 + 16 * w + 4 * g);
  const f4 wc2 = *(const f4*)(ga.Wz + WC2 + 16 * w + 4 * g);
  const f4 ba1 = *(const f4*)(ga.Wz + BA1 + 16 * w + 4 * g);
  const f4 bc1 = *(const f4*)(ga.Wz + BC1 + 16 * w + 4 * g);
  const f4 ba2 = *(const f4*)(ga.Wz + BA2 + 16 * w + 4 * g);
  const float b3g = ga.Wz[BA3 + g], bc2 = ga.Wz[BC2];

  float* const tt = lds + team * 2 * TB;  // this team's two chunk buffers
  // the SX tiles' constant columns: 12 = 1.0 (the bias column), 13..15 = 0
  if (w == 0 && g == 0) {
#pragma unroll
    for (int b = 0; b < 2; b++)
      *(f4*)(tt + b * TB + O_SX + n * RSX + 12) = f4{1.0f, 0.0f, 0.0f, 0.0f};
  }

  f4 a2[4], aw3[4], a1 = z4, a1c = z4, awc2 = z4, db2 = z4;
#pragma unroll
  for (int i = 0; i < 4; i++) { a2[i] = z4; aw3[i] = z4; }
  float db3 = 0.0f, dbc2 = 0.0f, diagC = 0.0f, diagA = 0.0f, skipped = 0.0f;

#pragma unroll 1
  for (int i = 0; i < kmax; i++) {
    const bool live = i < kp;  // team-uniform; a finished team still meets the barriers
    const int c = c0 + i * nt;
    float* const tb = tt + (i & 1) * TB;
    const Smp cur = nxt;
    if (i + 1 < kp) nxt = gather(c + nt);
    const bool valid = c * 16 + n < ga.samples;
    f4 h1 = z4, hc1 = z4;
    if (live) {
      if (w == 0) {
#pragma unroll
        for (int t = 0; t < 3; t++) tb[O_SX + n * RSX + 4 * t + g] = cur.s[t];
      }
      // ---- layer 1 of tile w ----
      f4 z1 = z4, zc1 = z4;
#pragma unroll
      for (int t = 0; t < 3; t++) {
        z1 = mfma(wa1[t], cur.s[t], z1);
        zc1 = mfma(wc1[t], cur.s[t], zc1);
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        h1[r] = mf_lrelu(z1[r] + ba1[r]);
        hc1[r] = mf_lrelu(zc1[r] + bc1[r]);
      }
      *(f4*)(tb + O_H1 + n * RT + 16 * w + 4 * g) = h1;
    }
    __syncthreads();  // B1: the team's H1 tile
    f4 h2 = z4;
    if (live) {
      // ---- layer 2 of tile w (k order (Mp, r), as k_ppo_grad_ws) ----
      f4 hb[4];
#pragma unroll
      for (int Mp = 0; Mp < 4; Mp++) hb[Mp] = *(const f4*)(tb + O_H1 + n * RT + 16 * Mp + 4 * g);
      f4 z2 = z4;
#pragma unroll
      for (int Mp = 0; Mp < 4; Mp++)
#pragma unroll
        for (int r = 0; r < 4; r++) z2 = mfma(w2f[Mp][r], hb[Mp][r], z2);
#pragma unroll
      for (int r = 0; r < 4; r++) h2[r] = mf_lrelu(z2[r] + ba2[r]);
      // ---- the output rows' partial dots over the tile ----
      float p3[4] = {0.0f, 0.0f, 0.0f, 0.0f}, pv = 0.0f;
#pragma unroll
      for (int d = 0; d < 4; d++)
#pragma unroll
        for (int r = 0; r < 4; r++) p3[d] = __builtin_fmaf(w3[d][r], h2[r], p3[d]);
#pragma unroll
      for (int r = 0; r < 4; r++) pv = __builtin_fmaf(wc2[r], hc1[r], pv);
      pv = rows_sum4(pv);
      // lane (n, g) stores dim g's partial, lanes of group 0 also V's
      tb[O_P + w * RP + g * 16 + n] = rows_rsum4(p3);
      if (g == 0) tb[O_P + w * RP + 64 + n] = pv;
    }
    __syncthreads();  // B2: the team's partial dots
    if (live) {
      float z3 = 0.0f, pv = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        z3 = z3 + tb[O_P + q * RP + g * 16 + n];
        pv = pv + tb[O_P + q * RP + 64 + n];
      }
      z3 = z3 + b3g;
      const float V = pv + bc2;
      // ---- PPO derivative for action dimension d = g (PPOAgent.cs:234-326) ----
      const float act = cur.act, lpo = cur.lpo, ret = cur.ret, adv = cur.adv;
      const float mean = tanhf(z3);
      float criticLoss = 2.0f * (V - ret);
      float fr = (act - mean) / ga.std_;
      fr *= fr;
      fr /= 2.0f;
      const float lp = ga.lp_const - fr;
      const float rr = expf(lp - lpo);
      const float cr = rr >= ga.upper ? ga.upper : (rr <= ga.lower ? ga.lower : rr);
      const float cra = cr * adv, ra = rr * adv;
      const float partA = (ra <= cra ? 1.0f : 0.0f) * adv;
      const float partB = (cra < ra ? 1.0f : 0.0f) * adv;
      const float partC = (rr >= ga.lower && rr <= ga.upper) ? 1.0f : 0.0f;
      float l = partA + (partB * partC);
      l = l * -1.0f;
      const float eo = expf(lpo);
      float zd = eo == 0.0f ? 1.0f : 0.0f;  // Matrix.HadamardDivision throws -> sample skipped
      zd = rows_max4(zd);
      const bool use = valid && zd == 0.0f;
      const float lcd = l / eo;
      const float prob = expf(lp);
      const float frac = (act - mean) / (ga.std_ * ga.std_);
      float actorLoss = (prob * frac) * lcd;
      criticLoss = use ? criticLoss / ga.b_div : 0.0f;
      actorLoss = use ? actorLoss / ga.b_div : 0.0f;
      const float th = mean;  // tanh(z3) again in the reference's backward pass
      const float gz3 = actorLoss * (1.0f - (th * th));
      float q[4];
      rows_bcast4(gz3, q);
      if (w == 0) {  // the sample-level terms, once per team
        float al[4];
        rows_bcast4(actorLoss, al);
        if (g == 0) {
          diagC += criticLoss;
          diagA += use ? ((((0.0f + al[0]) + al[1]) + al[2]) + al[3]) / 4.0f : 0.0f;
          skipped += (valid && !use) ? 1.0f : 0.0f;
          dbc2 += criticLoss;
        }
        db3 += gz3;
      }
      // ---- dW3 / dWc2 partials, gz2 / gzc1 of tile w ----
      f4 gz2, gzc1;
#pragma unroll
      for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int d = 0; d < 4; d++) aw3[d][r] = __builtin_fmaf(q[d], h2[r], aw3[d][r]);
        awc2[r] = __builtin_fmaf(criticLoss, hc1[r], awc2[r]);
        float gh = 0.0f;
#pragma unroll
        for (int d = 0; d < 4; d++) gh = __builtin_fmaf(w3[d][r], q[d], gh);
        gz2[r] = gh * mf_dlrelu(h2[r]);
        gzc1[r] = (0.0f + wc2[r] * criticLoss) * mf_dlrelu(hc1[r]);
      }
      db2 = db2 + gz2;
      *(f4*)(tb + O_G2 + n * RT + 16 * w + 4 * g) = gz2;
      *(f4*)(tb + O_GC1 + n * RT + 16 * w + 4 * g) = gzc1;
    }
    __syncthreads();  // B3: the team's G2 tile
    if (live) {
      // ---- dW2[tile w][:] += gz2^T H1 (samples on K: step r = samples 4 g + r) ----
      {
        float ag[4], bh[4][4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          ag[r] = tb[O_G2 + (4 * g + r) * RT + 16 * w + n];
#pragma unroll
          for (int Nk = 0; Nk < 4; Nk++) bh[r][Nk] = tb[O_H1 + (4 * g + r) * RT + 16 * Nk + n];
        }
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int Nk = 0; Nk < 4; Nk++) a2[Nk] = mfma(ag[r], bh[r][Nk], a2[Nk]);
      }
      // ---- gh1 of tile w = W2[:][tile w]^T gz2 (B = the G2 tile) -> gz1 ----
      f4 gb[4];
#pragma unroll
      for (int Mj = 0; Mj < 4; Mj++) gb[Mj] = *(const f4*)(tb + O_G2 + n * RT + 16 * Mj + 4 * g);
      f4 gh1 = z4;
#pragma unroll
      for (int Mj = 0; Mj < 4; Mj++)
#pragma unroll
        for (int r = 0; r < 4; r++) gh1 = mfma(w2b[Mj][r], gb[Mj][r], gh1);
      f4 gz1;
#pragma unroll
      for (int r = 0; r < 4; r++) gz1[r] = gh1[r] * mf_dlrelu(h1[r]);  // lrelu(z) < 0 iff z < 0
      *(f4*)(tb + O_G1 + n * RT + 16 * w + 4 * g) = gz1;  // this wave's columns only
      wave_sync();
      // ---- dW1 | db1, dWc1 | dbc1 rows of tile w += gz1^T [S | 1] ----
      float bx[4], av[4], acv[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        bx[r] = tb[O_SX + (4 * g + r) * RSX + n];
        av[r] = tb[O_G1 + (4 * g + r) * RT + 16 * w + n];
        acv[r] = tb[O_GC1 + (4 * g + r) * RT + 16 * w + n];
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        a1 = mfma(av[r], bx[r], a1);
        a1c = mfma(acv[r], bx[r], a1c);
      }
    }
  }

  // ---- totals over the 16 sample lanes of each row, then this wave's part of the slab ----
#pragma unroll
  for (int r = 0; r < 4; r++) {
    db2[r] = row_sum16(db2[r]);
    awc2[r] = row_sum16(awc2[r]);
#pragma unroll
    for (int d = 0; d < 4; d++) aw3[d][r] = row_sum16(aw3[d][r]);
  }
  db3 = row_sum16(db3);
  dbc2 = row_sum16(dbc2);
  diagC = row_sum16(diagC);
  diagA = row_sum16(diagA);
  skipped = row_sum16(skipped);
  // each team's slab in LDS in parameter order (every entry written by exactly one wave of
  // the team), then the block writes (t0 [+ t1]) with 16-byte coalesced stores
  __syncthreads();  // every wave is done with the tiles
  float* const slab = lds + team * SLAB;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int j = 16 * w + 4 * g + r;
#pragma unroll
    for (int Nk = 0; Nk < 4; Nk++) slab[OFF_A_W2 + j * 64 + 16 * Nk + n] = a2[Nk][r];
    if (n < 12) {
      slab[OFF_A_W1 + j * 12 + n] = a1[r];
      slab[OFF_C_W1 + j * 12 + n] = a1c[r];
    } else if (n == 12) {
      slab[OFF_A_B1 + j] = a1[r];
      slab[OFF_C_B1 + j] = a1c[r];
    } else if (n == 13) {
      slab[OFF_A_B2 + j] = db2[r];
      slab[OFF_C_W2 + j] = awc2[r];
    } else if (n == 14) {
#pragma unroll
      for (int d = 0; d < 4; d++) slab[OFF_A_W3 + d * 64 + j] = aw3[d][r];
    }
  }
  if (w == 0) {
    if (n == 15) slab[OFF_A_B3 + g] = db3;
    if (lane == 0) {
      slab[OFF_C_B2] = dbc2;
      slab[NPARAM] = diagC;
      slab[NPARAM + 1] = diagA;
      slab[NPARAM + 2] = skipped;
    }
    if (lane < SLAB - (NPARAM + 3)) slab[NPARAM + 3 + lane] = 0.0f;  // (the pads)
  }
  __syncthreads();
  {
    const SlabOut out(ga.partial + (size_t)blockIdx.x * SLAB);
    constexpr int NV = SLAB / 4, PER = (NV + 256 * TEAMS - 1) / (256 * TEAMS);
    f4 sv[PER][TEAMS];
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int i = tid + k * 256 * TEAMS;
#pragma unroll
      for (int t = 0; t < TEAMS; t++) sv[k][t] = i < NV ? ((const f4*)(lds + t * SLAB))[i] : z4;
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int i = tid + k * 256 * TEAMS;
      f4 acc = sv[k][0];
      if (TEAMS == 2) acc = acc + sv[k][TEAMS - 1];
      if (i < NV) out.put(i, acc);
    }
  }
}

// the weight image from the flat parameters (initialisation, wk_set_weights)
__global__ void k_swizzle(const float* __restrict__ W, float* __restrict__ Wz) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < NPARAM) mf_scatter_param(Wz, p, W[p]);
}

int mfma_image_floats() { return mf::WEND; }
hipError_t launch_swizzle(const float* W, float* Wz, hipStream_t s) {
  hipLaunchKernelGGL(k_swizzle, dim3((NPARAM + 255) / 256), dim3(256), 0, s, W, Wz);
  return hipGetLastError();
}

// Which matrix-core gradient kernel (WK_GRAD_IMPL = ws / tp / tp1 / mf, read per context at
// wk_create; default: by minibatch size).  The tile-parallel kernel has the shorter chain per
// chunk, the producer / consumer kernel the higher throughput once every SIMD pair has several
// chunks (measured, scripts/grad_impls.py: tp faster up to 24,576 samples, ws from 32,768).
int grad_impl_env() {
  if (const char* e = getenv("WK_GRAD_IMPL")) {
    if (!strcmp(e, "ws")) return GI_WS;
    if (!strcmp(e, "tp")) return GI_TP2;
    if (!strcmp(e, "tp1")) return GI_TP1;
    if (!strcmp(e, "mf")) return GI_MF;
  }
  return GI_AUTO;
}
int grad_impl_for(int impl, int samples) {
  if (impl != GI_AUTO) return impl;
  // one team per block up to 256 chunks (one chunk per block on every CU: 7.6 vs 9.5 us at
  // 4,096 samples), two from there (8,192: 10.5 vs 11.3 us), the producer / consumer kernel
  // from 32,768
  return samples <= 4096 ? GI_TP1 : samples < 32768 ? GI_TP2 : GI_WS;
}
hipError_t configure_mfma_kernels() {
  hipError_t e = hipFuncSetAttribute((const void*)k_ppo_grad_mfma, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(float) * mf::LDS_FLOATS));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_ppo_grad_ws, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(sizeof(float) * ws::LDS_FLOATS));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_ppo_grad_tp<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(sizeof(float) * tp::L<2>::FLOATS));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_ppo_grad_tp<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(sizeof(float) * tp::L<1>::FLOATS));
  return e;
}

// blocks of the kernel `impl` (resolved) for a minibatch; at most 256 (one per CU; the ordered
// reduction's one-launch form and the IPC exchange take up to 256 slabs)
int ppo_grad_mfma_blocks(int samples, int impl) {
  const int chunks = (samples + 15) / 16;
  const int per = impl == GI_TP2 ? 2 : impl == GI_TP1 ? 1 : mf::WAVES;
  const int blocks = (chunks + per - 1) / per;
  return blocks < 256 ? (blocks > 0 ? blocks : 1) : 256;
}

hipError_t launch_ppo_grad_mfma(const GradArgs& g, int nblocks, int impl, hipStream_t s) {
  switch (impl) {
    case GI_WS:
      hipLaunchKernelGGL(k_ppo_grad_ws, dim3(nblocks), dim3(64 * 2 * ws::PAIRS), sizeof(float) * ws::LDS_FLOATS, s, g);
      break;
    case GI_TP1:
      hipLaunchKernelGGL(k_ppo_grad_tp<1>, dim3(nblocks), dim3(256), sizeof(float) * tp::L<1>::FLOATS, s, g);
      break;
    case GI_MF:
      hipLaunchKernelGGL(k_ppo_grad_mfma, dim3(nblocks), dim3(64 * mf::WAVES), sizeof(float) * mf::LDS_FLOATS, s, g);
      break;
    default:
      hipLaunchKernelGGL(k_ppo_grad_tp<2>, dim3(nblocks), dim3(512), sizeof(float) * tp::L<2>::FLOATS, s, g);
  }
  return hipGetLastError();
}

}  // namespace wk
