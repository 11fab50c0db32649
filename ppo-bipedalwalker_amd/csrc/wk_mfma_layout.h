// wk_mfma_layout.h -- the matrix-core gradient kernel's weight image (wk_ppo_mfma.hip).
//
// The policy parameters (wk_common.h OFF_*) are kept a second time in HBM in the exact
// order the v_mfma_f32_16x16x4_f32 A operands read them (lane l = 16 g + n holds A[n][g]),
// so each gradient block stages them into LDS with a straight 16-byte copy.  The image is
// rewritten by every Adam step (k_adam scatters each updated parameter) and by the
// initialisation / set-weights paths (k_swizzle).
#pragma once
#include "wk_common.h"

namespace wk {
namespace mf {
enum : int {
  AW1F = 0,              // [Mt 4][t 3][lane 64]        W1[16Mt + n][4t + g]
  CW1F = AW1F + 768,     // critic W1, same order
  W2F = CW1F + 768,      // [Mt 4][Mp 4][lane 64][r 4]  W2[16Mt + n][16Mp + 4g + r]
  W2B = W2F + 4096,      // [Mk 4][Mj 4][lane 64][r 4]  W2[16Mj + 4g + r][16Mk + n]
  W3 = W2B + 4096,       // [4][64]
  WC2 = W3 + 256,        // [64]
  BA1 = WC2 + 64, BA2 = BA1 + 64, BC1 = BA2 + 64, BA3 = BC1 + 64, BC2 = BA3 + 4,
  WEND = BC2 + 4         // 10,248 floats
};
static_assert(WEND % 4 == 0, "16-byte copies");
}  // namespace mf

// a float store; WT: written through (relaxed agent-scope atomic store = global_store sc1: the
// line leaves the L2 clean, MI355X_MICROARCH.md), so a later release has nothing of it to write back
template <bool WT>
__device__ __forceinline__ void st_f(float* p, float v) {
  if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// Exchanges between the four 16-lane rows of a wave (lane l = 16 g + n: row g, the MFMA
// operands' lane group) on gfx950's permlane swaps -- two VALU instructions, no LDS round trip
// and no lane-index arithmetic as __shfl / __shfl_xor (ds_bpermute_b32) need.  Called with the
// whole wave active.
//   v_permlane16_swap(v, v): odd rows of the first copy <-> even rows of the second, so
//     a = rows [r0 r0 r2 r2], b = rows [r1 r1 r3 r3]
//   v_permlane32_swap(v, v): upper half of the first <-> lower half of the second, so
//     lo = halves [lo lo], hi = halves [hi hi]
__device__ __forceinline__ void rows_pair_swap(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void halves_swap(float v, float& lo, float& hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  lo = __uint_as_float(r[0]);
  hi = __uint_as_float(r[1]);
}
// (v + __shfl_xor(v, 16)) then + __shfl_xor(., 32), in every lane: the rows whose own value is
// the second operand here get the same sum, fp32 addition being commutative
__device__ __forceinline__ float rows_sum4(float v) {
  float a, b, lo, hi;
  rows_pair_swap(v, a, b);
  halves_swap(a + b, lo, hi);
  return lo + hi;
}
__device__ __forceinline__ float rows_max4(float v) {  // the same with fmaxf
  float a, b, lo, hi;
  rows_pair_swap(v, a, b);
  halves_swap(__builtin_fmaxf(a, b), lo, hi);
  return __builtin_fmaxf(lo, hi);
}
// rows_sum4(p[g]) in lane (n, g) -- the four sums with each lane keeping its own row's, as a
// reduce-scatter in three swaps: permlane16_swap(p0, p1) gives rows [p0.r0 p1.r0 p0.r2 p1.r2]
// and [p0.r1 p1.r1 p0.r3 p1.r3] (summed: row g holds p_{g&1} over rows {g&2, (g&2)+1}), the same
// for p2 / p3, then the halves' swap adds rows {0,1} + {2,3}: the association of rows_sum4
__device__ __forceinline__ float rows_rsum4(const float p[4]) {
  const auto u = __builtin_amdgcn_permlane16_swap(__float_as_uint(p[0]), __float_as_uint(p[1]), false, false);
  const auto w = __builtin_amdgcn_permlane16_swap(__float_as_uint(p[2]), __float_as_uint(p[3]), false, false);
  const float s01 = __uint_as_float(u[0]) + __uint_as_float(u[1]);
  const float s23 = __uint_as_float(w[0]) + __uint_as_float(w[1]);
  const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(s01), __float_as_uint(s23), false, false);
  return __uint_as_float(h[0]) + __uint_as_float(h[1]);
}
// o[d] = v of lane (n, d) in every lane (n, g): __shfl(v, n + 16 d)
__device__ __forceinline__ void rows_bcast4(float v, float o[4]) {
  float a, b;
  rows_pair_swap(v, a, b);
  halves_swap(a, o[0], o[2]);
  halves_swap(b, o[1], o[3]);
}

// the sum over the 16 lanes of a DPP row, in lane 0 of the row, as ((v0 + v4) + (v8 + v12)) +
// ((v1 + v5) + (v9 + v13)) + ... grouped ((t0 + t1) + (t2 + t3)): row_ror 12, 8, 15, 14 bring
// lanes j + 4, j + 8, j + 1, j + 2 to lane j
template <int CTRL>
__device__ __forceinline__ float dpp_row(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_tree16(float v) {
  v = v + dpp_row<0x12C>(v);
  v = v + dpp_row<0x128>(v);
  v = v + dpp_row<0x12F>(v);
  v = v + dpp_row<0x12E>(v);
  return v;
}

// write parameter p (value v) to its image position(s)
template <bool WT = false>
__device__ inline void mf_scatter_param(float* __restrict__ Wz, int p, float v) {
  using namespace mf;
  if (p < OFF_C_B1 || (p >= OFF_A_W1 && p < OFF_A_B1)) {  // W1 (critic / actor) [64][12]
    const bool critic = p < OFF_C_B1;
    const int q = p - (critic ? OFF_C_W1 : OFF_A_W1);
    const int j = q / 12, k = q % 12;
    st_f<WT>(&Wz[(critic ? CW1F : AW1F) + ((j >> 4) * 3 + (k >> 2)) * 64 + 16 * (k & 3) + (j & 15)], v);
  } else if (p < OFF_C_W2) {
    st_f<WT>(&Wz[BC1 + p - OFF_C_B1], v);
  } else if (p < OFF_C_B2) {
    st_f<WT>(&Wz[WC2 + p - OFF_C_W2], v);
  } else if (p < OFF_A_W1) {
    st_f<WT>(&Wz[BC2], v);
  } else if (p < OFF_A_W2) {
    st_f<WT>(&Wz[BA1 + p - OFF_A_B1], v);
  } else if (p < OFF_A_B2) {  // W2 [64 j][64 k], both operand orders
    const int q = p - OFF_A_W2;
    const int j = q >> 6, k = q & 63;
    st_f<WT>(&Wz[W2F + (((j >> 4) * 4 + (k >> 4)) * 64 + 16 * ((k & 15) >> 2) + (j & 15)) * 4 + (k & 3)], v);
    st_f<WT>(&Wz[W2B + (((k >> 4) * 4 + (j >> 4)) * 64 + 16 * ((j & 15) >> 2) + (k & 15)) * 4 + (j & 3)], v);
  } else if (p < OFF_A_W3) {
    st_f<WT>(&Wz[BA2 + p - OFF_A_B2], v);
  } else if (p < OFF_A_B3) {
    st_f<WT>(&Wz[W3 + p - OFF_A_W3], v);
  } else {
    st_f<WT>(&Wz[BA3 + p - OFF_A_B3], v);
  }
}

}  // namespace wk
