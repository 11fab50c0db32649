// rows_check.hip -- bit-equality of the cross-row exchange helpers of wk_mfma_layout.h (the
// gradient kernels' and the rollout policy's lane-group sums and broadcasts on the gfx950
// permlane swaps, and the DPP row tree of the gradient epilogue) against the ds_bpermute /
// LDS formulations they replaced, on hashed floats of every magnitude, signed zeros and
// infinities (an all-NaN result on both sides counts as equal: fp32 addition of an infinity
// pair gives the default NaN either way).  Built by ppo-bipedalwalker_amd/Makefile (target
// `check`), run by tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#include "wk_mfma_layout.h"

using namespace wk;

__device__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// a float from hash h: mostly finite of any exponent, some signed zeros and infinities
__device__ float sample(uint32_t h) {
  const uint32_t k = h & 63u;
  if (k == 0) return 0.0f;
  if (k == 1) return -0.0f;
  if (k == 2) return __uint_as_float(0x7f800000u);
  if (k == 3) return __uint_as_float(0xff800000u);
  uint32_t b = mix(h);
  if (((b >> 23) & 0xffu) == 0xffu) b &= ~0x00800000u;  // no NaN inputs
  return __uint_as_float(b);
}
__device__ bool same(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}
__device__ float ref_sum4(float v) {
  v = v + __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}
__device__ float ref_max4(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}
// the former LDS pass of k_ppo_grad_ws: lane 0 of each row, f4 groups q[i] = lanes 4i..4i+3
__device__ float ref_tree16(float v, float* lds) {
  const int lane = threadIdx.x & 63, row = lane >> 4;
  float* r = lds + (threadIdx.x >> 6) * 64;
  r[lane] = v;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const float* q = r + 16 * row;
  float t[4];
  for (int j = 0; j < 4; j++) t[j] = (q[j] + q[4 + j]) + (q[8 + j] + q[12 + j]);
  const float s = (t[0] + t[1]) + (t[2] + t[3]);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  return s;
}

// out[t]: mismatches seen by thread t (vector stores only)
__global__ __launch_bounds__(256) void k_check(uint32_t rounds, uint32_t* out) {
  __shared__ float lds[4 * 64];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, n = lane & 15, g = lane >> 4;
  uint32_t bad = 0;
  for (uint32_t it = 0; it < rounds; it++) {
    const uint32_t h = mix(t * 0x9e3779b9u + it * 0x85ebca6bu);
    const float v = sample(h);
    float p[4];
    for (int d = 0; d < 4; d++) p[d] = sample(mix(h + 0x1000193u * (d + 1)));
    bad += !same(rows_sum4(v), ref_sum4(v));
    bad += !same(rows_max4(v), ref_max4(v));
    float o[4];
    rows_bcast4(v, o);
    for (int d = 0; d < 4; d++) bad += !same(o[d], __shfl(v, n + 16 * d));
    float s[4];
    for (int d = 0; d < 4; d++) s[d] = ref_sum4(p[d]);
    bad += !same(rows_rsum4(p), g == 0 ? s[0] : g == 1 ? s[1] : g == 2 ? s[2] : s[3]);
    const float tr = row_tree16(v), rt = ref_tree16(v, lds);
    if (n == 0) bad += !same(tr, rt);
  }
  out[t] = bad;
}

int main() {
  const int blocks = 1024, threads = 256, total = blocks * threads;
  const uint32_t rounds = 256;
  uint32_t* d_out;
  if (hipMalloc(&d_out, total * sizeof(uint32_t)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k_check, dim3(blocks), dim3(threads), 0, 0, rounds, d_out);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  std::vector<uint32_t> h(total);
  if (hipMemcpy(h.data(), d_out, total * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  unsigned long long bad = 0;
  for (uint32_t x : h) bad += x;
  printf("row exchanges, %d lanes x %u rounds: %llu mismatches\n", total, rounds, bad);
  printf(bad ? "FAIL\n" : "OK\n");
  return bad ? 1 : 0;
}
