// Probe: cheaper sequences for the correctly rounded sqrt s = RN(sqrt(x)) and for the
// normalisation factor v = RN(1 / RN(sqrt(x))) (Vector2.Normalize), checked bit for bit
// against sqrt_core / rcp_core(sqrt_core) over every float of [2^-96, 2^126].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "wk_device.h"
using namespace wk;
__device__ float s1(float x) {  // rsq-based: s0 = x y, one FMA correction with h = y / 2
  const float y = __builtin_amdgcn_rsqf(x);
  const float s0 = x * y;
  const float e = __builtin_fmaf(-s0, s0, x);
  return __builtin_fmaf(e, 0.5f * y, s0);
}
__device__ float s3(float x) {  // hardware sqrt + one FMA correction with h = rcp(s0) / 2
  const float s0 = __builtin_amdgcn_sqrtf(x);
  const float e = __builtin_fmaf(-s0, s0, x);
  return __builtin_fmaf(e, 0.5f * __builtin_amdgcn_rcpf(s0), s0);
}
__device__ float s4(float x) {  // hardware sqrt + one FMA correction with h = rsq(x) / 2
  const float s0 = __builtin_amdgcn_sqrtf(x);
  const float e = __builtin_fmaf(-s0, s0, x);
  return __builtin_fmaf(e, 0.5f * __builtin_amdgcn_rsqf(x), s0);
}
__device__ float v3(float x) {  // rsqrt with one Newton-Raphson step (single rounding)
  const float y = __builtin_amdgcn_rsqf(x);
  const float h = 0.5f * y;
  const float r = __builtin_fmaf(-(x * y), h, 0.5f);
  return __builtin_fmaf(y, r, y);
}
__device__ float n1(float x) {  // Normalize factor: the reciprocal's NR step seeded with rsq
  const float y = __builtin_amdgcn_rsqf(x);
  const float s0 = x * y;
  const float e = __builtin_fmaf(-s0, s0, x);
  const float s = __builtin_fmaf(e, 0.5f * y, s0);
  const float r = __builtin_fmaf(-s, y, 1.0f);
  return __builtin_fmaf(r, y, y);
}
__global__ void k(uint32_t lo, uint32_t hi, unsigned long long* bad) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= hi; b += stride) {
    const float x = __uint_as_float((uint32_t)b);
    const float s = sqrt_core(x);
    const uint32_t su = __float_as_uint(s), vu = __float_as_uint(rcp_core(s));
    if (__float_as_uint(s1(x)) != su) atomicAdd(bad + 0, 1ull);
    if (__float_as_uint(s3(x)) != su) atomicAdd(bad + 1, 1ull);
    if (__float_as_uint(s4(x)) != su) atomicAdd(bad + 2, 1ull);
    if (__float_as_uint(rcp_core(s1(x))) != vu) atomicAdd(bad + 3, 1ull);
    if (__float_as_uint(v3(x)) != vu) atomicAdd(bad + 4, 1ull);
    if (__float_as_uint(sqrtf(x)) != su) atomicAdd(bad + 5, 1ull);  // sanity: sqrt_core == sqrtf
    if (__float_as_uint(n1(x)) != vu) atomicAdd(bad + 6, 1ull);
  }
}
int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 64);
  (void)hipMemset(d, 0, 64);
  hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, 0x0F800000u /*2^-96*/, 0x7E800000u /*2^126*/, d);
  unsigned long long h[8];
  (void)hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
  const char* names[] = {"s1 rsq+fma", "s3 sqrt+rcp fma", "s4 sqrt+rsq fma", "v(s1)", "v3 rsq NR", "sqrtf sanity", "n1 rsq-seeded rcp"};
  for (int i = 0; i < 7; i++) printf("%-18s mismatches over [2^-96, 2^126]: %llu\n", names[i], h[i]);
  return 0;
}
