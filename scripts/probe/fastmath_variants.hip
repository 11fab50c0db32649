// Probe: which shortened sqrt / reciprocal sequences still equal the correctly rounded
// results bit for bit over every float of the fast-path domain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ float r_full(float d) {
  float r = __builtin_amdgcn_rcpf(d);
  float e = __builtin_fmaf(-d, r, 1.0f); r = __builtin_fmaf(e, r, r);
  float q = r; float rem = __builtin_fmaf(-d, q, 1.0f); q = __builtin_fmaf(rem, r, q);
  rem = __builtin_fmaf(-d, q, 1.0f); return __builtin_fmaf(rem, r, q);
}
__device__ float r_v1(float d) {
  float r = __builtin_amdgcn_rcpf(d);
  float e = __builtin_fmaf(-d, r, 1.0f); return __builtin_fmaf(e, r, r);
}
__device__ float r_v2(float d) {
  float r = __builtin_amdgcn_rcpf(d);
  float e = __builtin_fmaf(-d, r, 1.0f); r = __builtin_fmaf(e, r, r);
  e = __builtin_fmaf(-d, r, 1.0f); return __builtin_fmaf(e, r, r);
}
__device__ float s_full(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
  float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
  s = (rd <= 0.0f) ? sd : s; s = (ru > 0.0f) ? su : s; return s;
}
__device__ float s_down(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  float sd = __uint_as_float(__float_as_uint(s) - 1u);
  float rd = __builtin_fmaf(-sd, s, x);
  return (rd <= 0.0f) ? sd : s;
}
__device__ float s_up(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  float su = __uint_as_float(__float_as_uint(s) + 1u);
  float ru = __builtin_fmaf(-su, s, x);
  return (ru > 0.0f) ? su : s;
}
__device__ float s_raw(float x) { return __builtin_amdgcn_sqrtf(x); }
__global__ void k(uint32_t lo, uint32_t hi, unsigned long long* bad) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= hi; b += stride) {
    const float x = __uint_as_float((uint32_t)b);
    const uint32_t q = __float_as_uint(1.0f / x), s = __float_as_uint(sqrtf(x));
    if (__float_as_uint(r_full(x)) != q) atomicAdd(bad + 0, 1ull);
    if (__float_as_uint(r_v1(x)) != q) atomicAdd(bad + 1, 1ull);
    if (__float_as_uint(r_v2(x)) != q) atomicAdd(bad + 2, 1ull);
    if (__float_as_uint(s_full(x)) != s) atomicAdd(bad + 3, 1ull);
    if (__float_as_uint(s_down(x)) != s) atomicAdd(bad + 4, 1ull);
    if (__float_as_uint(s_up(x)) != s) atomicAdd(bad + 5, 1ull);
    if (__float_as_uint(s_raw(x)) != s) atomicAdd(bad + 6, 1ull);
  }
}
int main() {
  unsigned long long* d; (void)hipMalloc(&d, 64); (void)hipMemset(d, 0, 64);
  // [2^-48, 2^63]: every value a reciprocal of a sqrt in the fast domain can take, and
  // the sqrt inputs [2^-96, 2^126] for the sqrt variants (superset range run below)
  hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, 0x0F800000u /*2^-96*/, 0x7E800000u /*2^126*/, d);
  unsigned long long h[8];
  (void)hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
  const char* names[] = {"rcp full", "rcp 1 NR", "rcp 2 NR", "sqrt full", "sqrt down-only", "sqrt up-only", "sqrt raw"};
  for (int i = 0; i < 7; i++) printf("%-16s mismatches over [2^-96, 2^126]: %llu\n", names[i], h[i]);
  return 0;
}
