// floor_face_check.hip -- bit-equality of the flat floor's closed-form contact face
// (floor_face_ax, csrc/wk_device.h) against the generic significant_face_ax over the floor
// polygon and its normalised axes (the path it replaces in contact_points_floor), for
// 2^26 hashed normals in [-2, 2]^2 and every pair of 24 special components (signed zeros,
// units, diagonals, tiny and huge values: the projection ties between corners).
// Built by ppo-bipedalwalker_amd/Makefile (target `check`), run by tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "wk_device.h"

using namespace wk;

__constant__ float kSpecial[24] = {0.0f, -0.0f, 1.0f, -1.0f, 0.70710677f, -0.70710677f,
                                   0.5f, -0.5f, 1e-30f, -1e-30f, 1e-45f, -1e-45f,
                                   0.13636364f, -0.13636364f, 7.3333335f, -7.3333335f,
                                   0.99999994f, -0.99999994f, 1e30f, -1e30f, 2.0f, -2.0f,
                                   0.1f, -0.1f};

__device__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__device__ bool same(V2 a, V2 b) {
  return __float_as_uint(a.x) == __float_as_uint(b.x) && __float_as_uint(a.y) == __float_as_uint(b.y);
}

// out[t]: the number of mismatching normals seen by thread t (vector stores only)
__global__ void k_check(uint32_t n_random, uint32_t* out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  Poly<4> F;
  floor_poly(F);
  const EdgeAxes<4> AX = floor_axes();
  uint32_t bad = 0;
  for (uint32_t i = t; i < n_random + 24u * 24u; i += stride) {
    V2 n;
    if (i < n_random) {
      n.x = ((float)(mix(2u * i) >> 8) * 0x1p-24f) * 4.0f - 2.0f;
      n.y = ((float)(mix(2u * i + 1u) >> 8) * 0x1p-24f) * 4.0f - 2.0f;
    } else {
      const uint32_t k = i - n_random;
      n = mk(kSpecial[k % 24u], kSpecial[k / 24u]);
    }
    V2 a0, b0, m0, d0, a1, b1, m1, d1;
    significant_face_ax(F, AX, n, a0, b0, m0, d0);
    floor_face_ax(n, a1, b1, m1, d1);
    bad += !(same(a0, a1) && same(b0, b1) && same(m0, m1) && same(d0, d1));
  }
  out[t] = bad;
}

int main() {
  const int blocks = 2048, threads = 256, total = blocks * threads;
  const uint32_t n_random = 1u << 26;
  uint32_t* d_out;
  if (hipMalloc(&d_out, total * sizeof(uint32_t)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k_check, dim3(blocks), dim3(threads), 0, 0, n_random, d_out);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  std::vector<uint32_t> h(total);
  if (hipMemcpy(h.data(), d_out, total * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  unsigned long long bad = 0;
  for (uint32_t v : h) bad += v;
  printf("floor face, %u hashed + %u special normals: %llu mismatches\n", n_random, 24u * 24u, bad);
  printf(bad ? "FAIL\n" : "OK\n");
  return bad ? 1 : 0;
}
