// Probe: operand / result layout of v_mfma_f32_16x16x4_f32 on gfx950.
// A[i][k] = i + 100 k (i<16, k<4), B[k][j] = (k == j % 4) ? 1 : 0 ... use exact small ints.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out, int mode) {
  int l = threadIdx.x;
  // hypothesis: A[i = l%16][k = l/16], B[k = l/16][j = l%16]
  int i = l % 16, kk = l / 16, j = l % 16;
  float a = (mode == 0) ? (float)(i + 16 * kk) : 0.0f;   // A[i][k] distinct
  float b = (mode == 0) ? ((kk == 0 && j == 0) ? 1.0f : 0.0f) : 0.0f;  // B = e_{k=0, j=0}
  if (mode == 1) { a = (kk == 0 && i == 0) ? 1.0f : 0.0f; b = (float)(kk + 4 * j); }
  f4 c = {0, 0, 0, 0};
  f4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; r++) out[l * 4 + r] = d[r];
}
int main() {
  float* d; hipMalloc(&d, 256 * 4);
  float h[256];
  for (int mode = 0; mode < 2; mode++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    // mode 0: D[i][j] = sum_k A[i][k] B[k][j] = A[i][0] if j == 0 -> expect D[i][0] = i
    // mode 1: D[i][j] = A[0][k=0] * B[0][j] = 4j for i == 0
    int bad = 0;
    for (int l = 0; l < 64; l++)
      for (int r = 0; r < 4; r++) {
        int row = 4 * (l / 16) + r, col = l % 16;
        float expect = mode == 0 ? (col == 0 ? (float)row : 0.0f) : (row == 0 ? (float)(4 * col) : 0.0f);
        if (h[l * 4 + r] != expect) bad++;
      }
    printf("mode %d mismatches %d (hypothesis D[4*(l/16)+r][l%%16])\n", mode, bad);
    if (bad) for (int l = 0; l < 64; l++) printf("l%d: %g %g %g %g\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
  }
  return 0;
}
