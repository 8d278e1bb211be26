// Operand-layout probe of v_mfma_i32_16x16x64_i8 on gfx950 (tool, not product): every lane passes 16
// distinct int8 of A and of B; the host tries candidate lane->element maps and reports which one
// reproduces the device's D exactly (C/D map assumed: col = lane & 15, row = 4 * (lane >> 4) + reg).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_probe(const int8_t* fa, const int8_t* fb, int* d) {
  const int l = threadIdx.x;
  v4i a, b;
  __builtin_memcpy(&a, fa + 16 * l, 16);
  __builtin_memcpy(&b, fb + 16 * l, 16);
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[4 * l + r] = c[r];
}

int main() {
  int8_t fa[64 * 16], fb[64 * 16];
  srand(3);
  for (int i = 0; i < 64 * 16; ++i) {
    fa[i] = (int8_t)(rand() % 255 - 127);
    fb[i] = (int8_t)(rand() % 255 - 127);
  }
  int8_t *dfa, *dfb;
  int* dd;
  hipMalloc(&dfa, sizeof(fa));
  hipMalloc(&dfb, sizeof(fb));
  hipMalloc(&dd, 64 * 4 * 4);
  hipMemcpy(dfa, fa, sizeof(fa), hipMemcpyHostToDevice);
  hipMemcpy(dfb, fb, sizeof(fb), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dfa, dfb, dd);
  int d[256];
  hipMemcpy(d, dd, sizeof(d), hipMemcpyDeviceToHost);
  // candidate k maps for element j of lane l (h = l >> 4):
  //   0: k = 16h + j            1: k = 8h + j (j < 8), 32 + 8h + (j - 8) (j >= 8)
  //   2: k = 4h + j%4 + 16*(j/4)   3: k = j*4 + h
  const char* names[] = {"k=16h+j", "k=8h+j | 32+8h+(j-8)", "k=4h+(j%4)+16(j/4)", "k=4j+h"};
  for (int cand = 0; cand < 4; ++cand) {
    int A[16][64], B[64][16];
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 16; ++j) {
        const int h = l >> 4;
        int k = 0;
        switch (cand) {
          case 0: k = 16 * h + j; break;
          case 1: k = j < 8 ? 8 * h + j : 32 + 8 * h + (j - 8); break;
          case 2: k = 4 * h + (j % 4) + 16 * (j / 4); break;
          case 3: k = 4 * j + h; break;
        }
        A[l & 15][k] = fa[16 * l + j];
        B[k][l & 15] = fb[16 * l + j];
      }
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * (l >> 4) + r, col = l & 15;
        int s = 0;
        for (int k = 0; k < 64; ++k) s += A[row][k] * B[k][col];
        bad += s != d[4 * l + r];
      }
    printf("candidate %d (%s): %d of 256 outputs differ\n", cand, names[cand], bad);
  }
  return 0;
}
