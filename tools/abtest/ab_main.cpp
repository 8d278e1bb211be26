// Interleaved A/B timing of fold-kernel variants in one process (rule: compare in one process).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
typedef hipError_t (*launch_t)(const uint32_t*, size_t, size_t, const uint32_t*, uint32_t, uint32_t*, size_t, size_t);
#define DECL(n) extern "C" hipError_t k_ab##n##_launch(const uint32_t*, size_t, size_t, const uint32_t*, uint32_t, uint32_t*, size_t, size_t);
DECL(0) DECL(1) DECL(2) DECL(3)
int main(int argc, char** argv) {
  const int S = 148, W = 28;
  size_t count = argc > 1 ? atoll(argv[1]) : 4000000;
  int rounds = argc > 2 ? atoi(argv[2]) : 5;
  int nvar = argc > 3 ? atoi(argv[3]) : 4;
  launch_t fns[4] = {k_ab0_launch, k_ab1_launch, k_ab2_launch, k_ab3_launch};
  size_t stride = (count + 63) / 64 * 64;
  std::vector<uint32_t> h((size_t)S * stride), hn((size_t)S * 5, 0);  // constant block (kConstCount*S)
  srand(1);
  for (int l = 0; l < S; ++l) hn[l] = (uint32_t)rand() & ((1u << W) - 1);  // kConstN
  hn[0] |= 1; hn[S - 1] = (1u << 10) | 5;   // ~4095-bit odd modulus (top limb small)
  for (int l = 0; l < S; ++l) for (size_t i = 0; i < count; ++i) h[(size_t)l * stride + i] = (uint32_t)rand() & ((1u << W) - 1);
  for (size_t i = 0; i < count; ++i) h[(size_t)(S - 1) * stride + i] = 3;  // value < N
  uint32_t inv = hn[0]; for (int i = 0; i < 5; ++i) inv *= 2u - hn[0] * inv;
  uint32_t n0 = (0u - inv) & ((1u << W) - 1);
  uint32_t *dX, *dN, *dP;
  hipMalloc(&dX, h.size() * 4); hipMalloc(&dN, hn.size() * 4);
  size_t G = 32768, ps = G;
  hipMalloc(&dP, (size_t)160 * ps * 4);  // production kernel zero-fills to s_out=160
  hipMemcpy(dX, h.data(), h.size() * 4, hipMemcpyHostToDevice); hipMemcpy(dN, hn.data(), hn.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  std::vector<std::vector<float>> t(nvar);
  for (int v = 0; v < nvar; ++v) fns[v](dX, stride, count, dN, n0, dP, ps, G);  // warm
  hipDeviceSynchronize();
  std::vector<uint32_t> ref((size_t)S * 4), got((size_t)S * 4);
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < nvar; ++v) {
      hipEventRecord(e0); fns[v](dX, stride, count, dN, n0, dP, ps, G); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); t[v].push_back(ms);
      hipMemcpy(got.data(), dP, got.size() * 4, hipMemcpyDeviceToHost);
      if (v == 0 && r == 0) ref = got; else if (got != ref) printf("variant %d output differs!\n", v);
    }
  for (int v = 0; v < nvar; ++v) {
    std::sort(t[v].begin(), t[v].end());
    double mm = (double)(count - G);
    printf("variant %d: median %.3f ms min %.3f ms  -> %.3e MonPro/s\n", v, t[v][t[v].size() / 2], t[v][0], mm / (t[v][t[v].size() / 2] * 1e-3));
  }
  return 0;
}
