// Interleaved A/B timing of builds of the production fold kernel k_fold<148, 4, 28, QP> in one process
// (tool, not product). The modulus is a QP modulus N~ = N·n0 (N~ = -1 mod 2^28) of an odd ~4095-bit N,
// as the engine uses at the committed key's shape, so every build computes the same residues: outputs
// must agree bit for bit. Usage: ab_fold [rows=10000000] [rounds=7] [groups=0: 256 CUs x 2 x 64]
// Built with -DAB_FOLD1: the k_fold1<74, 28, false> builds instead (a ~2048-bit odd N, plain CIOS quotient,
// one bignum per lane: groups default 256 CUs x 2 x 256).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>
typedef hipError_t (*launch_t)(const uint32_t*, size_t, size_t, const uint32_t*, uint32_t, uint32_t*, size_t, size_t);
#define DECL(n) \
  extern "C" hipError_t k_ab##n##_launch(const uint32_t*, size_t, size_t, const uint32_t*, uint32_t, uint32_t*, size_t, size_t);
DECL(0) DECL(1) DECL(2) DECL(3)
#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
#ifdef AB_FOLD1
  const int S = 74, W = 28;
  const bool qp = false;
#else
  const int S = 148, W = 28;
  const bool qp = true;
#endif
  const uint32_t mask = (1u << W) - 1;
  const size_t count = argc > 1 ? atoll(argv[1]) : 10000000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 7;
  size_t G = argc > 3 ? atoll(argv[3]) : 0;
  const char* names[4] = {getenv("AB_NAME0"), getenv("AB_NAME1"), getenv("AB_NAME2"), getenv("AB_NAME3")};
  launch_t fns[4] = {k_ab0_launch, k_ab1_launch, k_ab2_launch, k_ab3_launch};
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  if (!G) G = (size_t)prop.multiProcessorCount * 2 * (qp ? 64 : 256);  // 2 blocks of 256 threads per CU
  if (G > count) G = count;
  const size_t stride = (count + 63) / 64 * 64;
  // N: odd, ~4095 bits (top limb 2^10 | 5); N~ = N * n0 with n0 = -N^-1 mod 2^W (N~ = -1 mod 2^W, < 2^4123)
  std::vector<uint32_t> N(S, 0), C((size_t)S * 5, 0);
  srand(1);
  for (int l = 0; l < S; ++l) N[l] = (uint32_t)rand() & mask;
  N[0] |= 1;
  N[S - 1] = 0;
  N[S - 2] = (1u << 10) | 5;
  uint32_t inv = N[0];
  for (int i = 0; i < 5; ++i) inv *= 2u - N[0] * inv;
  const uint32_t n0 = (0u - inv) & mask;
  uint64_t carry = 0;
  for (int l = 0; l < S; ++l) {
    const uint64_t v = qp ? (uint64_t)N[l] * n0 + carry : N[l];
    C[l] = (uint32_t)v & mask;  // kConstN block = N~ (QP) or N
    carry = qp ? v >> W : 0;
  }
  if (carry || (qp && C[0] != mask)) {
    fprintf(stderr, "bad QP modulus\n");
    return 1;
  }
  // rows: random values < N (top limbs 0 / small)
  std::vector<uint32_t> h((size_t)S * stride, 0);
  for (int l = 0; l < S - 2; ++l)
    for (size_t i = 0; i < count; ++i) h[(size_t)l * stride + i] = (uint32_t)rand() & mask;
  for (size_t i = 0; i < count; ++i) h[(size_t)(S - 2) * stride + i] = (uint32_t)rand() & 0x3ff;
  uint32_t *dX, *dC, *dP;
  CK(hipMalloc(&dX, h.size() * 4));
  CK(hipMalloc(&dC, C.size() * 4));
  const size_t ps = (G + 63) / 64 * 64;
  CK(hipMalloc(&dP, (size_t)S * ps * 4));
  CK(hipMemcpy(dX, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int nvar = 0;
  while (nvar < 4 && names[nvar]) ++nvar;
  if (!nvar) nvar = 2;
  std::vector<std::vector<float>> t(nvar);
  std::vector<uint32_t> ref((size_t)S * ps), got((size_t)S * ps);
  for (int v = 0; v < nvar; ++v) CK(fns[v](dX, stride, count, dC, n0, dP, ps, G));  // warm
  CK(hipDeviceSynchronize());
  int bad = 0;
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < nvar; ++v) {
      CK(hipMemset(dP, 0, (size_t)S * ps * 4));
      CK(hipEventRecord(e0));
      CK(fns[v](dX, stride, count, dC, n0, dP, ps, G));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms);
      if (r == 0) {
        CK(hipMemcpy(got.data(), dP, got.size() * 4, hipMemcpyDeviceToHost));
        if (v == 0)
          ref = got;
        else if (got != ref) {
          printf("variant %d output differs!\n", v);
          bad = 1;
        }
      }
    }
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("rows %zu groups %zu rounds %d (device max clock %d MHz)\n", count, G, rounds, clk / 1000);
  for (int v = 0; v < nvar; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const double mm = (double)(count - G);
    printf("variant %d (%s): median %.3f ms min %.3f ms max %.3f ms -> %.4e MonPro/s\n", v, names[v] ? names[v] : "?",
           t[v][t[v].size() / 2], t[v][0], t[v].back(), mm / (t[v][t[v].size() / 2] * 1e-3));
  }
  return bad;
}
