// One fold-kernel variant per translation unit (A/B timing tool, not product).
// -DKNAME=<name> names the variant; switches live in ddshe_device.hpp behind DDSHE_AB_* macros.
// -DPROD times the production kernel (ddshe_fold.hpp's k_fold) compiled inside namespace KNAME,
// so several builds of it (different macros) can share one process.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#ifdef PROD
namespace KNAME {
#include "ddshe_fold.hpp"
}
extern "C" hipError_t CAT(KNAME, _launch)(const uint32_t* X, size_t xstride, size_t count, const uint32_t* C, uint32_t n0,
                                          uint32_t* P, size_t pstride, size_t ngroups) {
  // C: kConstCount*S constant block (only kConstN / kConstRmod are read by k_fold)
  hipLaunchKernelGGL((KNAME::ddshe::k_fold<148, 4, 28>), dim3((unsigned)((ngroups * 4 + 255) / 256)), dim3(256), 0, 0,
                     X, xstride, count, C, n0, P, pstride, ngroups);
  return hipGetLastError();
}
#else
#include "ddshe_device.hpp"
using namespace ddshe;
template <int S, int TPI, int W>
__global__ void __launch_bounds__(256, 2) KNAME(const uint32_t* __restrict__ X, size_t xstride, size_t count,
                                                 const uint32_t* __restrict__ N, uint32_t n0, uint32_t* __restrict__ P,
                                                 size_t pstride, size_t ngroups) {
  using M = Mont<S, TPI, W>;
  constexpr int L = M::L;
  const int r = threadIdx.x % TPI;
  const bool top = r == TPI - 1, bottom = r == 0;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= ngroups) return;
  uint32_t n[L], a[L];
  for (int l = 0; l < L; ++l) n[l] = N[r * L + l];
  size_t row = grp;
  for (int l = 0; l < L; ++l) a[l] = X[(size_t)(r * L + l) * xstride + row];
  row += ngroups;
  for (; row < count; row += ngroups) M::mul_col(a, n, X, xstride, (uint32_t)row, n0, top, bottom);
  M::normalize(a, bottom);
  for (int l = 0; l < L; ++l) P[(size_t)(r * L + l) * pstride + grp] = a[l];
}
extern "C" hipError_t CAT(KNAME, _launch)(const uint32_t* X, size_t xstride, size_t count, const uint32_t* N, uint32_t n0,
                                          uint32_t* P, size_t pstride, size_t ngroups) {
  hipLaunchKernelGGL((KNAME<148, 4, 28>), dim3((unsigned)((ngroups * 4 + 255) / 256)), dim3(256), 0, 0, X, xstride,
                     count, N, n0, P, pstride, ngroups);
  return hipGetLastError();
}
#endif
