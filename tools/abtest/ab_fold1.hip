// One build of the production one-bignum-per-lane fold k_fold1<74, 28, false> per translation unit (A/B
// tool, not product); -I picks whose headers, -DKNAME names the build (see ab_fold.hip).
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
namespace KNAME {
#include "ddshe_fold.hpp"
}
extern "C" hipError_t CAT(KNAME, _launch)(const uint32_t* X, size_t xstride, size_t count, const uint32_t* C, uint32_t n0,
                                          uint32_t* P, size_t pstride, size_t ngroups) {
  hipLaunchKernelGGL((KNAME::ddshe::k_fold1<74, 28, false>), dim3((unsigned)((ngroups + 255) / 256)), dim3(256), 0, 0, X,
                     xstride, count, C, n0, P, pstride, ngroups);
  return hipGetLastError();
}
