// One build of the production fold kernel k_fold<148, 4, 28, QP> per translation unit (A/B tool, not
// product). -I picks whose ddshe_fold.hpp / ddshe_device.hpp (HEAD's csrc or an older commit's copy
// extracted by tools/abtest/ab_fold.sh), -DKNAME names the build so several share one process.
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
  hipLaunchKernelGGL((KNAME::ddshe::k_fold<148, 4, 28, true>), dim3((unsigned)((ngroups * 4 + 255) / 256)), dim3(256),
                     0, 0, X, xstride, count, C, n0, P, pstride, ngroups);
  return hipGetLastError();
}
