// Deterministic-equality scans over a device-resident string table:
//   SearchEq / SearchNEq   DDSRestServer.scala:607-681  (contents(position) vs item)
//   SearchEntry/OR/AND     DDSRestServer.scala:831-938  (any element vs 1 or 3 items)
//   IsElement              DDSRestServer.scala:322-353  (one row)
// HomoDet.compare (hlib, absent) is taken as equality of the ciphertext strings.
//
// Layout in HBM (built once per table by dds_strtab_create): chars (all element strings back to
// back), elem_off[nelems+1] (u64 byte offsets), row_off[nrows+1] (u64 element offsets) and a
// resident 64-bit digest per element (k_str_digest). A scan then streams 8 B of digest per
// element it must look at (plus the row offsets); bytes are compared only on a digest hit, so
// the result stays exact. k_str_scan writes one int64 flag per row; the OPE compaction
// (k_ope_count / k_ope_scatter) turns the flags into ascending row ids.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ddshe_launch.hpp"

namespace ddshe {

__global__ void k_str_digest(const uint8_t* __restrict__ chars, const uint64_t* __restrict__ elem_off, size_t nelems,
                             uint64_t* __restrict__ digest) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nelems) return;
  const uint64_t a = elem_off[e], b = elem_off[e + 1];
  digest[e] = str_digest(chars + a, b - a);
}

__device__ __forceinline__ bool str_equal(const uint8_t* __restrict__ x, const uint8_t* __restrict__ y, uint64_t len) {
  for (uint64_t i = 0; i < len; ++i)
    if (x[i] != y[i]) return false;
  return true;
}

// mode 0: contents(position) == needle 0 (negate: !=), rows with length-1 > position only;
// mode 1: some element equals some needle; mode 2: every needle equals some element.
__global__ void k_str_scan(const uint64_t* __restrict__ row_off, size_t nrows, const uint64_t* __restrict__ elem_off,
                           const uint8_t* __restrict__ chars, const uint64_t* __restrict__ digest,
                           const uint8_t* __restrict__ nchars, StrNeedles nd, int mode, uint64_t position,
                           int negate, int64_t* __restrict__ flags) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  const uint64_t e0 = row_off[r], e1 = row_off[r + 1];
  auto hit = [&](uint64_t e, int j) {
    if (digest[e] != nd.h[j]) return false;
    const uint64_t a = elem_off[e], b = elem_off[e + 1];
    return b - a == nd.len[j] && str_equal(chars + a, nchars + nd.off[j], nd.len[j]);
  };
  int64_t f = 0;
  if (mode == 0) {
    if (e1 - e0 > position + 1) f = hit(e0 + position, 0) != (negate != 0);
  } else {
    uint32_t found = 0;
    for (uint64_t e = e0; e < e1; ++e)
      for (int j = 0; j < nd.n; ++j)
        if (!((found >> j) & 1u) && hit(e, j)) found |= 1u << j;
    f = mode == 1 ? found != 0 : found == (1u << nd.n) - 1u;
  }
  flags[r] = f;
}

hipError_t launch_str_digest(const uint8_t* chars, const uint64_t* elem_off, size_t nelems, uint64_t* digest,
                             hipStream_t st) {
  if (nelems == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_digest, dim3((unsigned)((nelems + 255) / 256)), dim3(256), 0, st, chars, elem_off, nelems,
                     digest);
  return hipGetLastError();
}

hipError_t launch_str_scan(const uint64_t* row_off, size_t nrows, const uint64_t* elem_off, const uint8_t* chars,
                           const uint64_t* digest, const uint8_t* nchars, const StrNeedles& nd, int mode,
                           uint64_t position, int negate, int64_t* flags, hipStream_t st) {
  if (nrows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_scan, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, st, row_off, nrows, elem_off,
                     chars, digest, nchars, nd, mode, position, negate, flags);
  return hipGetLastError();
}

}  // namespace ddshe
