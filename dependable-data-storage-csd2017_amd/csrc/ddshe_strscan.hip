// Deterministic-equality scans over a device-resident string table:
//   SearchEq / SearchNEq   DDSRestServer.scala:607-681  (contents(position) vs item)
//   SearchEntry/OR/AND     DDSRestServer.scala:831-938  (any element vs 1 or 3 items)
//   IsElement              DDSRestServer.scala:322-353  (one row)
// HomoDet.compare (hlib, absent) is taken as equality of the ciphertext strings.
//
// Layout in HBM (built once per table by dds_strtab_create): chars (all element strings back to
// back), elem_off[nelems+1] (u64 byte offsets), row_off[nrows+1] (u64 element offsets) and a
// resident 32-bit fingerprint per element (k_str_digest: top half of str_digest). A scan streams
// 4 B of fingerprint per element it must look at; bytes are compared only on a fingerprint hit
// (about nelems * needles / 2^32 false hits per scan), so results stay exact.
//   k_str_any: one thread per 4 consecutive elements (one 16-byte fingerprint load); a verified hit
//              finds its row by binary search in row_off (hits are rare) and ORs the needle bit
//              into the row's u32 flag;
//   SearchEq: the position index below (k_str_posfp) read by k_str_eq_count (ddshe_kernels.hip),
//              which writes the compaction masks directly;
// then k_flag_count (SearchEntry) / k_ope_scatter compact the flagged rows into ascending row ids.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ddshe_launch.hpp"

namespace ddshe {

__global__ void k_str_digest(const uint8_t* __restrict__ chars, const uint64_t* __restrict__ elem_off, size_t nelems,
                             uint32_t* __restrict__ fp) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nelems) return;
  const uint64_t a = elem_off[e], b = elem_off[e + 1];
  fp[e] = (uint32_t)(str_digest(chars + a, b - a) >> 32);
}

// SearchEq's position-major index (built on the first query at a position, kept with the table):
// posfp[r] = fingerprint of row r's element `position`, present bit r = the row passes the route's
// strict guard (length - 1 > position, DDSRestServer.scala:615). A query (k_str_eq_count) reads 4 B per
// row, coalesced, instead of gathering one 4-byte fingerprint per 32-byte sector (plus 8 B of row
// offsets); only fingerprint hits touch the row offsets and the bytes.
__global__ void k_str_posfp(const uint64_t* __restrict__ row_off, size_t nrows, const uint32_t* __restrict__ fp,
                            uint64_t position, uint32_t* __restrict__ posfp, uint64_t* __restrict__ present) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool pres = false;
  if (r < nrows) {
    const uint64_t e0 = row_off[r], e1 = row_off[r + 1];
    pres = e1 - e0 > position + 1;
    posfp[r] = pres ? fp[e0 + position] : 0u;
  }
  const uint64_t m = __ballot(pres);
  if ((threadIdx.x & 63) == 0 && r < nrows) present[r >> 6] = m;  // r: the wave's first row, a multiple of 64
}

// row holding element e: last r with row_off[r] <= e (row_off ascending, rows may be empty)
__device__ __forceinline__ size_t row_of(const uint64_t* __restrict__ row_off, size_t nrows, uint64_t e) {
  size_t lo = 0, hi = nrows;  // invariant: row_off[lo] <= e < row_off[hi]
  while (hi - lo > 1) {
    const size_t mid = (lo + hi) / 2;
    if (row_off[mid] <= e) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ void k_str_any(const uint32_t* __restrict__ fp, uint64_t e_first, size_t nelems,
                          const uint64_t* __restrict__ row_off, size_t nrows, const uint64_t* __restrict__ elem_off,
                          const uint8_t* __restrict__ chars, const uint8_t* __restrict__ nchars, StrNeedles nd,
                          uint32_t* __restrict__ flags) {
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // element quad
  const uint64_t e0 = e_first + 4 * q;
  if (4 * q >= nelems) return;
  uint32_t f[4];
  if (4 * q + 3 < nelems && e0 % 4 == 0) {
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(fp + e0));
    f[0] = x.x;
    f[1] = x.y;
    f[2] = x.z;
    f[3] = x.w;
  } else {
    for (int i = 0; i < 4; ++i) f[i] = 4 * q + i < nelems ? fp[e0 + i] : 0u;
  }
  const uint32_t h0 = (uint32_t)(nd.h[0] >> 32), h1 = (uint32_t)(nd.h[1] >> 32), h2 = (uint32_t)(nd.h[2] >> 32);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (4 * q + i >= nelems) break;
    const bool c0 = f[i] == h0, c1 = nd.n > 1 && f[i] == h1, c2 = nd.n > 2 && f[i] == h2;
    if (!(c0 | c1 | c2)) continue;  // the common case: no fingerprint hit
    const uint64_t e = e0 + i;
    uint32_t bits = 0;
    if (c0 && str_hit(e, 0, elem_off, chars, nchars, nd)) bits |= 1u;
    if (c1 && str_hit(e, 1, elem_off, chars, nchars, nd)) bits |= 2u;
    if (c2 && str_hit(e, 2, elem_off, chars, nchars, nd)) bits |= 4u;
    if (bits) atomicOr(&flags[row_of(row_off, nrows, e)], bits);
  }
}

hipError_t launch_str_digest(const uint8_t* chars, const uint64_t* elem_off, size_t nelems, uint32_t* fp,
                             hipStream_t st) {
  if (nelems == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_digest, dim3((unsigned)((nelems + 255) / 256)), dim3(256), 0, st, chars, elem_off, nelems,
                     fp);
  return hipGetLastError();
}

hipError_t launch_str_posfp(const uint64_t* row_off, size_t nrows, const uint32_t* fp, uint64_t position,
                            uint32_t* posfp, uint64_t* present, hipStream_t st) {
  if (nrows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_posfp, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, st, row_off, nrows, fp, position,
                     posfp, present);
  return hipGetLastError();
}

hipError_t launch_str_any(const uint32_t* fp, uint64_t e_first, size_t nelems, const uint64_t* row_off, size_t nrows,
                          const uint64_t* elem_off, const uint8_t* chars, const uint8_t* nchars, const StrNeedles& nd,
                          uint32_t* flags, hipStream_t st) {
  if (nrows == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(flags, 0, nrows * 4, st);
  if (e != hipSuccess || nelems == 0) return e;
  const size_t quads = (nelems + 3) / 4;
  hipLaunchKernelGGL(k_str_any, dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, st, fp, e_first, nelems, row_off,
                     nrows, elem_off, chars, nchars, nd, flags);
  return hipGetLastError();
}

}  // namespace ddshe
