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
//   k_str_any: four 16-byte fingerprint loads per thread (block-interleaved quads); a verified
//              hit finds its row by binary search in row_off (hits are rare) and ORs the needle bit
//              into the row's flag byte;
//   SearchEq: the position index below (k_str_posfp) read by k_str_eq_count (ddshe_kernels.hip),
//              which writes the compaction masks directly;
// then k_byte_count (SearchEntry) / k_ope_scatter compact the flagged rows into ascending row ids.
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

// one thread per kStrQuads element quads, block-interleaved (quad b*256*kStrQuads + k*256 + tid: each
// 16-byte load instruction of a wave covers 1 KiB contiguous; all kStrQuads loads in flight together);
// a verified hit ORs the needle bit into its row's flag byte (a 32-bit atomic on the byte's word:
// hits are rare)
constexpr int kStrQuads = 4;
__global__ void __launch_bounds__(256) k_str_any(const uint32_t* __restrict__ fp, uint64_t e_first, size_t nelems,
                                                 const uint64_t* __restrict__ row_off, size_t nrows,
                                                 const uint64_t* __restrict__ elem_off, const uint8_t* __restrict__ chars,
                                                 const uint8_t* __restrict__ nchars, StrNeedles nd,
                                                 uint8_t* __restrict__ flags) {
  const size_t qb = (size_t)blockIdx.x * 256 * kStrQuads + threadIdx.x;  // quad of k = 0
  uint32_t f[4 * kStrQuads];
#pragma unroll
  for (int k = 0; k < kStrQuads; ++k) {
    const size_t q = qb + (size_t)k * 256;
    const uint64_t e0 = e_first + 4 * q;
    if (e_first % 4 == 0 && 4 * q + 3 < nelems) {
      const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(fp + e0));
      f[4 * k] = x.x;
      f[4 * k + 1] = x.y;
      f[4 * k + 2] = x.z;
      f[4 * k + 3] = x.w;
    } else {
      for (int i = 0; i < 4; ++i) f[4 * k + i] = 4 * q + i < nelems ? fp[e0 + i] : 0u;
    }
  }
  const uint32_t h0 = (uint32_t)(nd.h[0] >> 32), h1 = (uint32_t)(nd.h[1] >> 32), h2 = (uint32_t)(nd.h[2] >> 32);
#pragma unroll
  for (int k = 0; k < kStrQuads; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t ei = 4 * (qb + (size_t)k * 256) + i;  // element index relative to e_first
      if (ei >= nelems) continue;
      const uint32_t v = f[4 * k + i];
      const bool c0 = v == h0, c1 = nd.n > 1 && v == h1, c2 = nd.n > 2 && v == h2;
      if (!(c0 | c1 | c2)) continue;  // the common case: no fingerprint hit
      const uint64_t e = e_first + ei;
      uint32_t bits = 0;
      if (c0 && str_hit(e, 0, elem_off, chars, nchars, nd)) bits |= 1u;
      if (c1 && str_hit(e, 1, elem_off, chars, nchars, nd)) bits |= 2u;
      if (c2 && str_hit(e, 2, elem_off, chars, nchars, nd)) bits |= 4u;
      if (bits) {
        const size_t r = row_of(row_off, nrows, e);
        atomicOr(reinterpret_cast<uint32_t*>(flags + (r & ~(size_t)3)), bits << (8 * (r & 3)));
      }
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
                          uint8_t* flags, hipStream_t st) {
  if (nrows == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(flags, 0, (nrows + 3) & ~(size_t)3, st);  // whole words (the atomics' unit)
  if (e != hipSuccess || nelems == 0) return e;
  const size_t quads = (nelems + 3) / 4, per_block = (size_t)256 * kStrQuads;
  hipLaunchKernelGGL(k_str_any, dim3((unsigned)((quads + per_block - 1) / per_block)), dim3(256), 0, st, fp, e_first, nelems, row_off,
                     nrows, elem_off, chars, nchars, nd, flags);
  return hipGetLastError();
}

}  // namespace ddshe
