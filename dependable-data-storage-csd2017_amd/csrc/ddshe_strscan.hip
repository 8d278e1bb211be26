// Deterministic-equality scans over a device-resident string table:
//   SearchEq / SearchNEq   DDSRestServer.scala:607-681  (contents(position) vs item)
//   SearchEntry/OR/AND     DDSRestServer.scala:831-938  (any element vs 1 or 3 items)
//   IsElement              DDSRestServer.scala:322-353  (one row)
// HomoDet.compare (hlib, absent) is taken as equality of the ciphertext strings.
//
// Layout in HBM (dds_strtab, ddshe_strtab.cpp): an element heap -- chars (element strings back to back),
// elem_off[nheap+1] (u64 byte offsets), a resident 16-bit fingerprint per element (k_str_digest: top
// 16 bits of str_digest) and the row owning each element (elem_row; kStrDead for a superseded version) --
// and per row its current version: row_beg (first heap element), row_len (element count) and a live
// byte (0: the set was removed, RemoveSet writes None). A row write appends a new version to the heap
// and kills the old one; the heap is compacted (k_str_compact) when it runs out of room. A scan
// streams 2 B of fingerprint per element it must look at; bytes are compared only on a fingerprint hit
// (about nelems * needles / 2^16 false hits per scan: ~3,700 for SearchEntryOR's 3 needles over 80M
// elements, each a row lookup and a 32-byte compare), so results stay exact.
//   k_str_any: four 16-byte loads of 8 fingerprints per thread (block-interleaved octets); a verified
//              hit of a live row's current version ORs the needle bit into the row's flag byte;
//   SearchEq: the position index below (k_str_posfp) read by k_str_eq_count (ddshe_kernels.hip),
//              which writes the compaction masks directly; writes patch it (k_str_posfp_ids);
// then k_byte_count (SearchEntry) / k_ope_scatter compact the flagged rows into ascending row ids.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ddshe_launch.hpp"

namespace ddshe {

__global__ void k_str_digest(const uint8_t* __restrict__ chars, const uint64_t* __restrict__ elem_off, size_t nelems,
                             StrFp* __restrict__ fp) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nelems) return;
  const uint64_t a = elem_off[e], b = elem_off[e + 1];
  fp[e] = str_fp(str_digest(chars + a, b - a));
}

// SearchEq's position-major index (built on the first query at a position, kept with the table and
// patched by every write): posfp[r] = fingerprint of row r's element `position`, present bit r = the
// row is live and passes the route's strict guard (length - 1 > position, DDSRestServer.scala:615). A
// query (k_str_eq_count) reads 2 B per row, coalesced, instead of gathering one fingerprint per
// 32-byte sector; only fingerprint hits touch the row descriptors and the bytes.
__device__ __forceinline__ bool str_present(const uint64_t* __restrict__ row_beg, const uint32_t* __restrict__ row_len,
                                            const uint8_t* __restrict__ live, const StrFp* __restrict__ fp,
                                            size_t r, uint64_t position, StrFp* f) {
  const bool pres = live[r] != 0 && (uint64_t)row_len[r] > position + 1;
  *f = pres ? fp[row_beg[r] + position] : (StrFp)0;
  return pres;
}
// rows [r_first, r_first + count), r_first a multiple of 64: whole present words
__global__ void k_str_posfp(const uint64_t* __restrict__ row_beg, const uint32_t* __restrict__ row_len,
                            const uint8_t* __restrict__ live, size_t r_first, size_t count,
                            const StrFp* __restrict__ fp, uint64_t position, StrFp* __restrict__ posfp,
                            uint64_t* __restrict__ present) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x, r = r_first + i;
  bool pres = false;
  if (i < count) {
    StrFp f;
    pres = str_present(row_beg, row_len, live, fp, r, position, &f);
    posfp[r] = f;
  }
  const uint64_t m = __ballot(pres);
  if ((threadIdx.x & 63) == 0 && i < count) present[r >> 6] = m;  // r: the wave's first row, a multiple of 64
}
// distinct rows ids[0..n) (after a write / live change): their entries and present bits
__global__ void k_str_posfp_ids(const uint32_t* __restrict__ ids, size_t n, const uint64_t* __restrict__ row_beg,
                                const uint32_t* __restrict__ row_len, const uint8_t* __restrict__ live,
                                const StrFp* __restrict__ fp, uint64_t position, StrFp* __restrict__ posfp,
                                uint64_t* __restrict__ present) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t r = ids[i];
  StrFp f;
  const bool pres = str_present(row_beg, row_len, live, fp, r, position, &f);
  posfp[r] = f;
  const unsigned long long bit = 1ull << (r & 63);
  auto* w = reinterpret_cast<unsigned long long*>(present + (r >> 6));
  if (pres) atomicOr(w, bit);
  else atomicAnd(w, ~bit);
}

// row descriptors of rows ids[0..n) <- (beg[i], len[i]), live (a written set is present again)
__global__ void k_str_rows_set(const uint32_t* __restrict__ ids, const uint64_t* __restrict__ beg,
                               const uint32_t* __restrict__ len, size_t n, uint64_t* __restrict__ row_beg,
                               uint32_t* __restrict__ row_len, uint8_t* __restrict__ live) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = ids[i];
  row_beg[r] = beg[i];
  row_len[r] = len[i];
  live[r] = 1;
}

// superseded versions: heap elements [beg[i], beg[i] + len[i]) belong to no row any more
__global__ void k_str_kill(const uint64_t* __restrict__ beg, const uint32_t* __restrict__ len, size_t n,
                           uint32_t* __restrict__ elem_row) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = beg[i];
  for (uint32_t k = 0; k < len[i]; ++k) elem_row[b + k] = kStrDead;
}

// Heap compaction into fresh buffers: one wave per row copies its current version's element
// descriptors (fingerprint, owner, rebased byte offset) and bytes to new_beg[r] / new_cbeg[r] (host
// prefix sums over the rows' versions); superseded versions are left behind.
__global__ void __launch_bounds__(256) k_str_compact(size_t nrows, const uint64_t* __restrict__ old_beg,
                                                     const uint32_t* __restrict__ len,
                                                     const uint64_t* __restrict__ new_beg,
                                                     const uint64_t* __restrict__ new_cbeg,
                                                     const uint64_t* __restrict__ elem_off,
                                                     const StrFp* __restrict__ fp, const uint8_t* __restrict__ chars,
                                                     uint64_t* __restrict__ nelem_off, StrFp* __restrict__ nfp,
                                                     uint32_t* __restrict__ nelem_row, uint8_t* __restrict__ nchars) {
  const size_t r = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (r >= nrows) return;
  const uint64_t ob = old_beg[r], nb = new_beg[r], cb = new_cbeg[r];
  const uint32_t L = len[r];
  if (L == 0) return;
  const uint64_t c0 = elem_off[ob], c1 = elem_off[ob + L];
  for (uint32_t k = lane; k < L; k += 64) {
    nfp[nb + k] = fp[ob + k];
    nelem_row[nb + k] = (uint32_t)r;
    nelem_off[nb + k] = cb + (elem_off[ob + k] - c0);
  }
  for (uint64_t b = lane; b < c1 - c0; b += 64) nchars[cb + b] = chars[c0 + b];
}

// one thread per kStrOcts element octets, block-interleaved (octet b*256*kStrOcts + k*256 + tid: each
// 16-byte load instruction of a wave covers 1 KiB contiguous; all kStrOcts loads in flight together);
// a verified hit of a live row r in [row0, row0 + nrows) ORs the needle bit into flag byte r - row0 (a
// 32-bit atomic on the byte's word: hits are rare)
constexpr int kStrOcts = 4;
__global__ void __launch_bounds__(256) k_str_any(const StrFp* __restrict__ fp, uint64_t e_first, size_t nelems,
                                                 const uint32_t* __restrict__ elem_row,
                                                 const uint8_t* __restrict__ live, size_t row0, size_t nrows,
                                                 const uint64_t* __restrict__ elem_off, const uint8_t* __restrict__ chars,
                                                 const uint8_t* __restrict__ nchars, StrNeedles nd,
                                                 uint8_t* __restrict__ flags) {
  const size_t ob = (size_t)blockIdx.x * 256 * kStrOcts + threadIdx.x;  // octet of k = 0
  uint32_t f[4 * kStrOcts];  // two fingerprints per word
#pragma unroll
  for (int k = 0; k < kStrOcts; ++k) {
    const size_t o = ob + (size_t)k * 256;
    const uint64_t e0 = e_first + 8 * o;
    if (e_first % 8 == 0 && 8 * o + 7 < nelems) {
      const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(fp + e0));
      f[4 * k] = x.x;
      f[4 * k + 1] = x.y;
      f[4 * k + 2] = x.z;
      f[4 * k + 3] = x.w;
    } else {
      for (int i = 0; i < 4; ++i) {
        const uint32_t lo = 8 * o + 2 * i < nelems ? fp[e0 + 2 * i] : 0u;
        const uint32_t hi = 8 * o + 2 * i + 1 < nelems ? fp[e0 + 2 * i + 1] : 0u;
        f[4 * k + i] = lo | (hi << 16);
      }
    }
  }
  const uint32_t h0 = str_fp(nd.h[0]), h1 = str_fp(nd.h[1]), h2 = str_fp(nd.h[2]);
  // the common case without per-element work: a zero-halfword test of (word ^ needle pair) per needle
  // ((t - 0x00010001) & ~t & 0x80008000 is non-zero iff a half of t is zero), no bounds checks (padding
  // reads as fingerprint 0; a hit on it drops to the exact loop below, which checks bounds)
  {
    uint32_t any = 0;
    const uint32_t p0 = h0 | (h0 << 16), p1 = h1 | (h1 << 16), p2 = h2 | (h2 << 16);
#pragma unroll
    for (int w = 0; w < 4 * kStrOcts; ++w) {
      uint32_t t = f[w] ^ p0;
      any |= (t - 0x00010001u) & ~t;
      if (nd.n > 1) {
        t = f[w] ^ p1;
        any |= (t - 0x00010001u) & ~t;
      }
      if (nd.n > 2) {
        t = f[w] ^ p2;
        any |= (t - 0x00010001u) & ~t;
      }
    }
    if ((any & 0x80008000u) == 0) return;
  }
#pragma unroll
  for (int k = 0; k < kStrOcts; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const size_t ei = 8 * (ob + (size_t)k * 256) + i;  // element index relative to e_first
      if (ei >= nelems) continue;
      const uint32_t v = (f[4 * k + i / 2] >> (16 * (i & 1))) & 0xFFFFu;
      const bool c0 = v == h0, c1 = nd.n > 1 && v == h1, c2 = nd.n > 2 && v == h2;
      if (!(c0 | c1 | c2)) continue;  // the common case: no fingerprint hit
      const uint64_t e = e_first + ei;
      const uint32_t row = elem_row[e];
      if (row == kStrDead || (size_t)row - row0 >= nrows || !live[row]) continue;
      uint32_t bits = 0;
      if (c0 && str_hit(e, 0, elem_off, chars, nchars, nd)) bits |= 1u;
      if (c1 && str_hit(e, 1, elem_off, chars, nchars, nd)) bits |= 2u;
      if (c2 && str_hit(e, 2, elem_off, chars, nchars, nd)) bits |= 4u;
      if (bits) {
        const size_t r = (size_t)row - row0;
        atomicOr(reinterpret_cast<uint32_t*>(flags + (r & ~(size_t)3)), bits << (8 * (r & 3)));
      }
    }
}

hipError_t launch_str_digest(const uint8_t* chars, const uint64_t* elem_off, size_t nelems, StrFp* fp,
                             hipStream_t st) {
  if (nelems == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_digest, dim3((unsigned)((nelems + 255) / 256)), dim3(256), 0, st, chars, elem_off, nelems,
                     fp);
  return hipGetLastError();
}

hipError_t launch_str_posfp(const uint64_t* row_beg, const uint32_t* row_len, const uint8_t* live, size_t r_first,
                            size_t count, const StrFp* fp, uint64_t position, StrFp* posfp, uint64_t* present,
                            hipStream_t st) {
  if (count == 0) return hipSuccess;
  if (r_first % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_str_posfp, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, row_beg, row_len, live,
                     r_first, count, fp, position, posfp, present);
  return hipGetLastError();
}

hipError_t launch_str_posfp_ids(const uint32_t* ids, size_t n, const uint64_t* row_beg, const uint32_t* row_len,
                                const uint8_t* live, const StrFp* fp, uint64_t position, StrFp* posfp,
                                uint64_t* present, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_posfp_ids, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids, n, row_beg, row_len,
                     live, fp, position, posfp, present);
  return hipGetLastError();
}

hipError_t launch_str_rows_set(const uint32_t* ids, const uint64_t* beg, const uint32_t* len, size_t n,
                               uint64_t* row_beg, uint32_t* row_len, uint8_t* live, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_rows_set, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids, beg, len, n, row_beg,
                     row_len, live);
  return hipGetLastError();
}

hipError_t launch_str_kill(const uint64_t* beg, const uint32_t* len, size_t n, uint32_t* elem_row, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_kill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, beg, len, n, elem_row);
  return hipGetLastError();
}

hipError_t launch_str_compact(size_t nrows, const uint64_t* old_beg, const uint32_t* len, const uint64_t* new_beg,
                              const uint64_t* new_cbeg, const uint64_t* elem_off, const StrFp* fp,
                              const uint8_t* chars, uint64_t* nelem_off, StrFp* nfp, uint32_t* nelem_row,
                              uint8_t* nchars, hipStream_t st) {
  if (nrows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_str_compact, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, st, nrows, old_beg, len, new_beg,
                     new_cbeg, elem_off, fp, chars, nelem_off, nfp, nelem_row, nchars);
  return hipGetLastError();
}

hipError_t launch_str_any(const StrFp* fp, uint64_t e_first, size_t nelems, const uint32_t* elem_row,
                          const uint8_t* live, size_t row0, size_t nrows, const uint64_t* elem_off, const uint8_t* chars,
                          const uint8_t* nchars, const StrNeedles& nd, uint8_t* flags, hipStream_t st,
                          bool flags_zeroed) {
  if (nrows == 0) return hipSuccess;
  hipError_t e = flags_zeroed ? hipSuccess : hipMemsetAsync(flags, 0, (nrows + 3) & ~(size_t)3, st);  // whole words
  if (e != hipSuccess || nelems == 0) return e;
  const size_t octs = (nelems + 7) / 8, per_block = (size_t)256 * kStrOcts;
  hipLaunchKernelGGL(k_str_any, dim3((unsigned)((octs + per_block - 1) / per_block)), dim3(256), 0, st, fp, e_first,
                     nelems, elem_row, live, row0, nrows, elem_off, chars, nchars, nd, flags);
  return hipGetLastError();
}

}  // namespace ddshe
