// Resident-row mutations (include/ddshe.h dds_col_write_rows / dds_col_set_live / dds_opecol_write_rows /
// dds_opecol_set_live): the write routes of the reference change stored sets in place —
// WriteElement overwrites contents(position) (DDSRestServer.scala:281-321), AddElement appends an
// element (:220-255), RemoveSet writes None (:207-218) — and the resident columns follow them with
// these scatters instead of a re-upload. All are HBM-trivial next to a fold: n rows x S limbs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ddshe_launch.hpp"

namespace ddshe {

namespace {
inline unsigned blocks_for(size_t threads) { return (unsigned)((threads + 255) / 256); }
}  // namespace

// thread t = (limb l, row i) with i fastest: src reads coalesce, dst writes land in row ids[i] of each limb
__global__ void __launch_bounds__(256) k_scatter_rows(const uint32_t* __restrict__ src, size_t sstride,
                                                      const uint32_t* __restrict__ ids, size_t n, int S,
                                                      uint32_t* __restrict__ dst, size_t dstride) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * (size_t)S) return;
  const size_t i = t % n, l = t / n;
  dst[l * dstride + ids[i]] = src[l * sstride + i];
}

__global__ void __launch_bounds__(256) k_scatter_bytes(const uint32_t* __restrict__ ids,
                                                       const uint8_t* __restrict__ vals, size_t n,
                                                       uint8_t* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[ids[i]] = vals[i];
}

__global__ void __launch_bounds__(256) k_scatter_u64(const uint32_t* __restrict__ ids,
                                                     const uint64_t* __restrict__ vals, size_t n,
                                                     uint64_t* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[ids[i]] = vals[i];
}

// Order over a column with removed sets: keep[p] = 1 unless the row at sorted position p is dead
__global__ void __launch_bounds__(256) k_perm_keep(const uint32_t* __restrict__ perm, const uint8_t* __restrict__ dead,
                                                   size_t n, uint8_t* __restrict__ keep) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) keep[p] = dead[perm[p]] ? 0 : 1;
}

__global__ void __launch_bounds__(256) k_gather_u32(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                    size_t n, uint32_t* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

hipError_t launch_scatter_rows(const uint32_t* src, size_t sstride, const uint32_t* ids, size_t n, int S, uint32_t* dst,
                               size_t dstride, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_rows, dim3(blocks_for(n * (size_t)S)), dim3(256), 0, st, src, sstride, ids, n, S, dst,
                     dstride);
  return hipGetLastError();
}

hipError_t launch_scatter_bytes(const uint32_t* ids, const uint8_t* vals, size_t n, uint8_t* dst, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_bytes, dim3(blocks_for(n)), dim3(256), 0, st, ids, vals, n, dst);
  return hipGetLastError();
}

hipError_t launch_scatter_u64(const uint32_t* ids, const uint64_t* vals, size_t n, uint64_t* dst, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_u64, dim3(blocks_for(n)), dim3(256), 0, st, ids, vals, n, dst);
  return hipGetLastError();
}

hipError_t launch_perm_keep(const uint32_t* perm, const uint8_t* dead, size_t n, uint8_t* keep, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_perm_keep, dim3(blocks_for(n)), dim3(256), 0, st, perm, dead, n, keep);
  return hipGetLastError();
}

hipError_t launch_gather_u32(const uint32_t* src, const uint32_t* idx, size_t n, uint32_t* dst, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_u32, dim3(blocks_for(n)), dim3(256), 0, st, src, idx, n, dst);
  return hipGetLastError();
}

}  // namespace ddshe
