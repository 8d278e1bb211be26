// Fold / finalize kernels and the lane-group helpers they share (gfx950).
// Kept in a header so tools/abtest can time the production kernel against variants in one process.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ddshe_device.hpp"
#include "ddshe_launch.hpp"  // kConst* block layout

namespace ddshe {

// ------------------------------------------------------------------------------
// group helpers
// ------------------------------------------------------------------------------
template <int S, int TPI, int W>
struct Grp {
  using M = Mont<S, TPI, W>;
  static constexpr uint32_t kMask = M::kMask;
  static constexpr int L = M::L;
  int r;        // lane index in group
  bool top;     // r == TPI-1
  bool bottom;  // r == 0
  __device__ __forceinline__ Grp() {
    r = (int)(threadIdx.x % TPI);
    top = r == TPI - 1;
    bottom = r == 0;
  }
  __device__ __forceinline__ void load_col(uint32_t (&a)[L], const uint32_t* __restrict__ col, size_t stride,
                                           size_t row) const {
#pragma unroll
    for (int l = 0; l < L; ++l) a[l] = col[(size_t)(r * L + l) * stride + row];
  }
  __device__ __forceinline__ void store_col(const uint32_t (&a)[L], uint32_t* __restrict__ col, size_t stride,
                                            size_t row) const {
#pragma unroll
    for (int l = 0; l < L; ++l) col[(size_t)(r * L + l) * stride + row] = a[l];
  }
  __device__ __forceinline__ void load_vec(uint32_t (&a)[L], const uint32_t* __restrict__ v) const {
#pragma unroll
    for (int l = 0; l < L; ++l) a[l] = v[r * L + l];
  }
  // sign(a - n) for fully normalised a (group-wide result)
  __device__ __forceinline__ int cmp(const uint32_t (&a)[L], const uint32_t (&n)[L]) const {
    int c = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) c = a[l] > n[l] ? 1 : (a[l] < n[l] ? -1 : c);
    int res = 0;
    for (int s = TPI - 1; s >= 0; --s) {
      int v = (int)M::group_read((uint32_t)c, s, r);
      res = res != 0 ? res : v;
    }
    return res;
  }
  // a -= n (a >= n, both fully normalised)
  __device__ __forceinline__ void sub(uint32_t (&a)[L], const uint32_t (&n)[L]) const {
    uint32_t br = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const uint32_t d = a[l] - n[l] - br;
      br = d >> 31;  // borrow iff wrapped (operands < 2^W)
      a[l] = d & kMask;
    }
    for (int round = 1; round < TPI; ++round) {
      uint32_t bin = grp_from_prev<TPI>(br);
      if (bottom) bin = 0;
#pragma unroll
      for (int l = 0; l < L; ++l) {
        const uint32_t d = a[l] - bin;
        bin = d >> 31;
        a[l] = d & kMask;
      }
      br = bin;
    }
  }
  // value < 2N, almost normalised -> canonical [0, N), fully normalised
  __device__ __forceinline__ void canon(uint32_t (&a)[L], const uint32_t (&n)[L]) const {
    M::normalize(a, bottom);
    if (cmp(a, n) >= 0) sub(a, n);
  }
};

// ------------------------------------------------------------------------------
// fold: each group folds rows g, g+G, g+2G, ... with Montgomery products.
// A group that folded c rows holds prod * R^(1-c). Requires 1 <= ngroups <= count (no empty
// group: the launcher checks), which keeps the kernel body to load, MonPro loop, store.
// ------------------------------------------------------------------------------
// Idx: the fold runs over the rows ids[0..count) of X instead of rows [0, count) (row-subset folds:
// the rows that pass a route's guard / dedup, DDSRestServer.scala:401-415). Sorted ids keep the
// lanes of a wave on nearby rows, so the limb loads stay mostly coalesced.
template <int S, int TPI, int W, bool QP = false, bool Idx = false>
__global__ void __launch_bounds__(256, 2) k_fold(const uint32_t* __restrict__ X, size_t xstride, size_t count,
                                              const uint32_t* __restrict__ consts, uint32_t n0,
                                              uint32_t* __restrict__ P, size_t pstride, size_t ngroups,
                                              const uint32_t* __restrict__ ids = nullptr) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W, QP>;
  constexpr int L = G::L;
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= ngroups) return;
  auto rowat = [&](size_t pos) -> uint32_t { return Idx ? ids[pos] : (uint32_t)pos; };
  uint32_t n[L], a[L];
  g.load_vec(n, consts + kConstN * S);
  g.load_col(a, X, xstride, rowat(grp));
  if (grp + ngroups < count) {
    uint32_t pre[2][M::kPF];  // first limb blocks of the next row, requested one row ahead
    uint32_t row = rowat(grp + ngroups);
    M::load_blocks2(pre, X, xstride, row);
    for (size_t pos = grp + ngroups; pos < count; pos += ngroups) {
      const uint32_t nxt = pos + ngroups < count ? rowat(pos + ngroups) : row;  // last row: a harmless re-read
      M::mul_col_chain(a, n, X, xstride, row, nxt, pre, n0, g.top, g.bottom);
      row = nxt;
    }
  }
  M::normalize(a, g.bottom);
  g.store_col(a, P, pstride, grp);
}

// result = canon(MonPro(P[0], Y)), Y = R^k mod N; writes S rW limbs to out
template <int S, int TPI, int W>
__global__ void __launch_bounds__(64) k_finalize(const uint32_t* __restrict__ P, size_t pstride,
                                                 const uint32_t* __restrict__ consts, const uint32_t* __restrict__ Y,
                                                 uint32_t n0, uint32_t* __restrict__ out) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W>;
  constexpr int L = G::L;
  G g;
  if (threadIdx.x >= TPI) return;
  uint32_t n[L], a[L];
  g.load_vec(n, consts + kConstN * S);
  g.load_col(a, P, pstride, 0);
  M::mul_col(a, n, Y, 1, 0, n0, g.top, g.bottom);
  g.canon(a, n);
#pragma unroll
  for (int l = 0; l < L; ++l) out[g.r * L + l] = a[l];
}

}  // namespace ddshe
