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
  // the column holds only its first `sin` limbs (the rest read as 0)
  __device__ __forceinline__ void load_col_narrow(uint32_t (&a)[L], const uint32_t* __restrict__ col, size_t stride,
                                                  size_t row, int sin) const {
#pragma unroll
    for (int l = 0; l < L; ++l) a[l] = r * L + l < sin ? col[(size_t)(r * L + l) * stride + row] : 0u;
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
// Narrow: X is a column of a narrower shape holding `sin` limbs per row (small folds run their first
// level in the latency shape straight from the main-shape rows; the missing top limbs read as 0).
// Partial g goes to P[l * pstride + g * pgs] (limb-major by default; row-major for a launch that hands
// its partials to the reduction tree, whose blocks then read each leaf as one contiguous run).
// InBlock: the block's 256 / TPI partials are folded together before the kernel ends (a tree through
// LDS: at each level the upper half of the live groups parks its values, the lower half multiplies them
// in with mul_lds), and group 0 writes ONE partial per block, row-major with pgs words per leaf (limbs
// S..pgs zeroed: the tree's leaf shape), at leaf blockIdx.x. Every group of every block must be live
// (ngroups a multiple of 256 / TPI: the launcher checks). The block partial holds prod * R^(1 - c) with
// c the block's rows, as a group's partial does (each in-block product contributes one R^-1 and one
// more group). This replaces the tail launches between level 1 and the tree.
template <int S, int TPI, int W, bool QP = false, bool Idx = false, bool Narrow = false, bool InBlock = false>
__global__ void __launch_bounds__(256, 2) k_fold(const uint32_t* __restrict__ X, size_t xstride, size_t count,
                                              const uint32_t* __restrict__ consts, uint32_t n0,
                                              uint32_t* __restrict__ P, size_t pstride, size_t ngroups,
                                              const uint32_t* __restrict__ ids = nullptr, int sin = S,
                                              size_t pgs = 1) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W, QP>;
  constexpr int L = G::L;
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= ngroups) return;
  auto rowat = [&](size_t pos) -> uint32_t { return Idx ? ids[pos] : (uint32_t)pos; };
  uint32_t n[L], a[L];
  g.load_vec(n, consts + kConstN * S);
  if constexpr (Narrow)
    g.load_col_narrow(a, X, xstride, rowat(grp), sin);
  else
    g.load_col(a, X, xstride, rowat(grp));
  if (grp + ngroups < count) {
    uint32_t pre[2][M::kPF];  // first limb blocks of the next row, requested one row ahead
    if constexpr (!Idx) {
      // rows grp, grp + G, ...: the loop of round 1 (the row is the loop variable)
      M::load_blocks2(pre, X, xstride, (uint32_t)(grp + ngroups));
      for (size_t row = grp + ngroups; row < count; row += ngroups) {
        const size_t nxt = row + ngroups < count ? row + ngroups : row;  // last row: a harmless re-read
        M::template mul_col_chain<Narrow>(a, n, X, xstride, (uint32_t)row, (uint32_t)nxt, pre, n0, g.top, g.bottom,
                                          sin);
      }
    } else {
      uint32_t row = rowat(grp + ngroups);
      M::load_blocks2(pre, X, xstride, row);
      for (size_t pos = grp + ngroups; pos < count; pos += ngroups) {
        const uint32_t nxt = pos + ngroups < count ? rowat(pos + ngroups) : row;  // last row: a harmless re-read
        M::template mul_col_chain<Narrow>(a, n, X, xstride, row, nxt, pre, n0, g.top, g.bottom, sin);
        row = nxt;
      }
    }
  }
  M::normalize(a, g.bottom);
  if constexpr (InBlock) {
    constexpr int GPB = 256 / TPI;  // groups per block
    __shared__ uint32_t slot[(GPB / 2) * S];
    const int gi = (int)(threadIdx.x / TPI);
    for (int h = GPB / 2; h >= 1; h >>= 1) {
      if (gi >= h && gi < 2 * h) {
        uint32_t* dst = slot + (gi - h) * S + g.r * L;
#pragma unroll
        for (int l = 0; l < L; ++l) dst[l] = a[l];
      }
      __syncthreads();
      if (gi < h) {
        M::mul_lds(a, n, slot + gi * S, n0, g.top, g.bottom);
        M::normalize(a, g.bottom);
      }
      __syncthreads();  // the slots are rewritten by the next level
    }
    if (gi == 0) {
      uint32_t* leaf = P + (size_t)blockIdx.x * pgs;
#pragma unroll
      for (int l = 0; l < L; ++l) leaf[g.r * L + l] = a[l];
      for (size_t l = S + g.r; l < pgs; l += TPI) leaf[l] = 0u;
    }
    return;
  }
  g.store_col(a, P, pstride, grp * pgs);  // pstride = 1, pgs = S: row-major partials (the tree's leaves)
}

// ------------------------------------------------------------------------------
// One bignum per lane (TPI = 1) for the narrow shapes (S <= 76: the 2048-bit RSA n of MultAll,
// DDSRestServer.scala:518, and the 2048-bit n² of a 1024-bit Paillier key, :423). A lane holds the
// whole accumulator (S 64-bit lazy sums + S limbs of a); N is wave-uniform and lives in SGPRs, so the
// m·N half of every CIOS step reads its multiplicand from the scalar file, and a step needs no lane
// exchange at all: 2S mads + 4 instructions, against 2S/TPI mads + ~20 exchange/quotient
// instructions per lane at TPI = 2. Rows of a wave are 64 consecutive rows (one 256-byte load per
// limb). Latency per product is TPI times longer, so the launcher uses it only for folds with many
// rows per lane (fold1_min_rows).
// ------------------------------------------------------------------------------
template <int S, int W, bool QP>
struct Mont1 {
  static constexpr uint32_t kMask = (1u << W) - 1u;
  static constexpr int PF = 4;      // limbs per block; two blocks in flight
  static constexpr int RM = S % PF;  // remainder limbs (S = 74: 2), one short block after the last full one
  static constexpr int SB = S - RM;  // limbs in full blocks
  static_assert(RM % 2 == 0 && SB >= 2 * PF, "S % PF");
  static_assert(3ull * S < (1ull << (65 - 2 * W)), "lazy 64-bit accumulation bound");

  // t = (t + a·b + m·N) / 2^W; QP: N ≡ -1 mod 2^W, so m = t0 mod 2^W
  __device__ __forceinline__ static void step(uint64_t (&t)[S], const uint32_t (&a)[S], const uint32_t (&n)[S],
                                              uint32_t b, uint32_t n0) {
    t[0] = (uint64_t)a[0] * b + t[0];
    const uint32_t m = (QP ? (uint32_t)t[0] : (uint32_t)t[0] * n0) & kMask;
#pragma unroll
    for (int l = 1; l < S; ++l) t[l] = (uint64_t)a[l] * b + t[l];
    const uint64_t u0 = (uint64_t)m * n[0] + t[0];
    t[0] = (uint64_t)m * n[1] + (t[1] + (u0 >> W));
#pragma unroll
    for (int l = 2; l < S; ++l) t[l - 1] = (uint64_t)m * n[l] + t[l];
    t[S - 1] = 0;
  }
  // t[S - 1] stays visibly zero between steps: the next step's first mad into it takes a 0 addend
  __device__ __forceinline__ static void fence_t(uint64_t (&t)[S]) {
#pragma unroll
    for (int l = 0; l < S - 1; ++l) asm volatile("" : "+v"(t[l]));
  }
  // lazy sums -> fully normalised limbs (the whole carry chain is in this lane; value < R: no carry out)
  __device__ __forceinline__ static void settle(const uint64_t (&t)[S], uint32_t (&a)[S]) {
    uint64_t c = 0;
#pragma unroll
    for (int l = 0; l < S; ++l) {
      const uint64_t v = t[l] + c;
      asm volatile("v_and_b32 %0, %1, %2" : "=&v"(a[l]) : "v"((uint32_t)v), "v"(kMask));
      c = v >> W;
    }
  }
  __device__ __forceinline__ static auto rsrc(const uint32_t* X, size_t stride, int i) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(X + (size_t)i * stride), (short)0,
                                             (int)(PF * (uint32_t)stride * 4u), 0x00020000);
  }
  __device__ __forceinline__ static void load_blocks2(uint32_t (&pre)[2][PF], const uint32_t* __restrict__ X,
                                                      size_t stride, uint32_t row) {
    const uint32_t voff = row * 4u, sstride = (uint32_t)stride * 4u;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const auto rs = rsrc(X, stride, d * PF);
#pragma unroll
      for (int q = 0; q < PF; ++q) pre[d][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
    }
  }
  // a <- MonPro(a, X[., row]); the first two blocks of `row` arrive in pre, those of `next` leave in it
  __device__ __forceinline__ static void mul_row_chain(uint32_t (&a)[S], const uint32_t (&n)[S],
                                                       const uint32_t* __restrict__ X, size_t stride, uint32_t row,
                                                       uint32_t next, uint32_t (&pre)[2][PF], uint32_t n0) {
    uint64_t t[S];
#pragma unroll
    for (int l = 0; l < S; ++l) t[l] = 0;
    const uint32_t voff = row * 4u, sstride = (uint32_t)stride * 4u;
    uint32_t bq[PF], bm[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      bq[q] = pre[0][q];
      bm[q] = pre[1][q];
    }
#pragma unroll 1
    for (int i = 0; i < SB - 2 * PF; i += PF) {
      // opaque redefinition of a[]: stops LICM hoisting zext(a[l]) out of the block loop as 64-bit
      // values (every limb pinned to an even register pair: +S VGPRs, which S = 76 cannot afford)
#pragma unroll
      for (int l = 0; l < S; ++l) asm volatile("" : "+v"(a[l]));
      const auto rs = rsrc(X, stride, i + 2 * PF);
      uint32_t bn[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) bn[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        step(t, a, n, bq[q], n0);
        fence_t(t);
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        bq[q] = bm[q];
        bm[q] = bn[q];
      }
    }
    uint32_t br[RM > 0 ? RM : 1];  // the short block (limbs SB..S-1), requested with the last full ones
    if constexpr (RM > 0) {
      const auto rs = rsrc(X, stride, SB);
#pragma unroll
      for (int q = 0; q < RM; ++q) br[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
    }
    const uint32_t nvoff = next * 4u;
    {
      const auto rs = rsrc(X, stride, 0);
#pragma unroll
      for (int q = 0; q < PF; ++q) pre[0][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, nvoff, q * sstride, 0);
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      step(t, a, n, bq[q], n0);
      fence_t(t);
    }
    {
      const auto rs = rsrc(X, stride, PF);
#pragma unroll
      for (int q = 0; q < PF; ++q) pre[1][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, nvoff, q * sstride, 0);
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      step(t, a, n, bm[q], n0);
      fence_t(t);
    }
    if constexpr (RM > 0) {
#pragma unroll
      for (int q = 0; q < RM; ++q) {
        step(t, a, n, br[q], n0);
        fence_t(t);
      }
    }
    settle(t, a);
  }
};

// Level-1 fold at one bignum per lane: lane g folds rows g, g+G, ... (same contract and partial layout
// as k_fold: limb-major, fully normalised, prod * R^(1-c)).
template <int S, int W, bool QP = true, bool Idx = false>
__global__ void __launch_bounds__(256, 2) k_fold1(const uint32_t* __restrict__ X, size_t xstride, size_t count,
                                               const uint32_t* __restrict__ consts, uint32_t n0,
                                               uint32_t* __restrict__ P, size_t pstride, size_t ngroups,
                                               const uint32_t* __restrict__ ids = nullptr) {
  using M = Mont1<S, W, QP>;
  const size_t grp = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (grp >= ngroups) return;
  auto rowat = [&](size_t pos) -> uint32_t { return Idx ? ids[pos] : (uint32_t)pos; };
  uint32_t n[S], a[S];
#pragma unroll
  for (int l = 0; l < S; ++l) n[l] = __builtin_amdgcn_readfirstlane(consts[kConstN * S + l]);
#pragma unroll
  for (int l = 0; l < S; ++l) asm volatile("" : "+s"(n[l]));
  const uint32_t r0 = rowat(grp);
#pragma unroll
  for (int l = 0; l < S; ++l) a[l] = X[(size_t)l * xstride + r0];
  if (grp + ngroups < count) {
    uint32_t pre[2][M::PF];
    if constexpr (!Idx) {  // the row is the loop variable (k_fold: the row-id loop form cost 4.5 % there)
      M::load_blocks2(pre, X, xstride, (uint32_t)(grp + ngroups));
      for (size_t row = grp + ngroups; row < count; row += ngroups) {
        const size_t nxt = row + ngroups < count ? row + ngroups : row;
        M::mul_row_chain(a, n, X, xstride, (uint32_t)row, (uint32_t)nxt, pre, n0);
      }
    } else {
      uint32_t row = rowat(grp + ngroups);
      M::load_blocks2(pre, X, xstride, row);
      for (size_t pos = grp + ngroups; pos < count; pos += ngroups) {
        const uint32_t nxt = pos + ngroups < count ? rowat(pos + ngroups) : row;
        M::mul_row_chain(a, n, X, xstride, row, nxt, pre, n0);
        row = nxt;
      }
    }
  }
#pragma unroll
  for (int l = 0; l < S; ++l) P[(size_t)l * pstride + grp] = a[l];
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
