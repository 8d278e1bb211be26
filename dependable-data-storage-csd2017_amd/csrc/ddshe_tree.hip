// Reduction tree of the fold (gfx950): every level after the first in ONE launch, each Montgomery
// product computed cooperatively by a whole workgroup (SumAll / MultAll fold, DDSRestServer.scala:
// 412-430 / 506-524; the tree replaces the per-level launches of round 1).
//
// Product ("SOS", separated operand scanning) on S limbs of W bits, R = 2^(W*S) >= 2^64 * N:
//   T  = a * b                      column sums, 64-bit lazy (one 1024-thread workgroup)
//   d  = T mod R                    as W-bit pieces: d_p = lo(T_p) + mid(T_{p-1}) + hi(T_{p-2}) < 3*2^W
//   m  = d * n' mod R               n' = -N^-1 mod R (full width), low-half column sums, split again
//   V  = T + m * N                  column sums; V == 0 mod R
//   U  = V / R                      high columns + the carry out of the low half, which is
//                                   ceil((V_{S-1} 2^2W + V_{S-2} 2^W + V_{S-3}) / 2^3W): the low half
//                                   is an exact multiple of R and lower columns add < 2^-48
//   two split passes give limbs < 2^W + 3 ("almost normalised")
// No step of it is sequential over the limbs: three convolutions spread over the workgroup's 16 waves
// (register-blocked, Sos::conv), 10 barriers, instead of S dependent CIOS steps. Bounds (static_assert): column sums < 7 S 2^2W < 2^64; any input below
// 2^31 N (leaves from the QP levels are < 2N~ <= 2^29 N) gives U < N/4 + 3.0001 N < 4N.
//
// Tree: block b starts with leaves (2b, 2b+1) and walks up. A node's first-arriving child stores
// its value and leaves; the second (agent-scope atomic on the node's flag, fences around) loads the
// sibling and multiplies. No block ever waits for another, so any grid size is safe. The root
// either multiplies by Y = 2^(W S - E) mod N and canonicalises (the result), or canonicalises and
// writes a radix-2^Wo partial (multi-GPU exchange).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include <map>
#include <mutex>
#include <utility>

#include "ddshe_launch.hpp"

namespace ddshe {

constexpr int kTreeThreads = 1024;

// Phase stamps (profiling aid, DDSHE_TREE_STAMPS=<file>; off: a null pointer and no cost): thread 0 of
// the first and the last block of a launch records the shader clock (s_memtime) after every barrier
// of its product(s) into LDS; wave 0 copies them out at the end (lane-divergent vector stores).
constexpr int kStamps = 48;
struct Stamps {
  uint64_t* sh = nullptr;  // LDS slots; null when off
  int k = 0;
  __device__ __forceinline__ void mark() {
    if (sh && threadIdx.x == 0 && k < kStamps - 2) sh[2 + k] = __builtin_amdgcn_s_memtime();
    ++k;
  }
};

template <int S, int W>
struct Sos {
  static_assert(S % 2 == 0 && S >= 4, "even limb count");
  static_assert(7ull * S < (1ull << (64 - 2 * W)), "64-bit column sums");
  static constexpr uint32_t kMask = (1u << W) - 1u;

  __device__ static __forceinline__ uint32_t split3(const uint64_t* c, int p) {
    uint32_t v = (uint32_t)c[p] & kMask;
    if (p >= 1) v += (uint32_t)(c[p - 1] >> W) & kMask;
    if (p >= 2) v += (uint32_t)(c[p - 2] >> (2 * W));
    return v;
  }

  // Column sums as a register-blocked convolution. Work unit = (chunk of C consecutive x limbs,
  // block of 4 consecutive columns): the lane loads the C + 4 y words its 4 columns meet in the chunk
  // once (128-bit reads of a native 4-vector: as 32-bit words the compiler pairs them into read2 with
  // 8-way bank conflicts, 1.7x slower), the chunk's x words as 128-bit reads, and runs 4 C mads on 4
  // independent accumulators, then adds its 4 sums into the columns (LDS 64-bit atomics: the chunks of
  // one column land from different lanes). Only the units that reach the requested columns
  // [c_lo, c_hi) work, flattened over all the workgroup's lanes (a lane per unit: S = 162 has 630 for a
  // full product, 1024 lanes), so a pass is one round of at most 4 C mads per lane; the m*N pass asks
  // only for the high half (+3 columns for the carry), about half the units.
  // tools/microbench/tree_conv.hip: 2700 -> 1420 cycles per full S = 162 pass (one chunk per wave with
  // 32-bit y reads before).
  static constexpr int C = S <= 64 ? 4 : S <= 128 ? 8 : S <= 192 ? 12 : S <= 256 ? 16 : S <= 384 ? 24 : 48;
  static constexpr int NCH = (S + C - 1) / C;    // chunks
  static constexpr int XL = (NCH * C + 3) / 4 * 4;    // x operands: zero words up to XL
  static constexpr int YL = (C + 8 + 3) / 4 * 4;      // zero words before y[0] (multiple of 4: aligned strips)
  static constexpr int YTOT = YL + S + S + 8;         // ... and S + 8 after y[S-1]
  static constexpr int BAND = (S + C + 2) / 4 + 1;    // column blocks a chunk can reach
  static_assert(YL % 4 == 0 && C % 4 == 0, "aligned strips");

  // acc[col] += sum_i x[i] * y[col - i] for c_lo <= col < c_hi; x: XL words (16-byte aligned, zero past
  // S); yz: y[0] (16-byte aligned), zero for indices in [-YL, 0) and [S, 2S + 8)
  template <int NT>
  __device__ static __forceinline__ void conv(const uint32_t* __restrict__ x, const uint32_t* __restrict__ yz,
                                              uint64_t* acc, int c_lo, int c_hi) {
    const int cb_lo = c_lo / 4, cb_hi = (c_hi + 3) / 4;
    const u32x4* const y4 = reinterpret_cast<const u32x4*>(yz);
    const u32x4* const x4 = reinterpret_cast<const u32x4*>(x);
    for (int u = threadIdx.x; u < NCH * BAND; u += NT) {
      // unit u -> (chunk, column block): a chunk reaches BAND blocks from i0/4 on; blocks outside the
      // requested columns or past the band's end (every term there has col - i >= S) are idle lanes
      const int ch = u / BAND, cb = ch * C / 4 + (u - ch * BAND);
      if (cb < cb_lo || cb >= cb_hi || 4 * cb > ch * C + C + S - 2) continue;
      const int i0 = ch * C;
      const int base = 4 * cb - i0 - C;  // ys[q] = y[base + q]; term (i0 + r, 4 cb + j) is ys[C + j - r]
      uint32_t ys[C + 4];
#pragma unroll
      for (int q = 0; q < C + 4; q += 4) {
        const u32x4 v = y4[(base + q) >> 2];
        ys[q] = v.x;
        ys[q + 1] = v.y;
        ys[q + 2] = v.z;
        ys[q + 3] = v.w;
      }
      uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
      for (int r4 = 0; r4 < C; r4 += 4) {
        const u32x4 xv = x4[(i0 + r4) >> 2];
        const uint32_t xr[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = r4 + q;
          c0 += (uint64_t)xr[q] * ys[C - r];
          c1 += (uint64_t)xr[q] * ys[C + 1 - r];
          c2 += (uint64_t)xr[q] * ys[C + 2 - r];
          c3 += (uint64_t)xr[q] * ys[C + 3 - r];
        }
      }
      const int col = 4 * cb;
      if (c0 && col >= c_lo) atomicAdd((unsigned long long*)&acc[col], (unsigned long long)c0);
      if (c1 && col + 1 >= c_lo && col + 1 < c_hi) atomicAdd((unsigned long long*)&acc[col + 1], (unsigned long long)c1);
      if (c2 && col + 2 >= c_lo && col + 2 < c_hi) atomicAdd((unsigned long long*)&acc[col + 2], (unsigned long long)c2);
      if (c3 && col + 3 >= c_lo && col + 3 < c_hi) atomicAdd((unsigned long long*)&acc[col + 3], (unsigned long long)c3);
    }
  }

  // a <- a * b * R^-1 (mod N), redundant limbs < 2^W + 3, value < 4N. LDS: by, ny, npy = b, N, n' at
  // their y[0] (zero-padded, see conv); a, d: XL words (zero past S); T2: two column buffers of 2S words
  // (the product sums into T2[par] and zeroes T2[par ^ 1] for the next product), M: S words. T2[par]
  // and M must be zero on entry (the kernel zeroes all three while it loads its leaves); par flips.
  // Ends with a barrier. 6 barriers: the carry out of the low half is recomputed by every thread of the
  // last phase instead of by one thread between two extra barriers.
  template <int NT>
  __device__ static void monpro(uint32_t* a, const uint32_t* by, const uint32_t* ny, const uint32_t* npy, uint64_t* T2,
                                uint32_t* d, uint64_t* M, int& par, Stamps& sp) {
    const int tid = threadIdx.x;
    uint64_t* T = T2 + (size_t)par * 2 * S;
    uint64_t* Tn = T2 + (size_t)(par ^ 1) * 2 * S;
    par ^= 1;
    conv<NT>(a, by, T, 0, 2 * S);  // T = a*b
    __syncthreads();
    sp.mark();
    for (int p = tid; p < S; p += NT) d[p] = split3(T, p);
    __syncthreads();
    sp.mark();
    conv<NT>(d, npy, M, 0, S);  // m = d * n' mod R (low columns)
    __syncthreads();
    sp.mark();
    for (int p = tid; p < S; p += NT) d[p] = split3(M, p);  // d now holds m (< 3*2^W limbs)
    __syncthreads();
    sp.mark();
    conv<NT>(d, ny, T, S - 3, 2 * S);  // V = T + m*N: the high half and the 3 columns of the carry
    __syncthreads();
    sp.mark();
    {
      // carry out of the low half (see the header): ceil(X / 2^3W), X < 2^(64+2W+1); it lands in column S
      const uint64_t v2 = T[S - 1], v1 = T[S - 2], v0 = T[S - 3];
      unsigned __int128 x = ((unsigned __int128)v2 << (2 * W)) + ((unsigned __int128)v1 << W) + v0;
      x += ((unsigned __int128)1 << (3 * W)) - 1;
      const uint64_t cy = (uint64_t)(x >> (3 * W));
      const uint64_t* U = T + S;
      // limb j of U = split3 of the high columns (column 0 plus the carry), then one normalising step
      auto col = [&](int p) -> uint64_t { return p < 0 ? 0ull : U[p] + (p == 0 ? cy : 0ull); };
      auto sp3 = [&](int p) -> uint32_t {
        if (p < 0) return 0u;
        return ((uint32_t)col(p) & kMask) + ((uint32_t)(col(p - 1) >> W) & kMask) + (uint32_t)(col(p - 2) >> (2 * W));
      };
      for (int j = tid; j < S; j += NT) a[j] = (sp3(j) & kMask) + (sp3(j - 1) >> W);
      for (int j = tid; j < 2 * S; j += NT) Tn[j] = 0;  // the next product's column sums
      for (int j = tid; j < S; j += NT) M[j] = 0;       // M was last read before the previous barrier
    }
    __syncthreads();
    sp.mark();
  }

  // carry-in bit of every limb for a generate/propagate pattern over S positions (wave 0, all lanes
  // get the same words): carries = (G + (G|P)) ^ G ^ (G|P), multiword. Returns the carry out of the top.
  static constexpr int kNW = (S + 63) / 64;
  __device__ static __forceinline__ uint32_t carries(const uint64_t (&G)[kNW], const uint64_t (&P)[kNW],
                                                     uint64_t (&C)[kNW]) {
    uint64_t cin = 0;
#pragma unroll
    for (int k = 0; k < kNW; ++k) {
      const uint64_t X = G[k] | P[k];
      const uint64_t s1 = G[k] + X;
      const uint64_t c1 = s1 < G[k];
      const uint64_t s2 = s1 + cin;
      const uint64_t c2 = s2 < s1;
      C[k] = s2 ^ G[k] ^ X;
      cin = c1 | c2;
    }
    // bit S of the vector (carry into position S): inside the last word when S % 64 != 0
    if (S % 64) return (uint32_t)((C[kNW - 1] >> (S % 64)) & 1u);
    return (uint32_t)cin;
  }

  // wave 0: a (limbs < 2^W + 3, value < 4N) -> canonical [0, N), fully normalised, in place.
  // kn: N, 2N, 3N (S normalised limbs each).
  __device__ static void canon(uint32_t* a, const uint32_t* kn) {
    const int lane = threadIdx.x;  // caller: threadIdx.x < 64
    uint32_t x[kNW];
    uint64_t G[kNW], P[kNW], C[kNW];
#pragma unroll
    for (int k = 0; k < kNW; ++k) {
      const int j = lane + 64 * k;
      x[k] = j < S ? a[j] : 0u;
      G[k] = __ballot(x[k] > kMask);
      P[k] = __ballot(x[k] == kMask);
    }
    (void)carries(G, P, C);  // value < R: no carry leaves the top
#pragma unroll
    for (int k = 0; k < kNW; ++k) x[k] = (x[k] + (uint32_t)((C[k] >> lane) & 1u)) & kMask;
    // largest k in {3, 2, 1} with value >= k*N: no borrow out of value - k*N
    for (int q = 2; q >= 0; --q) {
      const uint32_t* nq = kn + q * S;
      uint32_t y[kNW];
#pragma unroll
      for (int k = 0; k < kNW; ++k) {
        const int j = lane + 64 * k;
        y[k] = j < S ? nq[j] : 0u;
        G[k] = __ballot(x[k] < y[k]);
        P[k] = __ballot(x[k] == y[k]);
      }
      if (!carries(G, P, C)) {
#pragma unroll
        for (int k = 0; k < kNW; ++k) x[k] = (x[k] - y[k] - (uint32_t)((C[k] >> lane) & 1u)) & kMask;
        break;
      }
    }
#pragma unroll
    for (int k = 0; k < kNW; ++k) {
      const int j = lane + 64 * k;
      if (j < S) a[j] = x[k];
    }
  }
};

// limb j (radix 2^Wd) of a value given as radix-2^Ws limbs src[0..Ss); Wd <= 32
__device__ __forceinline__ uint32_t repack_limb(const uint32_t* src, int Ss, int Ws, int Wd, int j) {
  const int bit = j * Wd;
  int q = bit / Ws, s = bit % Ws;
  uint64_t v = 0;
  int have = -s;
  while (have < Wd && q < Ss) {
    v |= have >= 0 ? (uint64_t)src[q] << have : (uint64_t)src[q] >> (-have);
    have += Ws;
    ++q;
  }
  return (uint32_t)v & ((1u << Wd) - 1u);
}

// in-order index of internal node (h >= 1, i) of the tree over the leaves
__device__ __forceinline__ size_t node_row(int h, size_t i) { return (i << h) + ((size_t)1 << (h - 1)) - 1; }

// consts: N | n' | N | 2N | 3N (S limbs of W bits each); Y: S limbs (finalize mode)
// leaves: X[l * xstride + g * gstride], l < Sin limbs of Win bits (g -> ids[g] when ids), g < nleaves
// max_levels > 0: stop after reaching level max_levels (a node over 2^max_levels leaves) and write that
//   node's value (S limbs of W bits) to lvl_out[i * S] (next launch's leaves); 0: walk to the root.
// At the root: finalize (Y != nullptr): out = canonical result, S limbs of W bits;
//   else out = canonical partial, Sout limbs of Wout bits, consecutive.
// fence_mode 0: every wave releases / acquires at agent scope around a hand-off; 1: wave 0 only.
template <int S, int W, int NT>
__global__ void __launch_bounds__(NT) k_tree(const uint32_t* __restrict__ X, size_t xstride, size_t gstride,
                                                       int Sin, int Win, size_t nleaves,
                                                       const uint32_t* __restrict__ ids,
                                                       const uint32_t* __restrict__ consts,
                                                       const uint32_t* __restrict__ Y, uint32_t* __restrict__ nodes,
                                                       uint32_t* __restrict__ flags, uint32_t* __restrict__ out, int Sout,
                                                       int Wout, int max_levels, uint32_t* __restrict__ lvl_out,
                                                       int fence_mode, uint64_t* __restrict__ stamps,
                                                       uint32_t* __restrict__ clear, size_t nclear, int yleaf,
                                                       uint32_t* __restrict__ done, uint32_t seq) {
  using O = Sos<S, W>;
  // the next launch's hand-off counters, zeroed here instead of by a separate memset launch
  for (size_t j = (size_t)blockIdx.x * NT + threadIdx.x; j < nclear; j += (size_t)gridDim.x * NT) clear[j] = 0u;
  // y operands (b, N, n') zero-padded around y[0] (Sos::conv); x operands (a, d) zero past S
  __shared__ __attribute__((aligned(16))) uint32_t sa[O::XL], sd[O::XL], byp[O::YTOT], nyp[O::YTOT], npyp[O::YTOT];
  __shared__ uint32_t stmp[S + 64], stmp2[S + 64];
  __shared__ uint64_t sT[2 * 2 * S], sM[S];
  int par = 0;
  __shared__ int s_go;
  __shared__ uint64_t s_stamps[kStamps];
  Stamps sp;
  const bool stamped = stamps && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1);
  if (stamped) {
    sp.sh = s_stamps;
    if (threadIdx.x == 0) {
      s_stamps[0] = __builtin_amdgcn_s_memrealtime();
      s_stamps[2] = __builtin_amdgcn_s_memtime();
    }
    sp.k = 1;
  }
  uint32_t* const sb = byp + O::YL;
  const uint32_t* const ny = nyp + O::YL;
  const uint32_t* const npy = npyp + O::YL;
  const int tid = threadIdx.x;
  const size_t b = blockIdx.x;
  const bool pair = 2 * b + 1 < nleaves;
  // yleaf: the last leaf (index nleaves - 1) is Y, in this radix (the finalising factor enters as a
  // leaf instead of as a product after the root: same product count, one product less in sequence)
  const size_t nx = nleaves - (yleaf ? 1 : 0);  // leaves from X
  const bool y0 = yleaf && 2 * b == nx, y1 = yleaf && 2 * b + 1 == nx;
  const int n0 = y0 ? S : Sin, n1 = y1 ? S : Sin;  // words of each leaf
  // the leaves' words first (Sin <= S + 64), so their global loads are in flight together with the
  // constants' below: one memory round trip instead of two
  constexpr int LW = (S + 64 + NT - 1) / NT;  // leaf words per thread
  uint32_t lw0[LW], lw1[LW];
  {
    const size_t r0 = y0 ? 0 : (ids ? (size_t)ids[2 * b] : 2 * b);
    const size_t r1 = (pair && !y1) ? (ids ? (size_t)ids[2 * b + 1] : 2 * b + 1) : r0;
#pragma unroll
    for (int q = 0; q < LW; ++q) {
      const int j = tid + q * NT;
      lw0[q] = j < n0 ? (y0 ? Y[j] : X[(size_t)j * xstride + r0 * gstride]) : 0u;
      lw1[q] = (pair && j < n1) ? (y1 ? Y[j] : X[(size_t)j * xstride + r1 * gstride]) : 0u;
    }
  }
  for (int j = tid; j < O::YTOT; j += NT) {
    const int k = j - O::YL;  // logical index
    const bool in = k >= 0 && k < S;
    byp[j] = 0u;
    nyp[j] = in ? consts[k] : 0u;
    npyp[j] = in ? consts[S + k] : 0u;
  }
  for (int j = tid; j < O::XL; j += NT) {
    sa[j] = 0u;
    sd[j] = 0u;
  }
  for (int j = tid; j < 4 * S; j += NT) sT[j] = 0;  // both column buffers (Sos::monpro)
  for (int j = tid; j < S; j += NT) sM[j] = 0;
  {  // both leaves at once
#pragma unroll
    for (int q = 0; q < LW; ++q) {
      const int j = tid + q * NT;
      if (j < n0) stmp[j] = lw0[q];
      if (j < n1) stmp2[j] = lw1[q];
    }
    __syncthreads();
    // a previous launch's nodes (and Y) are in this radix: redundant limbs (< 2^W + 3), kept as they
    // are; rows / first-level partials are normalised limbs of another radix
    const bool same = Sin == S && Win == W;
    for (int j = tid; j < S; j += NT) {
      sa[j] = (same || y0) ? stmp[j] : repack_limb(stmp, Sin, Win, W, j);
      if (pair) sb[j] = (same || y1) ? stmp2[j] : repack_limb(stmp2, Sin, Win, W, j);
    }
    __syncthreads();
  }
  sp.mark();  // leaves loaded
  if (pair) O::template monpro<NT>(sa, sb, ny, npy, sT, sd, sM, par, sp);
  // walk up: node (h, i) holds this block's value
  int h = 1;
  size_t i = b;
  while (((size_t)1 << h) < nleaves) {
    if (max_levels > 0 && h >= max_levels) {  // hand the node to the next launch
      for (int j = tid; j < S; j += NT) lvl_out[i * S + j] = sa[j];
      if (stamped) {
        sp.mark();
        if (threadIdx.x == 0) s_stamps[1] = __builtin_amdgcn_s_memrealtime() | ((uint64_t)sp.k << 56);
        __syncthreads();
        if (threadIdx.x < kStamps) stamps[(blockIdx.x == 0 ? 0 : kStamps) + threadIdx.x] = s_stamps[threadIdx.x];
      }
      return;
    }
    const size_t sib = i ^ 1u;
    if ((sib << h) < nleaves) {  // the sibling subtree has leaves: meet it at the parent
      uint32_t* mine = nodes + node_row(h, i) * S;
      if (fence_mode == 2) {
        // no cache maintenance: the node words go through to memory as relaxed agent-scope atomic
        // stores (sc1, write-through), each wave waits for its stores to complete (workgroup-scope
        // release = s_waitcnt), and the sibling reads them with agent-scope atomic loads (sc1: not
        // served from a stale line of its own XCD's L2). tools/microbench/xcd_flag.hip: ~0.6 us per
        // hop this way against ~20 us with agent-scope release/acquire (L2 writeback + invalidate).
        for (int j = tid; j < S; j += NT)
          __hip_atomic_store(mine + j, sa[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores are done
      } else {
        for (int j = tid; j < S; j += NT) mine[j] = sa[j];
      }
      if (fence_mode == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // every wave: its stores
      __syncthreads();
      if (tid == 0) {
        if (fence_mode == 1) __threadfence();
        const uint32_t old = fence_mode == 2 ? __hip_atomic_fetch_add(flags + node_row(h + 1, i >> 1), 1u,
                                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                             : __hip_atomic_fetch_add(flags + node_row(h + 1, i >> 1), 1u,
                                                                      __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (fence_mode == 1) __threadfence();
        s_go = old != 0u;
      }
      __syncthreads();
      if (!s_go) return;  // first to arrive: the sibling's block continues
      if (fence_mode == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every wave: the sibling's stores
      const uint32_t* other = nodes + node_row(h, sib) * S;
      if (fence_mode == 2) {
        for (int j = tid; j < S; j += NT)
          sb[j] = __hip_atomic_load(const_cast<uint32_t*>(other) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        for (int j = tid; j < S; j += NT) sb[j] = __builtin_nontemporal_load(other + j);
      }
      __syncthreads();
      O::template monpro<NT>(sa, sb, ny, npy, sT, sd, sM, par, sp);
    }
    i >>= 1;
    ++h;
  }
  // root
  if (Y && !yleaf) {
    for (int j = tid; j < S; j += NT) sb[j] = Y[j];
    __syncthreads();
    sp.mark();
    O::template monpro<NT>(sa, sb, ny, npy, sT, sd, sM, par, sp);
  }
  if (tid < 64) O::canon(sa, consts + 2 * S);
  __syncthreads();
  sp.mark();
  if (Y) {
    for (int j = tid; j < S; j += NT) out[j] = sa[j];
  } else {
    for (int j = tid; j < Sout; j += NT) out[j] = repack_limb(sa, S, W, Wout, j);
  }
  if (done) {  // out is host memory a caller spins on: every storing thread's writes reach the system first,
               // then one system-scope release store of the call's sequence number
    __threadfence_system();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (stamped) {
    if (threadIdx.x == 0) s_stamps[1] = __builtin_amdgcn_s_memrealtime() | ((uint64_t)sp.k << 56);
    __syncthreads();
    if (threadIdx.x < kStamps) stamps[(blockIdx.x == 0 ? 0 : kStamps) + threadIdx.x] = s_stamps[threadIdx.x];
  }
}

// Pairwise products in the latency shape of the tree: block b computes out_b = A_b * B_b mod N
// (canonical, S limbs of W bits, row-major like A and B; operands < N) as MonPro(MonPro(a, b), R^2):
// two workgroup products of ~4 us each instead of two lane-group CIOS products of ~15 us (the /Sum and
// /Mult routes, DDSRestServer.scala:385, :479, coalesced by ddshe_pairs.cpp).
template <int S, int W>
__global__ void __launch_bounds__(kTreeThreads) k_pairs_sos(const uint32_t* __restrict__ A, const uint32_t* __restrict__ B,
                                                            const uint32_t* __restrict__ consts,
                                                            const uint32_t* __restrict__ R2, uint32_t* __restrict__ out) {
  using O = Sos<S, W>;
  constexpr int NT = kTreeThreads;
  __shared__ __attribute__((aligned(16))) uint32_t sa[O::XL], sd[O::XL], byp[O::YTOT], nyp[O::YTOT], npyp[O::YTOT];
  __shared__ uint64_t sT[2 * 2 * S], sM[S];
  uint32_t* const sb = byp + O::YL;
  const uint32_t* const ny = nyp + O::YL;
  const uint32_t* const npy = npyp + O::YL;
  const int tid = threadIdx.x;
  const size_t b = blockIdx.x;
  for (int j = tid; j < O::YTOT; j += NT) {
    const int k = j - O::YL;
    const bool in = k >= 0 && k < S;
    byp[j] = in ? B[b * S + k] : 0u;
    nyp[j] = in ? consts[k] : 0u;
    npyp[j] = in ? consts[S + k] : 0u;
  }
  for (int j = tid; j < O::XL; j += NT) {
    sa[j] = j < S ? A[b * S + j] : 0u;
    sd[j] = 0u;
  }
  for (int j = tid; j < 4 * S; j += NT) sT[j] = 0;
  for (int j = tid; j < S; j += NT) sM[j] = 0;
  __syncthreads();
  int par = 0;
  Stamps sp;
  O::template monpro<NT>(sa, sb, ny, npy, sT, sd, sM, par, sp);  // a b R^-1
  for (int j = tid; j < S; j += NT) sb[j] = R2[j];
  __syncthreads();
  O::template monpro<NT>(sa, sb, ny, npy, sT, sd, sM, par, sp);  // a b
  if (tid < 64) O::canon(sa, consts + 2 * S);
  __syncthreads();
  for (int j = tid; j < S; j += NT) out[b * S + j] = sa[j];
}

#define DDSHE_TREE_SWITCH(S_RT, ...)                 \
  switch (S_RT) {                                    \
    DDSHE_TREE_CASE(46, 26, __VA_ARGS__)             \
    DDSHE_TREE_CASE(84, 26, __VA_ARGS__)             \
    DDSHE_TREE_CASE(86, 26, __VA_ARGS__)             \
    DDSHE_TREE_CASE(124, 26, __VA_ARGS__)            \
    DDSHE_TREE_CASE(162, 26, __VA_ARGS__)            \
    DDSHE_TREE_CASE(244, 26, __VA_ARGS__)            \
    DDSHE_TREE_CASE(336, 26, __VA_ARGS__)            \
    DDSHE_TREE_CASE(694, 25, __VA_ARGS__)            \
    default: return hipErrorInvalidValue;            \
  }
#define DDSHE_TREE_CASE(S_, W_, ...)                 \
  case S_: {                                         \
    constexpr int S = S_, W = W_;                    \
    __VA_ARGS__;                                     \
  } break;

Shape tree_shape(size_t mod_bits) {
  // one class per main shape: R = 2^(W S) >= 2^64 * 2^(class max bits)
  static const struct { size_t maxbits; int S, W; } cls[] = {{1118, 46, 26},  {2070, 84, 26},  {2126, 86, 26},
                                                              {3134, 124, 26}, {4142, 162, 26}, {6262, 244, 26},
                                                              {8638, 336, 26}, {17278, 694, 25}};
  for (const auto& c : cls)
    if (mod_bits <= c.maxbits) return Shape{c.S, 0, c.W};
  return Shape{0, 0, 0};
}

// Launch plan of a tree over n leaves:
//   * wide levels (more than DDSHE_TREE_WIDE blocks, default 256 = one per CU): one level per launch on
//     256-thread workgroups (k_tree<S, W, 256>): 8 products resident per CU instead of 1-2, each product
//     slower than on 1024 threads but the level finishes in fewer rounds (512-thread workgroups for the
//     levels of <= 1024 blocks measured the same, tools/tree_sweep.sh);
//   * the rest on 1024-thread workgroups, DDSHE_TREE_LEVELS levels per launch (0 = to the root).
//     With in-kernel hand-offs (LEVELS != 1) the node words are handed over in the form MI355X_MICROARCH.md
//     (§ inter-workgroup visibility, "Valid forms", first table row) lists as measured valid: every node
//     word stored sc1 (relaxed agent-scope atomic store), every storing wave's s_waitcnt vmcnt(0), a
//     workgroup barrier, ONE lane's agent-scope atomic add on the parent's counter, the block whose add
//     returned 1 continues and its waves load the sibling with sc1 loads after a barrier; hipMalloc'd
//     memory; ONE workgroup per CU, enforced by the launch's dynamic LDS (> half of the CU's 160 KiB).
//     DDSHE_TREE_FENCE selects the hand-off style: 2 = that form, 0 = agent-scope release/acquire by
//     every wave (L2 writeback + L1 invalidate per hop), 1 = one level per launch only.
static int tree_env(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// DDSHE_TREE_STAMPS=<file>: after every tree launch, synchronise and append one line per stamped block:
// "S nleaves blocks block memtime_at_entry realtime_entry realtime_exit nmarks d1 d2 ..." (d = shader-clock
// deltas between consecutive marks). Profiling only: it serialises the stream.
static void dump_stamps(uint64_t* d_st, int S, size_t nleaves, size_t blocks, hipStream_t st) {
  static const char* path = getenv("DDSHE_TREE_STAMPS");
  uint64_t h[2 * kStamps];
  if (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(h, d_st, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
    return;
  FILE* f = fopen(path, "a");
  if (!f) return;
  for (int b = 0; b < (blocks > 1 ? 2 : 1); ++b) {
    const uint64_t* v = h + b * kStamps;
    const int nm = (int)(v[1] >> 56);
    fprintf(f, "%d %zu %zu %s %llu %llu %llu %d", S, nleaves, blocks, b ? "last" : "first", (unsigned long long)v[2],
            (unsigned long long)v[0], (unsigned long long)(v[1] & ((1ull << 56) - 1)), nm);
    for (int k = 1; k < nm && k + 2 < kStamps; ++k) fprintf(f, " %llu", (unsigned long long)(v[2 + k] - v[1 + k]));
    fprintf(f, "\n");
  }
  fclose(f);
}

hipError_t launch_pairs_sos(int S, const uint32_t* A, const uint32_t* B, size_t n, const uint32_t* consts,
                            const uint32_t* R2, uint32_t* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  DDSHE_TREE_SWITCH(S, hipLaunchKernelGGL((k_pairs_sos<S, W>), dim3((unsigned)n), dim3(kTreeThreads), 0, st, A, B,
                                          consts, R2, out));
  return hipGetLastError();
}

constexpr int kTreeWideThreads = 256;
constexpr size_t kOneWgPerCuLds = 96 * 1024;  // dynamic LDS of a hand-off launch: one workgroup per CU

// A hand-off launch asks for kOneWgPerCuLds of dynamic LDS on top of the kernel's static LDS (about
// 150 KiB in all at S = 694). Checked once per (device, kernel): a device whose workgroups cannot have
// that much (less than gfx950's 160 KiB per CU) runs the tree one level per launch instead of failing.
static bool handoff_fits(const void* fn) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, bool> known;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lk(mu);
  auto it = known.find({dev, fn});
  if (it != known.end()) return it->second;
  int lim = 0;
  for (hipDeviceAttribute_t a : {hipDeviceAttributeMaxSharedMemoryPerBlock, hipDeviceAttributeSharedMemPerBlockOptin,
                                 hipDeviceAttributeMaxSharedMemoryPerMultiprocessor}) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, a, dev) == hipSuccess) lim = std::max(lim, v);
  }
  hipFuncAttributes fa;
  bool ok = hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.sharedSizeBytes + kOneWgPerCuLds <= (size_t)lim &&
            hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kOneWgPerCuLds) == hipSuccess;
  (void)hipGetLastError();
  known[{dev, fn}] = ok;
  return ok;
}

hipError_t launch_tree(int S, const uint32_t* X, size_t xstride, int Sin, int Win, size_t nleaves, const uint32_t* ids,
                       const uint32_t* consts, const uint32_t* Y, uint32_t* nodes, uint32_t* flags, uint32_t* out,
                       int Sout, int Wout, hipStream_t st, size_t gstride, uint32_t* done, uint32_t seq) {
  static const int levels_env = tree_env("DDSHE_TREE_LEVELS", 0), fence = tree_env("DDSHE_TREE_FENCE", 2);
  static const size_t wide = (size_t)tree_env("DDSHE_TREE_WIDE", 256);
  static uint64_t* d_st = nullptr;
  static const bool stamping = getenv("DDSHE_TREE_STAMPS") && hipMalloc(&d_st, 2 * kStamps * 8) == hipSuccess;
  if (nleaves == 0 || Sin > S + 64) return hipErrorInvalidValue;
  // in-kernel hand-offs with wave-0-only fences rely on cache side effects the memory model does not
  // promise: only the every-wave (0) and sc1 write-through (2) styles may hand off in-kernel
  if (levels_env != 1 && fence == 1) return hipErrorInvalidValue;
  int levels = levels_env;
  if (levels != 1) DDSHE_TREE_SWITCH(S, if (!handoff_fits(reinterpret_cast<const void*>(&k_tree<S, W, kTreeThreads>))) levels = 1);
  // level buffers for multi-launch trees live after the nodes: two ping-pong halves of nleaves rows
  uint32_t* lvl[2] = {nodes + (2 * nleaves + 2) * (size_t)S, nodes + (3 * nleaves + 2) * (size_t)S};
  int flip = 0;
  bool flags_clear = false;  // a previous wide launch zeroed this launch's counters
  for (;;) {
    const size_t blocks = (nleaves + 1) / 2;
    const bool wide_level = blocks > wide;  // 256-thread workgroups, one level
    const int lv = wide_level ? 1 : levels;
    const bool last = lv <= 0 || nleaves <= ((size_t)1 << lv);
    // the launch that walks to the root with in-kernel hand-offs takes Y as one more leaf (not for
    // <= 2 leaves: the extra leaf would add the hand-off and its counter reset to a one-product tree)
    const int yleaf = (last && Y && lv != 1 && nleaves > 2) ? 1 : 0;
    const size_t nl = nleaves + yleaf;
    const bool handoff = nl > 2 && (last ? lv != 1 : lv > 1);  // hand-offs happen in this launch
    if (handoff && !flags_clear) {
      hipError_t e = hipMemsetAsync(flags, 0, (2 * nl + 2) * 4, st);
      if (e != hipSuccess) return e;
    }
    flags_clear = false;
    if (wide_level) {
      // the next launch: its leaves and whether it hands off in-kernel (then this one zeroes its counters)
      const size_t nn = (nleaves + 1) >> 1, nb = (nn + 1) / 2;
      const int nlv = nb > wide ? 1 : levels;
      const bool nlast = nlv <= 0 || nn <= ((size_t)1 << nlv);
      const size_t nnl = nn + ((nlast && Y && nlv != 1 && nn > 2) ? 1 : 0);  // its leaves, Y included
      const size_t nclear = (nnl > 2 && (nlast ? nlv != 1 : nlv > 1)) ? 2 * nnl + 2 : 0;
      flags_clear = nclear != 0;
      DDSHE_TREE_SWITCH(S, hipLaunchKernelGGL((k_tree<S, W, kTreeWideThreads>), dim3((unsigned)blocks),
                                              dim3(kTreeWideThreads), 0, st, X, xstride, gstride, Sin, Win, nleaves,
                                              ids, consts, Y, nodes, flags, out, Sout, Wout, last ? 0 : 1, lvl[flip],
                                              fence, stamping ? d_st : nullptr, flags, nclear, 0, done, seq));
    } else {
      const size_t dyn = handoff ? kOneWgPerCuLds : 0;
      DDSHE_TREE_SWITCH(S, {
        hipLaunchKernelGGL((k_tree<S, W, kTreeThreads>), dim3((unsigned)((nl + 1) / 2)), dim3(kTreeThreads), dyn, st,
                           X, xstride, gstride, Sin, Win, nl, ids, consts, Y, nodes, flags, out, Sout, Wout,
                           last ? 0 : lv, lvl[flip], fence, stamping ? d_st : nullptr, nullptr, (size_t)0, yleaf,
                           done, seq);
      });
    }
    hipError_t e = hipGetLastError();
    if (stamping && e == hipSuccess) dump_stamps(d_st, S, nleaves, blocks, st);
    if (e != hipSuccess || last) return e;
    X = lvl[flip];
    flip ^= 1;
    nleaves = (nleaves + ((size_t)1 << lv) - 1) >> lv;
    xstride = 1;
    gstride = S;
    Sin = S;
    Win = S == 694 ? 25 : 26;  // the tree radix of this class (DDSHE_TREE_SWITCH)
    ids = nullptr;
  }
}

}  // namespace ddshe
