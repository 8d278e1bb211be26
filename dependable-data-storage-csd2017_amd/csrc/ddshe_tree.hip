// Reduction tree of the fold (gfx950): every level after the first in ONE launch, each Montgomery
// product computed cooperatively by a whole workgroup (SumAll / MultAll fold, DDSRestServer.scala:
// 412-430 / 506-524; the tree replaces the per-level launches of round 1).
//
// Product ("SOS", separated operand scanning) on S limbs of W bits, R = 2^(W*S) >= 2^64 * N:
//   T  = a * b                      column sums, 64-bit lazy (one workgroup, S column pairs)
//   d  = T mod R                    as W-bit pieces: d_p = lo(T_p) + mid(T_{p-1}) + hi(T_{p-2}) < 3*2^W
//   m  = d * n' mod R               n' = -N^-1 mod R (full width), low-half column sums, split again
//   V  = T + m * N                  column sums; V == 0 mod R
//   U  = V / R                      high columns + the carry out of the low half, which is
//                                   ceil((V_{S-1} 2^2W + V_{S-2} 2^W + V_{S-3}) / 2^3W): the low half
//                                   is an exact multiple of R and lower columns add < 2^-48
//   two split passes give limbs < 2^W + 3 ("almost normalised")
// No step of it is sequential over the limbs: 3 passes of S mads per thread, 9 barriers, instead of
// S dependent CIOS steps. Bounds (static_assert): column sums < 7 S 2^2W < 2^64; any input below
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

#include "ddshe_launch.hpp"

namespace ddshe {

constexpr int kTreeThreads = 256;

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

  // Column sums with wave-uniform loop bounds. y operands are zero-padded in LDS (yz[S + j] = y[j],
  // yz[0..S) = yz[2S..3S) = 0), so a lane whose column does not contain a term reads a zero instead of
  // leaving the loop: each wave runs S + 64 mads (regions A | B | C below) with scalar loop control.
  // Full-product column pair of thread t (wave's first thread t0): c0 = col t, c1 = col S + t:
  //   A: i < t0        every lane's term is in col t
  //   B: t0 <= i < t0+64  both (one of the two reads hits a zero)
  //   C: i >= t0+64    every lane's term is in col S + t
  __device__ static __forceinline__ void colpair(const uint32_t* __restrict__ x, const uint32_t* __restrict__ yz, int t,
                                                 int t0, uint64_t& c0, uint64_t& c1) {
    t0 = __builtin_amdgcn_readfirstlane(t0);  // wave-uniform: scalar loop control
    const int eA = t0 < S ? t0 : S, eB = t0 + 64 < S ? t0 + 64 : S;
    const uint32_t* y0 = yz + S + t;      // y0[-i] = y[t - i] (zero when t - i < 0)
    const uint32_t* y1 = yz + 2 * S + t;  // y1[-i] = y[S + t - i] (zero when S + t - i >= S)
#pragma unroll 8
    for (int i = 0; i < eA; ++i) c0 += (uint64_t)x[i] * y0[-i];
#pragma unroll 8
    for (int i = eA; i < eB; ++i) {
      c0 += (uint64_t)x[i] * y0[-i];
      c1 += (uint64_t)x[i] * y1[-i];
    }
#pragma unroll 8
    for (int i = eB; i < S; ++i) c1 += (uint64_t)x[i] * y1[-i];
  }

  // a <- a * b * R^-1 (mod N), redundant limbs < 2^W + 3, value < 4N. LDS: bz, nz, npz zero-padded
  // (3S words, see colpair; b lives in bz[S..2S)), T: 2S words, d: S words, M: S words. Ends with a barrier.
  __device__ static void monpro(uint32_t* a, const uint32_t* bz, const uint32_t* nz, const uint32_t* npz, uint64_t* T,
                                uint32_t* d, uint64_t* M) {
    const int tid = threadIdx.x;
    // T = a*b: thread t owns columns t and S+t
    for (int t = tid; t < S; t += kTreeThreads) {
      uint64_t c0 = 0, c1 = 0;
      colpair(a, bz, t, t & ~63, c0, c1);
      T[t] = c0;
      T[S + t] = c1;
    }
    __syncthreads();
    for (int p = tid; p < S; p += kTreeThreads) d[p] = split3(T, p);
    __syncthreads();
    // m = d * n' mod R: low columns t and u = S-1-t; uniform bounds t0+64 and S-t0 (zeros beyond)
    for (int t = tid; t < S / 2; t += kTreeThreads) {
      const int t0 = __builtin_amdgcn_readfirstlane(t & ~63), u = S - 1 - t;
      const int e0 = t0 + 64 < S ? t0 + 64 : S, e1 = S - t0;
      const uint32_t* y0 = npz + S + t;
      const uint32_t* y1 = npz + S + u;
      uint64_t c0 = 0, c1 = 0;
#pragma unroll 8
      for (int i = 0; i < e0; ++i) c0 += (uint64_t)d[i] * y0[-i];
#pragma unroll 8
      for (int i = 0; i < e1; ++i) c1 += (uint64_t)d[i] * y1[-i];
      M[t] = c0;
      M[u] = c1;
    }
    __syncthreads();
    for (int p = tid; p < S; p += kTreeThreads) d[p] = split3(M, p);  // d now holds m (< 3*2^W limbs)
    __syncthreads();
    // V = T + m*N
    for (int t = tid; t < S; t += kTreeThreads) {
      uint64_t c0 = T[t], c1 = T[S + t];
      colpair(d, nz, t, t & ~63, c0, c1);
      T[t] = c0;
      T[S + t] = c1;
    }
    __syncthreads();
    if (tid == 0) {  // carry out of the low half (see the header): ceil(X / 2^3W), X < 2^(64+2W+1)
      const uint64_t v2 = T[S - 1], v1 = T[S - 2], v0 = T[S - 3];
      unsigned __int128 x = ((unsigned __int128)v2 << (2 * W)) + ((unsigned __int128)v1 << W) + v0;
      x += ((unsigned __int128)1 << (3 * W)) - 1;
      T[S] += (uint64_t)(x >> (3 * W));
    }
    __syncthreads();
    for (int j = tid; j < S; j += kTreeThreads) d[j] = split3(T + S, j);
    __syncthreads();
    for (int j = tid; j < S; j += kTreeThreads) a[j] = (d[j] & kMask) + (j >= 1 ? d[j - 1] >> W : 0u);
    __syncthreads();
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
template <int S, int W>
__global__ void __launch_bounds__(kTreeThreads) k_tree(const uint32_t* __restrict__ X, size_t xstride, size_t gstride,
                                                       int Sin, int Win, size_t nleaves,
                                                       const uint32_t* __restrict__ ids,
                                                       const uint32_t* __restrict__ consts,
                                                       const uint32_t* __restrict__ Y, uint32_t* __restrict__ nodes,
                                                       uint32_t* __restrict__ flags, uint32_t* __restrict__ out, int Sout,
                                                       int Wout, int max_levels, uint32_t* __restrict__ lvl_out,
                                                       int fence_mode) {
  using O = Sos<S, W>;
  // bz, nz, npz: zero-padded operands (Sos::colpair); b itself is sb = bz + S
  __shared__ uint32_t sa[S], bz[3 * S], nz[3 * S], npz[3 * S], sd[S], stmp[S + 64];
  __shared__ uint64_t sT[2 * S], sM[S];
  __shared__ int s_go;
  uint32_t* const sb = bz + S;
  const int tid = threadIdx.x;
  for (int j = tid; j < 3 * S; j += kTreeThreads) {
    const bool mid = j >= S && j < 2 * S;
    bz[j] = 0u;
    nz[j] = mid ? consts[j - S] : 0u;
    npz[j] = mid ? consts[j] : 0u;  // n' = consts[S + (j - S)]
  }
  auto load_leaf = [&](uint32_t* dst, size_t g) {
    const size_t row = ids ? (size_t)ids[g] : g;
    for (int l = tid; l < Sin; l += kTreeThreads) stmp[l] = X[(size_t)l * xstride + row * gstride];
    __syncthreads();
    for (int j = tid; j < S; j += kTreeThreads) dst[j] = repack_limb(stmp, Sin, Win, W, j);
    __syncthreads();
  };
  const size_t b = blockIdx.x;
  load_leaf(sa, 2 * b);
  if (2 * b + 1 < nleaves) {
    load_leaf(sb, 2 * b + 1);
    O::monpro(sa, bz, nz, npz, sT, sd, sM);
  }
  // walk up: node (h, i) holds this block's value
  int h = 1;
  size_t i = b;
  while (((size_t)1 << h) < nleaves) {
    if (max_levels > 0 && h >= max_levels) {  // hand the node to the next launch
      for (int j = tid; j < S; j += kTreeThreads) lvl_out[i * S + j] = sa[j];
      return;
    }
    const size_t sib = i ^ 1u;
    if ((sib << h) < nleaves) {  // the sibling subtree has leaves: meet it at the parent
      uint32_t* mine = nodes + node_row(h, i) * S;
      for (int j = tid; j < S; j += kTreeThreads) mine[j] = sa[j];
      if (fence_mode == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // every wave: its stores
      __syncthreads();
      if (tid == 0) {
        if (fence_mode != 0) __threadfence();
        const uint32_t old = __hip_atomic_fetch_add(flags + node_row(h + 1, i >> 1), 1u, __ATOMIC_ACQ_REL,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (fence_mode != 0) __threadfence();
        s_go = old != 0u;
      }
      __syncthreads();
      if (!s_go) return;  // first to arrive: the sibling's block continues
      if (fence_mode == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every wave: the sibling's stores
      const uint32_t* other = nodes + node_row(h, sib) * S;
      for (int j = tid; j < S; j += kTreeThreads) sb[j] = __builtin_nontemporal_load(other + j);
      __syncthreads();
      O::monpro(sa, bz, nz, npz, sT, sd, sM);
    }
    i >>= 1;
    ++h;
  }
  // root
  if (Y) {
    for (int j = tid; j < S; j += kTreeThreads) sb[j] = Y[j];
    __syncthreads();
    O::monpro(sa, bz, nz, npz, sT, sd, sM);
  }
  if (tid < 64) O::canon(sa, consts + 2 * S);
  __syncthreads();
  if (Y) {
    for (int j = tid; j < S; j += kTreeThreads) out[j] = sa[j];
  } else {
    for (int j = tid; j < Sout; j += kTreeThreads) out[j] = repack_limb(sa, S, W, Wout, j);
  }
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

// DDSHE_TREE_LEVELS (default 1; 0 = one launch walks to the root through in-kernel hand-offs, whose
// agent-scope L2 writeback/invalidate fences measured far slower than a launch per level): levels per launch;
// DDSHE_TREE_FENCE (default 1): hand-off fence style (k_tree)
static int tree_env(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

hipError_t launch_tree(int S, const uint32_t* X, size_t xstride, int Sin, int Win, size_t nleaves, const uint32_t* ids,
                       const uint32_t* consts, const uint32_t* Y, uint32_t* nodes, uint32_t* flags, uint32_t* out,
                       int Sout, int Wout, hipStream_t st) {
  static const int levels = tree_env("DDSHE_TREE_LEVELS", 1), fence = tree_env("DDSHE_TREE_FENCE", 1);
  if (nleaves == 0 || Sin > S + 64) return hipErrorInvalidValue;
  // level buffers for multi-launch trees live after the nodes: two ping-pong halves of nleaves rows
  uint32_t* lvl[2] = {nodes + (2 * nleaves + 2) * (size_t)S, nodes + (3 * nleaves + 2) * (size_t)S};
  size_t gstride = 1;
  int flip = 0;
  for (;;) {
    const bool last = levels <= 0 || nleaves <= ((size_t)1 << levels);
    const size_t blocks = (nleaves + 1) / 2;
    if (nleaves > 2) {
      hipError_t e = hipMemsetAsync(flags, 0, (2 * nleaves + 2) * 4, st);
      if (e != hipSuccess) return e;
    }
    DDSHE_TREE_SWITCH(S, hipLaunchKernelGGL((k_tree<S, W>), dim3((unsigned)blocks), dim3(kTreeThreads), 0, st, X,
                                            xstride, gstride, Sin, Win, nleaves, ids, consts, Y, nodes, flags, out,
                                            Sout, Wout, last ? 0 : levels, lvl[flip], fence));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || last) return e;
    X = lvl[flip];
    flip ^= 1;
    nleaves = (nleaves + ((size_t)1 << levels) - 1) >> levels;
    xstride = 1;
    gstride = S;
    Sin = S;
    Win = S == 694 ? 25 : 26;  // the tree radix of this class (DDSHE_TREE_SWITCH)
    ids = nullptr;
  }
}

}  // namespace ddshe
