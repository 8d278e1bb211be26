// Decimal ciphertext codec (gfx950): BigInteger.toString rows -> rW column, on the GPU.
//
// Reference: ciphertexts travel and are stored as decimal strings (DDSSet contents,
// dds/core/models/DDSSet.scala:3, dds/http/DDSJsonProtocol.scala:14-29) and every fold
// re-parses them with new BigInteger(String) (dds/http/DDSRestServer.scala:417,419,422,513).
// That parse costs about as much as one modmul per row, so once the fold is on
// the GPU it is the next bottleneck.
//
// Input: an Arrow-style string column (chars + offsets[count+1]) staged in HBM with a 16-byte
// zero pad on both sides. Output: column rows X[l*stride + row], fully normalised radix-2^W, plus
// one status byte per row (kDec* bits) and their OR in flags[0].
//
// k_dec_parse, one lane group (TPI lanes) per row:
//   1. digits -> base-10^8 words w_j (j = 0 least significant), 8 ASCII digits per word with a
//      SWAR validate + combine; words go to the group's LDS slice;
//   2. value = sum_j w_j * 10^(8j): limb l accumulates w_j * P_j[l] in a 64-bit lazy accumulator,
//      P_j = 10^(8j) in radix 2^W from a per-modulus table (L2-resident). Limbs are interleaved
//      over lanes (l = r + TPI*i) so every lane skips the same all-zero prefix of the triangle
//      (P_j has ~0.95j non-zero limbs): ~K^2/(2*1.05*TPI) MACs per lane for K words;
//   3. two carry rounds in the interleaved domain (limbs < 2^(W+1)), LDS transpose to the
//      contiguous group layout, exact normalisation, 2N compare, store.
// k_dec_fix: rows flagged negative (BigInteger.mod: x -> N - (|x| mod N)) or >= 2N
// (x -> x mod N by two Montgomery products) are rewritten in place.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ddshe_device.hpp"
#include "ddshe_fold.hpp"
#include "ddshe_launch.hpp"
#include "ddshe_shapes.hpp"

namespace ddshe {

// 8 ASCII bytes (byte 0 = most significant digit) -> value; *bad set if any byte is not a digit
__device__ __forceinline__ uint32_t dec8_swar(uint64_t x, bool* bad) {
  const uint64_t hi = 0xF0F0F0F0F0F0F0F0ull, z = 0x3030303030303030ull;
  *bad = ((x & hi) != z) || (((x + 0x0606060606060606ull) & hi) != z);
  uint64_t v = x & 0x0F0F0F0F0F0F0F0Full;
  v = (v * 10 + (v >> 8)) & 0x00FF00FF00FF00FFull;
  v = (v * 100 + (v >> 16)) & 0x0000FFFF0000FFFFull;
  v = (v * 10000 + (v >> 32)) & 0xFFFFFFFFull;
  return (uint32_t)v;
}

// 8 bytes at byte offset p of a 4-byte aligned buffer (p-0..p+11 in bounds: the staging pad)
__device__ __forceinline__ uint64_t load8_unaligned(const uint32_t* __restrict__ base, int64_t p) {
  const int64_t a = p >> 2;
  const uint32_t sh = (uint32_t)(p & 3);
  const uint32_t u0 = base[a], u1 = base[a + 1], u2 = base[a + 2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(u1, u0, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(u2, u1, sh);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// lane (r-1) mod TPI of the group
template <int TPI>
__device__ __forceinline__ uint32_t grp_rot_prev(uint32_t x, int r) {
  const int base = lane_id() - r;
  return (uint32_t)__builtin_amdgcn_ds_bpermute((base + (r + TPI - 1) % TPI) << 2, (int)x);
}

template <int TPI>
__device__ __forceinline__ uint32_t grp_or(uint32_t x, int r) {
  uint32_t o = x;
  const int base = lane_id() - r;
#pragma unroll
  for (int s = 0; s < TPI; ++s) o |= (uint32_t)__builtin_amdgcn_ds_bpermute((base + s) << 2, (int)x);
  return o;
}

// tab: Pt[l * jpad + j] = limb l of 10^(8j) (j < jfit, zero up to jpad), then jst[i] (i < L of the shape's
// own TPI): a multiple of 4 <= the first j whose power reaches limb TPI*i. A launch with a wider lane
// group (TL = jstep * TPI lanes) reads jst[i * jstep] for its limb TL*i. ldsw: LDS words per group.
template <int S, int TPI, int W>
__global__ void __launch_bounds__(256) k_dec_parse(const uint32_t* __restrict__ chars4, const uint64_t* __restrict__ offs,
                                                   uint64_t obase, size_t count, const uint32_t* __restrict__ tab,
                                                   int jfit, int jpad, int ldsw, int jstep,
                                                   const uint32_t* __restrict__ consts, uint32_t* __restrict__ X,
                                                   size_t stride, uint8_t* __restrict__ rowflags,
                                                   uint32_t* __restrict__ flags) {
  using G = Grp<S, TPI, W>;
  constexpr int L = G::L;
  constexpr uint32_t kMask = G::kMask;
  constexpr int GPB = 256 / TPI;
  extern __shared__ uint32_t lds[];
  const uint8_t* chars = reinterpret_cast<const uint8_t*>(chars4);
  G g;
  const int q = (int)(threadIdx.x / TPI);
  const size_t row = (size_t)blockIdx.x * GPB + q;
  const bool live = row < count;
  uint32_t* buf = lds + (size_t)q * ldsw;

  // ---- 1. digits -> base-10^8 words --------------------------------------------------
  uint32_t fl = 0;
  int kw = 0;  // words kept (<= jfit), rounded up to 4 below
  if (live) {
    const int64_t beg = (int64_t)(offs[row] - obase) + 16, end = (int64_t)(offs[row + 1] - obase) + 16;
    if (end <= beg) {
      fl = kDecFormat;  // "" -> NumberFormatException
    } else {
      const uint8_t c0 = chars[beg];
      const bool neg = c0 == '-';
      const int64_t ds = beg + ((neg || c0 == '+') ? 1 : 0);
      const int64_t nd = end - ds;
      if (nd <= 0) {
        fl = kDecFormat;  // "-" / "+"
      } else {
        if (neg) fl |= kDecNeg;
        const int64_t K = (nd + 7) / 8;
        kw = (int)(K < jfit ? K : jfit);
        for (int64_t j = g.r; j < K; j += TPI) {
          const int64_t p = end - 8 * (j + 1);
          uint64_t x = load8_unaligned(chars4, p);
          const int64_t k = ds - p;  // leading bytes before the first digit read as '0'
          if (k > 0) {
            const uint64_t m = k >= 8 ? ~0ull : ((1ull << (8 * k)) - 1);
            x = (x & ~m) | (0x3030303030303030ull & m);
          }
          bool bad;
          const uint32_t w = dec8_swar(x, &bad);
          if (bad) fl |= kDecFormat;
          if (j < jfit) buf[j] = w;
          else if (w) fl |= kDecWide;
        }
        const int kr = (kw + 3) & ~3;
        for (int j = kw + g.r; j < kr; j += TPI) buf[j] = 0u;
        kw = kr;
      }
    }
  }
  fl = grp_or<TPI>(fl, g.r);
  __syncthreads();

  // ---- 2. value = sum_j w_j * 10^(8j), interleaved limbs l = r + TPI*i ----------------
  uint64_t acc[L];
#pragma unroll
  for (int i = 0; i < L; ++i) acc[i] = 0;
  if (live && !(fl & kDecFormat)) {
    // QL limbs per pass: one LDS read of 4 words feeds QL table rows (independent loads in flight
    // instead of one dependent L2 round trip per 4 words of one limb). A pass starts at its lowest
    // limb's first non-zero word; the higher limbs' table entries below their own start are zero.
    constexpr int QL = 4;
    const uint32_t* jst = tab + (size_t)S * jpad;
    const uint4* wb = reinterpret_cast<const uint4*>(buf);
#pragma unroll
    for (int i0 = 0; i0 < L; i0 += QL) {
      const uint4* pl[QL];
      uint64_t s[QL];
#pragma unroll
      for (int q = 0; q < QL; ++q) {
        pl[q] = reinterpret_cast<const uint4*>(tab + (size_t)(g.r + TPI * (i0 + q < L ? i0 + q : i0)) * jpad);
        s[q] = 0;
      }
#pragma unroll 2
      for (int j4 = (int)jst[i0 * jstep] >> 2; j4 < (kw >> 2); ++j4) {
        const uint4 w = wb[j4];
#pragma unroll
        for (int q = 0; q < QL; ++q) {
          if (i0 + q < L) {
            const uint4 pv = pl[q][j4];
            s[q] += (uint64_t)w.x * pv.x;
            s[q] += (uint64_t)w.y * pv.y;
            s[q] += (uint64_t)w.z * pv.z;
            s[q] += (uint64_t)w.w * pv.w;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < QL; ++q)
        if (i0 + q < L) acc[i0 + q] = s[q];
    }
  }

  // ---- 3. carries: two interleaved rounds, LDS transpose, exact normalisation -----------
  uint32_t ovf = 0;
#pragma unroll
  for (int round = 0; round < 2; ++round) {
    uint32_t clo[L], chi[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const uint64_t c = acc[i] >> W;
      acc[i] &= kMask;
      clo[i] = grp_rot_prev<TPI>((uint32_t)c, g.r);
      chi[i] = grp_rot_prev<TPI>((uint32_t)(c >> 32), g.r);
    }
    // lane r >= 1 takes the carry of limb l-1 = (r-1) + TPI*i; lane 0 that of (TPI-1) + TPI*(i-1)
#pragma unroll
    for (int i = L - 1; i >= 0; --i) {
      uint64_t c = ((uint64_t)chi[i] << 32) | clo[i];
      if (g.bottom) c = i ? (((uint64_t)chi[i - 1] << 32) | clo[i - 1]) : 0ull;
      acc[i] += c;
    }
    if (g.bottom && (clo[L - 1] | chi[L - 1])) ovf = 1;  // carry out of limb S-1
  }
  __syncthreads();  // buf (words) no longer read
  if (live) {
#pragma unroll
    for (int i = 0; i < L; ++i) buf[g.r + TPI * i] = (uint32_t)acc[i];
  }
  __syncthreads();
  uint32_t a[L];
#pragma unroll
  for (int l = 0; l < L; ++l) a[l] = buf[g.r * L + l];
  // limbs < 2^(W+1): ripple carries across lanes (one boundary per round), top carry = overflow
#pragma unroll 1
  for (int round = 0; round < TPI; ++round) {
    uint32_t c = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const uint32_t v = a[l] + c;
      a[l] = v & kMask;
      c = v >> W;
    }
    if (g.top && c) ovf = 1;
    uint32_t cin = grp_from_prev<TPI>(c);
    if (g.bottom) cin = 0;
    a[0] += cin;
  }
  if (!live) return;
  if (grp_or<TPI>(ovf, g.r)) fl |= kDecWide;
  if (!(fl & (kDecFormat | kDecWide))) {
    uint32_t n2[L];
    g.load_vec(n2, consts + kConstN2x * S);
    if (g.cmp(a, n2) >= 0) fl |= kDecReduce;
  } else {
#pragma unroll
    for (int l = 0; l < L; ++l) a[l] = 0;
  }
  g.store_col(a, X, stride, row);
  if (g.bottom) {
    rowflags[row] = (uint8_t)fl;
    if (fl) atomicOr(flags, fl);
  }
}

// rows flagged kDecReduce: x <- x mod N; kDecNeg: x <- (N - (|x| mod N)) mod N
template <int S, int TPI, int W>
__global__ void __launch_bounds__(256, 2) k_dec_fix(uint32_t* __restrict__ X, size_t stride, size_t count,
                                                 const uint8_t* __restrict__ rowflags,
                                                 const uint32_t* __restrict__ consts, uint32_t n0) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W>;
  constexpr int L = G::L;
  G g;
  const size_t row = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (row >= count) return;
  const uint32_t f = rowflags[row];
  if (!(f & (kDecNeg | kDecReduce)) || (f & (kDecFormat | kDecWide))) return;
  uint32_t n[L], a[L];
  g.load_vec(n, consts + kConstN * S);
  g.load_col(a, X, stride, row);
  if (f & kDecReduce) {
    M::mul_col(a, n, consts + kConstR2 * S, 1, 0, n0, g.top, g.bottom);
    M::mul_col(a, n, consts + kConstOne * S, 1, 0, n0, g.top, g.bottom);
  }
  g.canon(a, n);  // [0, N)
  if (f & kDecNeg) {
    uint32_t t[L];
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = n[l];
    g.sub(t, a);                    // N - a in (0, N]
    if (g.cmp(t, n) == 0) {         // a == 0
#pragma unroll
      for (int l = 0; l < L; ++l) t[l] = 0;
    }
#pragma unroll
    for (int l = 0; l < L; ++l) a[l] = t[l];
  }
  g.store_col(a, X, stride, row);
}

hipError_t launch_dec_parse(int S, const uint32_t* chars4, const uint64_t* offs, uint64_t obase, size_t count,
                            const uint32_t* tab, int jfit, int jpad, const uint32_t* consts, uint32_t* X,
                            size_t stride, uint8_t* rowflags, uint32_t* flags, hipStream_t st) {
  if (count == 0) return hipSuccess;
  const int ldsw = ((jfit > S ? jfit : S) + 3) & ~3;
  // A batch too small to fill the chip (config 1: 10k rows at 2 lanes each is 0.3 waves per SIMD) is
  // latency-bound: per-lane work is ~K^2 / (2 TPI) MACs, so such batches take a wider lane group
  // where the shape divides (S = 40, 76, 112); the output layout (limb r * L + l) is the same.
  constexpr size_t kDecLatencyLanes = 131072;
  DDSHE_SWITCH(S, {
    constexpr int TL = (S % (4 * TPI) == 0 && 4 * TPI <= 16) ? 4 * TPI : (S % (2 * TPI) == 0 && 2 * TPI <= 16) ? 2 * TPI : TPI;
    if (TL != TPI && count * TPI < kDecLatencyLanes) {
      const size_t lds = (size_t)(256 / TL) * ldsw * 4;
      hipLaunchKernelGGL((k_dec_parse<S, TL, W>), dim3(grid_for(count * TL)), dim3(256), lds, st, chars4, offs,
                         obase, count, tab, jfit, jpad, ldsw, TL / TPI, consts, X, stride, rowflags, flags);
    } else {
      const size_t lds = (size_t)(256 / TPI) * ldsw * 4;
      hipLaunchKernelGGL((k_dec_parse<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256), lds, st, chars4, offs,
                         obase, count, tab, jfit, jpad, ldsw, 1, consts, X, stride, rowflags, flags);
    }
  });
  return hipGetLastError();
}

hipError_t launch_dec_fix(int S, uint32_t* X, size_t stride, size_t count, const uint8_t* rowflags,
                          const uint32_t* consts, uint32_t n0, hipStream_t st) {
  if (count == 0) return hipSuccess;
  DDSHE_SWITCH(S, hipLaunchKernelGGL((k_dec_fix<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256), 0, st, X, stride,
                                     count, rowflags, consts, n0));
  return hipGetLastError();
}

}  // namespace ddshe
