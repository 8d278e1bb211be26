// HIP kernels of the homomorphic aggregation engine (gfx950 only).
//
// Column layout in HBM ("rW column"): limb-transposed radix-2^W words (W = 28 or 27),
//   X[l * stride + row], l in [0, S), stride >= rows (multiple of 64),
// so that the lanes of a wave touch consecutive rows of one limb (coalesced).
//
// Reference operations accelerated (all in /root/reference/src/main/scala/):
//   SumAll fold   dds/http/DDSRestServer.scala:397-446  -> k_fold + k_finalize
//   MultAll fold  dds/http/DDSRestServer.scala:491-539  -> k_fold + k_finalize
//   Sum / Mult    dds/http/DDSRestServer.scala:355-395, 447-490 -> k_pairs
//   Search{Gt,GtEq,Lt,LtEq} DDSRestServer.scala:682-830 -> k_ope_count + k_ope_scatter
//   HomoAdd.encrypt  utils/SJHomoLibProvider.scala:58 -> k_modexp_pre + k_modexp_ladder (also HomoMult.encrypt, :59)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "ddshe_device.hpp"
#include "ddshe_fold.hpp"
#include "ddshe_launch.hpp"
#include "ddshe_shapes.hpp"

namespace ddshe {

// ------------------------------------------------------------------------------
// ingest: big-endian fixed-width rows -> rW column (+ range classification)
// ------------------------------------------------------------------------------
// flags[0] |= 1 if some row is >= 2N (needs k_reduce_rows), flags[0] |= 2 if some row does not fit
// in S rW limbs (boundary error DDS_E_RANGE). rowflags (nullable): per row, 1 if it is >= 2N (it is
// stored as its residue, so the column remembers which rows differ from what the caller passed).
// One thread per row, least-significant end first; rows of a multiple of 4 bytes at 4-byte
// alignment are read as big-endian dwords (a 4096-bit row: 128 loads instead of 512).
__global__ void k_ingest_be(const uint8_t* __restrict__ in, size_t width, size_t count, int S, int W,
                            const uint32_t* __restrict__ n2x /* 2N in rW, S+1 limbs */, uint32_t* __restrict__ X,
                            size_t stride, uint32_t* __restrict__ flags, uint8_t* __restrict__ rowflags) {
  const size_t row = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= count) return;
  const uint8_t* p = in + row * width;
  uint64_t bitbuf = 0;
  int nbits = 0, l = 0, cmpv = 0;
  bool overflow = false;
  const uint32_t kMask = (1u << W) - 1u;
  auto emit = [&]() {
    while (nbits >= W) {
      const uint32_t limb = (uint32_t)bitbuf & kMask;
      bitbuf >>= W;
      nbits -= W;
      if (l < S) {
        X[(size_t)l * stride + row] = limb;
        const uint32_t nl = n2x[l];
        cmpv = limb > nl ? 1 : (limb < nl ? -1 : cmpv);
      } else if (limb) {
        overflow = true;
      }
      ++l;
    }
  };
  const bool words = (width % 4 == 0) && (((uintptr_t)in) % 4 == 0);
  if (words) {
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(p);
    for (size_t i = width / 4; i-- > 0;) {
      bitbuf |= (uint64_t)__builtin_bswap32(pw[i]) << nbits;  // nbits < W <= 28: fits 64 bits
      nbits += 32;
      emit();
    }
  } else {
    for (size_t i = 0; i < width; ++i) {
      bitbuf |= (uint64_t)p[width - 1 - i] << nbits;
      nbits += 8;
      emit();
    }
  }
  while (l < S || bitbuf != 0) {  // flush: zero-pad to S limbs, any leftover bit beyond S overflows
    const uint32_t limb = (uint32_t)bitbuf & kMask;
    bitbuf >>= W;
    if (l < S) {
      X[(size_t)l * stride + row] = limb;
      const uint32_t nl = n2x[l];
      cmpv = limb > nl ? 1 : (limb < nl ? -1 : cmpv);
    } else if (limb) {
      overflow = true;
    }
    ++l;
  }
  // 2N may need limb S (if 2N >= 2^(W*S)); row limbs beyond S are zero here
  if (n2x[S] != 0) cmpv = -1;
  if (overflow) atomicOr(flags, 2u);
  else if (cmpv >= 0) atomicOr(flags, 1u);
  if (rowflags) rowflags[row] = (!overflow && cmpv >= 0) ? 1 : 0;
}

// Same conversion with the rows staged through LDS: the 64 rows of a block are loaded by its 256
// lanes as consecutive 16-byte pieces (a wave reads 1 KiB of contiguous row bytes per load, instead of
// 64 lanes each walking its own row 512 bytes from its neighbours'). Limb l of a row is bits
// [W·l, W·l + W) of the value, i.e. a funnel shift of two words of the big-endian row, so every limb is
// extracted independently: lane (q, j) of the block (j = lane % 64 = row) extracts limbs q, q+4, ... of
// row j, and the 64 lanes of a wave store one limb of 64 consecutive rows (coalesced). The compare with
// 2N (highest differing limb) and the overflow test (bits at or above W·S) are combined per row in LDS.
// Row pitch width + 4 bytes: lanes reading word k of consecutive rows hit consecutive banks. Used when
// width % 16 == 0, the input is 16-byte aligned and width <= kIngestMaxW.
constexpr int kIngestRows = 64, kIngestThreads = 256;
constexpr size_t kIngestMaxW = 1024;
__global__ void __launch_bounds__(kIngestThreads) k_ingest_be_lds(const uint8_t* __restrict__ in, size_t width,
                                                                  size_t count, int S, int W,
                                                                  const uint32_t* __restrict__ n2x,
                                                                  uint32_t* __restrict__ X, size_t stride,
                                                                  uint32_t* __restrict__ flags,
                                                                  uint8_t* __restrict__ rowflags) {
  extern __shared__ uint32_t srow[];  // kIngestRows rows of width/4 + 1 words
  __shared__ int sdiff[kIngestThreads / kIngestRows][kIngestRows];  // per lane: (highest differing limb + 1) * sign
  __shared__ uint32_t sover[kIngestRows];
  const int tid = threadIdx.x, j = tid % kIngestRows, q = tid / kIngestRows;
  constexpr int Q = kIngestThreads / kIngestRows;
  const size_t r0 = (size_t)blockIdx.x * kIngestRows;
  const size_t nrows = min((size_t)kIngestRows, count - r0);
  const uint32_t wq = (uint32_t)(width / 16), nw = (uint32_t)(width / 4), pitch = nw + 1;
  const u32x4* src = reinterpret_cast<const u32x4*>(in + r0 * width);
  const uint32_t npieces = (uint32_t)nrows * wq;
  for (uint32_t i = tid; i < npieces; i += kIngestThreads) {
    const u32x4 v = __builtin_nontemporal_load(src + i);
    const uint32_t rr = i / wq, k = (i % wq) * 4;
    uint32_t* d = srow + rr * pitch + k;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
  if (tid < kIngestRows) sover[tid] = 0;
  __syncthreads();
  const bool live = (size_t)j < nrows;
  const size_t row = r0 + j;
  const uint32_t* pw = srow + j * pitch;  // pw[nw - 1 - k]: word k counted from the least significant end
  auto word = [&](uint32_t k) -> uint32_t { return k < nw ? __builtin_bswap32(pw[nw - 1 - k]) : 0u; };
  const uint32_t kMask = (1u << W) - 1u;
  int diff = 0;  // (l + 1) * sign(limb - 2N limb) at the highest l of this lane that differs
  if (live) {
    for (int l = q; l < S; l += Q) {
      const uint32_t bit = (uint32_t)l * (uint32_t)W, k = bit >> 5, sh = bit & 31u;
      const uint64_t two = ((uint64_t)word(k + 1) << 32) | word(k);
      const uint32_t limb = (uint32_t)(two >> sh) & kMask;
      X[(size_t)l * stride + row] = limb;
      const uint32_t nl = n2x[l];
      if (limb != nl) diff = (l + 1) * (limb > nl ? 1 : -1);
    }
    // bits at or above W·S must be zero (lane q = 0 checks them)
    if (q == 0) {
      const uint32_t top = (uint32_t)S * (uint32_t)W, k0 = top >> 5;
      uint32_t over = k0 < nw ? (word(k0) >> (top & 31u)) : 0u;
      for (uint32_t k = k0 + 1; k < nw; ++k) over |= word(k);
      sover[j] = over;
    }
  }
  sdiff[q][j] = diff;
  __syncthreads();
  if (q != 0 || !live) return;
  int best = 0;
#pragma unroll
  for (int t = 0; t < Q; ++t) {
    const int d = sdiff[t][j];
    if ((d < 0 ? -d : d) > (best < 0 ? -best : best)) best = d;
  }
  int cmpv = best > 0 ? 1 : (best < 0 ? -1 : 0);
  const bool overflow = sover[j] != 0;
  if (n2x[S] != 0) cmpv = -1;  // 2N may need limb S (if 2N >= 2^(W*S)); row limbs beyond S are zero here
  if (overflow) atomicOr(flags, 2u);
  else if (cmpv >= 0) atomicOr(flags, 1u);
  if (rowflags) rowflags[row] = (!overflow && cmpv >= 0) ? 1 : 0;
}

// egress: rW column rows -> fixed-width big-endian bytes (the binary boundary's output: what a JNA shim
// turns into BigIntegers). kEgressRows rows per block: their limbs are read limb-major (coalesced over
// rows) into LDS, rows >= N (columns keep rows < 2N) get N subtracted by one lane per row, and every
// output byte is a funnel shift of at most two limbs, written row-major by consecutive lanes.
constexpr int kEgressRows = 32, kEgressMaxS = kEgressMaxLimbs;
__global__ void __launch_bounds__(256) k_egress_be(const uint32_t* __restrict__ X, size_t stride, size_t count, int S,
                                                   int W, const uint32_t* __restrict__ nmod, size_t width,
                                                   uint8_t* __restrict__ out) {
  __shared__ uint32_t sl[kEgressRows * (kEgressMaxS + 1)];
  const int tid = threadIdx.x, P = S + 1;
  const size_t r0 = (size_t)blockIdx.x * kEgressRows;
  const int nrows = (int)min((size_t)kEgressRows, count - r0);
  for (int idx = tid; idx < nrows * S; idx += 256) {
    const int l = idx / nrows, r = idx - l * nrows;
    sl[r * P + l] = X[(size_t)l * stride + r0 + r];
  }
  __syncthreads();
  if (nmod && tid < nrows) {  // value < 2N: subtract N once if value >= N
    uint32_t* a = sl + tid * P;
    int c = 0;
    for (int l = S - 1; l >= 0 && c == 0; --l) c = a[l] > nmod[l] ? 1 : (a[l] < nmod[l] ? -1 : 0);
    if (c >= 0) {
      const uint32_t mask = (1u << W) - 1u;
      uint32_t br = 0;
      for (int l = 0; l < S; ++l) {
        const uint32_t d = a[l] - nmod[l] - br;
        br = d >> 31;
        a[l] = d & mask;
      }
    }
  }
  __syncthreads();
  const size_t nb = (size_t)nrows * width;
  uint8_t* o = out + r0 * width;
  for (size_t idx = tid; idx < nb; idx += 256) {
    const size_t r = idx / width, b = idx - r * width;
    const uint32_t bit = (uint32_t)(8 * (width - 1 - b));
    const uint32_t l = bit / (uint32_t)W, sh = bit - l * (uint32_t)W;
    const uint32_t* a = sl + r * P;
    uint32_t v = l < (uint32_t)S ? a[l] >> sh : 0u;
    if (sh + 8 > (uint32_t)W && l + 1 < (uint32_t)S) v |= a[l + 1] << (W - sh);
    o[idx] = (uint8_t)v;
  }
}

// rows >= 2N: x <- MonPro(MonPro(x, R^2 mod N), 1) = x mod N
// gate (nullable): skip unless gate[0] & 1 (an ingest's flags word, read on the device: no host round trip)
template <int S, int TPI, int W>
__global__ void __launch_bounds__(256, 2) k_reduce_rows(uint32_t* __restrict__ X, size_t stride, size_t count,
                                                     const uint32_t* __restrict__ consts, uint32_t n0,
                                                     const uint32_t* __restrict__ gate) {
  if (gate && !(gate[0] & 1u)) return;
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W>;
  constexpr int L = G::L;
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= count) return;
  const uint32_t* N = consts + kConstN * S;
  const uint32_t* N2 = consts + kConstN2x * S;
  const uint32_t* R2 = consts + kConstR2 * S;
  const uint32_t* ONE = consts + kConstOne * S;
  uint32_t n[L], a[L], n2[L];
  g.load_vec(n, N);
  g.load_vec(n2, N2);
  g.load_col(a, X, stride, grp);
  // 2N fits in S limbs (S chosen with 2 bits of headroom)
  if (g.cmp(a, n2) < 0) return;
  M::mul_col(a, n, R2, 1, 0, n0, g.top, g.bottom);
  M::mul_col(a, n, ONE, 1, 0, n0, g.top, g.bottom);
  M::normalize(a, g.bottom);
  g.store_col(a, X, stride, grp);
}

// out[i] = A[i]*B[i] mod N (canonical), rW columns in and out
template <int S, int TPI, int W>
__global__ void __launch_bounds__(256, 2) k_pairs(const uint32_t* __restrict__ A, const uint32_t* __restrict__ B,
                                               size_t stride, size_t count, const uint32_t* __restrict__ consts,
                                               uint32_t n0, uint32_t* __restrict__ O) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W>;
  constexpr int L = G::L;
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= count) return;
  uint32_t n[L], a[L];
  g.load_vec(n, consts + kConstN * S);
  g.load_col(a, A, stride, grp);
  M::mul_col(a, n, B, stride, (uint32_t)grp, n0, g.top, g.bottom);       // a*b*R^-1
  M::mul_col(a, n, consts + kConstR2 * S, 1, 0, n0, g.top, g.bottom);   // a*b
  g.canon(a, n);
  g.store_col(a, O, stride, grp);
}

// ------------------------------------------------------------------------------
// batched modular exponentiation: c_i = g^m_i * x_i^E mod N
//   Paillier encrypt (HomoAdd.encrypt, SJHomoLibProvider.scala:58): N = n^2, E = n
//   RSA encrypt / generic x^E (HomoMult.encrypt, :59): g^m term disabled (m == nullptr)
// E is uniform over the batch, so the host turns it into a sliding-window schedule
// (window w <= 5) that every group walks in lockstep — no divergence:
//   k_modexp_pre:    Tab[j] = x^(2j+1)·R mod N, j < nodd (per row, limb-transposed in HBM)
//   k_modexp_ladder: acc = Tab[sched[0]]; per entry: `nsq` squarings (operand staged in the
//                    group's LDS slot, read by ds_read broadcast), then acc·Tab[idx] streamed
//                    from HBM through the fold's buffer-descriptor path; then g^m_i (binary,
//                    per-row exponent < 2^14), leave Montgomery form, canonicalise.
// A 3072-bit E costs 3072 squarings + ~512 multiplies + 16 table products instead of
// 3072 + ~1536 for the binary ladder (-22 % Montgomery products).
// ------------------------------------------------------------------------------
template <int S, int TPI, int W>
__device__ __forceinline__ void store_lds(uint32_t* dst, const uint32_t (&a)[S / TPI], int r) {
#pragma unroll
  for (int l = 0; l < S / TPI; ++l) dst[r * (S / TPI) + l] = a[l];
}

// QP: products against N~ = N·n0 (qp_mod, see Mont QP); table entries are then < 2N~.
template <int S, int TPI, int W, bool QP = false>
__global__ void __launch_bounds__(256, 2) k_modexp_pre(const uint32_t* __restrict__ Xcol, size_t xstride,
                                                    size_t count, const uint32_t* __restrict__ consts,
                                                    const uint32_t* __restrict__ qp_mod, uint32_t n0,
                                                    int nodd, uint32_t* __restrict__ Tab, size_t tstride) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W, QP>;
  constexpr int L = G::L;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= count) return;
  uint32_t* x1 = lds + (size_t)(threadIdx.x / TPI) * 2 * S;  // group-private operand slots
  uint32_t* x2 = x1 + S;
  uint32_t n[L], acc[L];
  g.load_vec(n, QP ? qp_mod : consts + kConstN * S);
  g.load_col(acc, Xcol, xstride, grp);
  M::mul_col(acc, n, consts + kConstR2 * S, 1, 0, n0, g.top, g.bottom);  // x*R
  M::normalize(acc, g.bottom);
  g.store_col(acc, Tab, tstride, grp);
  if (nodd == 1) return;
  store_lds<S, TPI, W>(x1, acc, g.r);
  M::mul_lds(acc, n, x1, n0, g.top, g.bottom);  // x^2*R
  M::normalize(acc, g.bottom);
  store_lds<S, TPI, W>(x2, acc, g.r);
#pragma unroll
  for (int l = 0; l < L; ++l) acc[l] = x1[g.r * L + l];
  for (int j = 1; j < nodd; ++j) {
    M::mul_lds(acc, n, x2, n0, g.top, g.bottom);
    M::normalize(acc, g.bottom);
    g.store_col(acc, Tab + (size_t)j * S * tstride, tstride, grp);
  }
}

// sched[0] = index of the leading window; sched[1..nsched) = (nsq << 16) | (idx + 1),
// idx + 1 == 0: squarings only. nsched == 0: E == 0 (x^0 = 1).
// QP: every product but the last against N~ = N·n0 (values < 2N~); the last one, against N,
// leaves the Montgomery form below 2N (R > 2N~) for the canonical reduction.
// Occupancy: one S-word LDS slot per group (x^E·R is parked in the group's output row in HBM while
// g^m is computed, not in a second slot) and at most 168 VGPRs, so three waves per SIMD hide the
// squarings' serial parts (the LDS round trip of the operand, the settle/normalise carry chains);
// DDSHE_LADDER_OCC2=1 builds the previous two-wave form (two slots, 172 VGPRs) for A/B.
// Shapes of more than 29 limbs per lane keep two waves (a 168-VGPR bound spills them heavily).
template <int S, int TPI>
constexpr int ladder_waves() {
#ifdef DDSHE_LADDER_OCC2
  return 2;
#else
  return S / TPI <= 29 ? 3 : 2;
#endif
}
template <int S, int TPI, int W, bool QP = false>
__global__ void __launch_bounds__(256, (ladder_waves<S, TPI>())) k_modexp_ladder(const uint32_t* __restrict__ Tab, size_t tstride,
                                                       const uint32_t* __restrict__ m, size_t count,
                                                       const uint32_t* __restrict__ consts,
                                                       const uint32_t* __restrict__ qp_mod,
                                                       const uint32_t* __restrict__ gR,
                                                       const uint32_t* __restrict__ sched, int nsched, uint32_t n0,
                                                       uint32_t* __restrict__ O, size_t ostride) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W, QP>;
  constexpr int L = G::L;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= count) return;
#ifdef DDSHE_LADDER_OCC2
  uint32_t* sq = lds + (size_t)(threadIdx.x / TPI) * 2 * S;  // group-private operand slots
  uint32_t* xs = sq + S;
#else
  uint32_t* sq = lds + (size_t)(threadIdx.x / TPI) * S;  // group-private operand slot
#endif
  uint32_t n[L], acc[L];
  g.load_vec(n, QP ? qp_mod : consts + kConstN * S);
  if (nsched > 0) g.load_col(acc, Tab + (size_t)sched[0] * S * tstride, tstride, grp);
  else g.load_vec(acc, consts + kConstRmod * S);  // 1*R
  for (int k = 1; k < nsched; ++k) {
    const uint32_t e = sched[k];
    for (uint32_t s = e >> 16; s > 0; --s) {
      M::normalize(acc, g.bottom);
      store_lds<S, TPI, W>(sq, acc, g.r);
      M::mul_lds(acc, n, sq, n0, g.top, g.bottom);
    }
    if (e & 0xFFFFu)
      M::mul_col(acc, n, Tab + (size_t)((e & 0xFFFFu) - 1) * S * tstride, tstride, (uint32_t)grp, n0, g.top,
                 g.bottom);
  }
  if (m != nullptr) {
    // g^m_i: per-row exponent; the ladder length is the wave's max bit length so the
    // branch stays uniform, the multiplier is g*R or 1*R selected per group
    const uint32_t mi = m[grp];
    uint32_t wb = mi ? 32u - (uint32_t)__builtin_clz(mi) : 0u;
    for (int off = 32; off >= 1; off >>= 1) wb = max(wb, (uint32_t)__shfl_xor((int)wb, off));
    M::normalize(acc, g.bottom);
#ifdef DDSHE_LADDER_OCC2
    store_lds<S, TPI, W>(xs, acc, g.r);  // park x^E*R in xs; acc is reused for g^m
#else
    // park x^E*R in this group's output row (read back by mul_col below: other lanes' limbs, so the
    // stores must have landed — workgroup fence: vmcnt(0), the write-through L1 serves the reloads)
    g.store_col(acc, O, ostride, grp);
    __threadfence_block();
#endif
    g.load_vec(acc, consts + kConstRmod * S);
    for (int i = (int)wb - 1; i >= 0; --i) {
      M::normalize(acc, g.bottom);
      store_lds<S, TPI, W>(sq, acc, g.r);
      M::mul_lds(acc, n, sq, n0, g.top, g.bottom);
      const uint32_t* sel = ((mi >> i) & 1u) ? gR : consts + kConstRmod * S;
#pragma unroll
      for (int l = 0; l < L; ++l) sq[g.r * L + l] = sel[g.r * L + l];
      M::mul_lds(acc, n, sq, n0, g.top, g.bottom);
    }
    // acc = (g^m R) * (x^E R) * R^-1
#ifdef DDSHE_LADDER_OCC2
    M::mul_lds(acc, n, xs, n0, g.top, g.bottom);
#else
    M::mul_col(acc, n, O, ostride, (uint32_t)grp, n0, g.top, g.bottom);
#endif
  }
  if constexpr (QP) g.load_vec(n, consts + kConstN * S);
  Mont<S, TPI, W>::mul_col(acc, n, consts + kConstOne * S, 1, 0, n0, g.top, g.bottom);  // leave Montgomery form
  g.canon(acc, n);
  g.store_col(acc, O, ostride, grp);
}

// ------------------------------------------------------------------------------
// synthetic Paillier rows (bench / tests): c_i = T[m_i] * P[a_i] * P[b_i] mod N
// T: table of g^m (plain), P: pool of r^n in Montgomery form (r^n * R mod N).
// Indices come from splitmix64(seed, row), so the host can recompute sum(m_i).
// ------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <int S, int TPI, int W>
__global__ void __launch_bounds__(256, 2) k_synth_rows(const uint32_t* __restrict__ T, size_t tstride, uint32_t tcount,
                                                    const uint32_t* __restrict__ P, size_t pstride, uint32_t pcount,
                                                    uint64_t seed, uint64_t row0, size_t count,
                                                    const uint32_t* __restrict__ consts, uint32_t n0,
                                                    uint32_t* __restrict__ X, size_t xstride, uint32_t shards,
                                                    uint32_t shard) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W>;
  constexpr int L = G::L;
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= count) return;
  // local row l of shard `shard` of a column sharded in 64-row blocks round-robin over `shards`
  // holds global row ((l/64)*shards + shard)*64 + l%64 (shards == 1: l itself)
  const uint64_t l = row0 + grp;
  const uint64_t grow = (((l >> 6) * shards + shard) << 6) | (l & 63u);
  const uint64_t h = splitmix64(seed ^ splitmix64(grow));
  const uint32_t mi = (uint32_t)(h % tcount);
  const uint32_t ai = (uint32_t)((h >> 20) % pcount);
  const uint32_t bi = (uint32_t)((h >> 42) % pcount);
  uint32_t n[L], a[L];
  g.load_vec(n, consts + kConstN * S);
  g.load_col(a, T, tstride, mi);
  M::mul_col(a, n, P, pstride, ai, n0, g.top, g.bottom);
  M::normalize(a, g.bottom);
  M::mul_col(a, n, P, pstride, bi, n0, g.top, g.bottom);
  g.canon(a, n);
  g.store_col(a, X, xstride, grp);
}

// ------------------------------------------------------------------------------
// CRT Paillier encryption (HomoAdd.encrypt with the private factors, SJHomoLibProvider.scala:58;
// the client holds the whole PaillierKey, :43-50): c = g^m r^n mod n^2 is computed as
// y_p = g^m r^n mod p^2 and y_q mod q^2 (half-width moduli: 1/4 of the Montgomery work
// each), then Garner: h = (y_p - y_q)·(q^2)^-1 mod p^2, c = y_q + q^2·h  (< n^2, exact).
// ------------------------------------------------------------------------------
// radix change between rW layouts, one row per thread: dst (Sd limbs of Wd bits) <- src
// (Ss limbs of Ws bits). flags[0] |= 1 if the value does not fit in Sd limbs.
__global__ void k_repack(const uint32_t* __restrict__ src, size_t sstride, int Ss, int Ws, uint32_t* __restrict__ dst,
                         size_t dstride, int Sd, int Wd, size_t count, uint32_t* __restrict__ flags) {
  const size_t row = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= count) return;
  const uint32_t dmask = (1u << Wd) - 1u;
  uint64_t buf = 0;
  int nb = 0, l = 0;
  bool over = false;
  for (int i = 0; i < Ss; ++i) {
    buf |= (uint64_t)src[(size_t)i * sstride + row] << nb;
    nb += Ws;
    while (nb >= Wd) {
      const uint32_t v = (uint32_t)buf & dmask;
      if (l < Sd) dst[(size_t)l * dstride + row] = v;
      else over |= v != 0;
      ++l;
      buf >>= Wd;
      nb -= Wd;
    }
  }
  for (; l < Sd; ++l) {
    dst[(size_t)l * dstride + row] = (uint32_t)buf & dmask;
    buf >>= Wd;
  }
  if (over || buf != 0) atomicOr(flags, 1u);
}

// h = MonPro(y_p, c1R) + MonPro(y_q, c2R) with c1R = (q^2)^-1·R, c2R = -(q^2)^-1·R (mod p^2)
//   == (y_p - y_q)·(q^2)^-1 (mod p^2); canonical h < p^2. The first term is parked in H
//   (each lane re-reads only its own limbs) so one bignum is live at a time.
template <int S, int TPI, int W>
__global__ void __launch_bounds__(256, 2) k_crt_h(const uint32_t* __restrict__ Yp, const uint32_t* __restrict__ Yq,
                                               size_t stride, size_t count, const uint32_t* __restrict__ consts,
                                               const uint32_t* __restrict__ c12, uint32_t n0, uint32_t* H) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W>;
  constexpr int L = G::L;
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= count) return;
  uint32_t n[L], u[L];
  g.load_vec(n, consts + kConstN * S);
  g.load_col(u, Yp, stride, grp);
  M::mul_col(u, n, c12, 1, 0, n0, g.top, g.bottom);
  g.canon(u, n);
  g.store_col(u, H, stride, grp);
  g.load_col(u, Yq, stride, grp);
  M::mul_col(u, n, c12 + S, 1, 0, n0, g.top, g.bottom);
  g.canon(u, n);
#pragma unroll
  for (int l = 0; l < L; ++l) u[l] += H[(size_t)(g.r * L + l) * stride + grp];  // < 2 p^2, limbs < 2^(W+1)
  g.canon(u, n);
  g.store_col(u, H, stride, grp);
}

// c = canon(MonPro(h, q^2·R mod n^2)) + y_q   (h·q^2 + y_q < n^2: no reduction)
template <int S, int TPI, int W>
__global__ void __launch_bounds__(256, 2) k_crt_out(const uint32_t* __restrict__ Hn, const uint32_t* __restrict__ Yqn,
                                                 size_t stride, size_t count, const uint32_t* __restrict__ consts,
                                                 const uint32_t* __restrict__ q2R, uint32_t n0,
                                                 uint32_t* __restrict__ O, size_t ostride) {
  using G = Grp<S, TPI, W>;
  using M = Mont<S, TPI, W>;
  constexpr int L = G::L;
  G g;
  const size_t grp = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / TPI;
  if (grp >= count) return;
  uint32_t n[L], a[L];
  g.load_vec(n, consts + kConstN * S);
  g.load_col(a, Hn, stride, grp);
  M::mul_col(a, n, q2R, 1, 0, n0, g.top, g.bottom);
  g.canon(a, n);
  asm volatile("" ::: "memory");  // keep the y_q loads after the product (no extra live bignum)
#pragma unroll
  for (int l = 0; l < L; ++l) a[l] += Yqn[(size_t)(g.r * L + l) * stride + grp];
  M::normalize(a, g.bottom);
  g.store_col(a, O, ostride, grp);
}

// seeded r column (bench / tests): limb l of row i = splitmix64(splitmix64(seed ^ (row0+i)) + l),
// truncated to `bits` bits (r < 2^bits), lowest bit forced to 1 (r != 0)
__global__ void k_fill_random(uint32_t* __restrict__ X, size_t stride, int S, int W, uint64_t seed, uint64_t row0,
                              size_t count, int bits) {
  const size_t row = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= count) return;
  const uint64_t h = splitmix64(seed ^ (row0 + row));
  const uint32_t mask = (1u << W) - 1u;
  for (int l = 0; l < S; ++l) {
    const int lo = l * W;
    uint32_t v = 0;
    if (lo < bits) {
      v = (uint32_t)splitmix64(h + (uint64_t)l) & mask;
      if (bits - lo < W) v &= (1u << (bits - lo)) - 1u;
      if (l == 0) v |= 1u;
    }
    X[(size_t)l * stride + row] = v;
  }
}

// table-driven synthetic rows: X[row] = T[h % tcount], h = splitmix64(seed ^ splitmix64(row0+row))
// (RSA config 3: T[j] = (j+1)^e mod n, DDSDataGenerator.scala:274 plaintexts)
__global__ void k_gather_rows(const uint32_t* __restrict__ T, size_t tstride, uint32_t tcount, int S, uint64_t seed,
                              uint64_t row0, size_t count, uint32_t* __restrict__ X, size_t xstride) {
  const size_t row = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= count) return;
  const uint32_t j = (uint32_t)(splitmix64(seed ^ splitmix64(row0 + row)) % tcount);
  for (int l = 0; l < S; ++l) X[(size_t)l * xstride + row] = T[(size_t)l * tstride + j];
}

// ------------------------------------------------------------------------------
// OPE range filter: keep row i iff valid[i] && col[i] <op> bound (signed int64)
// DDSRestServer.scala:704 (Gt), :742 (GtEq), :779 (Lt), :816 (LtEq)
// ------------------------------------------------------------------------------
// One compare for all four operators: the host turns (op, bound) into (t, code) with
// c <op> bound == ((c > t) != (code & 1)), or a constant (code 2: every row, 4: none)
// (launch_ope_filter) — no per-row branch on the operator.
__device__ __forceinline__ bool ope_pred(int64_t c, int64_t t, int code) {
  const bool r = (c > t) != (bool)(code & 1);
  return (code & 2) ? true : (code & 4) ? false : r;
}

constexpr int kOpeBlock = 256;
constexpr int kOpeItems = 32;  // rows per thread (bits of the per-thread match mask)
constexpr size_t kOpeTile = (size_t)kOpeBlock * kOpeItems;

// Row layout of a tile: group k (< kOpeGroups) covers rows [k*1024, (k+1)*1024); thread tid owns
// the 4 consecutive rows k*1024 + 4*tid + j (j < 4), bit 4k+j of its match mask. Full tiles of an
// aligned column read 4 rows as two 16-byte loads (+ one 4-byte load of their valid bytes); the
// last tile (or an unaligned column) uses scalar loads with the index clamped to n-1. All loads are
// issued before any predicate so they are in flight together.
constexpr int kOpeGroups = kOpeItems / 4;

// A row qualifies iff its valid byte v has (v & vmask) != 0 and (v & vbad) == 0 (raw arrays:
// vmask 0xFF, vbad 0 — valid != 0; a resident OPE column: its searchable bit, minus wide rows).
template <bool HasValid>
__device__ __forceinline__ uint32_t ope_thread_mask(const int64_t* __restrict__ col, const uint8_t* __restrict__ valid,
                                                    size_t n, int64_t bound, int op, size_t tile, bool vec,
                                                    uint32_t vmask, uint32_t vbad) {
  const size_t t0 = tile * kOpeTile + 4 * (size_t)threadIdx.x;
  int64_t c[kOpeItems];
  uint32_t v[kOpeGroups];
  if (vec && t0 + (kOpeGroups - 1) * 4 * kOpeBlock + 3 < n) {
#pragma unroll
    for (int k = 0; k < kOpeGroups; ++k) {
      const size_t r = t0 + (size_t)k * 4 * kOpeBlock;
      typedef long long i64x2 __attribute__((ext_vector_type(2)));
      const i64x2* p = reinterpret_cast<const i64x2*>(col + r);
      const i64x2 x = __builtin_nontemporal_load(p), y = __builtin_nontemporal_load(p + 1);
      c[4 * k] = x.x;
      c[4 * k + 1] = x.y;
      c[4 * k + 2] = y.x;
      c[4 * k + 3] = y.y;
      if constexpr (HasValid) v[k] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(valid + r));
      else v[k] = 0x01010101u;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kOpeGroups; ++k) {
      uint32_t vk = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t r = t0 + (size_t)k * 4 * kOpeBlock + j;
        const size_t i = min(r, n - 1);
        c[4 * k + j] = col[i];
        const uint32_t vb = HasValid ? (uint32_t)valid[i] : 1u;
        vk |= (r < n ? vb : 0u) << (8 * j);
      }
      v[k] = vk;
    }
  }
  uint32_t mask = 0;
#pragma unroll
  for (int k = 0; k < kOpeGroups; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((((v[k] >> (8 * j)) & vmask) != 0u) && (((v[k] >> (8 * j)) & vbad) == 0u) && ope_pred(c[4 * k + j], bound, op))
        mask |= 1u << (4 * k + j);
  return mask;
}

// Loads give thread tid the rows k*1024 + 4*tid + j (bit 4k + j of its mask: coalesced 16-byte loads).
// Stored mask words are transposed through LDS to row order: word w of a tile covers rows
// [32w, 32w + 32) (group k = w / 32, the nibbles of threads 8(w % 32) .. +7), so the scatter ranks a
// tile with one block-wide scan of 256 popcounts instead of 32 ballots per thread. Also writes the
// tile's match count.
// hlimit != 0: masks is a host buffer mapped into the device (a registered Search reply buffer) of hlimit
// words and counts a mapped host array: the words and the tile's count go out as system-scope stores
// (written through to host memory, the reply needs no copy; the host adds the counts up) and words
// past the buffer's end (the last tile's) are dropped
__device__ __forceinline__ void ope_store_mask(uint32_t m, uint32_t* __restrict__ masks, uint32_t* __restrict__ counts,
                                               size_t tile, unsigned long long* __restrict__ total = nullptr,
                                               size_t hlimit = 0, int hwide = 0) {
  __shared__ uint8_t nib[kOpeGroups * kOpeBlock];
  __shared__ uint32_t wsum[kOpeBlock / 64];
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kOpeGroups; ++k) nib[k * kOpeBlock + tid] = (uint8_t)((m >> (4 * k)) & 0xFu);
  uint32_t s = __builtin_popcount(m);
  for (int off = 32; off >= 1; off >>= 1) s += (uint32_t)__shfl_xor((int)s, off);
  if ((tid & 63) == 0) wsum[tid >> 6] = s;
  __syncthreads();
  const uint64_t eight = *reinterpret_cast<const uint64_t*>(&nib[(tid >> 5) * kOpeBlock + (tid & 31) * 8]);
  uint32_t word = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) word |= (uint32_t)((eight >> (8 * i)) & 0xFu) << (4 * i);
  const size_t wi = tile * kOpeBlock + tid;
  if (hlimit == 0) {
    masks[wi] = word;
  } else if (hwide) {
    // over PCIe: the tile's 1 KiB as wider stores (A/B: hwide 1 = 8-byte system-scope stores by the first
    // two waves, 2 = 16-byte non-temporal stores by the first wave); the buffer is 16-byte aligned (the
    // launcher checks), words past its end dropped
    __shared__ __attribute__((aligned(16))) uint32_t wbuf[kOpeBlock];
    wbuf[tid] = word;
    __syncthreads();
    if (hwide == 1) {
      if (tid < kOpeBlock / 2) {
        const size_t w0 = tile * kOpeBlock + 2 * (size_t)tid;
        const uint64_t v = reinterpret_cast<const uint64_t*>(wbuf)[tid];
        if (w0 + 1 < hlimit)
          __hip_atomic_store(reinterpret_cast<uint64_t*>(masks + w0), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else if (w0 < hlimit)
          __hip_atomic_store(masks + w0, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    } else if (tid < kOpeBlock / 4) {
      const size_t w0 = tile * kOpeBlock + 4 * (size_t)tid;
      const uint4 v = reinterpret_cast<const uint4*>(wbuf)[tid];
      if (w0 + 3 < hlimit) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u q = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(q, reinterpret_cast<v4u*>(masks + w0));
      } else {
        const uint32_t e[4] = {v.x, v.y, v.z, v.w};
        for (int j = 0; j < 4; ++j)
          if (w0 + j < hlimit) __hip_atomic_store(masks + w0 + j, e[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  } else if (wi < hlimit) {
    __hip_atomic_store(masks + wi, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid == 0) {
    uint32_t c = 0;
    for (int w = 0; w < kOpeBlock / 64; ++w) c += wsum[w];
    if (hlimit == 0)
      counts[tile] = c;
    else
      __hip_atomic_store(counts + tile, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (total && c) atomicAdd(total, (unsigned long long)c);  // the Search bitmask's match count
  }
}

// Stable compaction in two launches (no inter-block waiting: a decoupled look-back's tile-state
// probes are agent-scope atomics that cross the 8 XCDs' L2s, and measured slower here):
//   k_ope_count:   reads the column once; per-thread match mask (32 rows -> 1 u32, 1/72 of the
//                  column bytes) and per-tile match count;
//   k_ope_scatter: each block sums the counts of the tiles before it (<= a few thousand u32 from
//                  L2), reloads its masks, ranks its matches in row order (k*256 + tid) and
//                  writes the row ids; the last block writes the total.
// total (nullable, zeroed by the caller): every tile also adds its count to it (one atomic per tile),
// so the Search bitmask route has its match count without a reduction launch
template <bool HasValid>
__global__ void __launch_bounds__(kOpeBlock) k_ope_count(const int64_t* __restrict__ col,
                                                         const uint8_t* __restrict__ valid, size_t n, int64_t bound,
                                                         int op, uint32_t vmask, uint32_t vbad,
                                                         uint32_t* __restrict__ masks, uint32_t* __restrict__ counts,
                                                         unsigned long long* __restrict__ total, size_t hlimit,
                                                         int hwide) {
  const bool vec = ((uintptr_t)col % 16 == 0) && (!HasValid || (uintptr_t)valid % 4 == 0);
  const uint32_t m = ope_thread_mask<HasValid>(col, valid, n, bound, op, blockIdx.x, vec, vmask, vbad);
  ope_store_mask(m, masks, counts, blockIdx.x, total, hlimit, hwide);
}

// SearchEq/NEq front end (ddshe_strscan.hip's position index): same tile layout and masks as
// k_ope_count; row r = row0 + i matches iff its present bit is set (length - 1 > position) and its
// fingerprint equals the needle's (bytes verified on a hit), xor negate. Reads 2 B + 1 bit per row and
// writes no per-row flags.
__global__ void __launch_bounds__(kOpeBlock) k_str_eq_count(const StrFp* __restrict__ posfp,
                                                            const uint64_t* __restrict__ present, size_t row0, size_t n,
                                                            const uint64_t* __restrict__ row_beg,
                                                            const uint64_t* __restrict__ elem_off,
                                                            const uint8_t* __restrict__ chars,
                                                            const uint8_t* __restrict__ nchars, StrNeedles nd,
                                                            uint64_t position, int negate,
                                                            uint32_t* __restrict__ masks,
                                                            uint32_t* __restrict__ counts) {
  const size_t t0 = (size_t)blockIdx.x * kOpeTile + 4 * (size_t)threadIdx.x;
  const uint32_t want = str_fp(nd.h[0]);
  uint32_t f[kOpeItems];
  uint32_t pb[kOpeGroups];
  const bool vec = (row0 % 4 == 0) && t0 + (kOpeGroups - 1) * 4 * kOpeBlock + 3 < n;
#pragma unroll
  for (int k = 0; k < kOpeGroups; ++k) {
    const size_t i = t0 + (size_t)k * 4 * kOpeBlock;
    if (vec) {  // 4 fingerprints in one 8-byte load
      const uint64_t x = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(posfp + row0 + i));
      f[4 * k] = (uint32_t)x & 0xFFFFu;
      f[4 * k + 1] = (uint32_t)(x >> 16) & 0xFFFFu;
      f[4 * k + 2] = (uint32_t)(x >> 32) & 0xFFFFu;
      f[4 * k + 3] = (uint32_t)(x >> 48);
      const size_t r = row0 + i;  // 4 rows inside one present word (r % 4 == 0)
      pb[k] = (uint32_t)(present[r >> 6] >> (r & 63)) & 0xFu;
    } else {
      uint32_t b = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t r = row0 + min(i + j, n - 1);
        f[4 * k + j] = posfp[r];
        b |= (i + j < n ? (uint32_t)(present[r >> 6] >> (r & 63)) & 1u : 0u) << j;
      }
      pb[k] = b;
    }
  }
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < kOpeGroups; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!((pb[k] >> j) & 1u)) continue;
      const size_t r = row0 + t0 + (size_t)k * 4 * kOpeBlock + j;
      const bool eq = f[4 * k + j] == want && str_hit(row_beg[r] + position, 0, elem_off, chars, nchars, nd);
      if (eq != (negate != 0)) m |= 1u << (4 * k + j);
    }
  ope_store_mask(m, masks, counts, blockIdx.x);
}

// Byte-mask compaction front end (live rows of a resident column, dds_col_set_live; the string scans'
// needle bits): same tile layout and masks as k_ope_count, predicate (b[r] & vmask) != 0 and
// (b[r] & vall) == vall on a byte per row. `bytes` may start at any
// offset (a row range of the mask): 4-byte loads only when it is aligned.
// rezero: every non-zero word / byte read is stored back as 0 (the string scans' row flags stay zeroed
// between scans: no memset launch before the next one; matches are sparse, so are these stores)
__global__ void __launch_bounds__(kOpeBlock) k_byte_count(const uint8_t* __restrict__ bytes, size_t n, uint32_t vmask,
                                                          uint32_t vall, uint32_t* __restrict__ masks,
                                                          uint32_t* __restrict__ counts, bool rezero) {
  const size_t t0 = (size_t)blockIdx.x * kOpeTile + 4 * (size_t)threadIdx.x;
  uint32_t v[kOpeGroups];
  uint8_t* zb = const_cast<uint8_t*>(bytes);
  if ((uintptr_t)bytes % 4 == 0 && t0 + (kOpeGroups - 1) * 4 * kOpeBlock + 3 < n) {
#pragma unroll
    for (int k = 0; k < kOpeGroups; ++k)
      v[k] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(bytes + t0 + (size_t)k * 4 * kOpeBlock));
    if (rezero) {
#pragma unroll
      for (int k = 0; k < kOpeGroups; ++k)
        if (v[k]) *reinterpret_cast<uint32_t*>(zb + t0 + (size_t)k * 4 * kOpeBlock) = 0u;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kOpeGroups; ++k) {
      uint32_t vk = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t r = t0 + (size_t)k * 4 * kOpeBlock + j;
        const uint32_t b = r < n ? (uint32_t)bytes[r] : 0u;
        if (rezero && b) zb[r] = 0;
        vk |= b << (8 * j);
      }
      v[k] = vk;
    }
  }
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < kOpeGroups; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((((v[k] >> (8 * j)) & vmask) != 0u) && (((v[k] >> (8 * j)) & vall) == vall)) m |= 1u << (4 * k + j);
  ope_store_mask(m, masks, counts, blockIdx.x);
}

// Total of the per-tile match counts (one block): the match count of a bitmask-only Search
// (dds_opecol_search_mask), written next to the mask words so one copy brings both back.
__global__ void __launch_bounds__(1024) k_count_total(const uint32_t* __restrict__ counts, size_t ntiles,
                                                      uint64_t* __restrict__ total) {
  __shared__ uint64_t ws[16];
  uint64_t s = 0;
  for (size_t t = threadIdx.x; t < ntiles; t += 1024) s += counts[t];
  for (int off = 32; off >= 1; off >>= 1) s += (uint64_t)__shfl_xor((long long)s, off);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < 16; ++w) t += ws[w];
    *total = t;
  }
}

// inclusive prefix sum over the 64 lanes of a wave (DPP row shifts + row broadcasts: no LDS round trips)
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Thread tid owns mask word tid of its tile, i.e. rows [32 tid, 32 tid + 32) of the tile (ope_store_mask).
// Its matches' tile-local rank is an exclusive block-wide scan of the words' popcounts; the ids are
// staged in LDS at their rank and written out by consecutive threads as full-line nontemporal stores
// (the ids stream to memory instead of leaving ~20 MB of dirty L2 lines for the kernel boundary).
// The tile's global offset is the sum of the counts of the tiles before it (<= a few thousand u32,
// 8 independent loads per thread per pass).
__global__ void __launch_bounds__(kOpeBlock) k_ope_scatter(const uint32_t* __restrict__ masks,
                                                           const uint32_t* __restrict__ counts,
                                                           uint32_t* __restrict__ out, uint64_t* __restrict__ total) {
  constexpr int kWaves = kOpeBlock / 64;
  __shared__ uint32_t wtot[kWaves];
  __shared__ uint32_t s_part[kWaves];
  __shared__ uint32_t sids[kOpeTile];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const size_t tile = blockIdx.x;
  const uint32_t word = masks[tile * kOpeBlock + tid];
  // exclusive prefix of this tile: sum of the counts of tiles [0, tile) (< 2^32: n is)
  uint32_t pre = 0;
  for (size_t base = 0; base < tile; base += 8 * kOpeBlock) {
    uint32_t cv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const size_t t = base + (size_t)q * kOpeBlock + tid;
      cv[q] = counts[t < tile ? t : 0];  // unconditional loads (issued together), masked below
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) pre += (base + (size_t)q * kOpeBlock + tid < tile) ? cv[q] : 0u;
  }
  pre = (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_sum(pre), 63);  // wave total
  const uint32_t c = __builtin_popcount(word);
  const uint32_t inc = wave_inclusive_sum(c);
  if (lane == 63) wtot[wid] = inc;
  if (lane == 0) s_part[wid] = pre;
  __syncthreads();
  uint32_t rank = inc - c, loc = 0;
  uint64_t off = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    rank += (w < wid) ? wtot[w] : 0u;
    loc += wtot[w];
    off += s_part[w];
  }
  const uint32_t row0 = (uint32_t)(tile * kOpeTile) + 32u * (uint32_t)tid;
  uint32_t m = word;
  while (m) {
    sids[rank++] = row0 + (uint32_t)__builtin_ctz(m);
    m &= m - 1u;
  }
  __syncthreads();
  uint32_t* o = out + off;
  for (uint32_t k = tid; k < loc; k += kOpeBlock) __builtin_nontemporal_store(sids[k], o + k);
  if (tid == 0 && tile == gridDim.x - 1) *total = off + loc;
}

// ------------------------------------------------------------------------------
// plain (unmodular) big-integer sum: SumAll without nsqr (DDSRestServer.scala:425)
// Each thread accumulates 64-bit lazy limb sums over a strided slice of rows.
// ------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_plain_sum(const uint32_t* __restrict__ X, size_t stride, size_t count,
                                                   int S, size_t nthreads, uint64_t* __restrict__ part) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthreads) return;
  for (int l = 0; l < S; ++l) {
    uint64_t s = 0;
    for (size_t row = t; row < count; row += nthreads) s += X[(size_t)l * stride + row];
    part[(size_t)l * nthreads + t] = s;
  }
}

__global__ void __launch_bounds__(256) k_plain_sum_reduce(const uint64_t* __restrict__ part, size_t nthreads, int S,
                                                          uint64_t* __restrict__ out) {
  __shared__ uint64_t sh[256];
  const int l = blockIdx.x;
  uint64_t s = 0;
  for (size_t t = threadIdx.x; t < nthreads; t += 256) s += part[(size_t)l * nthreads + t];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off >= 1; off >>= 1) {
    if ((int)threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[l] = sh[0];
}

// ------------------------------------------------------------------------------
// unbounded big-integer product tree: MultAll without pubkey (DDSRestServer.scala:520,
// `mult.get.multiply(operand)`). Radix 2^16 limbs in 32-bit words; one tree level
// multiplies rows (2p, 2p+1) of a [count][len] matrix into row p of [count/2][2 len].
// ------------------------------------------------------------------------------
// column sums: S[p][k] = sum_{i+j=k} A[2p][i] * A[2p+1][j]  (< len * 2^32, 64-bit)
// outlen <= 2 len: columns [outlen, 2 len) are not computed (a product mod 2^(16 outlen), the
// truncated tree of an even modulus' power-of-two part)
__global__ void __launch_bounds__(256) k_bigmul_cols(const uint32_t* __restrict__ A, size_t count, size_t len,
                                                     uint64_t* __restrict__ Sk, size_t outlen) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t p = blockIdx.y;
  if (k >= outlen) return;
  const uint32_t* a = A + (2 * p) * len;
  uint64_t acc = 0;
  if (2 * p + 1 < count) {
    const uint32_t* b = a + len;
    const size_t i0 = k >= len ? k - len + 1 : 0;
    const size_t i1 = k < len ? k : len - 1;
    for (size_t i = i0; i <= i1; ++i) acc += (uint64_t)(a[i] * b[k - i]);  // 16x16 -> 32 bits
  } else {
    acc = k < len ? a[k] : 0;  // odd row passes through
  }
  Sk[p * outlen + k] = acc;
}

// spread each 64-bit column sum over four 16-bit limbs: v_k = sum_d piece_d(S_{k-d}) (< 2^18)
__global__ void __launch_bounds__(256) k_bigmul_spread(const uint64_t* __restrict__ Sk, size_t outlen,
                                                       uint32_t* __restrict__ V) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t p = blockIdx.y;
  if (k >= outlen) return;
  const uint64_t* s = Sk + p * outlen;
  uint32_t v = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d)
    if (k >= (size_t)d) v += (uint32_t)((s[k - d] >> (16 * d)) & 0xFFFFu);
  V[p * outlen + k] = v;
}

// one carry pass: w_k = (v_k & 0xFFFF) + (v_{k-1} >> 16); flags[0] = 1 if some w_k > 0xFFFF
__global__ void __launch_bounds__(256) k_bigmul_carry(const uint32_t* __restrict__ V, size_t outlen,
                                                      uint32_t* __restrict__ Wout, uint32_t* __restrict__ flag) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t p = blockIdx.y;
  if (k >= outlen) return;
  const uint32_t* v = V + p * outlen;
  const uint32_t w = (v[k] & 0xFFFFu) + (k ? v[k - 1] >> 16 : 0u);
  Wout[p * outlen + k] = w;
  if (w > 0xFFFFu) atomicOr(flag, 1u);
}

// ------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------
// 2048-bit moduli (RSA n) use S = 76, not the minimal 74: 4-limb blocks (fewer loop instructions per
// CIOS step) and room for the QP modulus (no v_mul_lo) outweigh the 5.5 % more mads: MultAll fold
// 4.08-4.11 -> 4.01 ms over 10M rows (profiles/r01_rsa76_ab.txt). DDSHE_RSA76=0 keeps S = 74.
static bool use_rsa76() {
  static const bool on = [] {
    const char* e = getenv("DDSHE_RSA76");
    return !(e && e[0] == '0');
  }();
  return on;
}

Shape pick_shape(size_t mod_bits) {
  for (const Shape& s : kShapes) {
    if (s.S == (use_rsa76() ? 74 : 76)) continue;
    if ((size_t)s.W * s.S >= mod_bits + 2) return s;
  }
  return Shape{0, 0, 0};
}

Shape tail_shape(const Shape& main) {
  static_assert(sizeof(kShapes) == sizeof(kTail), "one tail shape per main shape");
  for (size_t i = 0; i < sizeof(kShapes) / sizeof(kShapes[0]); ++i)
    if (kShapes[i].S == main.S) return kTail[i];
  return Shape{0, 0, 0};
}

size_t max_modulus_bits() {
  const Shape& s = kShapes[sizeof(kShapes) / sizeof(kShapes[0]) - 1];
  return (size_t)s.W * s.S - 2;
}

hipError_t launch_egress_be(const uint32_t* X, size_t stride, size_t count, int S, int W, const uint32_t* nmod,
                            size_t width, uint8_t* out, hipStream_t st) {
  if (count == 0) return hipSuccess;
  if (S > kEgressMaxS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_egress_be, dim3((unsigned)((count + kEgressRows - 1) / kEgressRows)), dim3(256), 0, st, X, stride,
                     count, S, W, nmod, width, out);
  return hipGetLastError();
}

hipError_t launch_ingest_be(const uint8_t* in, size_t width, size_t count, int S, int W, const uint32_t* n2x,
                            uint32_t* X, size_t stride, uint32_t* flags, hipStream_t st, uint8_t* rowflags) {
  if (count == 0) return hipSuccess;
  static const bool lds = [] {  // DDSHE_INGEST_LDS=0: per-thread row walk (A/B timing)
    const char* e = getenv("DDSHE_INGEST_LDS");
    return !(e && e[0] == '0');
  }();
  if (lds && width % 16 == 0 && width <= kIngestMaxW && (uintptr_t)in % 16 == 0) {
    const size_t smem = (size_t)kIngestRows * (width / 4 + 1) * 4;
    hipLaunchKernelGGL(k_ingest_be_lds, dim3((unsigned)((count + kIngestRows - 1) / kIngestRows)),
                       dim3(kIngestThreads), smem, st, in, width, count, S, W, n2x, X, stride, flags, rowflags);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_ingest_be, dim3(grid_for(count)), dim3(256), 0, st, in, width, count, S, W, n2x, X, stride,
                     flags, rowflags);
  return hipGetLastError();
}

hipError_t launch_reduce_rows(int S, uint32_t* X, size_t stride, size_t count, const uint32_t* consts, uint32_t n0,
                              hipStream_t st, const uint32_t* gate) {
  if (count == 0) return hipSuccess;
  DDSHE_SWITCH(S, hipLaunchKernelGGL((k_reduce_rows<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256), 0, st, X, stride,
                                     count, consts, n0, gate));
  return hipGetLastError();
}

hipError_t launch_fold(int S, const uint32_t* X, size_t xstride, size_t count, const uint32_t* consts,
                       const uint32_t* qp_mod, uint32_t n0, uint32_t* P, size_t pstride, size_t ngroups, int s_out,
                       hipStream_t st, const uint32_t* ids, int lane1, size_t inblock_pgs) {
  if (ngroups == 0 || ngroups > count) return hipErrorInvalidValue;
  if (inblock_pgs) s_out = 0;  // the kernel zeroes the leaves' upper limbs itself
  if (lane1 && !(fold1_shape(S) && (lane1 == S || (S == 76 && lane1 == 74)))) return hipErrorInvalidValue;
  const int sw = lane1 ? lane1 : S;  // limbs the kernel writes
  // limbs sw..s_out of the partials (tail shape is wider): zero, contiguous in the limb-major layout
  if (s_out > sw) {
    hipError_t e = hipMemsetAsync(P + (size_t)sw * pstride, 0, (size_t)(s_out - sw) * pstride * 4, st);
    if (e != hipSuccess) return e;
  }
  if (lane1) {
    // k_fold1 at the column's own S may reduce against N~ (QP); at S = 74 over a 76-limb column
    // (moduli of <= 2070 bits: the top two limbs of every row are zero) it uses N and the CIOS quotient
    const bool qp = qp_mod && lane1 == S;
    const uint32_t* c = qp ? qp_mod : consts;
#define DDSHE_FOLD1(S_)                                                                                            \
  case S_:                                                                                                         \
    if (qp && ids)                                                                                                 \
      hipLaunchKernelGGL((k_fold1<S_, 28, true, true>), dim3(grid_for(ngroups)), dim3(256), 0, st, X, xstride,     \
                         count, c, n0, P, pstride, ngroups, ids);                                                  \
    else if (qp)                                                                                                   \
      hipLaunchKernelGGL((k_fold1<S_, 28, true>), dim3(grid_for(ngroups)), dim3(256), 0, st, X, xstride, count, c, \
                         n0, P, pstride, ngroups, nullptr);                                                        \
    else if (ids)                                                                                                  \
      hipLaunchKernelGGL((k_fold1<S_, 28, false, true>), dim3(grid_for(ngroups)), dim3(256), 0, st, X, xstride,    \
                         count, c, n0, P, pstride, ngroups, ids);                                                  \
    else                                                                                                           \
      hipLaunchKernelGGL((k_fold1<S_, 28, false>), dim3(grid_for(ngroups)), dim3(256), 0, st, X, xstride, count,   \
                         c, n0, P, pstride, ngroups, nullptr);                                                     \
    break;
    switch (lane1) {
      DDSHE_FOLD1(40)
      DDSHE_FOLD1(74)
      DDSHE_FOLD1(76)
      default: return hipErrorInvalidValue;
    }
#undef DDSHE_FOLD1
    return hipGetLastError();
  }
  const uint32_t* c = qp_mod ? qp_mod : consts;  // N~ = N·n0 in place of N (Mont QP): no v_mul_lo per CIOS step
  if (inblock_pgs) {  // one partial per block (k_fold InBlock), row-major leaves of inblock_pgs words
    if (!qp_mod || ids || lane1) return hipErrorInvalidValue;
    DDSHE_SWITCH(S, {
      if (ngroups % (256 / TPI) != 0 || inblock_pgs < (size_t)S) return hipErrorInvalidValue;
      hipLaunchKernelGGL((k_fold<S, TPI, W, true, false, false, true>), dim3(grid_for(ngroups * TPI)), dim3(256), 0,
                         st, X, xstride, count, c, n0, P, 1, ngroups, nullptr, S, inblock_pgs);
    });
    return hipGetLastError();
  }
  if (qp_mod && ids) {
    DDSHE_SWITCH(S, hipLaunchKernelGGL((k_fold<S, TPI, W, true, true>), dim3(grid_for(ngroups * TPI)), dim3(256), 0, st, X, xstride, count, c,
                                       n0, P, pstride, ngroups, ids));
  } else if (qp_mod) {
    DDSHE_SWITCH(S, hipLaunchKernelGGL((k_fold<S, TPI, W, true>), dim3(grid_for(ngroups * TPI)), dim3(256), 0, st, X, xstride, count, c, n0, P,
                                       pstride, ngroups, nullptr));
  } else if (ids) {
    DDSHE_SWITCH(S, hipLaunchKernelGGL((k_fold<S, TPI, W, false, true>), dim3(grid_for(ngroups * TPI)), dim3(256), 0, st, X, xstride, count, c,
                                       n0, P, pstride, ngroups, ids));
  } else {
    DDSHE_SWITCH(S, hipLaunchKernelGGL((k_fold<S, TPI, W>), dim3(grid_for(ngroups * TPI)), dim3(256), 0, st, X, xstride, count, c, n0, P,
                                       pstride, ngroups, nullptr));
  }
  return hipGetLastError();
}

bool fold1_shape(int S) {
  static const bool on = [] {
    const char* e = getenv("DDSHE_FOLD1");
    return !(e && e[0] == '0');
  }();
  return on && (S == 40 || S == 76);
}
// limbs k_fold1 runs with for a modulus of `bits` in shape S: 2048-bit moduli (RSA n, a 1024-bit
// Paillier key's n^2) fit 74 limbs (74 * 28 >= bits + 2): 5 % fewer mads than 76 for one v_mul_lo per
// CIOS step (the QP modulus N~ needs 76). DDSHE_FOLD1_74=0 keeps 76 (A/B timing).
int fold1_limbs(int S, size_t bits) {
  static const bool s74 = [] {
    const char* e = getenv("DDSHE_FOLD1_74");
    return !(e && e[0] == '0');
  }();
  if (S == 76 && s74 && bits + 2 <= 74 * 28) return 74;
  return S;
}
// A product at one lane per bignum takes ~TPI times longer than at TPI lanes, so small folds (a few rows
// per lane) keep the lane-group kernel; from ~8 rows per lane of a full k_fold1 grid on, the fold is
// throughput-bound and k_fold1 issues fewer instructions per product.
size_t fold1_min_rows(int S, int cus) {
  static const long long env = [] {
    const char* e = getenv("DDSHE_FOLD1_MIN");
    return e ? atoll(e) : -1ll;
  }();
  if (env >= 0) return (size_t)env;
  int bpc = 0;
  if (fold1_occupancy(S, &bpc) != hipSuccess || bpc < 1) bpc = 1;
  return (size_t)8 * cus * bpc * 256;
}
hipError_t fold1_occupancy(int S, int* blocks_per_cu) {
  switch (S) {
    case 40: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (const void*)k_fold1<40, 28, true>, 256, 0);
    case 76: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (const void*)k_fold1<76, 28, true>, 256, 0);
    case 74: return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (const void*)k_fold1<74, 28, false>, 256, 0);
    default: return hipErrorInvalidValue;
  }
}

bool fold_qp_enabled() {  // DDSHE_FOLD_QP=0 disables (A/B timing)
  static const bool on = [] {
    const char* e = getenv("DDSHE_FOLD_QP");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Latency-bound tree levels of the 4096-bit tail shape (S = 160, W = 28) run with 32 lanes per
// bignum (L = 5 limbs per lane): a Montgomery step issues 10 mads per wave instead of 20, and
// these levels have at most one wave per SIMD, so the step time is the issue time of one wave.
// Levels with more groups stay at TPI = 16 (fewer exchange instructions per mad). Same limb
// layout and constants for both, so levels mix freely. DDSHE_TAIL32=0 disables (A/B timing).
constexpr size_t kTail32MaxGroups = 2048;
bool tail_qp(int S) {  // DDSHE_TAIL_QP=0 disables (A/B timing)
  static const bool on = [] {
    const char* e = getenv("DDSHE_TAIL_QP");
    return !(e && e[0] == '0');
  }();
  return on && S == 160;
}
static bool use_tail32(int S, size_t ngroups) {
  static const bool on = [] {
    const char* e = getenv("DDSHE_TAIL32");
    return !(e && e[0] == '0');
  }();
  return on && S == 160 && ngroups <= kTail32MaxGroups;
}

// The widest tail levels of the 4096-bit shape (>= 8192 products: throughput-bound, 2+ waves per SIMD at
// 8 lanes per bignum) run at TPI = 8: 40 mads per step against the same ~18 exchange/quotient
// instructions as at TPI = 16 (20 mads). DDSHE_TAIL8=0 disables (A/B timing).
constexpr size_t kTail8MinGroups = 8192;
static bool use_tail8(int S, size_t ngroups) {
  static const bool on = [] {
    const char* e = getenv("DDSHE_TAIL8");
    return !(e && e[0] == '0');
  }();
  return on && S == 160 && ngroups >= kTail8MinGroups;
}

// The 2048-bit tail shape (S = 80, 16 lanes per bignum) gets many more leaves since MultAll folds at one
// bignum per lane (131,072 level-1 partials at 10M rows): its widest levels are throughput-bound and run
// at 4 lanes per bignum (>= 32768 products: 40 mads per step against ~14 exchange/quotient instructions)
// or 8 (>= 16384). DDSHE_TAIL80=0 disables (A/B timing).
static int tail80_tpi(int S, size_t ngroups) {
  static const bool on = [] {
    const char* e = getenv("DDSHE_TAIL80");
    return !(e && e[0] == '0');
  }();
  if (!on || S != 80) return 0;
  return ngroups >= 32768 ? 4 : ngroups >= 16384 ? 8 : 0;
}

// First fold level of a small fold in the latency shape S2, straight from a main-shape column holding
// `sin` limbs per row (k_fold<..., Narrow>): one launch of wide lane groups instead of a main-shape level
// with one or two rows per group (long per-product latency at 2-4 lanes) plus the zeroing of the
// partials' extra limbs. TPI by the number of groups, as the tail levels choose it.
bool fold_narrow_shape(int S2) { return S2 == 48 || S2 == 80 || S2 == 160; }
hipError_t launch_fold_narrow(int S2, const uint32_t* X, size_t xstride, size_t count, int sin, const uint32_t* consts,
                              const uint32_t* qp_mod, uint32_t n0, uint32_t* P, size_t pstride, size_t ngroups,
                              hipStream_t st, size_t pgs) {
  if (ngroups == 0 || ngroups > count || !fold_narrow_shape(S2) || sin < 8 || sin % 4 || sin > S2)
    return hipErrorInvalidValue;
#define DDSHE_NARROW(S_, TPI_, QP_, C_)                                                                        \
  hipLaunchKernelGGL((k_fold<S_, TPI_, 28, QP_, false, true>), dim3(grid_for(ngroups * TPI_)), dim3(256), 0, st, X, \
                     xstride, count, C_, n0, P, pstride, ngroups, nullptr, sin, pgs)
  if (S2 == 48) {
    DDSHE_NARROW(48, 16, false, consts);
  } else if (S2 == 80) {
    if (ngroups >= 32768)
      DDSHE_NARROW(80, 4, false, consts);
    else if (ngroups >= 16384)
      DDSHE_NARROW(80, 8, false, consts);
    else
      DDSHE_NARROW(80, 16, false, consts);
  } else {
    const int tpi = ngroups >= kTail8MinGroups ? 8 : ngroups <= kTail32MaxGroups ? 32 : 16;
    if (qp_mod) {
      if (tpi == 8) DDSHE_NARROW(160, 8, true, qp_mod);
      else if (tpi == 32) DDSHE_NARROW(160, 32, true, qp_mod);
      else DDSHE_NARROW(160, 16, true, qp_mod);
    } else {
      if (tpi == 8) DDSHE_NARROW(160, 8, false, consts);
      else if (tpi == 32) DDSHE_NARROW(160, 32, false, consts);
      else DDSHE_NARROW(160, 16, false, consts);
    }
  }
#undef DDSHE_NARROW
  return hipGetLastError();
}

hipError_t launch_fold_tail(int S, const uint32_t* X, size_t xstride, size_t count, const uint32_t* consts,
                            const uint32_t* qp_mod, uint32_t n0, uint32_t* P, size_t pstride, size_t ngroups,
                            hipStream_t st, size_t pgs) {
  if (ngroups == 0 || ngroups > count) return hipErrorInvalidValue;
  if (const int t80 = tail80_tpi(S, ngroups)) {  // S = 80 has no QP modulus (tail_qp)
    if (t80 == 4)
      hipLaunchKernelGGL((k_fold<80, 4, 28>), dim3(grid_for(ngroups * 4)), dim3(256), 0, st, X, xstride, count, consts,
                         n0, P, pstride, ngroups, nullptr, 80, pgs);
    else
      hipLaunchKernelGGL((k_fold<80, 8, 28>), dim3(grid_for(ngroups * 8)), dim3(256), 0, st, X, xstride, count, consts,
                         n0, P, pstride, ngroups, nullptr, 80, pgs);
    return hipGetLastError();
  }
  if (use_tail8(S, ngroups)) {
    if (qp_mod)
      hipLaunchKernelGGL((k_fold<160, 8, 28, true>), dim3(grid_for(ngroups * 8)), dim3(256), 0, st, X, xstride, count,
                         qp_mod, n0, P, pstride, ngroups, nullptr, 160, pgs);
    else
      hipLaunchKernelGGL((k_fold<160, 8, 28>), dim3(grid_for(ngroups * 8)), dim3(256), 0, st, X, xstride, count,
                         consts, n0, P, pstride, ngroups, nullptr, 160, pgs);
    return hipGetLastError();
  }
  if (use_tail32(S, ngroups)) {
    if (qp_mod)  // N~ = N·n0 in place of N (Mont QP): the quotient needs no multiply
      hipLaunchKernelGGL((k_fold<160, 32, 28, true>), dim3(grid_for(ngroups * 32)), dim3(256), 0, st, X, xstride,
                         count, qp_mod, n0, P, pstride, ngroups, nullptr, 160, pgs);
    else
      hipLaunchKernelGGL((k_fold<160, 32, 28>), dim3(grid_for(ngroups * 32)), dim3(256), 0, st, X, xstride, count,
                         consts, n0, P, pstride, ngroups, nullptr, 160, pgs);
    return hipGetLastError();
  }
  if (qp_mod) {
    DDSHE_TAIL_SWITCH(S, hipLaunchKernelGGL((k_fold<S, TPI, W, true>), dim3(grid_for(ngroups * TPI)), dim3(256), 0, st,
                                            X, xstride, count, qp_mod, n0, P, pstride, ngroups, nullptr, S, pgs));
  } else {
    DDSHE_TAIL_SWITCH(S, hipLaunchKernelGGL((k_fold<S, TPI, W>), dim3(grid_for(ngroups * TPI)), dim3(256), 0, st, X,
                                            xstride, count, consts, n0, P, pstride, ngroups, nullptr, S, pgs));
  }
  return hipGetLastError();
}

hipError_t launch_finalize_tail(int S, const uint32_t* P, size_t pstride, const uint32_t* consts, const uint32_t* Y,
                                uint32_t n0, uint32_t* out, hipStream_t st) {
  if (use_tail32(S, 1)) {
    hipLaunchKernelGGL((k_finalize<160, 32, 28>), dim3(1), dim3(64), 0, st, P, pstride, consts, Y, n0, out);
    return hipGetLastError();
  }
  DDSHE_TAIL_SWITCH(S, hipLaunchKernelGGL((k_finalize<S, TPI, W>), dim3(1), dim3(64), 0, st, P, pstride, consts, Y, n0,
                                          out));
  return hipGetLastError();
}

int tail_tpi() { return 16; }

hipError_t launch_pairs(int S, const uint32_t* A, const uint32_t* B, size_t stride, size_t count,
                        const uint32_t* consts, uint32_t n0, uint32_t* O, hipStream_t st) {
  if (count == 0) return hipSuccess;
  DDSHE_SWITCH(S, hipLaunchKernelGGL((k_pairs<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256), 0, st, A, B, stride,
                                     count, consts, n0, O));
  return hipGetLastError();
}

hipError_t launch_pairs_tail(int S, const uint32_t* A, const uint32_t* B, size_t stride, size_t count,
                             const uint32_t* consts, uint32_t n0, uint32_t* O, hipStream_t st) {
  if (count == 0) return hipSuccess;
  DDSHE_TAIL_SWITCH(S, hipLaunchKernelGGL((k_pairs<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256), 0, st, A, B,
                                          stride, count, consts, n0, O));
  return hipGetLastError();
}

hipError_t launch_modexp_pre(int S, const uint32_t* Xcol, size_t xstride, size_t count, const uint32_t* consts,
                             const uint32_t* qp_mod, uint32_t n0, int nodd, uint32_t* Tab, size_t tstride,
                             hipStream_t st) {
  if (count == 0) return hipSuccess;
  if (qp_mod) {
    DDSHE_SWITCH(S, hipLaunchKernelGGL((k_modexp_pre<S, TPI, W, true>), dim3(grid_for(count * TPI)), dim3(256),
                                       (256 / TPI) * 2 * S * 4, st, Xcol, xstride, count, consts, qp_mod, n0, nodd,
                                       Tab, tstride));
  } else {
    DDSHE_SWITCH(S, hipLaunchKernelGGL((k_modexp_pre<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256),
                                       (256 / TPI) * 2 * S * 4, st, Xcol, xstride, count, consts, nullptr, n0, nodd,
                                       Tab, tstride));
  }
  return hipGetLastError();
}

#ifdef DDSHE_LADDER_OCC2
constexpr int kLadderSlots = 2;
#else
constexpr int kLadderSlots = 1;
#endif
hipError_t launch_modexp_ladder(int S, const uint32_t* Tab, size_t tstride, const uint32_t* m, size_t count,
                                const uint32_t* consts, const uint32_t* qp_mod, const uint32_t* gR,
                                const uint32_t* sched, int nsched, uint32_t n0, uint32_t* O, size_t ostride,
                                hipStream_t st) {
  if (count == 0) return hipSuccess;
  if (qp_mod) {
    DDSHE_SWITCH(S, hipLaunchKernelGGL((k_modexp_ladder<S, TPI, W, true>), dim3(grid_for(count * TPI)), dim3(256),
                                       (256 / TPI) * kLadderSlots * S * 4, st, Tab, tstride, m, count, consts, qp_mod, gR, sched,
                                       nsched, n0, O, ostride));
  } else {
    DDSHE_SWITCH(S, hipLaunchKernelGGL((k_modexp_ladder<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256),
                                       (256 / TPI) * kLadderSlots * S * 4, st, Tab, tstride, m, count, consts, nullptr, gR, sched,
                                       nsched, n0, O, ostride));
  }
  return hipGetLastError();
}

hipError_t launch_synth_rows(int S, const uint32_t* T, size_t tstride, uint32_t tcount, const uint32_t* P,
                             size_t pstride, uint32_t pcount, uint64_t seed, uint64_t row0, size_t count,
                             const uint32_t* consts, uint32_t n0, uint32_t* X, size_t xstride, hipStream_t st,
                             uint32_t shards, uint32_t shard) {
  if (count == 0) return hipSuccess;
  DDSHE_SWITCH(S, hipLaunchKernelGGL((k_synth_rows<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256), 0, st, T, tstride,
                                     tcount, P, pstride, pcount, seed, row0, count, consts, n0, X, xstride, shards,
                                     shard));
  return hipGetLastError();
}

hipError_t launch_repack(const uint32_t* src, size_t sstride, int Ss, int Ws, uint32_t* dst, size_t dstride, int Sd,
                         int Wd, size_t count, uint32_t* flags, hipStream_t st) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(k_repack, dim3(grid_for(count)), dim3(256), 0, st, src, sstride, Ss, Ws, dst, dstride, Sd, Wd,
                     count, flags);
  return hipGetLastError();
}

hipError_t launch_crt_h(int S, const uint32_t* Yp, const uint32_t* Yq, size_t stride, size_t count,
                        const uint32_t* consts, const uint32_t* c12, uint32_t n0, uint32_t* H, hipStream_t st) {
  if (count == 0) return hipSuccess;
  DDSHE_SWITCH(S, hipLaunchKernelGGL((k_crt_h<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256), 0, st, Yp, Yq,
                                     stride, count, consts, c12, n0, H));
  return hipGetLastError();
}

hipError_t launch_crt_out(int S, const uint32_t* Hn, const uint32_t* Yqn, size_t stride, size_t count,
                          const uint32_t* consts, const uint32_t* q2R, uint32_t n0, uint32_t* O, size_t ostride,
                          hipStream_t st) {
  if (count == 0) return hipSuccess;
  DDSHE_SWITCH(S, hipLaunchKernelGGL((k_crt_out<S, TPI, W>), dim3(grid_for(count * TPI)), dim3(256), 0, st, Hn, Yqn,
                                     stride, count, consts, q2R, n0, O, ostride));
  return hipGetLastError();
}

hipError_t launch_fill_random(uint32_t* X, size_t stride, int S, int W, uint64_t seed, uint64_t row0, size_t count,
                              int bits, hipStream_t st) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_random, dim3(grid_for(count)), dim3(256), 0, st, X, stride, S, W, seed, row0, count, bits);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const uint32_t* T, size_t tstride, uint32_t tcount, int S, uint64_t seed, uint64_t row0,
                              size_t count, uint32_t* X, size_t xstride, hipStream_t st) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_rows, dim3(grid_for(count)), dim3(256), 0, st, T, tstride, tcount, S, seed, row0, count, X,
                     xstride);
  return hipGetLastError();
}

size_t ope_blocks(size_t n) { return (n + kOpeTile - 1) / kOpeTile; }

size_t ope_scratch_bytes(size_t n) { return ope_blocks(n) * (4 + 4 * kOpeBlock) + 8; }

hipError_t launch_str_eq_compact(const StrFp* posfp, const uint64_t* present, size_t row0, size_t nrows,
                                 const uint64_t* row_beg, const uint64_t* elem_off, const uint8_t* chars,
                                 const uint8_t* nchars, const StrNeedles& nd, uint64_t position, int negate,
                                 void* scratch, uint64_t* total, uint32_t* out, hipStream_t st) {
  const size_t nb = ope_blocks(nrows);
  if (nb == 0) return hipSuccess;
  uint32_t* counts = (uint32_t*)scratch;
  uint32_t* masks = counts + nb;
  hipLaunchKernelGGL(k_str_eq_count, dim3((unsigned)nb), dim3(kOpeBlock), 0, st, posfp, present, row0, nrows, row_beg,
                     elem_off, chars, nchars, nd, position, negate, masks, counts);
  hipLaunchKernelGGL(k_ope_scatter, dim3((unsigned)nb), dim3(kOpeBlock), 0, st, masks, counts, out, total);
  return hipGetLastError();
}

hipError_t launch_byte_compact(const uint8_t* bytes, size_t n, uint32_t vmask, void* scratch, uint64_t* total,
                               uint32_t* out, hipStream_t st, uint32_t vall, bool rezero) {
  const size_t nb = ope_blocks(n);
  if (nb == 0) return hipSuccess;
  uint32_t* counts = (uint32_t*)scratch;
  uint32_t* masks = counts + nb;
  hipLaunchKernelGGL(k_byte_count, dim3((unsigned)nb), dim3(kOpeBlock), 0, st, bytes, n, vmask, vall, masks, counts,
                     rezero);
  hipLaunchKernelGGL(k_ope_scatter, dim3((unsigned)nb), dim3(kOpeBlock), 0, st, masks, counts, out, total);
  return hipGetLastError();
}

namespace {
// gt: c > b; le: !(c > b); ge: c > b-1; lt: !(c > b-1); b-1 underflows only for b = INT64_MIN, where
// ge keeps every row and lt none
void ope_code(int64_t bound, int op, int64_t* t, int* code) {
  *t = bound;
  *code = 0;
  switch (op) {
    case 0: break;
    case 3: *code = 1; break;
    case 1: if (bound == INT64_MIN) *code = 2; else *t = bound - 1; break;
    default: if (bound == INT64_MIN) *code = 4; else { *t = bound - 1; *code = 1; } break;
  }
}
void ope_count(const int64_t* col, const uint8_t* valid, size_t n, int64_t bound, int op, uint32_t* masks,
               uint32_t* counts, hipStream_t st, uint32_t vmask, uint32_t vbad,
               unsigned long long* total = nullptr, size_t hlimit = 0) {
  // zero-copy mask store width (DDSHE_MASK_STORE, A/B: 16 = 16-byte non-temporal stores by the tile's
  // first wave (default: 0.0445-0.0457 ms per 10M-row Search route against 0.046-0.055 for one word per
  // lane on the same box); 8 = 8-byte system-scope stores; 4 = one word per lane, system-scope; plain
  // 16-byte stores were slower, 0.058 ms: the lines sit in L2 until the kernel's end-of-kernel write-back).
  // The wider forms need a 16-byte aligned buffer, else one word per lane
  static const int wide_mode = [] {
    const char* e = getenv("DDSHE_MASK_STORE");
    const int v = e ? atoi(e) : 16;
    return v == 8 ? 1 : v == 16 ? 2 : 0;
  }();
  const int hwide = (hlimit && ((uintptr_t)masks & 15) == 0) ? wide_mode : 0;
  const size_t nb = ope_blocks(n);
  int64_t t;
  int code;
  ope_code(bound, op, &t, &code);
  if (valid)
    hipLaunchKernelGGL(k_ope_count<true>, dim3((unsigned)nb), dim3(kOpeBlock), 0, st, col, valid, n, t, code, vmask,
                       vbad, masks, counts, total, hlimit, hwide);
  else
    hipLaunchKernelGGL(k_ope_count<false>, dim3((unsigned)nb), dim3(kOpeBlock), 0, st, col, valid, n, t, code, vmask,
                       vbad, masks, counts, total, hlimit, hwide);
}
}  // namespace

hipError_t launch_ope_filter(const int64_t* col, const uint8_t* valid, size_t n, int64_t bound, int op, void* scratch,
                             uint64_t* total, uint32_t* out, hipStream_t st, uint32_t vmask, uint32_t vbad) {
  const size_t nb = ope_blocks(n);
  if (nb == 0) return hipSuccess;
  uint32_t* counts = (uint32_t*)scratch;
  uint32_t* masks = counts + nb;
  ope_count(col, valid, n, bound, op, masks, counts, st, vmask, vbad);
  hipLaunchKernelGGL(k_ope_scatter, dim3((unsigned)nb), dim3(kOpeBlock), 0, st, masks, counts, out, total);
  return hipGetLastError();
}

uint32_t* ope_mask_words(void* scratch, size_t n) { return (uint32_t*)scratch + ope_blocks(n); }

hipError_t launch_ope_mask(const int64_t* col, const uint8_t* valid, size_t n, int64_t bound, int op, void* scratch,
                           uint64_t* total, hipStream_t st, uint32_t vmask, uint32_t vbad, bool total_zeroed,
                           uint32_t* hmask, size_t hwords, uint32_t* hcounts) {
  const size_t nb = ope_blocks(n);
  if (nb == 0) return hipSuccess;
  uint32_t* counts = (uint32_t*)scratch;
  if (hmask) {  // words and tile counts straight into mapped host memory (hwords u32 words, nb counts)
    if (!hcounts || hwords < (n + 31) / 32) return hipErrorInvalidValue;
    ope_count(col, valid, n, bound, op, hmask, hcounts, st, vmask, vbad, nullptr, hwords);
    return hipGetLastError();
  }
  if (total_zeroed) {  // the tiles add their counts into *total themselves
    ope_count(col, valid, n, bound, op, counts + nb, counts, st, vmask, vbad, (unsigned long long*)total);
    return hipGetLastError();
  }
  ope_count(col, valid, n, bound, op, counts + nb, counts, st, vmask, vbad);
  hipLaunchKernelGGL(k_count_total, dim3(1), dim3(1024), 0, st, counts, nb, total);
  return hipGetLastError();
}

hipError_t launch_plain_sum(const uint32_t* X, size_t stride, size_t count, int S, size_t nthreads, uint64_t* part,
                            uint64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_plain_sum, dim3(grid_for(nthreads)), dim3(256), 0, st, X, stride, count, S, nthreads, part);
  hipLaunchKernelGGL(k_plain_sum_reduce, dim3(S), dim3(256), 0, st, part, nthreads, S, out);
  return hipGetLastError();
}

hipError_t launch_bigmul_level(const uint32_t* A, size_t count, size_t len, uint64_t* Sk, uint32_t* V, hipStream_t st,
                               size_t cap) {
  const size_t pairs = (count + 1) / 2, outlen = cap ? std::min(2 * len, cap) : 2 * len;
  dim3 grid((unsigned)((outlen + 255) / 256), (unsigned)pairs);
  hipLaunchKernelGGL(k_bigmul_cols, grid, dim3(256), 0, st, A, count, len, Sk, outlen);
  hipLaunchKernelGGL(k_bigmul_spread, grid, dim3(256), 0, st, Sk, outlen, V);
  return hipGetLastError();
}

hipError_t launch_bigmul_carry(const uint32_t* V, size_t pairs, size_t outlen, uint32_t* Wout, uint32_t* flag,
                               hipStream_t st) {
  dim3 grid((unsigned)((outlen + 255) / 256), (unsigned)pairs);
  hipLaunchKernelGGL(k_bigmul_carry, grid, dim3(256), 0, st, V, outlen, Wout, flag);
  return hipGetLastError();
}

// dst[r*drs + c*dcs] = src[r*srs + c*scs]: partials between the limb-major tree layout and packed rows
__global__ void k_strided_copy(const uint32_t* __restrict__ src, size_t srs, size_t scs, uint32_t* __restrict__ dst,
                               size_t drs, size_t dcs, size_t rows, size_t cols) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  const size_t r = i / cols, c = i % cols;
  dst[r * drs + c * dcs] = src[r * srs + c * scs];
}

hipError_t launch_strided_copy(const uint32_t* src, size_t srs, size_t scs, uint32_t* dst, size_t drs, size_t dcs,
                               size_t rows, size_t cols, hipStream_t st) {
  if (rows * cols == 0) return hipSuccess;
  hipLaunchKernelGGL(k_strided_copy, dim3(grid_for(rows * cols)), dim3(256), 0, st, src, srs, scs, dst, drs, dcs, rows,
                     cols);
  return hipGetLastError();
}

hipError_t fold_occupancy(int S, int* blocks_per_cu) {
  DDSHE_SWITCH(S, return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, (const void*)k_fold<S, TPI, W>, 256,
                                                                       0));
  return hipSuccess;
}

}  // namespace ddshe
