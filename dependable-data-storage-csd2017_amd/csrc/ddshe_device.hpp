// Device-side Montgomery arithmetic for the homomorphic aggregation engine (gfx950).
//
// Replaces the per-element BigInteger work of the reference fold loops:
//   HomoAdd.sum(acc, x, nsquare)   DDSRestServer.scala:423  (c1·c2 mod n²)
//   HomoMult.multiply(acc, x, pk)  DDSRestServer.scala:518  (c1·c2 mod n)
//
// Number representation:
//   * radix 2^27 limbs held in 32-bit words ("r27"). A modulus of B bits uses
//     S ≥ ceil((B+2)/27) limbs so that R = 2^(27·S) > 4N.
//   * the Montgomery accumulator t[] is kept as 64-bit LAZY sums: every limb
//     product is a single v_mad_u64_u32 (measured half-rate, the same rate as
//     v_add_co/v_addc — so carry-free accumulation halves the instruction
//     count vs. 32-bit limbs with carry chains). With 27-bit limbs a column
//     receives at most 2S products < 2^55, so 2S·2^55 < 2^64 for S < 256.
//   * a bignum is owned by a GROUP of TPI consecutive lanes; lane r holds limbs
//     [r·L, (r+1)·L), L = S/TPI. Per CIOS step the group exchanges two words
//     (the Montgomery quotient m, broadcast from lane 0, and the limb shifted
//     across the lane boundary) with DPP/ds_swizzle.
//   * values are kept < 2N and "almost normalised" (limbs < 2^28) between
//     Montgomery products; anything written to HBM is fully normalised
//     (limbs < 2^27). Canonical reduction to [0, N) happens once per result.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ddshe {

constexpr int kW = 27;
constexpr uint32_t kMask = (1u << kW) - 1u;

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// ---- intra-group lane exchange -----------------------------------------------
// value of lane 0 of this lane's group
template <int TPI>
__device__ __forceinline__ uint32_t grp_bcast0(uint32_t x) {
  if constexpr (TPI == 1) return x;
  else if constexpr (TPI == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xA0, 0xF, 0xF, false);  // quad_perm [0,0,2,2]
  else if constexpr (TPI == 4) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x00, 0xF, 0xF, false);  // quad_perm [0,0,0,0]
  else if constexpr (TPI == 8) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x18);                      // and_mask 0b11000
  else { static_assert(TPI == 16, "TPI"); return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x10); }
}
// value of lane r+1 (caller masks the group's top lane)
template <int TPI>
__device__ __forceinline__ uint32_t grp_from_next(uint32_t x) {
  if constexpr (TPI == 1) return 0u;
  else if constexpr (TPI == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xF5, 0xF, 0xF, false);  // [1,1,3,3]
  else if constexpr (TPI == 4) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xF9, 0xF, 0xF, false);  // [1,2,3,3]
  else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, true);                          // row_shl:1
}
// value of lane r-1 (caller masks the group's bottom lane)
template <int TPI>
__device__ __forceinline__ uint32_t grp_from_prev(uint32_t x) {
  if constexpr (TPI == 1) return 0u;
  else if constexpr (TPI == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xA0, 0xF, 0xF, false);  // [0,0,2,2]
  else if constexpr (TPI == 4) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x90, 0xF, 0xF, false);  // [0,0,1,2]
  else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);                          // row_shr:1
}

// ---- Montgomery product on a lane group --------------------------------------
template <int S, int TPI>
struct Mont {
  static_assert(S % TPI == 0, "S must divide into TPI lanes");
  static constexpr int L = S / TPI;
  static_assert(L >= 2, "need at least two limbs per lane");
  static_assert(S < 256, "lazy 64-bit accumulation bound");

  // One CIOS step with multiplier limb b: t = (t + a·b + m·N) / 2^27.
  __device__ __forceinline__ static void step(uint64_t (&t)[L], const uint32_t (&a)[L], const uint32_t (&n)[L],
                                              uint32_t b, uint32_t n0, bool top) {
    // pass 1: t += a*b, in place (no 64-bit temporaries live across the pass)
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = (uint64_t)a[l] * b + t[l];
    const uint32_t m = grp_bcast0<TPI>(((uint32_t)t[0] * n0) & kMask);
    // pass 2: t = (t + m*N) / 2^27, shifting down one limb in place
    const uint64_t u0 = (uint64_t)m * n[0] + t[0];
    const uint32_t lo0 = (uint32_t)u0 & kMask;  // == 0 on the group's lane 0
    t[0] = (uint64_t)m * n[1] + (t[1] + (u0 >> kW));
#pragma unroll
    for (int l = 2; l < L; ++l) t[l - 1] = (uint64_t)m * n[l] + t[l];
    const uint32_t up = grp_from_next<TPI>(lo0);
    t[L - 1] = top ? 0ull : (uint64_t)up;
  }

  // 64-bit lazy sums -> almost-normalised limbs (< 2^28) in a[].
  __device__ __forceinline__ static void settle(const uint64_t (&t)[L], uint32_t (&a)[L], bool bottom) {
    uint64_t c = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const uint64_t v = t[l] + c;
      a[l] = (uint32_t)v & kMask;
      c = v >> kW;
    }
    uint32_t clo = grp_from_prev<TPI>((uint32_t)c & kMask);
    uint32_t chi = grp_from_prev<TPI>((uint32_t)(c >> kW));
    if (bottom) { clo = 0; chi = 0; }
    a[0] += clo;
    a[1] += chi;
  }

  // a <- MonPro(a, B), B streamed limb by limb from bcol[i*stride] (fully normalised, value < 2N).
  __device__ __forceinline__ static void mul_col(uint32_t (&a)[L], const uint32_t (&n)[L],
                                                 const uint32_t* __restrict__ bcol, size_t stride, uint32_t n0,
                                                 bool top, bool bottom) {
    uint64_t t[L];
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = 0;
    constexpr int PF = 4;  // prefetch distance (b loads in flight)
    uint32_t bq[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) bq[q] = __builtin_nontemporal_load(bcol + (size_t)q * stride);
    const uint32_t* bnext = bcol + (size_t)PF * stride;
    // not unrolled: unrolling lets LLVM re-associate the u64 sums of several steps
    // into mad(x,y,0)+add trees, which costs registers and extra 64-bit adds
#pragma unroll 1
    for (int i = 0; i < S; ++i) {
      const uint32_t b = bq[0];
#pragma unroll
      for (int q = 0; q < PF - 1; ++q) bq[q] = bq[q + 1];
      bq[PF - 1] = i + PF < S ? __builtin_nontemporal_load(bnext) : 0u;
      bnext += stride;
      step(t, a, n, b, n0, top);
    }
    settle(t, a, bottom);
  }

  // a <- MonPro(a, B) with B held by the group in registers (same layout as a).
  __device__ __forceinline__ static void mul_reg(uint32_t (&a)[L], const uint32_t (&bv)[L], const uint32_t (&n)[L],
                                                 uint32_t n0, int r, bool top, bool bottom) {
    uint64_t t[L];
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = 0;
    for (int src = 0; src < TPI; ++src) {
#pragma unroll
      for (int l = 0; l < L; ++l) {
        // limb src*L + l of B lives in lane `src` of the group
        const uint32_t b = group_read(bv[l], src, r);
        step(t, a, n, b, n0, top);
      }
    }
    settle(t, a, bottom);
  }

  // read x from lane `src` of the group (all lanes receive it)
  __device__ __forceinline__ static uint32_t group_read(uint32_t x, int src, int r) {
    if constexpr (TPI == 1) return x;
    else {
      const int base = lane_id() - r;
      return (uint32_t)__builtin_amdgcn_ds_bpermute((base + src) << 2, (int)x);
    }
  }

  // Almost-normalised (limbs < 2^28) -> fully normalised (limbs < 2^27); value unchanged.
  __device__ __forceinline__ static void normalize(uint32_t (&a)[L], bool bottom) {
    for (int round = 0; round < TPI; ++round) {
      uint32_t c = 0;
#pragma unroll
      for (int l = 0; l < L; ++l) {
        const uint32_t v = a[l] + c;
        a[l] = v & kMask;
        c = v >> kW;
      }
      uint32_t cin = grp_from_prev<TPI>(c);
      if (bottom) cin = 0;
      a[0] += cin;  // at most one carry-propagation round per lane boundary
    }
  }
};

}  // namespace ddshe
