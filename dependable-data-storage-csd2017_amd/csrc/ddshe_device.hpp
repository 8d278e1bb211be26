// Device-side Montgomery arithmetic for the homomorphic aggregation engine (gfx950).
//
// Replaces the per-element BigInteger work of the reference fold loops:
//   HomoAdd.sum(acc, x, nsquare)   DDSRestServer.scala:423  (c1·c2 mod n²)
//   HomoMult.multiply(acc, x, pk)  DDSRestServer.scala:518  (c1·c2 mod n)
//
// Number representation:
//   * radix 2^W limbs held in 32-bit words ("rW", W = 28 up to 4142-bit moduli,
//     27 above). A modulus of B bits uses S >= ceil((B+2)/W) limbs so that
//     R = 2^(W·S) > 4N.
//   * the Montgomery accumulator t[] is kept as 64-bit LAZY sums: every limb
//     product is a single v_mad_u64_u32 (measured half-rate, the same rate as
//     v_add_co/v_addc — so carry-free accumulation halves the instruction
//     count vs. 32-bit limbs with carry chains). Per CIOS step a position gains
//     a·b + m·N < 2^(2W+1) + 2^(2W) (a almost normalised, < 2^(W+1)); over S
//     steps that stays < 2^64 when 1.5·S·2^(2W) < 2^64: S <= 170 at W = 28,
//     S <= 682 at W = 27 (checked by static_assert).
//   * a bignum is owned by a GROUP of TPI consecutive lanes; lane r holds limbs
//     [r·L, (r+1)·L), L = S/TPI. Per CIOS step the group exchanges two words
//     (the Montgomery quotient m, broadcast from lane 0, and the limb shifted
//     across the lane boundary) with DPP/ds_swizzle.
//   * values are kept < 2N and "almost normalised" (limbs < 2^(W+1)) between
//     Montgomery products; anything written to HBM is fully normalised
//     (limbs < 2^W). Canonical reduction to [0, N) happens once per result.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ddshe {


__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// ---- intra-group lane exchange -----------------------------------------------
// value of lane 0 of this lane's group
// (mov_dpp: every source lane is valid for quad_perm, so no "old" value is materialised)
template <int TPI>
__device__ __forceinline__ uint32_t grp_bcast0(uint32_t x) {
  if constexpr (TPI == 1) return x;
  else if constexpr (TPI == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xA0, 0xF, 0xF, false);  // quad_perm [0,0,2,2]
  else if constexpr (TPI == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x00, 0xF, 0xF, false);  // quad_perm [0,0,0,0]
  else if constexpr (TPI == 8) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x18);  // and_mask 0b11000
  else if constexpr (TPI == 16) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150, 0xF, 0xF, false);  // row_newbcast:0
  else {
    static_assert(TPI == 32, "TPI");
    // row_newbcast:0 gives every row its lane 0; row_bcast:15 then hands row 0's (row 2's) value,
    // now in its lane 15, to row 1 (row 3) — rows 0 and 2 keep theirs (row_mask 0b1010)
    const int r0 = __builtin_amdgcn_mov_dpp((int)x, 0x150, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(r0, r0, 0x142, 0xA, 0xF, false);
  }
}
// value of lane r+1; the group's top lane receives the value of a group's lane 0 (TPI <= 4: its own
// group's, quad_perm wraps; TPI 8: the next group's; TPI 16: 0 via bound_ctrl at the row end;
// TPI 32: wave_shl:1 crosses rows, lane 31 reads lane 32 (forced to 0 by the select: the next
// group may have exited), lane 63 gets 0 via bound_ctrl).
// Montgomery steps pass lo0 through this, and lo0 == 0 on every group's lane 0, so the top lane
// gets 0 without a select.
template <int TPI>
__device__ __forceinline__ uint32_t grp_from_next(uint32_t x) {
  if constexpr (TPI == 1) return 0u;
  else if constexpr (TPI == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  else if constexpr (TPI == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x39, 0xF, 0xF, false);  // [1,2,3,0]
  else if constexpr (TPI == 32) {
    const uint32_t v = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x130, 0xF, 0xF, true);  // wave_shl:1
    return (lane_id() & 31) == 31 ? 0u : v;
  }
  else return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x101, 0xF, 0xF, true);                          // row_shl:1
}
// value of lane r-1 (caller masks the group's bottom lane)
template <int TPI>
__device__ __forceinline__ uint32_t grp_from_prev(uint32_t x) {
  if constexpr (TPI == 1) return 0u;
  else if constexpr (TPI == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xA0, 0xF, 0xF, false);  // [0,0,2,2]
  else if constexpr (TPI == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x90, 0xF, 0xF, false);  // [0,0,1,2]
  else if constexpr (TPI == 32) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x138, 0xF, 0xF, true);  // wave_shr:1
  else return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xF, 0xF, true);                          // row_shr:1
}

// ---- Montgomery product on a lane group --------------------------------------
// QP ("quotient pipelining" modulus): the caller passes N~ = N·n0 instead of N, so that
// N~ ≡ -1 mod 2^W and the CIOS quotient is the low limb of t itself — no v_mul_lo on the
// step's dependent chain. Products are then correct mod N~, hence mod N (N | N~), with values
// < 2N~ (needs R > 4N~, i.e. W·S >= bits(N) + W + 2); a final product against N brings them
// back below 2N. Used by the latency-bound tree levels.
template <int S, int TPI, int W, bool QP = false>
struct Mont {
  static_assert(S % TPI == 0, "S must divide into TPI lanes");
  static constexpr int L = S / TPI;
  static constexpr int kW = W;
  static constexpr uint32_t kMask = (1u << W) - 1u;
  static_assert(L >= 2, "need at least two limbs per lane");
  static_assert(W == 27 || W == 28, "radix");
  // 1.5 * S * 2^(2W) < 2^64  <=>  3 * S < 2^(65 - 2W)
  static_assert(3ull * S < (1ull << (65 - 2 * W)), "lazy 64-bit accumulation bound");

  // One CIOS step with multiplier limb b: t = (t + a·b + m·N) / 2^W.
  __device__ __forceinline__ static void step(uint64_t (&t)[L], const uint32_t (&a)[L], const uint32_t (&n)[L],
                                              uint32_t b, uint32_t n0, bool top) {
    // pass 1: t += a*b, in place (no 64-bit temporaries live across the pass). The
    // quotient m depends only on limb 0, so it is issued first and its latency
    // (mul_lo -> and -> DPP) hides under the remaining L-1 mads.
#ifndef DDSHE_AB_M_LATE
    t[0] = (uint64_t)a[0] * b + t[0];
    const uint32_t m = grp_bcast0<TPI>((QP ? (uint32_t)t[0] : (uint32_t)t[0] * n0) & kMask);
#pragma unroll
    for (int l = 1; l < L; ++l) t[l] = (uint64_t)a[l] * b + t[l];
#else
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = (uint64_t)a[l] * b + t[l];
    const uint32_t m = grp_bcast0<TPI>(((uint32_t)t[0] * n0) & kMask);
#endif
    // pass 2: t = (t + m*N) / 2^W, shifting down one limb in place
    const uint64_t u0 = (uint64_t)m * n[0] + t[0];
    const uint32_t lo0 = (uint32_t)u0 & kMask;  // == 0 on the group's lane 0
    t[0] = (uint64_t)m * n[1] + (t[1] + (u0 >> kW));
#pragma unroll
    for (int l = 2; l < L; ++l) t[l - 1] = (uint64_t)m * n[l] + t[l];
    // top lane: lo0 of a group's lane 0, which is 0 (see grp_from_next) — no select needed
    (void)top;
    t[L - 1] = (uint64_t)grp_from_next<TPI>(lo0);
  }

  // 64-bit lazy sums -> almost-normalised limbs (< 2^(W+1)) in a[].
  __device__ __forceinline__ static void settle(const uint64_t (&t)[L], uint32_t (&a)[L], bool bottom) {
    uint64_t c = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const uint64_t v = t[l] + c;
      // early-clobber output: a[l] must not inherit the low half of the 64-bit pair v,
      // otherwise a[] ends up on even registers only and wastes ~L VGPRs
      asm volatile("v_and_b32 %0, %1, %2" : "=&v"(a[l]) : "v"((uint32_t)v), "v"(kMask));
      c = v >> kW;
    }
    uint32_t clo = grp_from_prev<TPI>((uint32_t)c & kMask);
    uint32_t chi = grp_from_prev<TPI>((uint32_t)(c >> kW));
    if (bottom) { clo = 0; chi = 0; }
    a[0] += clo;
    a[1] += chi;
  }

  // opaque register barrier: stops LLVM re-associating the u64 sums of consecutive
  // unrolled steps into mad(x,y,0)+add trees (extra registers and 64-bit adds)
  __device__ __forceinline__ static void fence_t(uint64_t (&t)[L]) {
#ifdef DDSHE_AB_NO_FENCE_T
    return;
#endif
#pragma unroll
    for (int l = 0; l < L; ++l) asm volatile("" : "+v"(t[l]));
  }
  // opaque redefinition of the 32-bit operands once per Montgomery product: stops LICM
  // from hoisting zext(a[l]) / zext(n[l]) out of the step loop as 64-bit values, which
  // would pin every operand to an even register and waste ~2L VGPRs
  __device__ __forceinline__ static void fence_ops(uint32_t (&a)[L], const uint32_t (&n)[L]) {
#ifdef DDSHE_AB_NO_FENCE_OPS
    return;
#endif
#pragma unroll
    for (int l = 0; l < L; ++l) asm volatile("" : "+v"(a[l]));
    if constexpr (TPI == 1) {  // N is wave-uniform: keep it in SGPRs (one SGPR operand per mad)
#pragma unroll
      for (int l = 0; l < L; ++l) asm volatile("" : "+s"(const_cast<uint32_t&>(n[l])));
    } else {
#pragma unroll
      for (int l = 0; l < L; ++l) asm volatile("" : "+v"(const_cast<uint32_t&>(n[l])));
    }
  }

  // a <- MonPro(a, B), B = column `row` of the limb-transposed matrix X (limb i at
  // X[i*stride + row]; fully normalised, value < 2N). X and stride are wave-uniform:
  // each block of PF limbs is read through a buffer descriptor whose base is
  // X + i*stride (SGPRs), voffset = 4*row, soffset = 4*q*stride — no per-lane 64-bit
  // address arithmetic in the loop.
  // FenceOps: see fence_ops. The single-product fold loop runs faster without it (the
  // operand redefinitions also pin the schedule; measured -6 % time at 2-block prefetch),
  // kernels with several products in sequence need it to stay spill-free.
  template <bool FenceOps = true>
  __device__ __forceinline__ static void mul_col(uint32_t (&a)[L], const uint32_t (&n)[L],
                                                 const uint32_t* __restrict__ X, size_t stride, uint32_t row,
                                                 uint32_t n0, bool top, bool bottom) {
    uint64_t t[L];
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = 0;
#ifdef DDSHE_AB_PF
    constexpr int PF = DDSHE_AB_PF;
#else
    constexpr int PF = (S % 4 == 0) ? 4 : 2;  // limbs per unrolled block = loads in flight
#endif
    static_assert(S % PF == 0 && S >= 2 * PF, "S % PF");
    const uint32_t voff = row * 4u;
    const uint32_t sstride = (uint32_t)stride * 4u;  // host guarantees PF*stride*4 < 2^32
    auto block_rsrc = [&](int i) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(X + (size_t)i * stride), (short)0, (int)(PF * sstride),
                                               0x00020000);
    };
#ifndef DDSHE_AB_SHALLOW_PF
    // two blocks in flight: limbs of block i+2 are requested while block i is computed
    // (one block = PF steps ~ 1.4k cycles per wave is short of an HBM miss under load)
    uint32_t bq[PF], bm[PF];
    {
      const auto rs0 = block_rsrc(0), rs1 = block_rsrc(PF);
#pragma unroll
      for (int q = 0; q < PF; ++q) bq[q] = __builtin_amdgcn_raw_buffer_load_b32(rs0, voff, q * sstride, 0);
#pragma unroll
      for (int q = 0; q < PF; ++q) bm[q] = __builtin_amdgcn_raw_buffer_load_b32(rs1, voff, q * sstride, 0);
    }
#pragma unroll 1
    for (int i = 0; i < S - 2 * PF; i += PF) {
      if constexpr (FenceOps) fence_ops(a, n);
      const auto rs = block_rsrc(i + 2 * PF);
      uint32_t bn[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) bn[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        step(t, a, n, bq[q], n0, top);
        fence_t(t);
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        bq[q] = bm[q];
        bm[q] = bn[q];
      }
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      step(t, a, n, bq[q], n0, top);
      fence_t(t);
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      step(t, a, n, bm[q], n0, top);
      fence_t(t);
    }
#else
    uint32_t bq[PF];
    {
      const auto rs = block_rsrc(0);
#pragma unroll
      for (int q = 0; q < PF; ++q) bq[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
    }
#pragma unroll 1
    for (int i = 0; i < S - PF; i += PF) {
      if constexpr (FenceOps) fence_ops(a, n);
      const auto rs = block_rsrc(i + PF);
      uint32_t bn[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) bn[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        step(t, a, n, bq[q], n0, top);
        fence_t(t);
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) bq[q] = bn[q];
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      step(t, a, n, bq[q], n0, top);
      fence_t(t);
    }
#endif
    settle(t, a, bottom);
  }

  // Row-chained form of mul_col for the fold's row loop: the first two limb blocks of `row` arrive
  // in `pre` (requested during the previous row), and the first two blocks of `next` are requested
  // during this row's last two blocks and returned in `pre`, so no row starts on an HBM miss.
  static constexpr int kPF = (S % 4 == 0) ? 4 : 2;
  __device__ __forceinline__ static void load_blocks2(uint32_t (&pre)[2][kPF], const uint32_t* __restrict__ X,
                                                      size_t stride, uint32_t row) {
    const uint32_t voff = row * 4u, sstride = (uint32_t)stride * 4u;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (size_t)d * kPF * stride), (short)0,
                                                        (int)(kPF * sstride), 0x00020000);
#pragma unroll
      for (int q = 0; q < kPF; ++q) pre[d][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
    }
  }
  // Narrow: X holds only its first `sin` limbs (sin a multiple of kPF, >= 2 kPF; a main-shape column
  // read in a wider shape): blocks from sin on get an empty descriptor, so their loads return 0
  template <bool Narrow = false>
  __device__ __forceinline__ static void mul_col_chain(uint32_t (&a)[L], const uint32_t (&n)[L],
                                                       const uint32_t* __restrict__ X, size_t stride, uint32_t row,
                                                       uint32_t next, uint32_t (&pre)[2][kPF], uint32_t n0,
                                                       bool top, bool bottom, int sin = S) {
    constexpr int PF = kPF;
    static_assert(S % PF == 0 && S >= 2 * PF, "S % PF");
    uint64_t t[L];
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = 0;
    const uint32_t voff = row * 4u;
    const uint32_t sstride = (uint32_t)stride * 4u;
    auto block_rsrc = [&](int i) {
      const int bytes = (!Narrow || i < sin) ? (int)(PF * sstride) : 0;
      return __builtin_amdgcn_make_buffer_rsrc((void*)(X + (size_t)i * stride), (short)0, bytes, 0x00020000);
    };
    uint32_t bq[PF], bm[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      bq[q] = pre[0][q];
      bm[q] = pre[1][q];
    }
#pragma unroll 1
    for (int i = 0; i < S - 2 * PF; i += PF) {
      const auto rs = block_rsrc(i + 2 * PF);
      uint32_t bn[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) bn[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        step(t, a, n, bq[q], n0, top);
        fence_t(t);
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        bq[q] = bm[q];
        bm[q] = bn[q];
      }
    }
    const uint32_t nvoff = next * 4u;
    {
      const auto rs = block_rsrc(0);
#pragma unroll
      for (int q = 0; q < PF; ++q) pre[0][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, nvoff, q * sstride, 0);
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      step(t, a, n, bq[q], n0, top);
      fence_t(t);
    }
    {
      const auto rs = block_rsrc(PF);
#pragma unroll
      for (int q = 0; q < PF; ++q) pre[1][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, nvoff, q * sstride, 0);
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      step(t, a, n, bm[q], n0, top);
      fence_t(t);
    }
    settle(t, a, bottom);
  }

  // a <- MonPro(a, B), B in LDS (limb i at lb[i], fully normalised, value < 2N). The TPI
  // lanes of a group read the same address (broadcast); group arrays sit S dwords apart.
  __device__ __forceinline__ static void mul_lds(uint32_t (&a)[L], const uint32_t (&n)[L], const uint32_t* lb,
                                                 uint32_t n0, bool top, bool bottom) {
    uint64_t t[L];
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = 0;
    constexpr int PF = (S % 4 == 0) ? 4 : 2;
    uint32_t bq[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) bq[q] = lb[q];
#pragma unroll 1
    for (int i = 0; i < S - PF; i += PF) {
      fence_ops(a, n);
      uint32_t bn[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) bn[q] = lb[i + PF + q];
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        step(t, a, n, bq[q], n0, top);
        fence_t(t);
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) bq[q] = bn[q];
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      step(t, a, n, bq[q], n0, top);
      fence_t(t);
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

  // Almost-normalised (limbs < 2^(W+1)) -> fully normalised (limbs < 2^W); value unchanged.
  // After one round only limb 0 of a lane can hold 2^W (its carry-in landed on 2^W - 1); further
  // rounds run only while some lane of the wave has that (wave-uniform test, almost never taken).
  __device__ __forceinline__ static void normalize(uint32_t (&a)[L], bool bottom) {
    for (int round = 0; round < TPI; ++round) {
      if (round > 0 && !__builtin_amdgcn_ballot_w64((a[0] >> kW) != 0u)) break;
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
