#!/usr/bin/env python3
"""A/B tool (not product): copy the production ddshe_device.hpp / ddshe_fold.hpp into <outdir> with the row
chain of Mont::mul_col_chain rewritten for a prefetch depth D (limb blocks of the row requested D blocks
ahead) and the block loop unrolled by D + 1, so the ring of D + 1 block buffers rotates by renaming
instead of register moves. usage: make_depth_variant.py <outdir> <D>"""
import os
import re
import sys

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "dependable-data-storage-csd2017_amd", "csrc")
out, D = sys.argv[1], int(sys.argv[2])
os.makedirs(out, exist_ok=True)
dev = open(os.path.join(SRC, "ddshe_device.hpp")).read()
fold = open(os.path.join(SRC, "ddshe_fold.hpp")).read()

a = dev.index("  // Row-chained form of mul_col for the fold's row loop")
b = dev.index("  // a <- MonPro(a, B), B in LDS")
new = r'''  // Row-chained form of mul_col (A/B variant): prefetch depth kDepth, ring of kDepth + 1 block buffers
  static constexpr int kPF = (S % 4 == 0) ? 4 : 2;
  static constexpr int kDepth = AB_DEPTH;
  template <int N, class F>
  __device__ __forceinline__ static void sfor(F&& f) {
    if constexpr (N > 0) {
      sfor<N - 1>(f);
      f(std::integral_constant<int, N - 1>{});
    }
  }
  __device__ __forceinline__ static void load_blocks2(uint32_t (&pre)[kDepth][kPF], const uint32_t* __restrict__ X,
                                                      size_t stride, uint32_t row) {
    const uint32_t voff = row * 4u, sstride = (uint32_t)stride * 4u;
#pragma unroll
    for (int d = 0; d < kDepth; ++d) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (size_t)d * kPF * stride), (short)0,
                                                        (int)(kPF * sstride), 0x00020000);
#pragma unroll
      for (int q = 0; q < kPF; ++q) pre[d][q] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, q * sstride, 0);
    }
  }
  template <bool Narrow = false>
  __device__ __forceinline__ static void mul_col_chain(uint32_t (&a)[L], const uint32_t (&n)[L],
                                                       const uint32_t* __restrict__ X, size_t stride, uint32_t row,
                                                       uint32_t next, uint32_t (&pre)[kDepth][kPF], uint32_t n0,
                                                       bool top, bool bottom, int sin = S) {
    constexpr int PF = kPF, NB = S / PF, DD = kDepth, R = DD + 1, NMAIN = NB - DD;
    static_assert(S % PF == 0 && NB > DD, "S % PF");
    uint64_t t[L];
#pragma unroll
    for (int l = 0; l < L; ++l) t[l] = 0;
    const uint32_t voff = row * 4u, nvoff = next * 4u;
    const uint32_t sstride = (uint32_t)stride * 4u;
    auto block_rsrc = [&](int i) {
      const int bytes = (!Narrow || i < sin) ? (int)(PF * sstride) : 0;
      return __builtin_amdgcn_make_buffer_rsrc((void*)(X + (size_t)i * stride), (short)0, bytes, 0x00020000);
    };
    uint32_t buf[R][PF];
#pragma unroll
    for (int d = 0; d < DD; ++d)
#pragma unroll
      for (int q = 0; q < PF; ++q) buf[d][q] = pre[d][q];
    auto load = [&](uint32_t(&bb)[PF], int blk, uint32_t vo) {  // blk: block number (limbs blk*PF ..)
      const auto rs = block_rsrc(blk * PF);
#pragma unroll
      for (int q = 0; q < PF; ++q) bb[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, q * sstride, 0);
    };
    auto compute = [&](const uint32_t(&bb)[PF]) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        step(t, a, n, bb[q], n0, top);
        fence_t(t);
      }
    };
    int b = 0;
#pragma unroll 1
    for (; b + R <= NMAIN; b += R) {
      sfor<R>([&](auto j) {
        constexpr int J = decltype(j)::value;
        load(buf[(J + DD) % R], b + J + DD, voff);
        compute(buf[J]);
      });
    }
    sfor<NMAIN % R>([&](auto j) {
      constexpr int J = decltype(j)::value;
      load(buf[(J + DD) % R], b + J + DD, voff);
      compute(buf[J]);
    });
    sfor<DD>([&](auto j) {
      constexpr int J = decltype(j)::value;
      load(pre[J], J, nvoff);
      compute(buf[(NMAIN + J) % R]);
    });
    settle(t, a, bottom);
  }

'''
dev = dev[:a] + new + dev[b:]
if "#include <type_traits>" not in dev:
    dev = dev.replace("#pragma once", "#pragma once\n#include <type_traits>", 1)
fold = fold.replace("uint32_t pre[2][M::kPF];  // first limb blocks of the next row, requested one row ahead",
                    "uint32_t pre[M::kDepth][M::kPF];  // first limb blocks of the next row, requested one row ahead")
assert "pre[M::kDepth]" in fold
open(os.path.join(out, "ddshe_device.hpp"), "w").write("#define AB_DEPTH %d\n" % D + dev)
open(os.path.join(out, "ddshe_fold.hpp"), "w").write(fold)
for f in ("ddshe_launch.hpp", "ddshe_shapes.hpp"):
    open(os.path.join(out, f), "w").write(open(os.path.join(SRC, f)).read())
print("wrote", out, "depth", D)
