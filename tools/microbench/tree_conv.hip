// Reduction-tree convolution microbenchmark (tool, not product; VERDICT r02 "next" 3). One 1024-thread
// workgroup runs R column-sum convolutions (T = x * y, 2S columns, as Sos::conv in ddshe_tree.hip) back
// to back and records s_memtime per convolution: the mapping of work units to lanes (one chunk per
// wave, as in the product, vs. units flattened over all 1024 lanes), the chunk length C, and LDS
// atomics vs. none (sums kept in registers, to price the atomics). Checks every variant's columns
// against the host. Prints cycles per convolution.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tree_conv.hip -o tree_conv && ./tree_conv
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int NT = 1024;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// acc[col] += sum_i x[i] y[col - i]; x zero past S, y zero outside [0, S) (YL words before y[0])
template <int S, int C, bool FLAT, bool ATOM, bool EMPTY = false, bool FENCE = false>
__device__ __forceinline__ void conv(const uint32_t* __restrict__ x, const uint32_t* __restrict__ yz, uint64_t* acc,
                                     uint64_t& sink) {
  constexpr int NCH = (S + C - 1) / C;
  constexpr int BAND = (S + C + 2) / 4 + 1;
  constexpr int ncols = 2 * S, ncb = (ncols + 3) / 4;
  if (EMPTY) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nunits = FLAT ? NCH * BAND : NCH * ((BAND + 63) / 64);
  const int step = FLAT ? NT : NT / 64;
  for (int u = FLAT ? (int)threadIdx.x : wave; u < nunits; u += step) {
    int ch, cb;
    if (FLAT) {
      ch = u / BAND;
      cb = ch * C / 4 + (u - ch * BAND);
    } else {
      constexpr int NGR = (BAND + 63) / 64;
      ch = u / NGR;
      cb = ch * C / 4 + (u - ch * NGR) * 64 + lane;
    }
    const int i0 = ch * C;
    if (cb >= ncb || 4 * cb > i0 + C + S - 2) continue;
    const int base = 4 * cb - i0 - C;
    uint32_t ys[C + 4];
    const u32x4* yv = reinterpret_cast<const u32x4*>(__builtin_assume_aligned(yz, 16)) + (base >> 2);
#pragma unroll
    for (int q = 0; q < C + 4; q += 4) {
      u32x4 v = yv[q >> 2];
      if (FENCE) asm volatile("" : "+v"(v));  // one 128-bit LDS read (no per-word read2 with 8-way bank conflicts)
      ys[q] = v.x;
      ys[q + 1] = v.y;
      ys[q + 2] = v.z;
      ys[q + 3] = v.w;
    }
    uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int r4 = 0; r4 < C; r4 += 4) {
      const uint4 xv = reinterpret_cast<const uint4*>(__builtin_assume_aligned(x, 16))[(i0 + r4) >> 2];
      const uint32_t xr[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = r4 + q;
        c0 += (uint64_t)xr[q] * ys[C - r];
        c1 += (uint64_t)xr[q] * ys[C + 1 - r];
        c2 += (uint64_t)xr[q] * ys[C + 2 - r];
        c3 += (uint64_t)xr[q] * ys[C + 3 - r];
        if (FENCE) asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3));  // keep the 4 chains interleaved
      }
    }
    const int col = 4 * cb;
    if (ATOM) {
      if (c0) atomicAdd((unsigned long long*)&acc[col], (unsigned long long)c0);
      if (c1 && col + 1 < ncols) atomicAdd((unsigned long long*)&acc[col + 1], (unsigned long long)c1);
      if (c2 && col + 2 < ncols) atomicAdd((unsigned long long*)&acc[col + 2], (unsigned long long)c2);
      if (c3 && col + 3 < ncols) atomicAdd((unsigned long long*)&acc[col + 3], (unsigned long long)c3);
    } else {
      sink += c0 ^ (c1 << 1) ^ (c2 << 2) ^ (c3 << 3);
    }
  }
}

template <int S, int C, bool FLAT, bool ATOM, bool EMPTY = false, bool FENCE = false>
__global__ void __launch_bounds__(NT) k_bench(const uint32_t* gx, const uint32_t* gy, int R, uint64_t* out,
                                               uint64_t* cycles) {
  constexpr int YL = (C + 8 + 3) / 4 * 4;
  constexpr int NCH = (S + C - 1) / C;
  constexpr int XL = (NCH * C + 3) / 4 * 4;
  __shared__ __attribute__((aligned(16))) uint32_t sx[XL + 64], sy[YL + 2 * S + 64];
  __shared__ uint64_t acc[2 * S + 8];
  for (int j = threadIdx.x; j < XL + 64; j += NT) sx[j] = j < S ? gx[j] : 0u;
  for (int j = threadIdx.x; j < YL + 2 * S + 64; j += NT) {
    const int k = j - YL;
    sy[j] = (k >= 0 && k < S) ? gy[k] : 0u;
  }
  uint64_t sink = 0;
  __syncthreads();
  uint64_t t0 = 0;
  for (int r = 0; r < R; ++r) {
    for (int j = threadIdx.x; j < 2 * S + 8; j += NT) acc[j] = 0;
    __syncthreads();
    if (r == 1) t0 = __builtin_amdgcn_s_memtime();  // round 0 warms up
    conv<S, C, FLAT, ATOM, EMPTY, FENCE>(sx, sy + YL, acc, sink);
    __syncthreads();
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  for (int j = threadIdx.x; j < 2 * S; j += NT) out[j] = acc[j];
  if (!ATOM) out[2 * S + threadIdx.x] = sink;
  if (threadIdx.x == 0) cycles[0] = t1 - t0;
}

template <int S, int C, bool FLAT, bool ATOM, bool EMPTY = false, bool FENCE = false>
void run(const char* name, int R) {
  std::vector<uint32_t> x(S), y(S);
  srand(S);
  for (int i = 0; i < S; ++i) {
    x[i] = (uint32_t)rand() & ((1u << 26) - 1);
    y[i] = (uint32_t)rand() & ((1u << 26) - 1);
  }
  uint32_t *dx, *dy;
  uint64_t *dout, *dc;
  CK(hipMalloc(&dx, S * 4));
  CK(hipMalloc(&dy, S * 4));
  CK(hipMalloc(&dout, (2 * S + NT) * 8));
  CK(hipMalloc(&dc, 8));
  CK(hipMemcpy(dx, x.data(), S * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, y.data(), S * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL((k_bench<S, C, FLAT, ATOM, EMPTY, FENCE>), dim3(1), dim3(NT), 0, 0, dx, dy, R, dout, dc);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> out(2 * S);
  uint64_t cyc;
  CK(hipMemcpy(out.data(), dout, 2 * S * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost));
  bool ok = true;
  if (ATOM && !EMPTY)
    for (int c = 0; c < 2 * S; ++c) {
      uint64_t want = 0;
      for (int i = 0; i < S; ++i)
        if (c - i >= 0 && c - i < S) want += (uint64_t)x[i] * y[c - i];
      ok = ok && want == out[c];
    }
  printf("%-34s S=%d C=%2d: %7.0f cycles / conv %s\n", name, S, C, (double)cyc / (R - 1), ok ? "" : "MISMATCH");
  CK(hipFree(dx));
  CK(hipFree(dy));
  CK(hipFree(dout));
  CK(hipFree(dc));
}

int main() {
  const int R = 201;
  run<162, 12, false, true, true>("loop overhead only (zero + 2 barriers)", R);
  run<162, 12, false, true>("chunk per wave (product)", R);
  run<162, 12, false, true, false, true>("chunk per wave + chain fences", R);
  run<162, 12, true, true, false, true>("flattened + chain fences", R);
  run<162, 16, true, true, false, true>("flattened + chain fences", R);
  run<162, 8, true, true, false, true>("flattened + chain fences", R);
  run<86, 8, false, true, false, true>("chunk per wave + chain fences", R);
  run<86, 8, true, true, false, true>("flattened + chain fences", R);
  run<86, 4, true, true, false, true>("flattened + chain fences", R);
  run<162, 12, false, false>("chunk per wave, no atomics", R);
  run<162, 12, true, true>("flattened units", R);
  run<162, 8, true, true>("flattened units", R);
  run<162, 4, true, true>("flattened units", R);
  run<162, 16, true, true>("flattened units", R);
  run<162, 8, true, false>("flattened units, no atomics", R);
  run<86, 8, false, true>("chunk per wave (product)", R);
  run<86, 8, true, true>("flattened units", R);
  run<86, 4, true, true>("flattened units", R);
  return 0;
}
