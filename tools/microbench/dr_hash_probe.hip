// Distinct-key hash set insertion rate on gfx950 (tool, not product): 10M int64 rows drawing from D
// distinct keys, inserted into one global open-addressing table (2^17 slots) by every row. Variants:
//   0: plain load of the slot first, CAS only when it reads empty (stale L2 lines of other XCDs may
//      read empty: the CAS then answers),
//   1: CAS on every probe,
//   2: wave-level dedup first (lanes with the key of a lower lane skip), then as 0.
// Reports ms per pass and the distinct count found (must equal D).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

constexpr int kBits = 17;
constexpr uint32_t kSlots = 1u << kBits;
constexpr uint64_t kEmpty = ~0ull;

__device__ __forceinline__ uint32_t hsh(uint64_t u) { return (uint32_t)((u * 0x9E3779B97F4A7C15ull) >> (64 - kBits)); }

template <int V>
__global__ void __launch_bounds__(256) k_ins(const uint64_t* __restrict__ keys, size_t n, uint64_t* T, uint32_t* cnt) {
  constexpr int R = 8;
  const size_t base = (size_t)blockIdx.x * 256 * R + threadIdx.x;
  uint64_t u[R];
#pragma unroll
  for (int k = 0; k < R; ++k) u[k] = keys[min(base + (size_t)k * 256, n - 1)];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    if (base + (size_t)k * 256 >= n) continue;
    if (V == 2) {  // skip when a lower lane of the wave holds the same key
      const int lane = threadIdx.x & 63;
      bool dup = false;
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t v = (uint64_t)__shfl((long long)u[k], lane ^ o);
        if ((lane ^ o) < lane && v == u[k]) dup = true;
      }
      if (dup) continue;
    }
    uint32_t h = hsh(u[k]);
    for (int p = 0; p < 64; ++p) {
      uint64_t v = (V == 1) ? kEmpty : T[h];
      if (v == u[k]) break;
      if (v == kEmpty) {
        const uint64_t old = atomicCAS((unsigned long long*)&T[h], (unsigned long long)kEmpty, (unsigned long long)u[k]);
        if (old == kEmpty) {
          atomicAdd(cnt, 1u);
          break;
        }
        if (old == u[k]) break;
      }
      h = (h + 1) & (kSlots - 1);
    }
  }
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? atoll(argv[1]) : 10000000;
  const int D = argc > 2 ? atoi(argv[2]) : 10000;
  std::vector<uint64_t> vals(D), rows(n);
  srand(5);
  for (int i = 0; i < D; ++i) vals[i] = ((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 11) ^ (uint64_t)rand();
  for (size_t i = 0; i < n; ++i) rows[i] = vals[(size_t)rand() % D];
  uint64_t *dk, *T;
  uint32_t* cnt;
  hipMalloc(&dk, n * 8);
  hipMalloc(&T, kSlots * 8);
  hipMalloc(&cnt, 4);
  hipMemcpy(dk, rows.data(), n * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const unsigned grid = (unsigned)((n + 2047) / 2048);
  for (int v = 0; v < 3; ++v) {
    std::vector<float> ts;
    uint32_t got = 0;
    for (int r = 0; r < 6; ++r) {
      hipMemset(T, 0xFF, kSlots * 8);
      hipMemset(cnt, 0, 4);
      hipEventRecord(a);
      if (v == 0) hipLaunchKernelGGL(k_ins<0>, dim3(grid), dim3(256), 0, 0, dk, n, T, cnt);
      if (v == 1) hipLaunchKernelGGL(k_ins<1>, dim3(grid), dim3(256), 0, 0, dk, n, T, cnt);
      if (v == 2) hipLaunchKernelGGL(k_ins<2>, dim3(grid), dim3(256), 0, 0, dk, n, T, cnt);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ts.push_back(ms);
      hipMemcpy(&got, cnt, 4, hipMemcpyDeviceToHost);
    }
    std::sort(ts.begin(), ts.end());
    printf("variant %d: median %.4f ms min %.4f ms, distinct %u (want %d)\n", v, ts[ts.size() / 2], ts[0], got, D);
  }
  return 0;
}
