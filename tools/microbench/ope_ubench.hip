// OPE filter microbenchmark (tool, not product): shapes of the two-pass stable compaction
// (count pass + scatter pass) over a 10M-row int64 column with 1-byte valid flags, 50 % selectivity.
// Prints one line per variant: device ms per call (HIP events, 50 reps) and GB/s of algorithmic bytes
// (9 B per row + 4 B per match), and checks the row ids against a host compaction.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 ope_ubench.hip -o ope_ubench && ./ope_ubench
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

typedef long long i64x2 __attribute__((ext_vector_type(2)));

// count: thread owns ITEMS rows as ITEMS/4 groups of 4 consecutive rows, groups B*4 rows apart
template <int B, int ITEMS>
__global__ void __launch_bounds__(B) k_count(const int64_t* __restrict__ col, const uint8_t* __restrict__ valid,
                                             size_t n, int64_t bound, uint32_t* __restrict__ masks,
                                             uint32_t* __restrict__ counts) {
  constexpr int G = ITEMS / 4;
  constexpr size_t TILE = (size_t)B * ITEMS;
  __shared__ uint32_t wsum[B / 64];
  const size_t t0 = blockIdx.x * TILE + 4 * (size_t)threadIdx.x;
  int64_t c[ITEMS];
  uint32_t v[G];
  if (t0 + (G - 1) * 4 * B + 3 < n) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const size_t r = t0 + (size_t)k * 4 * B;
      const i64x2* p = reinterpret_cast<const i64x2*>(col + r);
      const i64x2 x = __builtin_nontemporal_load(p), y = __builtin_nontemporal_load(p + 1);
      c[4 * k] = x.x;
      c[4 * k + 1] = x.y;
      c[4 * k + 2] = y.x;
      c[4 * k + 3] = y.y;
      v[k] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(valid + r));
    }
  } else {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      uint32_t vk = 0;
      for (int j = 0; j < 4; ++j) {
        const size_t r = t0 + (size_t)k * 4 * B + j;
        const size_t i = r < n ? r : n - 1;
        c[4 * k + j] = col[i];
        vk |= (r < n ? (uint32_t)valid[i] : 0u) << (8 * j);
      }
      v[k] = vk;
    }
  }
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < G; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (((v[k] >> (8 * j)) & 0xFFu) && c[4 * k + j] > bound) m |= 1u << (4 * k + j);
  masks[blockIdx.x * (size_t)B + threadIdx.x] = m;
  uint32_t s = __builtin_popcount(m);
  for (int off = 32; off >= 1; off >>= 1) s += (uint32_t)__shfl_xor((int)s, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < B / 64; ++w) t += wsum[w];
    counts[blockIdx.x] = t;
  }
}

// exclusive scan of the tile counts in one block (variant "scan")
__global__ void __launch_bounds__(1024) k_scan(const uint32_t* __restrict__ counts, size_t nb, uint64_t* __restrict__ offs) {
  __shared__ uint64_t part[1024];
  const int tid = threadIdx.x;
  const size_t per = (nb + 1023) / 1024;
  uint64_t s = 0;
  for (size_t i = 0; i < per; ++i) {
    const size_t t = tid * per + i;
    if (t < nb) s += counts[t];
  }
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint64_t x = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  uint64_t run = tid ? part[tid - 1] : 0;
  for (size_t i = 0; i < per; ++i) {
    const size_t t = tid * per + i;
    if (t < nb) {
      offs[t] = run;
      run += counts[t];
    }
  }
  if (tid == 1023) offs[nb] = part[1023];
}

// scatter: PREFIX 0 = sum the counts of earlier tiles (8 independent loads per pass), 1 = read offs[tile]
template <int B, int ITEMS, int PREFIX>
__global__ void __launch_bounds__(B) k_scatter(const uint32_t* __restrict__ masks, const uint32_t* __restrict__ counts,
                                               const uint64_t* __restrict__ offs, uint32_t* __restrict__ out,
                                               uint64_t* __restrict__ total) {
  constexpr int G = ITEMS / 4, NW = B / 64;
  constexpr size_t TILE = (size_t)B * ITEMS;
  __shared__ uint32_t wtot[G][NW];
  __shared__ uint64_t s_part[NW];
  __shared__ uint32_t sids[TILE];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  const size_t tile = blockIdx.x;
  const size_t t0 = tile * TILE + 4 * (size_t)tid;
  const uint32_t mask = masks[tile * B + tid];
  uint64_t off = 0;
  if (PREFIX == 0) {
    uint64_t pre = 0;
    for (size_t base = 0; base < tile; base += 8 * B) {
      uint32_t cv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const size_t t = base + (size_t)q * B + tid;
        cv[q] = t < tile ? counts[t] : 0u;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) pre += cv[q];
    }
    for (int o = 32; o >= 1; o >>= 1) pre += (uint64_t)__shfl_xor((long long)pre, o);
    if (lane == 0) s_part[wid] = pre;
  }
  uint32_t below[G];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    uint32_t b = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t bal = __ballot((mask >> (4 * k + j)) & 1u);
      b += (uint32_t)__popcll(bal & lt);
      tot += (uint32_t)__popcll(bal);
    }
    below[k] = b;
    if (lane == 0) wtot[k][wid] = tot;
  }
  __syncthreads();
  if (PREFIX == 0) {
#pragma unroll
    for (int w = 0; w < NW; ++w) off += s_part[w];
  } else {
    off = offs[tile];
  }
  uint32_t loc = 0;
#pragma unroll
  for (int k = 0; k < G; ++k) {
    uint32_t pw = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      pw += (w < wid) ? wtot[k][w] : 0u;
      tot += wtot[k][w];
    }
    const uint32_t q = (mask >> (4 * k)) & 0xFu;
    uint32_t dst = loc + pw + below[k];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((q >> j) & 1u) sids[dst++] = (uint32_t)(t0 + (size_t)k * 4 * B + j);
    loc += tot;
  }
  __syncthreads();
  uint32_t* o = out + off;
  for (uint32_t k = tid; k < loc; k += B) o[k] = sids[k];
  if (tid == 0 && tile == gridDim.x - 1) *total = off + loc;
}

struct Bufs {
  int64_t* col;
  uint8_t* valid;
  uint32_t *masks, *counts, *out;
  uint64_t *offs, *total;
  size_t n;
  int64_t bound;
};

// single pass, decoupled look-back (variant "lookback"): tile state words packed (flag << 62 | value),
// flag 1 = aggregate, 2 = inclusive prefix, read and written with agent-scope atomics (coherent across
// the XCDs' L2s). Tiles are taken in blockIdx order; the host only launches it when every block of
// the grid is co-resident (occupancy x CUs), and a spin limit turns a lost wait into an error flag.
template <int B, int ITEMS>
__global__ void __launch_bounds__(B) k_lookback(const int64_t* __restrict__ col, const uint8_t* __restrict__ valid,
                                                size_t n, int64_t bound, uint64_t* __restrict__ state,
                                                uint32_t* __restrict__ out, uint64_t* __restrict__ total,
                                                uint32_t* __restrict__ err) {
  constexpr int G = ITEMS / 4, NW = B / 64;
  constexpr size_t TILE = (size_t)B * ITEMS;
  constexpr uint64_t kVal = (1ull << 62) - 1;
  __shared__ uint32_t wtot[G][NW];
  __shared__ uint32_t sids[TILE];
  __shared__ uint64_t s_excl;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  const size_t tile = blockIdx.x;
  const size_t t0 = tile * TILE + 4 * (size_t)tid;
  int64_t c[ITEMS];
  uint32_t v[G];
  if (t0 + (G - 1) * 4 * B + 3 < n) {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const size_t r = t0 + (size_t)k * 4 * B;
      const i64x2* p = reinterpret_cast<const i64x2*>(col + r);
      const i64x2 x = __builtin_nontemporal_load(p), y = __builtin_nontemporal_load(p + 1);
      c[4 * k] = x.x;
      c[4 * k + 1] = x.y;
      c[4 * k + 2] = y.x;
      c[4 * k + 3] = y.y;
      v[k] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(valid + r));
    }
  } else {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      uint32_t vk = 0;
      for (int j = 0; j < 4; ++j) {
        const size_t r = t0 + (size_t)k * 4 * B + j;
        const size_t i = r < n ? r : n - 1;
        c[4 * k + j] = col[i];
        vk |= (r < n ? (uint32_t)valid[i] : 0u) << (8 * j);
      }
      v[k] = vk;
    }
  }
  uint32_t mask = 0;
#pragma unroll
  for (int k = 0; k < G; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (((v[k] >> (8 * j)) & 0xFFu) && c[4 * k + j] > bound) mask |= 1u << (4 * k + j);
  uint32_t below[G];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    uint32_t bb = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t bal = __ballot((mask >> (4 * k + j)) & 1u);
      bb += (uint32_t)__popcll(bal & lt);
      tot += (uint32_t)__popcll(bal);
    }
    below[k] = bb;
    if (lane == 0) wtot[k][wid] = tot;
  }
  __syncthreads();
  uint32_t agg = 0;
#pragma unroll
  for (int k = 0; k < G; ++k)
#pragma unroll
    for (int w = 0; w < NW; ++w) agg += wtot[k][w];
  if (wid == 0) {
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&state[0], (2ull << 62) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0) s_excl = 0;
    } else {
      if (lane == 0) __hip_atomic_store(&state[tile], (1ull << 62) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint64_t excl = 0;
      long pos = (long)tile - 1;
      int spins = 0;
      for (;;) {
        const long i = pos - lane;
        uint64_t st = i >= 0 ? __hip_atomic_load(&state[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (2ull << 62);
        while (__ballot((st >> 62) == 0)) {
          if (++spins > (1 << 22)) {
            if (lane == 0) atomicOr(err, 1u);
            st = 2ull << 62;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if ((st >> 62) == 0) st = __hip_atomic_load(&state[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint64_t inc = __ballot((st >> 62) == 2);
        uint64_t val = st & kVal;
        if (inc) {
          const int k = __builtin_ctzll(inc);  // nearest predecessor holding an inclusive prefix
          if (lane > k) val = 0;
          for (int o = 32; o >= 1; o >>= 1) val += (uint64_t)__shfl_xor((long long)val, o);
          excl += val;
          break;
        }
        for (int o = 32; o >= 1; o >>= 1) val += (uint64_t)__shfl_xor((long long)val, o);
        excl += val;
        pos -= 64;
      }
      if (lane == 0) {
        __hip_atomic_store(&state[tile], (2ull << 62) | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_excl = excl;
      }
    }
  }
  uint32_t loc = 0;
#pragma unroll
  for (int k = 0; k < G; ++k) {
    uint32_t pw = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      pw += (w < wid) ? wtot[k][w] : 0u;
      tot += wtot[k][w];
    }
    const uint32_t q = (mask >> (4 * k)) & 0xFu;
    uint32_t dst = loc + pw + below[k];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((q >> j) & 1u) sids[dst++] = (uint32_t)(t0 + (size_t)k * 4 * B + j);
    loc += tot;
  }
  __syncthreads();
  const uint64_t off = s_excl;
  uint32_t* o = out + off;
  for (uint32_t k = tid; k < loc; k += B) o[k] = sids[k];
  if (tid == 0 && tile == gridDim.x - 1) *total = off + loc;
}

template <int B, int ITEMS>
void run_lookback(Bufs& b, const std::vector<uint32_t>& want, hipStream_t st, uint64_t* state, uint32_t* err) {
  constexpr size_t TILE = (size_t)B * ITEMS;
  const size_t nb = (b.n + TILE - 1) / TILE;
  int per_cu = 0, dev = 0, cus = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_lookback<B, ITEMS>, B, 0));
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  if ((size_t)per_cu * cus < nb) {
    printf("{\"variant\": \"lookback\", \"block\": %d, \"items\": %d, \"skipped\": \"%zu tiles > %d resident\"}\n", B,
           ITEMS, nb, per_cu * cus);
    return;
  }
  auto once = [&]() {
    CK(hipMemsetAsync(state, 0, nb * 8, st));
    hipLaunchKernelGGL((k_lookback<B, ITEMS>), dim3(nb), dim3(B), 0, st, b.col, b.valid, b.n, b.bound, state, b.out,
                       b.total, err);
  };
  CK(hipMemset(err, 0, 4));
  once();
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 50;
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) once();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  uint32_t he = 0;
  CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
  uint64_t tot = 0;
  CK(hipMemcpy(&tot, b.total, 8, hipMemcpyDeviceToHost));
  std::vector<uint32_t> got(tot);
  CK(hipMemcpy(got.data(), b.out, tot * 4, hipMemcpyDeviceToHost));
  const double bytes = 9.0 * b.n + 4.0 * want.size();
  printf("{\"variant\": \"lookback\", \"block\": %d, \"items\": %d, \"tiles\": %zu, \"resident\": %d, \"ms\": %.5f, "
         "\"GBps\": %.1f, \"ok\": %s, \"err\": %u}\n",
         B, ITEMS, nb, per_cu * cus, ms, bytes / ms / 1e6, got == want ? "true" : "false", he);
  fflush(stdout);
}

// reference stream: sum the column (achievable read rate of the same bytes)
__global__ void __launch_bounds__(256) k_read(const int64_t* __restrict__ col, const uint8_t* __restrict__ valid,
                                              size_t n, uint64_t* __restrict__ sink) {
  const size_t t0 = (blockIdx.x * 256 * (size_t)32) + 4 * (size_t)threadIdx.x;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const size_t r = t0 + (size_t)k * 1024;
    if (r + 3 < n) {
      const i64x2* p = reinterpret_cast<const i64x2*>(col + r);
      const i64x2 x = __builtin_nontemporal_load(p), y = __builtin_nontemporal_load(p + 1);
      s += x.x ^ x.y ^ y.x ^ y.y ^ __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(valid + r));
    }
  }
  if (s == 0x123456789ull) *sink = s;
}



template <int B, int ITEMS, int PREFIX>
void run(const char* name, Bufs& b, const std::vector<uint32_t>& want, hipStream_t st) {
  constexpr size_t TILE = (size_t)B * ITEMS;
  const size_t nb = (b.n + TILE - 1) / TILE;
  auto once = [&]() {
    hipLaunchKernelGGL((k_count<B, ITEMS>), dim3(nb), dim3(B), 0, st, b.col, b.valid, b.n, b.bound, b.masks, b.counts);
    if (PREFIX) hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, b.counts, nb, b.offs);
    hipLaunchKernelGGL((k_scatter<B, ITEMS, PREFIX>), dim3(nb), dim3(B), 0, st, b.masks, b.counts, b.offs, b.out,
                       b.total);
  };
  once();
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 50;
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) once();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  // the two passes timed alone (the scatter re-reads the masks and counts of the last call)
  float ms_count = 0, ms_scatter = 0;
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_count<B, ITEMS>), dim3(nb), dim3(B), 0, st, b.col, b.valid, b.n, b.bound, b.masks, b.counts);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms_count, e0, e1));
  if (PREFIX) hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, b.counts, nb, b.offs);
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_scatter<B, ITEMS, PREFIX>), dim3(nb), dim3(B), 0, st, b.masks, b.counts, b.offs, b.out,
                       b.total);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms_scatter, e0, e1));
  printf("  {\"count_ms\": %.5f, \"scatter_ms\": %.5f}\n", ms_count / reps, ms_scatter / reps);
  uint64_t tot = 0;
  CK(hipMemcpy(&tot, b.total, 8, hipMemcpyDeviceToHost));
  std::vector<uint32_t> got(tot);
  CK(hipMemcpy(got.data(), b.out, tot * 4, hipMemcpyDeviceToHost));
  const bool ok = got == want;
  const double bytes = 9.0 * b.n + 4.0 * want.size();
  printf("{\"variant\": \"%s\", \"block\": %d, \"items\": %d, \"tiles\": %zu, \"ms\": %.5f, \"GBps\": %.1f, \"ok\": %s}\n",
         name, B, ITEMS, nb, ms, bytes / ms / 1e6, ok ? "true" : "false");
  fflush(stdout);
}

int main() {
  const size_t n = 10000000;
  std::vector<int64_t> h(n);
  std::vector<uint8_t> hv(n, 1);
  uint64_t x = 88172645463325252ull;
  for (size_t i = 0; i < n; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    h[i] = (int64_t)(x >> 1) - (int64_t)(1ull << 62);
  }
  const int64_t bound = 0;
  std::vector<uint32_t> want;
  for (size_t i = 0; i < n; ++i)
    if (hv[i] && h[i] > bound) want.push_back((uint32_t)i);
  Bufs b;
  b.n = n;
  b.bound = bound;
  CK(hipMalloc(&b.col, n * 8));
  CK(hipMalloc(&b.valid, n));
  CK(hipMalloc(&b.masks, n / 2 + 65536));
  CK(hipMalloc(&b.counts, n / 64 + 4096));
  CK(hipMalloc(&b.offs, n / 32 + 8192));
  CK(hipMalloc(&b.out, n * 4));
  CK(hipMalloc(&b.total, 8));
  CK(hipMemcpy(b.col, h.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(b.valid, hv.data(), n, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  {  // read-only reference
    uint64_t* sink;
    CK(hipMalloc(&sink, 8));
    const size_t nb = (n + 8191) / 8192;
    hipLaunchKernelGGL(k_read, dim3(nb), dim3(256), 0, st, b.col, b.valid, n, sink);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 50; ++r) hipLaunchKernelGGL(k_read, dim3(nb), dim3(256), 0, st, b.col, b.valid, n, sink);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"variant\": \"read_only\", \"ms\": %.5f, \"GBps\": %.1f}\n", ms / 50, 9.0 * n / (ms / 50) / 1e6);
  }
  {
    uint64_t* state;
    uint32_t* err;
    CK(hipMalloc(&state, (n / 1024 + 64) * 8));
    CK(hipMalloc(&err, 4));
    run_lookback<256, 32>(b, want, st, state, err);
    run_lookback<256, 64>(b, want, st, state, err);
    run_lookback<512, 32>(b, want, st, state, err);
    run_lookback<1024, 16>(b, want, st, state, err);
  }
  run<256, 32, 0>("prefix", b, want, st);
  run<256, 32, 1>("scan", b, want, st);
  run<256, 16, 0>("prefix", b, want, st);
  run<256, 16, 1>("scan", b, want, st);
  run<128, 32, 0>("prefix", b, want, st);
  run<512, 32, 0>("prefix", b, want, st);
  run<512, 16, 1>("scan", b, want, st);
  run<1024, 16, 1>("scan", b, want, st);
  run<256, 8, 1>("scan", b, want, st);
  return 0;
}
