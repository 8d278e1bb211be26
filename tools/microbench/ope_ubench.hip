// OPE filter microbenchmark (tool, not product): shapes of the two-pass stable compaction
// (count pass + scatter pass) over a 10M-row int64 column with 1-byte valid flags, 50 % selectivity.
// (A single-pass decoupled look-back over agent-scope tile states was tried here and hung past 90 s on
// MI355X: spinning on a state another XCD published does not see it in time. Not retried.)
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
                                             uint32_t* __restrict__ counts, size_t tile0 = 0) {
  constexpr int G = ITEMS / 4;
  constexpr size_t TILE = (size_t)B * ITEMS;
  __shared__ uint32_t wsum[B / 64];
  const size_t tile = tile0 + blockIdx.x;
  const size_t t0 = tile * TILE + 4 * (size_t)threadIdx.x;
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
  masks[tile * (size_t)B + threadIdx.x] = m;
  uint32_t s = __builtin_popcount(m);
  for (int off = 32; off >= 1; off >>= 1) s += (uint32_t)__shfl_xor((int)s, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < B / 64; ++w) t += wsum[w];
    counts[tile] = t;
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
template <int B, int ITEMS, int PREFIX, int STORE = 0>
__global__ void __launch_bounds__(B) k_scatter(const uint32_t* __restrict__ masks, const uint32_t* __restrict__ counts,
                                               const uint64_t* __restrict__ offs, uint32_t* __restrict__ out,
                                               uint64_t* __restrict__ total, size_t tile0 = 0, size_t ntiles = 0) {
  constexpr int G = ITEMS / 4, NW = B / 64;
  constexpr size_t TILE = (size_t)B * ITEMS;
  __shared__ uint32_t wtot[G][NW];
  __shared__ uint64_t s_part[NW];
  __shared__ uint32_t sids[TILE];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  const size_t tile = tile0 + blockIdx.x;
  const size_t t0 = tile * TILE + 4 * (size_t)tid;
  const uint32_t mask = masks[tile * B + tid];
  uint64_t off = 0;
  if (STORE == 3) {  // floor: load the mask, store one word
    if (mask == 0xFFFFFFFFu && tid == 0) out[tile] = mask;
    if (tid == 0 && tile == (ntiles ? ntiles : gridDim.x) - 1) *total = 0;
    return;
  }
  if (STORE == 4) {  // floor + prefix of the earlier tiles' counts
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
    if (pre == 0x12345 || mask == 0xFFFFFFFFu) out[tile] = (uint32_t)pre;
    if (tid == 0 && tile == (ntiles ? ntiles : gridDim.x) - 1) *total = 0;
    return;
  }
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
  if (STORE == 0) {
    for (uint32_t k = tid; k < loc; k += B) o[k] = sids[k];
  } else if (STORE == 1) {
    for (uint32_t k = tid; k < loc; k += B) __builtin_nontemporal_store(sids[k], o + k);
  } else {  // compute only: one word per block
    if (tid == 0) o[0] = sids[0];
  }
  if (tid == 0 && tile == (ntiles ? ntiles : gridDim.x) - 1) *total = off + loc;
}

struct Bufs {
  int64_t* col;
  uint8_t* valid;
  uint32_t *masks, *counts, *out;
  uint64_t *offs, *total;
  size_t n;
  int64_t bound;
};

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



template <int B, int ITEMS, int PREFIX, int STORE = 0>
void run(const char* name, Bufs& b, const std::vector<uint32_t>& want, hipStream_t st) {
  constexpr size_t TILE = (size_t)B * ITEMS;
  const size_t nb = (b.n + TILE - 1) / TILE;
  auto once = [&]() {
    hipLaunchKernelGGL((k_count<B, ITEMS>), dim3(nb), dim3(B), 0, st, b.col, b.valid, b.n, b.bound, b.masks, b.counts);
    if (PREFIX) hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, b.counts, nb, b.offs);
    hipLaunchKernelGGL((k_scatter<B, ITEMS, PREFIX, STORE>), dim3(nb), dim3(B), 0, st, b.masks, b.counts, b.offs, b.out,
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
    hipLaunchKernelGGL((k_scatter<B, ITEMS, PREFIX, STORE>), dim3(nb), dim3(B), 0, st, b.masks, b.counts, b.offs, b.out,
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

// count and scatter in K chunks of tiles on two streams: the scatter of chunk c (stream B) runs while
// the count of chunk c+1 (stream A) streams the column
template <int B, int ITEMS, int K>
void run_pipe(Bufs& b, const std::vector<uint32_t>& want, hipStream_t sa, hipStream_t sb) {
  constexpr size_t TILE = (size_t)B * ITEMS;
  const size_t nb = (b.n + TILE - 1) / TILE;
  const size_t per = (nb + K - 1) / K;
  hipEvent_t ev[K], done;
  for (int c = 0; c < K; ++c) CK(hipEventCreateWithFlags(&ev[c], hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  auto once = [&]() {
    for (int c = 0; c < K; ++c) {
      const size_t t0 = c * per, cnt = t0 >= nb ? 0 : (nb - t0 < per ? nb - t0 : per);
      if (!cnt) break;
      hipLaunchKernelGGL((k_count<B, ITEMS>), dim3(cnt), dim3(B), 0, sa, b.col, b.valid, b.n, b.bound, b.masks, b.counts,
                         t0);
      CK(hipEventRecord(ev[c], sa));
      CK(hipStreamWaitEvent(sb, ev[c], 0));
      hipLaunchKernelGGL((k_scatter<B, ITEMS, 0>), dim3(cnt), dim3(B), 0, sb, b.masks, b.counts, b.offs, b.out, b.total,
                         t0, nb);
    }
    CK(hipEventRecord(done, sb));
    CK(hipStreamWaitEvent(sa, done, 0));
  };
  once();
  CK(hipStreamSynchronize(sa));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 50;
  CK(hipEventRecord(e0, sa));
  for (int r = 0; r < reps; ++r) once();
  CK(hipEventRecord(e1, sa));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  uint64_t tot = 0;
  CK(hipMemcpy(&tot, b.total, 8, hipMemcpyDeviceToHost));
  std::vector<uint32_t> got(tot);
  CK(hipMemcpy(got.data(), b.out, tot * 4, hipMemcpyDeviceToHost));
  const double bytes = 9.0 * b.n + 4.0 * want.size();
  printf("{\"variant\": \"pipe\", \"block\": %d, \"items\": %d, \"chunks\": %d, \"ms\": %.5f, \"GBps\": %.1f, \"ok\": %s}\n",
         B, ITEMS, K, ms, bytes / ms / 1e6, got == want ? "true" : "false");
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
    fflush(stdout);
    printf("{\"variant\": \"read_only\", \"ms\": %.5f, \"GBps\": %.1f}\n", ms / 50, 9.0 * n / (ms / 50) / 1e6);
  }
  run<256, 32, 0>("prefix", b, want, st);
  run<256, 32, 0, 1>("prefix_ntstore", b, want, st);
  run<256, 32, 0, 2>("prefix_nostore", b, want, st);
  run<256, 32, 0, 3>("floor_maskload", b, want, st);
  run<256, 32, 0, 4>("floor_plus_prefix", b, want, st);
  return 0;
}
