// OPE ordering (OrderLS / OrderSL, DDSRestServer.scala:541-606): stable LSD radix sort of the
// int64 OPE column (ciphertexts are Java Long, SJHomoLibProvider.scala:55; sort key
// `contents(position).toLong`, :562 / :595) carrying the row ids.
//   OrderLS: descending (`a > b`), rows lacking the position (`length-1 < position`) last;
//   OrderSL: ascending  (`a < b`), rows lacking the position first.
// scala's sortWith is a stable merge sort, so equal keys keep their input order: LSD radix with
// a stable per-tile rank reproduces that. Descending order sorts ~key (still stable for ties).
//
// Keys are offset by the smallest key of a holder (k_rs_prep / k_rs_red: min and max over the rows that
// hold the position), so only the bytes of (max - min) are sorted: ceil(bits(max - min) / 8) passes
// (an OPE column spanning 2^54 values needs 7, not 8). Per 8-bit digit pass (the last executed one
// has 257 buckets: the validity of the row moves it to the end / front): k_rs_hist (per-tile digit counts, digit-major) -> k_rs_scan_digits (per-digit
// scan over tiles, one block per digit, coalesced 1024-count chunks; the scatter blocks scan the 257
// digit totals themselves) -> k_rs_scatter (stable rank inside the tile: each wave walks a contiguous
// quarter of the tile, peers with equal digits are found with 9 ballots, per-wave digit counters in
// LDS; the ranked rows are staged in LDS in tile-local digit order and written out by consecutive
// threads, so a store instruction covers a few digit runs instead of 64 buckets). HBM traffic per
// pass: 8 B/row read by hist, 12 B/row read + 12 B/row written by scatter; the validity of a row
// rides in bit 31 of its id (no random gather of valid[] in the last pass).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ddshe_launch.hpp"

namespace ddshe {

constexpr int kRsBlock = 256;
constexpr int kRsWaves = kRsBlock / 64;
constexpr int kRsItems = 8;                       // rows per lane
constexpr size_t kRsTile = (size_t)kRsBlock * kRsItems;
constexpr int kRsDigits = 257;                    // 256 + the validity bucket of the last pass
constexpr uint32_t kRsNone = 511;                 // digit of a lane past the end (never counted)
constexpr uint64_t kSign = 0x8000000000000000ull;

// Sort key of a holder: its value in unsigned order (descending: complemented), minus the smallest
// such key (kmin). Rows lacking the position get key 0 so that earlier passes keep them in input
// order; the last pass moves them to their bucket (256 / 0). The first executed pass derives the keys
// from the column itself (no separate key buffer is written up front).
__device__ __forceinline__ uint64_t rs_ukey(uint64_t raw, int desc) {
  const uint64_t u = raw ^ kSign;  // signed order -> unsigned order
  return desc ? ~u : u;
}
__device__ __forceinline__ uint64_t rs_key_of(uint64_t raw, const uint8_t* __restrict__ valid, size_t i, int desc,
                                              uint64_t kmin) {
  return (valid && !valid[i]) ? 0ull : rs_ukey(raw, desc) - kmin;
}

// min / max of the holders' keys (per block, then k_rs_red): only the bytes of max - min are sorted.
// Reads the column once, writes nothing per row.
constexpr int kRsPrepRows = 16;  // rows per thread of k_rs_prep

__device__ __forceinline__ void rs_minmax_block(uint64_t lo, uint64_t hi, uint64_t* __restrict__ out) {
  __shared__ uint64_t slo[16], shi[16];
  for (int off = 32; off >= 1; off >>= 1) {
    lo = min(lo, (uint64_t)__shfl_xor((long long)lo, off));
    hi = max(hi, (uint64_t)__shfl_xor((long long)hi, off));
  }
  if ((threadIdx.x & 63) == 0) {
    slo[threadIdx.x >> 6] = lo;
    shi[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      lo = min(lo, slo[w]);
      hi = max(hi, shi[w]);
    }
    out[0] = min(lo, slo[0]);
    out[1] = max(hi, shi[0]);
  }
}

__global__ void __launch_bounds__(256) k_rs_prep(const int64_t* __restrict__ col, const uint8_t* __restrict__ valid,
                                                 size_t n, int desc, uint64_t* __restrict__ part) {
  uint64_t lo = ~0ull, hi = 0;
  const size_t base = (size_t)blockIdx.x * 256 * kRsPrepRows + threadIdx.x;
#pragma unroll 4
  for (int k = 0; k < kRsPrepRows; ++k) {
    const size_t i = base + (size_t)k * 256;
    if (i < n && (!valid || valid[i])) {
      const uint64_t key = rs_ukey((uint64_t)col[i], desc);
      lo = min(lo, key);
      hi = max(hi, key);
    }
  }
  rs_minmax_block(lo, hi, part + 2 * blockIdx.x);
}

// min / max of the per-block partials -> red[0..1] (one block; no holder at all: red[0] > red[1])
__global__ void __launch_bounds__(1024) k_rs_red(const uint64_t* __restrict__ part, size_t nparts,
                                                 uint64_t* __restrict__ red) {
  uint64_t lo = ~0ull, hi = 0;
  for (size_t i = threadIdx.x; i < nparts; i += 1024) {
    lo = min(lo, part[2 * i]);
    hi = max(hi, part[2 * i + 1]);
  }
  rs_minmax_block(lo, hi, red);
}

__global__ void k_rs_iota(uint32_t* __restrict__ ids, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ids[i] = (uint32_t)i;
}

// Row id as carried between passes. vbit (n <= 2^31): bit 31 holds "row lacks the position", set
// from a coalesced valid[i] read where the identity ids start, so the last pass reads it from the
// id instead of gathering valid[id] at random; the last pass strips it.
constexpr uint32_t kRsLack = 0x80000000u;
__device__ __forceinline__ uint32_t rs_load_id(const uint32_t* __restrict__ ids, size_t i,
                                               const uint8_t* __restrict__ valid, bool vbit) {
  if (ids) return ids[i];
  return (uint32_t)i | ((vbit && valid && !valid[i]) ? kRsLack : 0u);
}

__device__ __forceinline__ uint32_t rs_digit(uint64_t k, uint32_t id, const uint8_t* __restrict__ valid, int pass,
                                             bool last, int desc, bool vbit) {
  uint32_t d = (uint32_t)(k >> (8 * pass)) & 0xFFu;
  if (last && valid) {
    const bool v = vbit ? (id & kRsLack) == 0 : valid[id] != 0;
    d = desc ? (v ? d : 256u) : (v ? d + 1u : 0u);
  }
  return d;
}

// row of item k of a lane: each wave owns a contiguous quarter of the tile
__device__ __forceinline__ size_t rs_row(size_t tile, int wid, int k, int lane) {
  return tile * kRsTile + (size_t)wid * (kRsTile / kRsWaves) + (size_t)k * 64 + lane;
}

__global__ void __launch_bounds__(kRsBlock) k_rs_hist(const uint64_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ ids,
                                                      const uint8_t* __restrict__ valid, size_t n, int pass,
                                                      bool last, int desc, bool vbit, uint64_t kmin,
                                                      uint32_t* __restrict__ hist, size_t nblocks) {
  __shared__ uint32_t cnt[kRsDigits];
  for (int d = threadIdx.x; d < kRsDigits; d += kRsBlock) cnt[d] = 0;
  __syncthreads();
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  const bool need_id = last && valid;
  // all loads first (independent, in flight together), then the LDS counting
  uint64_t key[kRsItems];
  uint32_t id[kRsItems];
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {  // unconditional loads (index clamped), masked below
    const size_t i = min(rs_row(blockIdx.x, wid, k, lane), n - 1);
    key[k] = ids ? keys[i] : rs_key_of(keys[i], valid, i, desc, kmin);  // first pass: keys = the column
    id[k] = need_id ? rs_load_id(ids, i, valid, vbit) : 0u;
  }
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const size_t i = rs_row(blockIdx.x, wid, k, lane);
    const uint32_t d = i < n ? rs_digit(key[k], id[k], valid, pass, last, desc, vbit) : kRsNone;
    // one LDS atomic per distinct digit of the wave (OPE columns repeat digits a lot; measured
    // faster than per-wave histograms with one atomic per row)
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    if (d != kRsNone && (peers & lt) == 0) atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kRsDigits; d += kRsBlock) hist[(size_t)d * nblocks + blockIdx.x] = cnt[d];
}

// per digit d (one block each): exclusive scan of the tile counts hist[d][0..nblocks) in place,
// digit total -> dtot[d]. Chunks of 1024 counts: thread t owns counts 4t..4t+3 of a chunk (a wave's
// loads cover 1 KiB contiguous); up to kScanRegChunks chunks are loaded before any is scanned.
constexpr int kScanRegChunks = 8;
__global__ void __launch_bounds__(256) k_rs_scan_digits(uint32_t* __restrict__ hist, size_t nblocks,
                                                        uint32_t* __restrict__ dtot) {
  __shared__ uint32_t wtot[4];
  uint32_t* h = hist + (size_t)blockIdx.x * nblocks;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  uint32_t carry = 0;
  for (size_t c0 = 0; c0 < nblocks; c0 += (size_t)1024 * kScanRegChunks) {
    uint32_t v[kScanRegChunks][4];
#pragma unroll
    for (int c = 0; c < kScanRegChunks; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t b = c0 + (size_t)c * 1024 + 4 * tid + j;
        v[c][j] = b < nblocks ? h[b] : 0u;
      }
#pragma unroll
    for (int c = 0; c < kScanRegChunks; ++c) {
      if (c0 + (size_t)c * 1024 >= nblocks) break;  // block-uniform
      const uint32_t s = v[c][0] + v[c][1] + v[c][2] + v[c][3];
      uint32_t inc = s;
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, off);
        if (lane >= off) inc += y;
      }
      if (lane == 63) wtot[wid] = inc;
      __syncthreads();
      uint32_t run = carry + inc - s;
      for (int w = 0; w < wid; ++w) run += wtot[w];
      const uint32_t ctot = wtot[0] + wtot[1] + wtot[2] + wtot[3];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t b = c0 + (size_t)c * 1024 + 4 * tid + j;
        if (b < nblocks) h[b] = run;
        run += v[c][j];
      }
      carry += ctot;
    }
  }
  if (tid == 0) dtot[blockIdx.x] = carry;
}

// The ranked rows are first placed in tile-local digit order in LDS, then written out by
// consecutive threads: lanes of a store instruction hit consecutive addresses of a digit run
// (runs average kRsTile/256 = 16 rows), instead of 64 different buckets per store.
__global__ void __launch_bounds__(kRsBlock) k_rs_scatter(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ ids,
                                                         const uint8_t* __restrict__ valid, size_t n, int pass,
                                                         int desc, bool vbit, bool last, uint64_t kmin,
                                                         const uint32_t* __restrict__ hist,
                                                         const uint32_t* __restrict__ dtot, size_t nblocks,
                                                         uint64_t* __restrict__ keys_out,
                                                         uint32_t* __restrict__ ids_out) {
  __shared__ uint32_t cnt[kRsWaves][kRsDigits];
  __shared__ uint32_t dbase[kRsDigits + 1];   // global start of digit d, then of this tile's run of d
  __shared__ uint32_t lstart[kRsDigits + 1];  // tile-local start of digit d
  __shared__ uint64_t skey[kRsTile];
  __shared__ uint32_t sid[kRsTile];
  __shared__ uint16_t sdig[kRsTile];
  for (int d = threadIdx.x; d < kRsWaves * kRsDigits; d += kRsBlock) (&cnt[0][0])[d] = 0;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  // exclusive scan of kRsDigits values v(d) into out[] by one wave (5 digits per lane)
  auto wave_scan = [&](auto v_of, uint32_t* out) {
    uint32_t v[5], s = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int d = lane * 5 + q;
      v[q] = d < kRsDigits ? v_of(d) : 0u;
      s += v[q];
    }
    uint32_t inc = s;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, off);
      if (lane >= off) inc += y;
    }
    uint32_t run = inc - s;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int d = lane * 5 + q;
      if (d <= kRsDigits) out[d] = run;
      run += v[q];
    }
  };
  if (wid == 0) wave_scan([&](int d) { return dtot[d]; }, dbase);  // digit bases over all tiles
  __syncthreads();
  uint64_t key[kRsItems];
  uint32_t id[kRsItems], dr[kRsItems];  // dr = digit | rank << 9
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {  // all loads first, unconditional (index clamped), masked below
    const size_t i = min(rs_row(blockIdx.x, wid, k, lane), n - 1);
    key[k] = ids ? keys[i] : rs_key_of(keys[i], valid, i, desc, kmin);  // first pass: keys = the column
    id[k] = rs_load_id(ids, i, valid, vbit);  // ids == nullptr: first executed pass, identity
  }
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const size_t i = rs_row(blockIdx.x, wid, k, lane);
    dr[k] = i < n ? rs_digit(key[k], id[k], valid, pass, last, desc, vbit) : kRsNone;
  }
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const uint32_t d = dr[k];
    // lanes holding the same digit: AND of 9 bit-ballots (bit 8 only set in the last pass)
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    uint32_t rank = 0;
    if (d != kRsNone) {
      const uint32_t before = cnt[wid][d];  // every peer reads before the leader writes (wave order)
      rank = before + (uint32_t)__popcll(peers & lt);
      if ((peers & lt) == 0) cnt[wid][d] = before + (uint32_t)__popcll(peers);
    }
    dr[k] = d | (rank << 9);
  }
  __syncthreads();
  if (wid == 0) wave_scan([&](int d) { return cnt[0][d] + cnt[1][d] + cnt[2][d] + cnt[3][d]; }, lstart);
  __syncthreads();
  // cnt[w][d] <- tile-local start of wave w's rows of digit d; dbase[d] <- global start of the tile's run
  for (int d = threadIdx.x; d < kRsDigits; d += kRsBlock) {
    uint32_t run = lstart[d];
    for (int w = 0; w < kRsWaves; ++w) {
      const uint32_t c = cnt[w][d];
      cnt[w][d] = run;
      run += c;
    }
    dbase[d] += hist[(size_t)d * nblocks + blockIdx.x];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const uint32_t d = dr[k] & 511u;
    if (d == kRsNone) continue;
    const uint32_t lp = cnt[wid][d] + (dr[k] >> 9);
    if (keys_out) skey[lp] = key[k];
    sid[lp] = (last && vbit) ? (id[k] & ~kRsLack) : id[k];
    sdig[lp] = (uint16_t)d;
  }
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * kRsTile;
  const uint32_t rows = (uint32_t)min(kRsTile, n - t0);
  for (uint32_t q = threadIdx.x; q < rows; q += kRsBlock) {
    const uint32_t d = sdig[q];
    const uint32_t dst = dbase[d] + (q - lstart[d]);
    if (keys_out) keys_out[dst] = skey[q];
    ids_out[dst] = sid[q];
  }
}

size_t rs_blocks(size_t n) { return (n + kRsTile - 1) / kRsTile; }
size_t rs_scratch_bytes(size_t n) {
  // keys x2 (8 B), ids x1 extra (4 B; the other id buffer is the caller's output), histogram, OR/AND
  return 2 * n * 8 + n * 4 + (size_t)kRsDigits * (rs_blocks(n) + 2) * 4 + 1024 +
         16 * ((n + 256 * kRsPrepRows - 1) / (256 * kRsPrepRows));
}

hipError_t launch_ope_order(const int64_t* col, const uint8_t* valid, size_t n, int desc, void* scratch,
                            uint32_t* out_ids, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const size_t nb = rs_blocks(n);
  uint64_t* ka = (uint64_t*)scratch;
  uint64_t* kb = ka + n;
  uint32_t* ib = (uint32_t*)(kb + n);
  uint32_t* hist = (uint32_t*)(((uintptr_t)(ib + n) + 255) & ~(uintptr_t)255);
  uint32_t* dtot = hist + (size_t)kRsDigits * nb;
  uint64_t* red = (uint64_t*)(((uintptr_t)(dtot + kRsDigits) + 15) & ~(uintptr_t)15);
  uint64_t* part = red + 2;
  const size_t pb = (n + 256 * kRsPrepRows - 1) / (256 * kRsPrepRows);
  hipLaunchKernelGGL(k_rs_prep, dim3((unsigned)pb), dim3(256), 0, st, col, valid, n, desc, part);
  hipLaunchKernelGGL(k_rs_red, dim3(1), dim3(1024), 0, st, part, pb, red);
  uint64_t hred[2];
  hipError_t e = hipMemcpyAsync(hred, red, sizeof(hred), hipMemcpyDeviceToHost, st);
  if (e != hipSuccess) return e;
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
  // the bytes of max - min (at least one pass when rows may lack the position: its last pass buckets them)
  const uint64_t kmin = hred[0] <= hred[1] ? hred[0] : 0ull;
  const uint64_t span = hred[0] <= hred[1] ? hred[1] - hred[0] : 0ull;
  int passes[8], np = 0;
  for (int p = 0; p < 8 && (span >> (8 * p)) != 0; ++p) passes[np++] = p;
  if (np == 0 && valid) passes[np++] = 0;
  if (np == 0) {
    hipLaunchKernelGGL(k_rs_iota, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out_ids, n);
    return hipGetLastError();
  }
  // executed pass j writes ids to out_ids when (np-1-j) is even, so the last one lands there
  const uint32_t* ids_in = nullptr;  // identity before the first pass
  const uint64_t* kin = (const uint64_t*)col;  // raw column before the first pass
  uint64_t* kout = ka;
  for (int j = 0; j < np; ++j) {
    const int pass = passes[j];
    uint32_t* ids_out = ((np - 1 - j) % 2 == 0) ? out_ids : ib;
    const bool last = j == np - 1;
    const bool vbit = valid && n <= (size_t)kRsLack;
    hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)nb), dim3(kRsBlock), 0, st, kin, ids_in, valid, n, pass, last, desc,
                       vbit, kmin, hist, nb);
    hipLaunchKernelGGL(k_rs_scan_digits, dim3(kRsDigits), dim3(256), 0, st, hist, nb, dtot);
    hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)nb), dim3(kRsBlock), 0, st, kin, ids_in, valid, n, pass, desc,
                       vbit, last, kmin, hist, dtot, nb, last ? nullptr : kout, ids_out);
    kin = kout;
    kout = kout == ka ? kb : ka;
    ids_in = ids_out;
  }
  return hipGetLastError();
}

}  // namespace ddshe
