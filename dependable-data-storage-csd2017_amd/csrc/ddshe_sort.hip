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
// has 257 buckets: the validity of the row moves it to the end / front): k_rs_hist (per-tile digit counts, tile-major) -> k_rs_scan_tiles +
// k_rs_scan_chunks (per-digit scan over tiles in chunks of 64 tiles; the scatter blocks scan the 257
// digit totals themselves) -> k_rs_scatter (stable rank inside the tile: each wave walks a contiguous
// quarter of the tile, peers with equal digits are found with 9 ballots, per-wave digit counters in
// LDS; the ranked rows are staged in LDS in tile-local digit order and written out by consecutive
// threads, so a store instruction covers a few digit runs instead of 64 buckets). HBM traffic per
// pass: 8 B/row read by hist, 12 B/row read + 12 B/row written by scatter; the validity of a row
// rides in bit 31 of its id (no random gather of valid[] in the last pass).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

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

// the same over rows one at a time (a column not 16-byte aligned, or valid bytes at an odd address)
__global__ void __launch_bounds__(256) k_rs_prep_rows(const int64_t* __restrict__ col, const uint8_t* __restrict__ valid,
                                                      size_t n, int desc, uint64_t* __restrict__ part) {
  uint64_t lo = ~0ull, hi = 0;
  const size_t base = (size_t)blockIdx.x * 256 * kRsPrepRows + threadIdx.x;
  int64_t raw[kRsPrepRows];
  uint8_t hold[kRsPrepRows];
#pragma unroll
  for (int k = 0; k < kRsPrepRows; ++k) {
    const size_t i = min(base + (size_t)k * 256, n - 1);
    raw[k] = col[i];
    hold[k] = valid ? valid[i] : 1;
  }
#pragma unroll
  for (int k = 0; k < kRsPrepRows; ++k) {
    if (base + (size_t)k * 256 < n && hold[k]) {
      const uint64_t key = rs_ukey((uint64_t)raw[k], desc);
      lo = min(lo, key);
      hi = max(hi, key);
    }
  }
  rs_minmax_block(lo, hi, part + 2 * blockIdx.x);
}

__global__ void __launch_bounds__(256) k_rs_prep(const int64_t* __restrict__ col, const uint8_t* __restrict__ valid,
                                                 size_t n, int desc, uint64_t* __restrict__ part) {
  uint64_t lo = ~0ull, hi = 0;
  // rows in pairs: a wave instruction reads 64 consecutive 16-byte key pairs (and their 2 valid bytes);
  // all loads first (unconditional, index clamped: no load waits on a valid byte), then the min/max
  constexpr int P = kRsPrepRows / 2;
  const size_t base = (size_t)blockIdx.x * 256 * kRsPrepRows;
  const size_t npair = n / 2;  // whole pairs; an odd last row is read on its own
  ulonglong2 kv[P];
  uint16_t hv[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const size_t q = min(base / 2 + (size_t)k * 256 + threadIdx.x, npair ? npair - 1 : 0);
    kv[k] = npair ? reinterpret_cast<const ulonglong2*>(col)[q] : make_ulonglong2(0, 0);
    hv[k] = (valid && npair) ? reinterpret_cast<const uint16_t*>(valid)[q] : (uint16_t)0x0101;
  }
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const size_t q = base / 2 + (size_t)k * 256 + threadIdx.x;
    if (q < npair) {
      if (hv[k] & 0xFFu) {
        const uint64_t key = rs_ukey(kv[k].x, desc);
        lo = min(lo, key);
        hi = max(hi, key);
      }
      if (hv[k] >> 8) {
        const uint64_t key = rs_ukey(kv[k].y, desc);
        lo = min(lo, key);
        hi = max(hi, key);
      }
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0 && (!valid || valid[n - 1])) {  // odd last row
    const uint64_t key = rs_ukey((uint64_t)col[n - 1], desc);
    lo = min(lo, key);
    hi = max(hi, key);
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

__device__ __forceinline__ uint32_t rs_digit(uint64_t k, uint32_t id, const uint8_t* __restrict__ valid, int shift,
                                             bool last, int desc, bool vbit) {
  uint32_t d = (uint32_t)(k >> shift) & 0xFFu;
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
                                                      const uint8_t* __restrict__ valid, size_t n, int shift,
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
    const uint32_t d = i < n ? rs_digit(key[k], id[k], valid, shift, last, desc, vbit) : kRsNone;
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
  for (int d = threadIdx.x; d < kRsDigits; d += kRsBlock) hist[(size_t)blockIdx.x * kRsDigits + d] = cnt[d];  // 1 KiB, coalesced
}

// Tile counts are tile-major (hist[tile][digit]: each histogram block writes 1 KiB in one go; the
// digit-major layout cost one 32-byte sector per 4-byte count, 8x the bytes, PMC round 2). The
// exclusive scan over tiles per digit then runs in two steps:
//   k_rs_scan_tiles: one block per chunk of kScanTiles tiles, one thread per digit: the chunk's
//     counts of that digit (coalesced rows across the digit threads) are replaced in place by their
//     exclusive prefix within the chunk, and the chunk total goes to ctot[chunk][digit];
//   k_rs_scan_chunks: one block, one thread per digit: exclusive prefix of the chunk totals in place,
//     digit total -> dtot[digit].
// A tile's offset for digit d is then dbase[d] + ctot[chunk][d] + hist[tile][d] (k_rs_scatter).
constexpr int kScanTiles = 64;
constexpr int kScanThreads = 320;  // >= kRsDigits
__global__ void __launch_bounds__(kScanThreads) k_rs_scan_tiles(uint32_t* __restrict__ hist, size_t nblocks,
                                                                uint32_t* __restrict__ ctot) {
  const int d = threadIdx.x;
  if (d >= kRsDigits) return;
  const size_t t0 = (size_t)blockIdx.x * kScanTiles;
  uint32_t v[kScanTiles];
#pragma unroll
  for (int r = 0; r < kScanTiles; ++r) v[r] = t0 + r < nblocks ? hist[(t0 + r) * kRsDigits + d] : 0u;
  uint32_t run = 0;
#pragma unroll
  for (int r = 0; r < kScanTiles; ++r) {
    if (t0 + r < nblocks) hist[(t0 + r) * kRsDigits + d] = run;
    run += v[r];
  }
  ctot[(size_t)blockIdx.x * kRsDigits + d] = run;
}

__global__ void __launch_bounds__(kScanThreads) k_rs_scan_chunks(uint32_t* __restrict__ ctot, size_t nchunks,
                                                                 uint32_t* __restrict__ dtot) {
  const int d = threadIdx.x;
  if (d >= kRsDigits) return;
  uint32_t run = 0;
  for (size_t c0 = 0; c0 < nchunks; c0 += 16) {
    uint32_t v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = c0 + q < nchunks ? ctot[(c0 + q) * kRsDigits + d] : 0u;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (c0 + q < nchunks) ctot[(c0 + q) * kRsDigits + d] = run;
      run += v[q];
    }
  }
  dtot[d] = run;
}

// The ranked rows are first placed in tile-local digit order in LDS, then written out by
// consecutive threads: lanes of a store instruction hit consecutive addresses of a digit run
// (runs average kRsTile/256 = 16 rows), instead of 64 different buckets per store.
__global__ void __launch_bounds__(kRsBlock) k_rs_scatter(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ ids,
                                                         const uint8_t* __restrict__ valid, size_t n, int shift,
                                                         int desc, bool vbit, bool last, uint64_t kmin,
                                                         const uint32_t* __restrict__ hist,
                                                         const uint32_t* __restrict__ ctot,
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
    dr[k] = i < n ? rs_digit(key[k], id[k], valid, shift, last, desc, vbit) : kRsNone;
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
    dbase[d] += ctot[(size_t)(blockIdx.x / kScanTiles) * kRsDigits + d] + hist[(size_t)blockIdx.x * kRsDigits + d];
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

// ---- MSD split + in-bucket sort (OPE columns whose key span needs > 3 LSD passes) ----------------
// Two stable LSD passes over the TOP 16 bits of the span group the rows by those bits (65,536
// buckets), each bucket in input order. Each bucket with two distinct keys is then put in its final
// order, one wave per bucket (k_msd_local):
//   * stable partition by distinct key: round r writes, in input order, the rows whose key is the
//     r-th smallest of the bucket (ballot compaction) and finds the next smallest; a bucket of one key
//     is a single copy round. OPE columns repeat values (the generator's plaintexts are < 10^4), so
//     their buckets hold a few distinct keys however many rows they have.
//   * when a bucket needs more rounds (2 for <= 512 rows, 16 above): a bitonic network over the packed
//     value (rest of the key << pos bits | position in the bucket), unique, so the unstable network
//     yields the stable order: one wave in registers up to 512 rows (<= 8 per lane), one 1024-thread
//     workgroup up to 8192 rows (k_msd_big, 8 per thread, partners in other waves through LDS);
//   * a bucket of > 8192 rows with > 16 distinct keys raises a flag and the host redoes the sort with
//     the LSD passes (never seen on OPE data: it needs > 16 distinct keys among > 8192 rows whose
//     keys agree on the top 16 bits of the span).
// The last top pass writes each id to its final place if its bucket holds one key (OPE columns:
// most buckets); a multi-key bucket's wave first copies its ids to the first pass's (now free) id
// buffer and reads them from there, so nothing is sorted in place.
// Bucket bounds come from one pass over the sorted keys (k_msd_bounds: the first and the last row of
// every non-empty bucket and whether it holds two distinct keys); only those buckets are touched.
// Per row: 2 LSD passes + 8 B of bounds read, and for rows of multi-key buckets a 4 B id copy plus
// (8 B key + 4 B id read, 4 B id written) per partition round or sort, against
// ceil(bits(span) / 8) LSD passes (7 for a 2^54 span).
constexpr int kMsdBits = 16;
constexpr uint32_t kMsdBuckets = 1u << kMsdBits;
constexpr uint32_t kMsdWaveMax = 512;
constexpr uint32_t kMsdBlockMax = 8192;
constexpr int kMsdBigBlocks = 256;  // grid of the block path (grid-stride over the big buckets; one per CU:
                                     // a launch that finds no big bucket costs its dispatch, 13 us at 512)
enum { kMsdCtlBig = 0, kMsdCtlOverflow = 1 };

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

// Ascending bitonic sort of G*E values, element e = t*E + r held by thread t in v[r]. Partners at
// distance j < E are in the same thread, E <= j < 64E in the same wave (lane xor j/E), j >= 64E in
// another wave: exchanged through xch (r-major, G*E slots; only when G > 64).
template <int E, int LOGP, int G>
__device__ __forceinline__ void bitonic(uint64_t (&v)[E], int t, uint64_t* xch) {
#pragma unroll
  for (int kk = 1; kk <= LOGP; ++kk) {
#pragma unroll
    for (int jj = kk - 1; jj >= 0; --jj) {
      const int k = 1 << kk, j = 1 << jj;
      if (j < E) {
#pragma unroll
        for (int r = 0; r < E; ++r) {
          if ((r & j) == 0) {
            const bool up = ((t * E + r) & k) == 0;
            const uint64_t a = v[r], b = v[r | j];
            const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
            v[r] = up ? lo : hi;
            v[r | j] = up ? hi : lo;
          }
        }
      } else {
        uint64_t p[E];
        if (j < 64 * E) {
#pragma unroll
          for (int r = 0; r < E; ++r) p[r] = shfl_xor_u64(v[r], j / E);
        } else {
          __syncthreads();  // the previous exchange's reads are done
#pragma unroll
          for (int r = 0; r < E; ++r) xch[r * G + t] = v[r];
          __syncthreads();
#pragma unroll
          for (int r = 0; r < E; ++r) p[r] = xch[r * G + (t ^ (j / E))];
        }
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const int e = t * E + r;
          const bool take_min = ((e & j) == 0) == ((e & k) == 0);
          const uint64_t a = v[r], b = p[r];
          v[r] = take_min ? (a < b ? a : b) : (a < b ? b : a);
        }
      }
    }
  }
}

__device__ __forceinline__ uint32_t msd_bucket_of(uint64_t key, int s1) { return (uint32_t)(key >> s1); }

// Holder range of the sorted rows: the last (validity) pass put the rows lacking the position in
// bucket 256 (descending: at the end) or 0 (ascending: in front).
__device__ __forceinline__ void msd_holders(const uint32_t* __restrict__ dtot, size_t n, int desc, bool has_valid,
                                            size_t* h0, size_t* h1) {
  *h0 = 0;
  *h1 = n;
  if (has_valid) {
    if (desc) *h1 = n - dtot[256];
    else *h0 = dtot[0];
  }
}

// first[b] / end[b]: first row / one past the last row of non-empty bucket b (read only where multi[b]);
// multi[b] = 1 when bucket b holds two distinct keys (preset to 0). Neighbouring keys come from the
// adjacent lanes; 4 rows per thread (loads in flight together); block 0 also clears the control words.
constexpr int kMsdBoundsRows = 4;
__global__ void __launch_bounds__(256) k_msd_bounds(const uint64_t* __restrict__ keys, size_t n, int s1,
                                                    const uint32_t* __restrict__ dtot, int desc, bool has_valid,
                                                    uint32_t* __restrict__ first, uint32_t* __restrict__ end,
                                                    uint32_t* __restrict__ multi) {
  size_t h0, h1;
  msd_holders(dtot, n, desc, has_valid, &h0, &h1);
  const int lane = threadIdx.x & 63;
  const size_t base = h0 + (size_t)blockIdx.x * 256 * kMsdBoundsRows + threadIdx.x;
  uint64_t k[kMsdBoundsRows];
#pragma unroll
  for (int r = 0; r < kMsdBoundsRows; ++r) k[r] = keys[min(base + (size_t)r * 256, h1 - 1)];
#pragma unroll
  for (int r = 0; r < kMsdBoundsRows; ++r) {
    const size_t i = base + (size_t)r * 256;
    const bool in = i < h1;
    uint64_t kp = (uint64_t)__shfl_up((long long)k[r], 1), kn = (uint64_t)__shfl_down((long long)k[r], 1);
    if (!in) continue;
    if (lane == 0 && i > h0) kp = keys[i - 1];
    if (lane == 63 && i + 1 < h1) kn = keys[i + 1];
    const uint32_t b = msd_bucket_of(k[r], s1);
    const bool head = i == h0 || msd_bucket_of(kp, s1) != b;
    if (head) first[b] = (uint32_t)i;
    else if (kp != k[r]) multi[b] = 1u;
    if (i == h1 - 1 || msd_bucket_of(kn, s1) != b) end[b] = (uint32_t)(i + 1);
  }
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  for (int off = 32; off >= 1; off >>= 1) {
    const uint64_t o = shfl_xor_u64(v, off);
    v = o < v ? o : v;
  }
  return v;
}

// Stable partition of bucket [lo, lo + m) by distinct key, at most max_rounds rounds; returns whether
// every row was written. Round: kPartRows chunks of 64 rows in flight, the rows whose key is cur compacted by
// ballot, the next larger key found on the way. The first round takes cur = the bucket's first key
// (a one-key bucket is then a single copy); a smaller key seen in it restarts from the smallest.
constexpr int kPartRows = 16;  // rows per lane in flight (8: the same kernel time within noise)
__device__ __forceinline__ bool msd_wave_partition(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ src,
                                                   uint32_t* __restrict__ ids, uint32_t lo, uint32_t m, int lane,
                                                   int max_rounds) {
  const uint64_t lt = (1ull << lane) - 1ull;
  uint64_t cur = keys[lo];
  uint32_t out = lo;
  bool restarted = false;
  for (int round = 0; round < max_rounds; ++round) {
    uint64_t nxt = ~0ull, below = ~0ull;
    for (uint32_t p0 = 0; p0 < m; p0 += 64 * kPartRows) {
      uint64_t k[kPartRows];
      uint32_t id[kPartRows];
#pragma unroll
      for (int r = 0; r < kPartRows; ++r) {
        const uint32_t pos = min(p0 + (uint32_t)(r * 64 + lane), m - 1);
        k[r] = keys[lo + pos];
        id[r] = src[lo + pos];
      }
#pragma unroll
      for (int r = 0; r < kPartRows; ++r) {
        const bool in = p0 + (uint32_t)(r * 64) + lane < m;
        const bool hit = in && k[r] == cur;
        const uint64_t bal = __ballot(hit);
        if (hit) ids[out + __popcll(bal & lt)] = id[r];
        out += (uint32_t)__popcll(bal);
        if (in && k[r] > cur && k[r] < nxt) nxt = k[r];
        if (in && k[r] < below) below = k[r];
      }
    }
    if (!restarted) {
      restarted = true;
      below = wave_min_u64(below);
      if (below < cur) {  // the first key was not the smallest: start over from the smallest
        cur = below;
        out = lo;
        continue;
      }
    }
    if (out == lo + m) return true;
    cur = wave_min_u64(nxt);
  }
  return false;
}

// one wave sorts a bucket of m <= 64E rows by bitonic network (input positions r*64 + lane: coalesced)
template <int E, int LOGP>
__device__ __forceinline__ void msd_wave_sort(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ src,
                                              uint32_t* __restrict__ ids, uint32_t lo, uint32_t m, uint64_t rmask,
                                              int lane) {
  uint64_t v[E];
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const uint32_t pos = (uint32_t)r * 64 + lane;
    v[r] = pos < m ? ((keys[lo + pos] & rmask) << 10) | pos : ~0ull;
  }
  bitonic<E, LOGP, 64>(v, lane, nullptr);
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const uint32_t e = (uint32_t)lane * E + r;
    if (e < m) ids[lo + e] = src[lo + (uint32_t)(v[r] & 1023u)];
  }
}

__global__ void __launch_bounds__(256) k_msd_local(const uint64_t* __restrict__ keys, uint32_t* __restrict__ src,
                                                   uint32_t* __restrict__ ids, const uint32_t* __restrict__ first,
                                                   const uint32_t* __restrict__ end,
                                                   const uint32_t* __restrict__ multi, int s1,
                                                   uint32_t* __restrict__ ctl, uint32_t* __restrict__ big) {
  const int lane = threadIdx.x & 63;
  {  // one wave per bucket (a grid-stride loop over the buckets measured 34 -> 56 us: the multi-key
     // buckets' rounds serialise within a wave)
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (!multi[b]) return;  // empty, or one key: the last pass already put its rows in their place
    const uint32_t lo = first[b], m = end[b] - lo;
    // this bucket's grouped ids to the side buffer (free after the last pass), read from there below
    for (uint32_t p0 = 0; p0 < m; p0 += 512) {  // 8 loads in flight per lane, then their stores
      uint32_t v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const uint32_t p = p0 + (uint32_t)(r * 64 + lane);
        v[r] = p < m ? ids[lo + p] : 0u;
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const uint32_t p = p0 + (uint32_t)(r * 64 + lane);
        if (p < m) src[lo + p] = v[r];
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wave's copies land before its lanes read them
    if (msd_wave_partition(keys, src, ids, lo, m, lane, m <= kMsdWaveMax ? 2 : 16)) return;
    if (m > kMsdWaveMax) {
      if (lane == 0) big[atomicAdd(&ctl[kMsdCtlBig], 1u)] = b;
      return;
    }
    const uint64_t rmask = (1ull << s1) - 1ull;
    if (m <= 64) msd_wave_sort<1, 6>(keys, src, ids, lo, m, rmask, lane);
    else if (m <= 128) msd_wave_sort<2, 7>(keys, src, ids, lo, m, rmask, lane);
    else if (m <= 256) msd_wave_sort<4, 8>(keys, src, ids, lo, m, rmask, lane);
    else msd_wave_sort<8, 9>(keys, src, ids, lo, m, rmask, lane);
  }
}

template <int E, int LOGP>
__device__ __forceinline__ void msd_block_sort(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ src,
                                               uint32_t* __restrict__ ids, uint32_t lo, uint32_t m, uint64_t rmask,
                                               uint64_t* xch) {
  const int t = threadIdx.x;
  uint64_t v[E];
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const uint32_t pos = (uint32_t)r * 1024 + t;
    v[r] = pos < m ? ((keys[lo + pos] & rmask) << 13) | pos : ~0ull;
  }
  bitonic<E, LOGP, 1024>(v, t, xch);
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const uint32_t e = (uint32_t)t * E + r;
    if (e < m) ids[lo + e] = src[lo + (uint32_t)(v[r] & 8191u)];
  }
}

// buckets of 513..8192 rows with more distinct keys than k_msd_local's partition rounds: one
// workgroup each (grid-stride over the list); larger ones: overflow flag (host falls back to LSD)
__global__ void __launch_bounds__(1024) k_msd_big(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ src,
                                                  uint32_t* __restrict__ ids, const uint32_t* __restrict__ first,
                                                  const uint32_t* __restrict__ end, int s1, uint32_t* __restrict__ ctl,
                                                  const uint32_t* __restrict__ big) {
  __shared__ uint64_t xch[kMsdBlockMax];
  const uint32_t nbig = ctl[kMsdCtlBig];
  const uint64_t rmask = (1ull << s1) - 1ull;
  for (uint32_t q = blockIdx.x; q < nbig; q += gridDim.x) {
    const uint32_t b = big[q];
    const uint32_t lo = first[b], m = end[b] - lo;
    if (m > kMsdBlockMax) {
      if (threadIdx.x == 0) atomicOr(&ctl[kMsdCtlOverflow], 1u);
      continue;
    }
    if (m <= 2048) msd_block_sort<2, 11>(keys, src, ids, lo, m, rmask, xch);
    else if (m <= 4096) msd_block_sort<4, 12>(keys, src, ids, lo, m, rmask, xch);
    else msd_block_sort<8, 13>(keys, src, ids, lo, m, rmask, xch);
    __syncthreads();  // xch is free for the next bucket
  }
}

size_t rs_blocks(size_t n) { return (n + kRsTile - 1) / kRsTile; }
size_t rs_scratch_bytes(size_t n) {
  // keys x2 (8 B), ids x1 extra (4 B; the other id buffer is the caller's output), histogram, OR/AND,
  // MSD bucket starts + control words + big-bucket list
  return 2 * n * 8 + n * 4 + (size_t)kRsDigits * (rs_blocks(n) + 2) * 4 + 1024 +
         (size_t)kRsDigits * ((rs_blocks(n) + kScanTiles - 1) / kScanTiles) * 4 + 256 +
         16 * ((n + 256 * kRsPrepRows - 1) / (256 * kRsPrepRows)) + 768 + (4 * (size_t)kMsdBuckets + 8) * 4;
}

// the MSD path pays off from 4 LSD passes on (a span of > 24 bits) and enough rows to fill the buckets
static bool msd_enabled(size_t n, int sb) {
  static const int mode = [] {
    const char* s = getenv("DDSHE_ORDER_MSD");  // 0: LSD passes only (A/B)
    return s ? atoi(s) : 1;
  }();
  return mode != 0 && n >= ((size_t)1 << 16) && sb > 24;
}

hipError_t launch_ope_order(const int64_t* col, const uint8_t* valid, size_t n, int desc, void* scratch,
                            uint32_t* out_ids, hipStream_t st, const uint64_t* ubounds) {
  if (n == 0) return hipSuccess;
  const size_t nb = rs_blocks(n);
  uint64_t* ka = (uint64_t*)scratch;
  uint64_t* kb = ka + n;
  uint32_t* ib = (uint32_t*)(kb + n);
  uint32_t* hist = (uint32_t*)(((uintptr_t)(ib + n) + 255) & ~(uintptr_t)255);
  uint32_t* dtot = hist + (size_t)kRsDigits * nb;
  const size_t nch = (nb + kScanTiles - 1) / kScanTiles;
  uint32_t* ctot = (uint32_t*)(((uintptr_t)(dtot + kRsDigits) + 255) & ~(uintptr_t)255);
  uint64_t* red = (uint64_t*)(((uintptr_t)(ctot + (size_t)kRsDigits * nch) + 15) & ~(uintptr_t)15);
  uint64_t* part = red + 2;
  const size_t pb = (n + 256 * kRsPrepRows - 1) / (256 * kRsPrepRows);
  uint32_t* mfirst = (uint32_t*)(((uintptr_t)(part + 2 * pb) + 255) & ~(uintptr_t)255);
  uint32_t* mend = mfirst + kMsdBuckets;
  uint32_t* mmulti = mend + kMsdBuckets;
  uint32_t* mctl = mmulti + kMsdBuckets;  // right after the multi flags: one memset clears both
  uint32_t* mbig = mctl + 8;
  uint64_t hred[2];
  hipError_t e = hipSuccess;
  if (ubounds) {  // bounds of the raw values from the caller: the keys' bounds follow (desc: complemented)
    hred[0] = ubounds[0] <= ubounds[1] ? (desc ? ~ubounds[1] : ubounds[0]) : 1;
    hred[1] = ubounds[0] <= ubounds[1] ? (desc ? ~ubounds[0] : ubounds[1]) : 0;
  } else {
    if (((uintptr_t)col & 15) == 0 && ((uintptr_t)valid & 1) == 0)
      hipLaunchKernelGGL(k_rs_prep, dim3((unsigned)pb), dim3(256), 0, st, col, valid, n, desc, part);
    else
      hipLaunchKernelGGL(k_rs_prep_rows, dim3((unsigned)pb), dim3(256), 0, st, col, valid, n, desc, part);
    hipLaunchKernelGGL(k_rs_red, dim3(1), dim3(1024), 0, st, part, pb, red);
    e = hipMemcpyAsync(hred, red, sizeof(hred), hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
  }
  // the bytes of max - min (at least one pass when rows may lack the position: its last pass buckets them)
  const uint64_t kmin = hred[0] <= hred[1] ? hred[0] : 0ull;
  const uint64_t span = hred[0] <= hred[1] ? hred[1] - hred[0] : 0ull;
  const int sb = span ? 64 - __builtin_clzll(span) : 0;  // bits of the span
  const bool vbit = valid && n <= (size_t)kRsLack;
  // executed pass j writes ids to fin when (np-1-j) is even, so the last one lands there
  auto run_passes = [&](const int* shifts, int np, bool keep_keys, uint32_t* fin, uint32_t* tmp) -> const uint64_t* {
    const uint32_t* ids_in = nullptr;  // identity before the first pass
    const uint64_t* kin = (const uint64_t*)col;  // raw column before the first pass
    uint64_t* kout = ka;
    for (int j = 0; j < np; ++j) {
      uint32_t* ids_out = ((np - 1 - j) % 2 == 0) ? fin : tmp;
      const bool last = j == np - 1;
      hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)nb), dim3(kRsBlock), 0, st, kin, ids_in, valid, n, shifts[j], last,
                         desc, vbit, kmin, hist, nb);
      hipLaunchKernelGGL(k_rs_scan_tiles, dim3((unsigned)nch), dim3(kScanThreads), 0, st, hist, nb, ctot);
      hipLaunchKernelGGL(k_rs_scan_chunks, dim3(1), dim3(kScanThreads), 0, st, ctot, nch, dtot);
      hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)nb), dim3(kRsBlock), 0, st, kin, ids_in, valid, n, shifts[j],
                         desc, vbit, last, kmin, hist, ctot, dtot, nb, (last && !keep_keys) ? nullptr : kout, ids_out);
      kin = kout;
      kout = kout == ka ? kb : ka;
      ids_in = ids_out;
    }
    return kin;
  };
  if (msd_enabled(n, sb)) {
    const int s1 = sb - kMsdBits;
    const int shifts[2] = {s1, sb - 8};
    // grouped ids -> out_ids (one-key buckets are final there); ib (the first pass's ids) is then free
    // and serves as the side copy of the multi-key buckets (k_msd_local)
    const uint64_t* sorted = run_passes(shifts, 2, true, out_ids, ib);
    if ((e = hipMemsetAsync(mmulti, 0, (kMsdBuckets + 8) * 4, st)) != hipSuccess) return e;  // flags + control
    const size_t nbd = (n + 256 * kMsdBoundsRows - 1) / (256 * kMsdBoundsRows);  // over <= n holder rows
    hipLaunchKernelGGL(k_msd_bounds, dim3((unsigned)nbd), dim3(256), 0, st, sorted, n, s1, dtot, desc, valid != nullptr,
                       mfirst, mend, mmulti);
    hipLaunchKernelGGL(k_msd_local, dim3(kMsdBuckets / 4), dim3(256), 0, st, sorted, ib, out_ids, mfirst, mend, mmulti,
                       s1, mctl, mbig);
    hipLaunchKernelGGL(k_msd_big, dim3(kMsdBigBlocks), dim3(1024), 0, st, sorted, ib, out_ids, mfirst, mend, s1, mctl,
                       mbig);
    uint32_t hctl[2];
    if ((e = hipMemcpyAsync(hctl, mctl, sizeof(hctl), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    if (!hctl[kMsdCtlOverflow]) return hipGetLastError();
    // a bucket of > 8192 rows with > 16 distinct keys: redo the whole sort with the LSD passes
  }
  int shifts[8], np = 0;
  for (int p = 0; p < 8 && (span >> (8 * p)) != 0; ++p) shifts[np++] = 8 * p;
  if (np == 0 && valid) shifts[np++] = 0;
  if (np == 0) {
    hipLaunchKernelGGL(k_rs_iota, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out_ids, n);
    return hipGetLastError();
  }
  run_passes(shifts, np, false, out_ids, ib);
  return hipGetLastError();
}

}  // namespace ddshe
