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

#include <algorithm>
#include <atomic>
#include <mutex>

#include "ddshe_launch.hpp"

namespace ddshe {

constexpr int kRsBlock = 256;
constexpr int kRsItems = 8;                       // rows per lane
constexpr size_t kRsTile = (size_t)kRsBlock * kRsItems;
constexpr int kRsDigits = 257;                    // 256 + the validity bucket of the last pass
constexpr uint32_t kRsNone = 511;                 // digit of a lane past the end (never counted)
constexpr uint64_t kSign = 0x8000000000000000ull;
constexpr int kScanTiles = 64;                    // tiles per chunk of the scan over tiles (k_rs_hist)
constexpr int kMsdBits = 16;                      // MSD split: buckets of the top 16 bits of the key span
constexpr uint32_t kMsdBuckets = 1u << kMsdBits;

// Sort key of a holder: its value in unsigned order (descending: complemented), minus the smallest
// such key (kmin). Rows lacking the position get key 0 so that earlier passes keep them in input
// order; the last pass moves them to their bucket (256 / 0). The first executed pass derives the keys
// from the column itself (no separate key buffer is written up front).
__device__ __forceinline__ uint64_t rs_ukey(uint64_t raw, int desc) {
  const uint64_t u = raw ^ kSign;  // signed order -> unsigned order
  return desc ? ~u : u;
}
// kbit (span < 2^56): a row lacking the position gets key 2^63 instead of 0. Its digit is still 0 in
// every pass but the last (whose shift is <= 48), and the last pass reads its validity from that bit: no
// id (vbit) or valid[] read there.
constexpr uint64_t kRsNoHold = 1ull << 63;
__device__ __forceinline__ uint64_t rs_key_of(uint64_t raw, const uint8_t* __restrict__ valid, size_t i, int desc,
                                              uint64_t kmin, bool kbit) {
  return (valid && !valid[i]) ? (kbit ? kRsNoHold : 0ull) : rs_ukey(raw, desc) - kmin;
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
// hout (host-mapped, nullable): red[0..1] also stored to host memory (read after the stream synchronises,
// no copy). spec_lo <= spec_hi: the plan of a speculative MSD call (launch_ope_order) to red[2..3]:
// red[2] = kmin, red[3] = s1 (the first pass's shift, span bits - 16) when the span has spec_lo..spec_hi
// bits, else kRsNoPlan (every later kernel of the call then returns at once).
constexpr uint64_t kRsNoPlan = ~0ull;
constexpr int kCarryWords = 64;  // the carried plan's max words (k_rs_hist atomicMax, k_rs_scan_chunks check)
__global__ void __launch_bounds__(1024) k_rs_red(const uint64_t* __restrict__ part, size_t nparts,
                                                 uint64_t* __restrict__ red, int spec_lo, int spec_hi,
                                                 uint64_t* __restrict__ hout) {
  uint64_t lo = ~0ull, hi = 0;
  for (size_t i = threadIdx.x; i < nparts; i += 1024) {
    lo = min(lo, part[2 * i]);
    hi = max(hi, part[2 * i + 1]);
  }
  rs_minmax_block(lo, hi, red);
  if (threadIdx.x == 0) {  // the thread that stored red[0..1]
    const uint64_t mn = red[0], mx = red[1];
    if (hout) {
      hout[0] = mn;
      hout[1] = mx;
    }
    if (spec_lo <= spec_hi) {
      const uint64_t span = mn <= mx ? mx - mn : 0ull;
      const int sb = span ? 64 - __builtin_clzll(span) : 0;
      red[2] = mn <= mx ? mn : 0ull;
      red[3] = (sb >= spec_lo && sb <= spec_hi) ? (uint64_t)(sb - kMsdBits) : kRsNoPlan;
    }
  }
}

// the end of a call's device work: plan and overflow flag to host memory (one thread)
__global__ void k_rs_publish(const uint32_t* __restrict__ ctl, const uint64_t* __restrict__ plan,
                             uint64_t* __restrict__ hout) {
  hout[2] = ctl[1];  // kMsdCtlOverflow
  hout[3] = plan ? plan[1] : 0ull;
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
                                             bool last, int desc, bool vbit, bool kbit) {
  uint32_t d = (uint32_t)(k >> shift) & 0xFFu;
  if (last && valid) {
    const bool v = kbit ? (k >> 63) == 0 : vbit ? (id & kRsLack) == 0 : valid[id] != 0;
    d = desc ? (v ? d : 256u) : (v ? d + 1u : 0u);
  }
  return d;
}

// Tile of a block. xcd != 0: blocks are dealt round-robin over the 8 XCDs (observed; speed only, never
// correctness), so block b works on tile (b % 8)-th eighth + b / 8: each XCD walks a contiguous range of
// tiles and neighbouring tiles' writes to one digit run meet in the same L2.
__device__ __forceinline__ size_t rs_tile(size_t nblocks, int xcd) {
  const size_t b = blockIdx.x;
  if (!xcd) return b;
  const size_t q = nblocks >> 3, r = nblocks & 7, x = b & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

// Tile geometry of a pass: BLK threads x kRsItems rows. Bigger tiles give longer digit runs in the
// scatter's write-out (2048-row tiles: ~8 rows per digit on random digits, the first pass's case).
template <int BLK>
struct RsTile {
  static constexpr int kWaves = BLK / 64;
  static constexpr size_t kRows = (size_t)BLK * kRsItems;
  // row of item k of a lane: each wave owns a contiguous 1/kWaves of the tile
  static __device__ __forceinline__ size_t row(size_t tile, int wid, int k, int lane) {
    return tile * kRows + (size_t)wid * (kRows / kWaves) + (size_t)k * 64 + lane;
  }
};

// Per-tile digit counts of the scatter's tiles (BLK x kRsItems rows) by HB threads (the counts do not
// depend on which lane holds which row). HB = 64, a whole tile per wave (every tile of 10M rows resident
// at once instead of 2.4 rounds of 256-thread blocks), measured slower: 30 -> 43 us on the first pass.
template <int BLK, int HB>
__global__ void __launch_bounds__(HB) k_rs_hist(const uint64_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ ids,
                                                     const uint8_t* __restrict__ valid, size_t n, int shift,
                                                     bool last, int desc, bool vbit, bool kbit, uint64_t kmin,
                                                     uint32_t* __restrict__ hist, size_t nblocks,
                                                     uint32_t* __restrict__ clr, uint32_t nclr, bool pairs,
                                                     const uint32_t* __restrict__ khi,
                                                     const uint64_t* __restrict__ plan, bool rowatom,
                                                     uint64_t* __restrict__ mm = nullptr) {
  if (plan) {  // speculative call: kmin and the shift (relative to s1) from k_rs_red's plan
    const uint64_t s1 = plan[1];
    if (s1 == kRsNoPlan) return;
    kmin = plan[0];
    shift += (int)s1;
  }
  constexpr size_t kRows = RsTile<BLK>::kRows;
  constexpr int kIt = (int)(kRows / HB);  // rows per thread
  constexpr int kW = HB / 64;
  // rowatom: one LDS atomic per row into the wave's own copy of the counts (digits of a wave mostly
  // distinct), else one per distinct digit of the wave found by 9 ballots (digits repeating)
  __shared__ uint32_t wcnt[kW][kRsDigits];
  uint32_t* cnt = &wcnt[0][0];
  for (int d = threadIdx.x; d < kW * kRsDigits; d += HB) cnt[d] = 0;
  if (clr) {  // first pass of the MSD path: the bucket tables of the last scatter start at their identities
    const size_t g = (size_t)blockIdx.x * HB + threadIdx.x;
    for (size_t g2 = g; g2 < nclr; g2 += (size_t)gridDim.x * HB)
      clr[g2] = g2 < 3 * (size_t)kMsdBuckets ? ~0u : 0u;  // first[], kmin[] (2 words each): ~0; the rest 0
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  const bool need_id = last && valid && !kbit;
  // all loads first (independent, in flight together), then the LDS counting
  uint64_t key[kIt];
  uint32_t id[kIt];
  size_t rix[kIt];
  uint64_t mhi = 0;  // mm: the block's largest holder key (offset by the carried kmin)
  if (khi) {
    // split keys (the MSD path's last pass, digit and validity bits >= 32): only the high words, four rows
    // per 16-byte load; an unaligned tail row by row
    const size_t nq = n / 4;
#pragma unroll
    for (int k = 0; k < kIt / 4; ++k) {
      const size_t q = (size_t)blockIdx.x * (kRows / 4) + (size_t)k * HB + threadIdx.x;
      uint4 h = nq ? reinterpret_cast<const uint4*>(khi)[min(q, nq - 1)] : make_uint4(0, 0, 0, 0);
      const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const size_t r = 4 * q + e;
        uint32_t w = hw[e];
        if (q >= nq && r < n) w = khi[r];  // the last n % 4 rows
        key[4 * k + e] = (uint64_t)w << 32;
        id[4 * k + e] = 0u;
        rix[4 * k + e] = r;
      }
    }
  } else if (pairs) {
    // 16-byte key pairs (a wave instruction reads 1 KiB): pair q = 2 rows; an odd last row on its own.
    // keys 16-byte aligned, valid 2-byte aligned, no id needed (host-checked)
    const size_t np = n / 2;
#pragma unroll
    for (int k = 0; k < kIt / 2; ++k) {
      const size_t q = (size_t)blockIdx.x * (kRows / 2) + (size_t)k * HB + threadIdx.x;
      const size_t qc = min(q, np ? np - 1 : 0);
      ulonglong2 kv = np ? reinterpret_cast<const ulonglong2*>(keys)[qc] : make_ulonglong2(0, 0);
      uint32_t hv = (!ids && valid && np) ? reinterpret_cast<const uint16_t*>(valid)[qc] : 0x0101u;
      rix[2 * k] = q < np ? 2 * q : ~(size_t)0;
      rix[2 * k + 1] = q < np ? 2 * q + 1 : ~(size_t)0;
      if ((n & 1) && q == np) {  // the odd last row
        kv.x = keys[n - 1];
        hv = (!ids && valid) ? valid[n - 1] : 1u;
        rix[2 * k] = n - 1;
      }
      key[2 * k] = ids ? kv.x : (hv & 0xFFu) ? rs_ukey(kv.x, desc) - kmin : (kbit ? kRsNoHold : 0ull);
      key[2 * k + 1] = ids ? kv.y : (hv >> 8) ? rs_ukey(kv.y, desc) - kmin : (kbit ? kRsNoHold : 0ull);
      id[2 * k] = id[2 * k + 1] = 0u;
      if (mm) {  // the largest offset key of a holder (k_rs_scan_chunks checks the carried plan with it)
        if (rix[2 * k] < n && (hv & 0xFFu)) mhi = max(mhi, key[2 * k]);
        if (rix[2 * k + 1] < n && (hv >> 8)) mhi = max(mhi, key[2 * k + 1]);
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kIt; ++k) {  // unconditional loads (index clamped), masked below
      const size_t r = (size_t)blockIdx.x * kRows + (size_t)k * HB + threadIdx.x;
      const size_t i = min(r, n - 1);
      key[k] = ids ? keys[i] : rs_key_of(keys[i], valid, i, desc, kmin, kbit);  // first pass: keys = the column
      id[k] = need_id ? rs_load_id(ids, i, valid, vbit) : 0u;
      rix[k] = r;
      if (mm && r < n && (!valid || valid[i])) mhi = max(mhi, key[k]);
    }
  }
  if (mm) {  // block max, folded into mm[block % kCarryWords] (k_rs_scan_chunks reads and re-zeroes them)
    for (int off = 32; off >= 1; off >>= 1) mhi = max(mhi, (uint64_t)__shfl_xor((long long)mhi, off));
    __shared__ uint64_t smax[kW];
    if (lane == 0) smax[threadIdx.x >> 6] = mhi;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t v = smax[0];
      for (int w = 1; w < kW; ++w) v = max(v, smax[w]);
      atomicMax(reinterpret_cast<unsigned long long*>(mm) + (blockIdx.x % kCarryWords), (unsigned long long)v);
    }
  }
  if (rowatom) {
    uint32_t* mine = &wcnt[threadIdx.x >> 6][0];
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const size_t i = rix[k];
      if (i < n) atomicAdd(&mine[rs_digit(key[k], id[k], valid, shift, last, desc, vbit, kbit)], 1u);
    }
  } else {
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const size_t i = rix[k];
      const uint32_t d = i < n ? rs_digit(key[k], id[k], valid, shift, last, desc, vbit, kbit) : kRsNone;
      // one LDS atomic per distinct digit of the wave
      uint64_t peers = ~0ull;
#pragma unroll
      for (int b = 0; b < 9; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bal : ~bal;
      }
      if (d != kRsNone && (peers & lt) == 0) atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kRsDigits; d += HB) {  // 1 KiB, coalesced
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < kW; ++w) c += wcnt[w][d];
    hist[(size_t)blockIdx.x * kRsDigits + d] = c;
  }
}

constexpr int kScanThreads = 320;  // >= kRsDigits
// Exclusive scan over tiles per digit, in two launches: k_rs_scan_tiles, one block per chunk of
// kScanTiles tiles and one thread per digit (coalesced rows across the digit threads), replaces the
// chunk's counts by their exclusive prefix within the chunk and stores the chunk total to
// ctot[chunk][digit]; k_rs_scan_chunks, one block, replaces the chunk totals by their exclusive prefix
// and stores the digit totals to dtot. A tile's offset for digit d is then dbase[d] + ctot[chunk][d] +
// hist[tile][d]. One launch instead (the chunks' last block scanning the totals after a ticket, with
// write-through chunk totals) measured slower on one box: 14-18 us against 6.4 + 5.9 us; the scans
// inside the histogram's last blocks made the histogram 2x slower (every block waits for its
// write-through row before its ticket).
__global__ void __launch_bounds__(kScanThreads) k_rs_scan_tiles(uint32_t* __restrict__ hist, size_t nblocks,
                                                                uint32_t* __restrict__ ctot) {
  const int d = threadIdx.x;
  if (d >= kRsDigits) return;
  const size_t t0 = (size_t)blockIdx.x * kScanTiles;
  uint32_t* p = hist + t0 * kRsDigits + d;
  uint32_t run = 0;
  if (t0 + kScanTiles <= nblocks) {
    uint32_t v[kScanTiles];
#pragma unroll
    for (int r = 0; r < kScanTiles; ++r) v[r] = p[r * kRsDigits];
#pragma unroll
    for (int r = 0; r < kScanTiles; ++r) {
      p[r * kRsDigits] = run;
      run += v[r];
    }
  } else {
    for (size_t r = 0; t0 + r < nblocks; ++r) {
      const uint32_t v = p[r * kRsDigits];
      p[r * kRsDigits] = run;
      run += v;
    }
  }
  ctot[(size_t)blockIdx.x * kRsDigits + d] = run;
}

// Carried plan (mm != nullptr, the first pass of launch_ope_order's prep-free path): thread 0 also reads
// the largest holder key of the first histogram (keys offset by the carried kmin, atomicMax'ed by its
// blocks into kCarryWords words: one word for all 4,883 blocks of 10M rows serialised the atomics, 23 ->
// 64 us), re-zeroes the words for the next call, and keeps the plan (plan[0..1] = kmin, s1) iff it
// fits: every holder key in [kmin, kmin + 2^(s1+16)) with the top bit used, i.e. 2^(s1+15) <= max <
// 2^(s1+16) and max <= ~kmin (a key below kmin wraps to at least 2^64 - kmin = ~kmin + 1); else plan[1]
// = kRsNoPlan and every later kernel of the call returns. A word that was not zero before the call (a
// fresh buffer, a scratch layout of another row count) only raises the max: the check then fails, or
// passes for a range that still holds every key.
__global__ void __launch_bounds__(kScanThreads) k_rs_scan_chunks(uint32_t* __restrict__ ctot, size_t nchunks,
                                                                 uint32_t* __restrict__ dtot,
                                                                 uint64_t* __restrict__ mm = nullptr,
                                                                 uint64_t* __restrict__ plan = nullptr,
                                                                 uint64_t ckmin = 0, int cs1 = -1) {
  if (mm && threadIdx.x < 64) {  // wave 0: the kCarryWords maxima
    uint64_t v = threadIdx.x < kCarryWords ? mm[threadIdx.x] : 0ull;
    if (threadIdx.x < kCarryWords) mm[threadIdx.x] = 0ull;
    for (int off = 32; off >= 1; off >>= 1) v = max(v, (uint64_t)__shfl_xor((long long)v, off));
    if (threadIdx.x == 0) {
      const bool ok = v <= ~ckmin && (v >> (cs1 + kMsdBits)) == 0 && (v >> (cs1 + kMsdBits - 1)) == 1;
      plan[0] = ckmin;
      plan[1] = ok ? (uint64_t)cs1 : kRsNoPlan;
    }
  }
  const int d = threadIdx.x;
  if (d >= kRsDigits) return;
  uint32_t run = 0;
  uint32_t* p = ctot + d;
  size_t c0 = 0;
  for (; c0 + 32 <= nchunks; c0 += 32, p += 32 * kRsDigits) {
    uint32_t v[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = p[q * kRsDigits];
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      p[q * kRsDigits] = run;
      run += v[q];
    }
  }
  for (; c0 < nchunks; ++c0, p += kRsDigits) {
    const uint32_t v = *p;
    *p = run;
    run += v;
  }
  dtot[d] = run;
}

// Tile counts are tile-major (hist[tile][digit]: each histogram block writes 1 KiB in one go; the
// digit-major layout cost one 32-byte sector per 4-byte count, 8x the bytes, PMC round 2); k_rs_scan
// (above) turns them into per-tile offsets.

// The ranked rows are first placed in tile-local digit order in LDS, then written out by
// consecutive threads: lanes of a store instruction hit consecutive addresses of a digit run
// (runs average kRsTile/256 = 16 rows), instead of 64 different buckets per store.
// Bucket table of the MSD split, filled by the last LSD pass's scatter (k_rs_scatter with runs.first set):
// rows of one top-16-bit bucket form one run in each tile's digit run, so per (tile, bucket) run the
// scatter takes first[b] = min(run start), end[b] = max(run end), kmin/kmax[b] = min/max(run's first key),
// and stores multi[b] = 1 where two adjacent rows of a run differ. A bucket holds two distinct keys iff
// multi[b] or kmin[b] != kmax[b]. Layout (one clear): first | kmin (~0) | end | kmax | multi | ctl (0).
struct MsdRuns {
  uint32_t* first;
  unsigned long long* kmin;
  uint32_t* end;
  unsigned long long* kmax;
  uint32_t* multi;
  int s1;  // bucket = key >> s1
};
constexpr uint32_t kMsdTableWords = 7 * kMsdBuckets + 8;

template <int BLK>
__global__ void __launch_bounds__(BLK) k_rs_scatter(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ ids,
                                                         const uint8_t* __restrict__ valid, size_t n, int shift,
                                                         int desc, bool vbit, bool kbit, bool last, uint64_t kmin,
                                                         const uint32_t* __restrict__ hist,
                                                         const uint32_t* __restrict__ ctot,
                                                         const uint32_t* __restrict__ dtot, size_t nblocks,
                                                         uint64_t* __restrict__ keys_out,
                                                         uint32_t* __restrict__ ids_out, int xcd, MsdRuns runs,
                                                         const uint32_t* __restrict__ khi,
                                                         uint32_t* __restrict__ khi_out,
                                                         const uint64_t* __restrict__ plan) {
  if (plan) {
    const uint64_t s1 = plan[1];
    if (s1 == kRsNoPlan) return;
    kmin = plan[0];
    shift += (int)s1;
    runs.s1 = (int)s1;
  }
  const size_t tile = rs_tile(nblocks, xcd);
  using T = RsTile<BLK>;
  constexpr int W = T::kWaves;
  __shared__ uint32_t cnt[W][kRsDigits];
  __shared__ uint32_t dbase[kRsDigits + 1];   // global start of digit d, then of this tile's run of d
  __shared__ uint32_t lstart[kRsDigits + 1];  // tile-local start of digit d
  __shared__ uint64_t skey[T::kRows];
  __shared__ uint32_t sid[T::kRows];
  __shared__ uint16_t sdig[T::kRows];
  for (int d = threadIdx.x; d < W * kRsDigits; d += BLK) (&cnt[0][0])[d] = 0;
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
    const size_t i = min(T::row(tile, wid, k, lane), n - 1);
    if (khi)  // split keys: high words + low words (keys points at the low words)
      key[k] = ((uint64_t)khi[i] << 32) | reinterpret_cast<const uint32_t*>(keys)[i];
    else
      key[k] = ids ? keys[i] : rs_key_of(keys[i], valid, i, desc, kmin, kbit);  // first pass: keys = the column
    id[k] = rs_load_id(ids, i, valid, vbit);  // ids == nullptr: first executed pass, identity
  }
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const size_t i = T::row(tile, wid, k, lane);
    dr[k] = i < n ? rs_digit(key[k], id[k], valid, shift, last, desc, vbit, kbit) : kRsNone;
  }
  // bit 8 of a digit is set only by the last pass's validity bucket and by lanes past the column's end
  // (kRsNone): a full tile of another pass ranks on 8 ballots
  const bool nine = (last && valid) || (tile + 1) * T::kRows > n;
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const uint32_t d = dr[k];
    // lanes holding the same digit: AND of the bit-ballots
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    if (nine) {
      const uint64_t bal = __ballot((d >> 8) & 1u);
      peers &= ((d >> 8) & 1u) ? bal : ~bal;
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
  if (wid == 0)
    wave_scan(
        [&](int d) {
          uint32_t c = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) c += cnt[w][d];
          return c;
        },
        lstart);
  __syncthreads();
  // cnt[w][d] <- tile-local start of wave w's rows of digit d; dbase[d] <- global start of the tile's run
  for (int d = threadIdx.x; d < kRsDigits; d += BLK) {
    uint32_t run = lstart[d];
    for (int w = 0; w < W; ++w) {
      const uint32_t c = cnt[w][d];
      cnt[w][d] = run;
      run += c;
    }
    dbase[d] += ctot[(tile / kScanTiles) * kRsDigits + d] + hist[tile * kRsDigits + d];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kRsItems; ++k) {
    const uint32_t d = dr[k] & 511u;
    if (d == kRsNone) continue;
    const uint32_t lp = cnt[wid][d] + (dr[k] >> 9);
    if (keys_out || runs.first) skey[lp] = key[k];
    sid[lp] = (last && vbit) ? (id[k] & ~kRsLack) : id[k];
    sdig[lp] = (uint16_t)d;
  }
  __syncthreads();
  const size_t t0 = tile * T::kRows;
  const uint32_t rows = (uint32_t)min(T::kRows, n - t0);
  for (uint32_t q = threadIdx.x; q < rows; q += BLK) {
    const uint32_t d = sdig[q];
    const uint32_t dst = dbase[d] + (q - lstart[d]);
    if (khi_out) {  // split: high and low words to their own arrays (keys_out points at the low words)
      const uint64_t kk = skey[q];
      khi_out[dst] = (uint32_t)(kk >> 32);
      reinterpret_cast<uint32_t*>(keys_out)[dst] = (uint32_t)kk;
    } else if (keys_out) {
      keys_out[dst] = skey[q];
    }
    ids_out[dst] = sid[q];
    // bucket runs (last pass of the MSD path; rows lacking the position sit in digit 256 / 0: skipped)
    if (runs.first && !(valid && d == (desc ? 256u : 0u))) {
      const uint64_t k = skey[q];
      const uint32_t b = (uint32_t)(k >> runs.s1);
      const bool head = q == lstart[d] || (uint32_t)(skey[q - 1] >> runs.s1) != b;
      const bool tail = q + 1 == lstart[d + 1] || (uint32_t)(skey[q + 1] >> runs.s1) != b;
      if (head) {
        atomicMin(&runs.first[b], dst);
        atomicMin(&runs.kmin[b], (unsigned long long)k);
        atomicMax(&runs.kmax[b], (unsigned long long)k);
      } else if (skey[q - 1] != k) {
        runs.multi[b] = 1u;
      }
      if (tail) atomicMax(&runs.end[b], dst + 1);
    }
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
constexpr uint32_t kMsdWaveMax = 512;
constexpr uint32_t kMsdBlockMax = 8192;
constexpr int kMsdBigBlocks = 256;  // grid of the block path (grid-stride over the big buckets; one per CU:
                                     // a launch that finds no big bucket costs its dispatch, 13 us at 512)
enum { kMsdCtlBig = 0, kMsdCtlOverflow = 1, kMsdCtlTicket = 2 };
static_assert(kMsdBigBlocks < (1 << 16), "k_msd_big ticket: block count in 16 bits");

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
constexpr int kMsdBlkThreads = 256;  // k_msd_local_blk: a block per bucket,
constexpr int kMsdBlkRows = 16;       // kMsdBlkRows rows per lane: up to 4,096 rows from registers
// fuse: the bucket's ids are still only in ids[] (not copied to src yet): round 0 reads them there and
// writes the copy to src as it goes. Its compacted writes land at positions it has already read (out never
// passes the rows loaded so far), and later rounds read src.
__device__ __forceinline__ bool msd_wave_partition(const uint64_t* __restrict__ keys, uint32_t* __restrict__ src,
                                                   uint32_t* __restrict__ ids, uint32_t lo, uint32_t m, int lane,
                                                   int max_rounds, bool fuse = false) {
  const uint64_t lt = (1ull << lane) - 1ull;
  uint64_t cur = keys[lo];
  uint32_t out = lo;
  bool restarted = false;
  for (int round = 0; round < max_rounds; ++round) {
    uint64_t nxt = ~0ull, below = ~0ull;
    const bool copy = fuse && round == 0;
    for (uint32_t p0 = 0; p0 < m; p0 += 64 * kPartRows) {
      uint64_t k[kPartRows];
      uint32_t id[kPartRows];
#pragma unroll
      for (int r = 0; r < kPartRows; ++r) {
        const uint32_t pos = min(p0 + (uint32_t)(r * 64 + lane), m - 1);
        k[r] = keys[lo + pos];
        id[r] = copy ? ids[lo + pos] : src[lo + pos];
      }
      if (copy) {
#pragma unroll
        for (int r = 0; r < kPartRows; ++r) {
          const uint32_t pos = p0 + (uint32_t)(r * 64 + lane);
          if (pos < m) src[lo + pos] = id[r];
        }
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
    if (copy) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the copy lands before later rounds read it
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

// The same partition for a bucket of m <= 256E rows by a 256-thread block, the rows held in registers
// (wave w: rows [64E w, 64E (w + 1)), element r of a lane at 64E w + 64 r + lane): one load phase (every
// row's key and id in flight together), the smallest key by a block minimum (no restart round), then per
// round each wave counts its rows of the key, a block prefix over the four counts gives the waves' output
// offsets (one barrier, double-buffered counts), and the waves store their ids by ballot compaction. The
// memory rounds pay one load latency per 1024-row chunk and round on one wave (the bench column's
// buckets: 2 keys ~1,900 rows, 3 keys ~2,900, up to ~3,950 with 4). Rows past m read as key ~0: they never
// lower the minimum or the next key, and as hits of a round whose key is ~0 (a real key only at a full
// 64-bit span) they sit in the last positions, after every real row: their stores past the bucket are
// dropped. fuse: ids[] is overwritten only after every wave holds its rows (a barrier); the side copy
// src[] is written only if the rounds run out (k_msd_big reads it).
template <int E, int NW>
__device__ __forceinline__ bool msd_block_partition(const uint64_t* __restrict__ keys, uint32_t* __restrict__ src,
                                                    uint32_t* __restrict__ ids, uint32_t lo, uint32_t m,
                                                    int max_rounds, bool fuse, uint32_t (*scnt)[NW],
                                                    uint64_t (*smin)[NW]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t w0 = (uint32_t)wid * 64 * E;
  uint64_t k[E];
  uint32_t id[E];
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const uint32_t pos = min(w0 + (uint32_t)(r * 64 + lane), m - 1);
    k[r] = keys[lo + pos];
    id[r] = fuse ? ids[lo + pos] : src[lo + pos];
  }
  uint64_t below = ~0ull;
#pragma unroll
  for (int r = 0; r < E; ++r) {
    if (w0 + (uint32_t)(r * 64 + lane) >= m) k[r] = ~0ull;
    below = k[r] < below ? k[r] : below;
  }
  below = wave_min_u64(below);
  if (lane == 0) smin[1][wid] = below;
  __syncthreads();  // every row in registers (ids[] may be written from here) and the four minima
  uint64_t cur = smin[1][0];
#pragma unroll
  for (int w = 1; w < NW; ++w) cur = smin[1][w] < cur ? smin[1][w] : cur;
  uint32_t out = lo;
  const uint32_t end = lo + m;
  for (int round = 0; round < max_rounds; ++round) {
    const int buf = round & 1;
    uint64_t nxt = ~0ull;
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < E; ++r) {
      c += (uint32_t)__popcll(__ballot(k[r] == cur));
      if (k[r] > cur && k[r] < nxt) nxt = k[r];
    }
    nxt = wave_min_u64(nxt);
    if (lane == 0) {
      scnt[buf][wid] = c;
      smin[buf][wid] = nxt;
    }
    __syncthreads();
    uint32_t base = out, tot = 0;
    uint64_t nb = ~0ull;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      base += w < wid ? scnt[buf][w] : 0u;
      tot += scnt[buf][w];
      nb = smin[buf][w] < nb ? smin[buf][w] : nb;
    }
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const bool hit = k[r] == cur;
      const uint64_t bal = __ballot(hit);
      const uint32_t dst = base + (uint32_t)__popcll(bal & lt);
      if (hit && dst < end) ids[dst] = id[r];
      base += (uint32_t)__popcll(bal);
    }
    out += tot;
    if (out >= end) return true;  // block-uniform
    cur = nb;
  }
  if (fuse) {
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const uint32_t pos = w0 + (uint32_t)(r * 64 + lane);
      if (pos < m) src[lo + pos] = id[r];
    }
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

// One wave's work on multi-key bucket b (rows [lo, lo + m)): copy its ids (and, gather mode, its keys)
// to the side buffers, then the stable partition, or the in-register network, or the big-bucket list.
__device__ __forceinline__ void msd_bucket(const int64_t* __restrict__ col, int desc, uint64_t kmin,
                                           uint64_t* __restrict__ keys, uint32_t* __restrict__ src,
                                           uint32_t* __restrict__ ids, uint32_t b, uint32_t lo, uint32_t m, int s1,
                                           uint32_t* __restrict__ ctl, uint32_t* __restrict__ big, int lane,
                                           bool fuse_copy) {
  // this bucket's grouped ids to the side buffer (free after the last pass), and (gather mode) their keys
  // gathered from the column by id, read from there below; with the sorted keys written by the last pass
  // the copy rides on the first partition round instead (DDSHE_ORDER_FUSECOPY=0: this loop, A/B)
  const bool fuse = col == nullptr && fuse_copy;
  for (uint32_t p0 = 0; p0 < (fuse ? 0u : m); p0 += 512) {  // 8 loads in flight per lane, then their stores
    uint32_t v[8];
    int64_t c[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint32_t p = p0 + (uint32_t)(r * 64 + lane);
      v[r] = ids[lo + min(p, m - 1)];
    }
    if (col) {
#pragma unroll
      for (int r = 0; r < 8; ++r) c[r] = col[v[r]];
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint32_t p = p0 + (uint32_t)(r * 64 + lane);
      if (p < m) {
        src[lo + p] = v[r];
        if (col) keys[lo + p] = rs_ukey((uint64_t)c[r], desc) - kmin;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wave's copies land before its lanes read them
  const int rounds = m <= kMsdWaveMax ? 2 : 16;
  const bool done = msd_wave_partition(keys, src, ids, lo, m, lane, rounds, fuse);
  if (done) return;
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

// Bucket ranges (DDSHE_ORDER_MSDLIST=0, round 6's A/B path): one wave per `per_wave` consecutive buckets:
// the wave's first lanes read their buckets' table entries
// together, a ballot marks the buckets holding two distinct keys, and the wave orders those one after
// another (bucket bounds made wave-uniform, so its addressing stays scalar). Round 5 ran one wave per
// bucket: 65,536 waves, most reading one word and exiting. Same box, k_msd_local per 10M-row call on the
// bench's OPE column (profiles/r06_msdwave_ab.txt): 1 bucket per wave 42.8 us, 2: 39.9, 4: 45.0, 8: ~51
// (neighbouring multi-key buckets serialise); uniform 54-bit keys (every bucket multi-key): call 0.709 ->
// 0.683 ms at 2.
// (per_wave: DDSHE_ORDER_MSDWAVE, 2 by default; 1 is round 5's one wave per bucket, A/B; a power of 2 <= 64)
// Lists (DDSHE_ORDER_MSDLIST=1, default; same box, profiles/r06_msdlist_ab.txt: raw call 0.270 -> 0.257 ms
// on the bench column, uniform 54-bit keys within 1 %): k_msd_list first gathers the multi-key buckets, block i of 64
// (1024 threads, one per bucket) writing its buckets of <= kMsdWaveMax rows to the front of list[1024 i ..
// 1024 i + 1024), the larger ones to the back, and the two counts to count[i] / count[64 + i] (no atomics:
// one atomic counter serialised 1,024 waves, 7.4 us). Then k_msd_local's waves take the small entries
// (wave w: entries w, w + waves, ...; each wave scans the 64 counts itself to find entry w) and
// k_msd_local_blk's blocks the large ones, one 256-thread block per bucket partitioning from registers up
// to 4,096 rows (msd_block_partition; wave 0 on the memory rounds above that). The bench column's ~600
// multi-key buckets of ~1,900 (2 keys) to ~3,950 rows (4 keys) then run one per block instead of one per
// wave on the memory rounds, queued behind the 65,536 / per_wave bucket ranges, most of which find nothing.
constexpr int kMsdListBlocks = 64;
constexpr int kMsdSmallBlocks = 1024;  // small list: 4,096 waves
constexpr int kMsdLargeBlocks = 768;   // large list: 3 blocks per CU, one bucket each at a time
// counts (small, large), then the small and the large segments (uint4 {bucket, first row, rows, 0} entries)
constexpr uint32_t kMsdListWords = 2 * kMsdListBlocks + 8 * kMsdBuckets;
static_assert(kMsdListBlocks * 1024 == (int)kMsdBuckets, "k_msd_list: one thread per bucket");
__global__ void __launch_bounds__(1024) k_msd_list(MsdRuns runs, uint32_t* __restrict__ list,
                                                   const uint64_t* __restrict__ plan) {
  if (plan && plan[1] == kRsNoPlan) return;
  __shared__ uint32_t wsmall[16], wlarge[16];
  const uint32_t b = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t lo = runs.first[b];
  const bool need = lo != ~0u && (runs.multi[b] != 0u || runs.kmin[b] != runs.kmax[b]);
  const bool large = need && runs.end[b] - lo > kMsdWaveMax;
  const uint64_t bs = __ballot(need && !large), bl = __ballot(large);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    wsmall[wid] = (uint32_t)__popcll(bs);
    wlarge[wid] = (uint32_t)__popcll(bl);
  }
  __syncthreads();
  uint32_t ps = 0, pl = 0, ts = 0, tl = 0;
  for (int w = 0; w < 16; ++w) {
    ps += w < wid ? wsmall[w] : 0u;
    pl += w < wid ? wlarge[w] : 0u;
    ts += wsmall[w];
    tl += wlarge[w];
  }
  const uint64_t lt = (1ull << lane) - 1ull;
  uint4* segs = reinterpret_cast<uint4*>(list + 2 * kMsdListBlocks) + blockIdx.x * 1024;
  if (large) segs[kMsdBuckets + pl + (uint32_t)__popcll(bl & lt)] = make_uint4(b, lo, runs.end[b] - lo, 0u);
  else if (need) segs[ps + (uint32_t)__popcll(bs & lt)] = make_uint4(b, lo, runs.end[b] - lo, 0u);
  if (threadIdx.x == 0) {
    list[blockIdx.x] = ts;
    list[kMsdListBlocks + blockIdx.x] = tl;
  }
}

// entry q of one kind of k_msd_list's output (uint4 {bucket, first row, rows, 0}: the bucket's bounds ride
// in its entry, no dependent load for them), by one wave: the 64 counts' prefix, kept in registers across
// the wave's entries
struct MsdListView {
  uint32_t incl, c, n;
  const uint4* segs;
  __device__ MsdListView(const uint32_t* list, bool large, int lane) {
    c = list[(large ? kMsdListBlocks : 0) + lane];
    segs = reinterpret_cast<const uint4*>(list + 2 * kMsdListBlocks) + (large ? kMsdBuckets : 0u);
    incl = c;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
      if (lane >= off) incl += y;
    }
    n = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)incl, 63));
  }
  __device__ uint4 entry(uint32_t q) const {  // q < n, wave-uniform
    const int seg = __popcll(__ballot(incl <= q));
    return segs[(uint32_t)seg * 1024 + q - (uint32_t)__shfl((int)(incl - c), seg)];
  }
};

__global__ void __launch_bounds__(256) k_msd_local(const int64_t* __restrict__ col, int desc, uint64_t kmin,
                                                   uint64_t* __restrict__ keys, uint32_t* __restrict__ src,
                                                   uint32_t* __restrict__ ids, MsdRuns runs,
                                                   uint32_t* __restrict__ ctl, uint32_t* __restrict__ big,
                                                   const uint64_t* __restrict__ plan, uint32_t per_wave,
                                                   bool fuse_copy, const uint32_t* __restrict__ list = nullptr) {
  if (plan) {
    const uint64_t s1 = plan[1];
    if (s1 == kRsNoPlan) return;
    kmin = plan[0];
    runs.s1 = (int)s1;
  }
  const int lane = threadIdx.x & 63;
  if (list) {  // the small entries of k_msd_list
    const MsdListView lv(list, false, lane);
    const uint32_t step = gridDim.x * 4;
    uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint4 e = q < lv.n ? lv.entry(q) : make_uint4(0, 0, 0, 0);
    while (q < lv.n) {  // the next entry's load in flight behind this bucket's work
      const uint32_t qn = q + step;
      const uint4 en = qn < lv.n ? lv.entry(qn) : make_uint4(0, 0, 0, 0);
      const uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)e.x);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)e.y);
      const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)e.z);
      msd_bucket(col, desc, kmin, keys, src, ids, b, lo, m, runs.s1, ctl, big, lane, fuse_copy);
      e = en;
      q = qn;
    }
    return;
  }
  const uint32_t b0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * per_wave;
  const uint32_t bl = b0 + ((uint32_t)lane & (per_wave - 1));
  const uint32_t lo_l = runs.first[bl];
  const bool need = lane < (int)per_wave && lo_l != ~0u &&
                    (runs.multi[bl] != 0u || runs.kmin[bl] != runs.kmax[bl]);
  const uint32_t m_l = need ? runs.end[bl] - lo_l : 0u;
  uint64_t mask = __ballot(need);
  while (mask) {
    const int j = __builtin_ctzll(mask);
    mask &= mask - 1ull;
    // wave-uniform (SGPRs): the bucket's addressing stays scalar in msd_bucket
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)lo_l, j));
    const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)m_l, j));
    msd_bucket(col, desc, kmin, keys, src, ids, b0 + (uint32_t)j, lo, m, runs.s1, ctl, big, lane, fuse_copy);
  }
}

// the large entries of k_msd_list (> kMsdWaveMax rows), one block per bucket: the register partition up to
// 256 x kMsdBlkRows rows with the fused side copy (the default); above that, or with the copy loop (gather
// mode, DDSHE_ORDER_FUSECOPY=0), wave 0 alone as k_msd_local would; a bucket whose 16 rounds run out goes
// to k_msd_big's list
__global__ void __launch_bounds__(kMsdBlkThreads) k_msd_local_blk(const int64_t* __restrict__ col, int desc, uint64_t kmin,
                                                       uint64_t* __restrict__ keys, uint32_t* __restrict__ src,
                                                       uint32_t* __restrict__ ids, MsdRuns runs,
                                                       uint32_t* __restrict__ ctl, uint32_t* __restrict__ big,
                                                       const uint64_t* __restrict__ plan, bool fuse_copy,
                                                       const uint32_t* __restrict__ list) {
  if (plan) {
    const uint64_t s1 = plan[1];
    if (s1 == kRsNoPlan) return;
    kmin = plan[0];
    runs.s1 = (int)s1;
  }
  constexpr int NW = kMsdBlkThreads / 64;
  __shared__ uint32_t scnt[2][NW];
  __shared__ uint64_t smin[2][NW];
  const int lane = threadIdx.x & 63;
  const bool fuse = col == nullptr && fuse_copy;
  const MsdListView lv(list, true, lane);  // every wave of the block: the same entries
  for (uint32_t q = blockIdx.x; q < lv.n; q += gridDim.x) {
    const uint4 e = lv.entry(q);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)e.x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)e.y);
    const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)e.z);
    if (fuse && m <= (uint32_t)kMsdBlkThreads * kMsdBlkRows) {
      if (!msd_block_partition<kMsdBlkRows, NW>(keys, src, ids, lo, m, 16, true, scnt, smin) && threadIdx.x == 0)
        big[atomicAdd(&ctl[kMsdCtlBig], 1u)] = b;
      __syncthreads();  // scnt / smin free for the next bucket
    } else if (threadIdx.x < 64) {
      msd_bucket(col, desc, kmin, keys, src, ids, b, lo, m, runs.s1, ctl, big, lane, fuse_copy);
    }
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
// hout (nullable): the call's read-back words (overflow flag, plan) stored to the host-mapped words by the
// last block to finish (a ticket in ctl, cleared with the table by the call's first histogram), instead
// of a k_rs_publish launch after it (DDSHE_ORDER_PUBLISH=1, A/B). kMsdBigBlocks < 2^16 (ticket bits).
__global__ void __launch_bounds__(1024) k_msd_big(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ src,
                                                  uint32_t* __restrict__ ids, MsdRuns runs, uint32_t* __restrict__ ctl,
                                                  const uint32_t* __restrict__ big, const uint64_t* __restrict__ plan,
                                                  uint64_t* __restrict__ hout) {
  bool planned = true;
  if (plan) {
    const uint64_t s1 = plan[1];
    planned = s1 != kRsNoPlan;
    runs.s1 = planned ? (int)s1 : 0;
  }
  __shared__ uint64_t xch[kMsdBlockMax];
  const uint32_t nbig = planned ? ctl[kMsdCtlBig] : 0u;
  const uint64_t rmask = (1ull << runs.s1) - 1ull;
  bool ovf_blk = false;  // this block raised the overflow flag
  for (uint32_t q = blockIdx.x; q < nbig; q += gridDim.x) {
    const uint32_t b = big[q];
    const uint32_t lo = runs.first[b], m = runs.end[b] - lo;
    if (m > kMsdBlockMax) {
      if (threadIdx.x == 0) atomicOr(&ctl[kMsdCtlOverflow], 1u);
      ovf_blk = true;
      continue;
    }
    if (m <= 2048) msd_block_sort<2, 11>(keys, src, ids, lo, m, rmask, xch);
    else if (m <= 4096) msd_block_sort<4, 12>(keys, src, ids, lo, m, rmask, xch);
    else msd_block_sort<8, 13>(keys, src, ids, lo, m, rmask, xch);
    __syncthreads();  // xch is free for the next bucket
  }
  if (hout && threadIdx.x == 0) {
    if (!planned) {  // nothing ran (the table was not cleared this call): block 0 reports the missing plan
      if (blockIdx.x == 0) {
        hout[2] = 0ull;
        hout[3] = kRsNoPlan;
      }
      return;
    }
    // planned: the call's first histogram cleared the ticket with the table. One atomic per block carries
    // both the ticket (low 16 bits) and whether the block overflowed (bits 16+), so the last block reads
    // the overflow verdict from its own atomic's result: no fence, no second word to order against.
    const uint32_t add = 1u + (ovf_blk ? 0x10000u : 0u);
    const uint32_t v = atomicAdd(&ctl[kMsdCtlTicket], add) + add;
    if ((v & 0xFFFFu) == gridDim.x) {  // every other block is done
      hout[2] = (v >> 16) != 0u ? 1ull : 0ull;
      hout[3] = plan ? plan[1] : 0ull;
      ctl[kMsdCtlTicket] = 0u;
    }
  }
}

size_t rs_blocks(size_t n) { return (n + kRsTile - 1) / kRsTile; }
size_t rs_scratch_bytes(size_t n) {
  // keys x2 (8 B), ids x1 extra (4 B; the other id buffer is the caller's output), histogram, OR/AND,
  // MSD bucket starts + control words + big-bucket list
  return 2 * n * 8 + 32 + n * 4 + (size_t)kRsDigits * (rs_blocks(n) + 2) * 4 + 1024 +
         (size_t)kRsDigits * ((rs_blocks(n) + kScanTiles - 1) / kScanTiles) * 4 + 256 +
         16 * std::max((n + 256 * kRsPrepRows - 1) / (256 * kRsPrepRows), rs_blocks(n)) + 8 * kCarryWords + 800 +
         (8 * (size_t)kMsdBuckets + 8 + kMsdListWords) * 4;
}

// the MSD path pays off from 4 LSD passes on (a span of > 24 bits) and enough rows to fill the buckets
static bool msd_enabled(size_t n, int sb) {
  static const int mode = [] {
    const char* s = getenv("DDSHE_ORDER_MSD");  // 0: LSD passes only (A/B)
    return s ? atoi(s) : 1;
  }();
  return mode != 0 && n >= ((size_t)1 << 16) && sb > 24;
}

static int order_env(const char* name, int dflt) {
  const char* s = getenv(name);
  return s ? atoi(s) : dflt;
}
static int order_xcd() {
  static const int mode = [] {
    const char* s = getenv("DDSHE_ORDER_XCD");  // 0: tile = block (A/B)
    return s ? atoi(s) : 1;
  }();
  return mode;
}

// one LSD pass: per-tile digit counts, their scan over tiles, the stable scatter (tiles of BLK x kRsItems
// rows; 256 threads measured fastest: 512 / 1024-thread tiles lengthen the write-out's digit runs but
// cut the blocks per CU, +0 / +10 us on the first pass of 10M rows)
// First pass of a carried plan (launch_ope_order's prep-free path): the histogram runs with the carried
// kmin and shift (absolute) and atomicMax's each block's largest holder key into *mm; k_rs_scan_chunks checks
// the plan with it before the scatter (which, like every later kernel, reads the plan from red + 2).
struct CarryPass {
  uint64_t* mm = nullptr;  // nullptr: no carried plan; else the word the first histogram's blocks atomicMax into
  uint64_t* red = nullptr;  // the plan goes to red + 2
  uint64_t kmin = 0;
  int s1 = -1;
};

template <int BLK>
static void rs_pass(hipStream_t st, const uint64_t* kin, const uint32_t* ids_in, const uint8_t* valid, size_t n,
                    int shift, bool last, int desc, bool vbit, bool kbit, uint64_t kmin, uint32_t* hist,
                    uint32_t* ctot, uint32_t* dtot, uint64_t* kout, uint32_t* ids_out, uint32_t* clr,
                    const MsdRuns& runs, const uint32_t* khi, uint32_t* khi_out, const uint64_t* plan,
                    const CarryPass& cp = CarryPass{}) {
  const size_t nb = (n + RsTile<BLK>::kRows - 1) / RsTile<BLK>::kRows;
  // 16-byte key pairs for the counts: aligned keys (and valid bytes when the first pass reads them), no
  // id read (DDSHE_ORDER_HPAIR=0: one row per lane, A/B)
  static const int hpair = order_env("DDSHE_ORDER_HPAIR", 1);
  const bool pairs = hpair && ((uintptr_t)kin & 15) == 0 && (ids_in || !valid || ((uintptr_t)valid & 1) == 0) &&
                     !(last && valid && !kbit);
  // digit counts by per-row LDS atomics into per-wave copies (DDSHE_ORDER_HATOM=0: one atomic per distinct
  // digit of a wave, found by 9 ballots, A/B): same box, 10M rows, raw call 0.318 -> 0.287 ms on the bench's
  // OPE column, 0.675 -> 0.652 on uniform 54-bit keys, 0.265 -> 0.275 with every wave's digits equal
  static const int hatom = order_env("DDSHE_ORDER_HATOM", 1);
  if (cp.mm) {  // carried plan: checked by k_rs_scan_chunks, before the scatter reads it
    hipLaunchKernelGGL((k_rs_hist<BLK, BLK>), dim3((unsigned)nb), dim3(BLK), 0, st, kin, ids_in, valid, n,
                       shift + cp.s1, last, desc, vbit, kbit, cp.kmin, hist, nb, clr, clr ? kMsdTableWords : 0u,
                       pairs && !khi, khi, nullptr, hatom != 0, cp.mm);
  } else {
    hipLaunchKernelGGL((k_rs_hist<BLK, BLK>), dim3((unsigned)nb), dim3(BLK), 0, st, kin, ids_in, valid, n, shift, last,
                       desc, vbit, kbit, kmin, hist, nb, clr, clr ? kMsdTableWords : 0u, pairs && !khi, khi, plan,
                       hatom != 0);
  }
  const size_t nch = (nb + kScanTiles - 1) / kScanTiles;
  hipLaunchKernelGGL(k_rs_scan_tiles, dim3((unsigned)nch), dim3(kScanThreads), 0, st, hist, nb, ctot);
  if (cp.mm)
    hipLaunchKernelGGL(k_rs_scan_chunks, dim3(1), dim3(kScanThreads), 0, st, ctot, nch, dtot, cp.mm, cp.red + 2,
                       cp.kmin, cp.s1);
  else
    hipLaunchKernelGGL(k_rs_scan_chunks, dim3(1), dim3(kScanThreads), 0, st, ctot, nch, dtot, nullptr, nullptr, 0ull,
                       -1);
  hipLaunchKernelGGL(k_rs_scatter<BLK>, dim3((unsigned)nb), dim3(BLK), 0, st, kin, ids_in, valid, n, shift, desc, vbit,
                     kbit, last, kmin, hist, ctot, dtot, nb, kout, ids_out, order_xcd(), runs, khi, khi_out, plan);
}

// Spans of kSpecLo..kSpecHi bits take the MSD path with split keys and (with a valid array) the key-bit
// validity; a raw call whose previous raw call had such a span launches that plan right after the
// min / max pass without reading the bounds back first (speculative: the plan's shifts and kmin come
// from k_rs_red on the device; another span makes every kernel of the plan return at once and the
// call continues on the host-planned path from the bounds the same pass stored to host memory).
constexpr int kSpecLo = 40, kSpecHi = 56;
static std::atomic<int> g_order_spec{0};
// The plan of the last raw call that ran the MSD path (kmin, s1, direction), carried to the next raw call:
// that call skips the min / max pass (k_rs_prep + k_rs_red before the passes) — its first histogram uses
// the carried plan and takes its largest holder key, k_rs_scan_chunks checks the plan with it
// before the first scatter, and a plan that no longer fits (keys below kmin, or a span of another bit
// length) makes every later kernel return; the call then runs the min / max pass and goes on as a call
// without a carried plan. Shared by every caller (a race only costs a failed check).
// DDSHE_ORDER_CARRY=0: the min / max pass every call (A/B).
struct CarriedPlan {
  uint64_t kmin;
  int s1;   // -1: none
  int desc;
};
static std::mutex g_carry_mu;
static CarriedPlan g_carry{0, -1, 0};
static CarriedPlan carry_get() {
  std::lock_guard<std::mutex> lk(g_carry_mu);
  return g_carry;
}
static void carry_set(CarriedPlan p) {
  std::lock_guard<std::mutex> lk(g_carry_mu);
  g_carry = p;
}

hipError_t launch_ope_order(const int64_t* col, const uint8_t* valid, size_t n, int desc, void* scratch,
                            uint32_t* out_ids, hipStream_t st, const uint64_t* ubounds, const MappedWords* hw) {
  if (n == 0) return hipSuccess;
  const size_t nb = rs_blocks(n);
  uint64_t* ka = (uint64_t*)scratch;
  // split keys keep their high words at word round_up(n, 4) of ka (16-byte aligned: the last histogram
  // reads them four rows per uint4), so kb starts 16 bytes past an even row count
  const size_t hi_word = (n + 3) & ~(size_t)3;
  uint64_t* kb = ka + ((n + 1) & ~(size_t)1) + 2;
  uint32_t* ib = (uint32_t*)(kb + n);
  uint32_t* hist = (uint32_t*)(((uintptr_t)(ib + n) + 255) & ~(uintptr_t)255);
  uint32_t* dtot = hist + (size_t)kRsDigits * nb;
  const size_t nch = (nb + kScanTiles - 1) / kScanTiles;
  uint32_t* ctot = (uint32_t*)(((uintptr_t)(dtot + kRsDigits) + 255) & ~(uintptr_t)255);
  uint64_t* red = (uint64_t*)(((uintptr_t)(ctot + (size_t)kRsDigits * nch) + 15) & ~(uintptr_t)15);
  uint64_t* part = red + 4;  // red[0..1] min / max, red[2..3] the speculative plan
  const size_t pb = (n + 256 * kRsPrepRows - 1) / (256 * kRsPrepRows);
  // MSD bucket table (MsdRuns layout), then the control words and the big-bucket list (part: the prep
  // blocks' bounds; cword: the carried plan's max word)
  uint64_t* cword = part + 2 * std::max(pb, nb);  // the carried plan's max words (nothing else writes them)
  uint32_t* mtab = (uint32_t*)(((uintptr_t)(cword + kCarryWords) + 255) & ~(uintptr_t)255);
  MsdRuns runs{mtab, (unsigned long long*)(mtab + kMsdBuckets), mtab + 3 * kMsdBuckets,
               (unsigned long long*)(mtab + 4 * kMsdBuckets), mtab + 6 * kMsdBuckets, 0};
  uint32_t* mctl = mtab + 7 * kMsdBuckets;
  uint32_t* mbig = mctl + 8;
  uint32_t* mlist = mbig + kMsdBuckets;  // k_msd_list's counts, then its multi-key buckets (kMsdListWords)
  hipError_t e = hipSuccess;
  // the last pass writes the sorted keys too (DDSHE_ORDER_KEYS2=0: k_msd_local gathers its buckets' keys
  // from the column by id instead: 80 MB less written, but k_msd_local 42 -> 59 us against scatter 76 -> 66)
  static const int keys2 = order_env("DDSHE_ORDER_KEYS2", 1);
  // the MSD path's first pass writes its keys as high and low 32-bit words in two arrays (the first n
  // words of ka: low, the next n: high) when the last pass's digit and the validity bit are in the high
  // words (span >= 2^40): the last histogram then reads 4 B per row (DDSHE_ORDER_SPLIT=0: 8 B, A/B)
  static const int split_env = order_env("DDSHE_ORDER_SPLIT", 1);
  static const int spec_env = order_env("DDSHE_ORDER_SPEC", 1);  // 0: bounds always read back first (A/B)
  // executed pass j writes ids to fin when (np-1-j) is even, so the last one lands there; with msd.first
  // set the first pass clears the bucket table and the last fills it. plan: shifts relative to s1, kmin
  // and s1 from the device
  auto run_passes = [&](const int* shifts, int np, uint32_t* fin, uint32_t* tmp, const MsdRuns& msd, bool split,
                        bool kbit, bool vbit, uint64_t kmin, const uint64_t* plan,
                        const CarryPass& cp = CarryPass{}) {
    const uint32_t* ids_in = nullptr;  // identity before the first pass
    const uint64_t* kin = (const uint64_t*)col;  // raw column before the first pass
    uint64_t* kout = ka;
    const MsdRuns none{};
    uint32_t* hi = split ? reinterpret_cast<uint32_t*>(ka) + hi_word : nullptr;  // ka = [low n words | high n words]
    for (int j = 0; j < np; ++j) {
      uint32_t* ids_out = ((np - 1 - j) % 2 == 0) ? fin : tmp;
      const bool last = j == np - 1;
      rs_pass<256>(st, kin, ids_in, valid, n, shifts[j], last, desc, vbit, kbit, kmin, hist, ctot, dtot,
                   last ? (msd.first && keys2 ? kout : nullptr) : kout, ids_out, j == 0 ? msd.first : nullptr,
                   last ? msd : none, j == 1 ? hi : nullptr, j == 0 ? hi : nullptr, plan,
                   j == 0 ? cp : CarryPass{});
      kin = kout;
      kout = kout == ka ? kb : ka;
      ids_in = ids_out;
    }
  };
  static const int publish_env = order_env("DDSHE_ORDER_PUBLISH", 0);  // 1: k_rs_publish launch (A/B)
  auto msd_tail = [&](uint64_t kmin, const uint64_t* plan) {
    static const int fuse_copy = order_env("DDSHE_ORDER_FUSECOPY", 1);
    static const uint32_t per_wave = [] {
      const int v = order_env("DDSHE_ORDER_MSDWAVE", 2);
      return (v >= 1 && v <= 64 && (v & (v - 1)) == 0) ? (uint32_t)v : 2u;
    }();
    static const int list_env = order_env("DDSHE_ORDER_MSDLIST", 1);  // 0: bucket ranges per wave (A/B)
    if (list_env) {
      hipLaunchKernelGGL(k_msd_list, dim3(kMsdListBlocks), dim3(1024), 0, st, runs, mlist, plan);
      hipLaunchKernelGGL(k_msd_local, dim3(kMsdSmallBlocks), dim3(256), 0, st, keys2 ? nullptr : col, desc, kmin, kb,
                         ib, out_ids, runs, mctl, mbig, plan, per_wave, fuse_copy != 0, mlist);
      hipLaunchKernelGGL(k_msd_local_blk, dim3(kMsdLargeBlocks), dim3(kMsdBlkThreads), 0, st, keys2 ? nullptr : col, desc, kmin,
                         kb, ib, out_ids, runs, mctl, mbig, plan, fuse_copy != 0, mlist);
    } else {
      hipLaunchKernelGGL(k_msd_local, dim3(kMsdBuckets / (4 * per_wave)), dim3(256), 0, st, keys2 ? nullptr : col,
                         desc, kmin, kb, ib, out_ids, runs, mctl, mbig, plan, per_wave, fuse_copy != 0, nullptr);
    }
    hipLaunchKernelGGL(k_msd_big, dim3(kMsdBigBlocks), dim3(1024), 0, st, kb, ib, out_ids, runs, mctl, mbig, plan,
                       (hw && !publish_env) ? hw->d : nullptr);
  };
  // words 2..3 of hw after the call's device work: overflow flag, plan
  auto read_ctl = [&](const uint64_t* plan, uint64_t* ovf, uint64_t* pl) -> hipError_t {
    if (hw) {
      if (publish_env) hipLaunchKernelGGL(k_rs_publish, dim3(1), dim3(1), 0, st, mctl, plan, hw->d);
      hipError_t r = hipStreamSynchronize(st);
      *ovf = hw->h[2];
      *pl = hw->h[3];
      return r;
    }
    uint32_t hctl[2];
    hipError_t r = hipMemcpyAsync(hctl, mctl, sizeof(hctl), hipMemcpyDeviceToHost, st);
    if (r == hipSuccess) r = hipStreamSynchronize(st);
    *ovf = hctl[kMsdCtlOverflow];
    *pl = 0;
    return r;
  };
  uint64_t hred[2];
  bool skip_msd = false;  // a speculative call's MSD plan ran and overflowed: straight to the LSD passes
  if (ubounds) {  // bounds of the raw values from the caller: the keys' bounds follow (desc: complemented)
    hred[0] = ubounds[0] <= ubounds[1] ? (desc ? ~ubounds[1] : ubounds[0]) : 1;
    hred[1] = ubounds[0] <= ubounds[1] ? (desc ? ~ubounds[0] : ubounds[1]) : 0;
  } else {
    static const int carry_env = order_env("DDSHE_ORDER_CARRY", 1);
    const CarriedPlan cpl = carry_get();
    bool carried = false;  // a carried plan ran and did not stand: the bounds come from the min / max pass now
    if (hw && carry_env && spec_env && split_env && msd_enabled(n, kSpecLo) && cpl.s1 >= 0 && cpl.desc == desc) {
      const uint64_t* plan = red + 2;
      CarryPass cp;
      cp.mm = cword;
      cp.red = red;
      cp.kmin = cpl.kmin;
      cp.s1 = cpl.s1;
      const int rel[2] = {0, 8};
      run_passes(rel, 2, out_ids, ib, runs, true, valid != nullptr, false, 0, plan, cp);
      msd_tail(0, plan);
      uint64_t ovf = 0, pl = 0;
      if ((e = read_ctl(plan, &ovf, &pl)) != hipSuccess) return e;
      if (pl != kRsNoPlan && !ovf) return hipGetLastError();  // the carried plan stands for the next call too
      carry_set(CarriedPlan{0, -1, 0});
      if (pl != kRsNoPlan) skip_msd = true;  // a crowded bucket overflowed: straight to the LSD passes
      carried = true;
    }
    const bool spec = !carried && hw && spec_env && split_env && msd_enabled(n, kSpecLo) &&
                      g_order_spec.load(std::memory_order_relaxed);
    if (((uintptr_t)col & 15) == 0 && ((uintptr_t)valid & 1) == 0)
      hipLaunchKernelGGL(k_rs_prep, dim3((unsigned)pb), dim3(256), 0, st, col, valid, n, desc, part);
    else
      hipLaunchKernelGGL(k_rs_prep_rows, dim3((unsigned)pb), dim3(256), 0, st, col, valid, n, desc, part);
    hipLaunchKernelGGL(k_rs_red, dim3(1), dim3(1024), 0, st, part, pb, red, spec ? kSpecLo : 1, spec ? kSpecHi : 0,
                       hw ? hw->d : nullptr);
    if (spec) {
      const uint64_t* plan = red + 2;
      const int rel[2] = {0, 8};
      run_passes(rel, 2, out_ids, ib, runs, true, valid != nullptr, false, 0, plan);
      msd_tail(0, plan);
      uint64_t ovf = 0, pl = 0;
      if ((e = read_ctl(plan, &ovf, &pl)) != hipSuccess) return e;
      if (pl != kRsNoPlan && !ovf) return hipGetLastError();
      if (pl == kRsNoPlan) g_order_spec.store(0, std::memory_order_relaxed);
      else skip_msd = true;
      hred[0] = hw->h[0];
      hred[1] = hw->h[1];
    } else if (hw) {
      if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
      hred[0] = hw->h[0];
      hred[1] = hw->h[1];
    } else {
      if ((e = hipMemcpyAsync(hred, red, sizeof(hred), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
      if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    }
  }
  // the bytes of max - min (at least one pass when rows may lack the position: its last pass buckets them)
  const uint64_t kmin = hred[0] <= hred[1] ? hred[0] : 0ull;
  const uint64_t span = hred[0] <= hred[1] ? hred[1] - hred[0] : 0ull;
  const int sb = span ? 64 - __builtin_clzll(span) : 0;  // bits of the span
  const bool kbit = valid && sb <= 56;                    // validity in key bit 63 (every shift <= 48)
  const bool vbit = valid && !kbit && n <= (size_t)kRsLack;
  if (!ubounds && hw) {
    g_order_spec.store(sb >= kSpecLo && sb <= kSpecHi, std::memory_order_relaxed);
    // the next raw call may carry this plan (the MSD path below runs it with split keys and, with a
    // valid array, the key-bit validity: what the carried path runs)
    const bool carriable = sb >= kSpecLo && sb <= kSpecHi && !skip_msd && msd_enabled(n, sb) && split_env &&
                           (!valid || sb <= 56);
    carry_set(carriable ? CarriedPlan{kmin, sb - kMsdBits, desc} : CarriedPlan{0, -1, 0});
  }
  if (!skip_msd && msd_enabled(n, sb)) {
    runs.s1 = sb - kMsdBits;
    const int shifts[2] = {runs.s1, sb - 8};
    const bool split = split_env && (!valid || kbit) && shifts[1] >= 32;
    // grouped ids -> out_ids (one-key buckets are final there) + the bucket table; ib (the first pass's
    // ids) and kb are then free: the side copies of the multi-key buckets' ids and keys (k_msd_local)
    run_passes(shifts, 2, out_ids, ib, runs, split, kbit, vbit, kmin, nullptr);
    msd_tail(kmin, nullptr);
    uint64_t ovf = 0, pl = 0;
    if ((e = read_ctl(nullptr, &ovf, &pl)) != hipSuccess) return e;
    if (!ovf) return hipGetLastError();
    // a bucket of > 8192 rows with > 16 distinct keys: redo the whole sort with the LSD passes
  }
  int shifts[8], np = 0;
  for (int p = 0; p < 8 && (span >> (8 * p)) != 0; ++p) shifts[np++] = 8 * p;
  if (np == 0 && valid) shifts[np++] = 0;
  if (np == 0) {
    hipLaunchKernelGGL(k_rs_iota, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out_ids, n);
    return hipGetLastError();
  }
  run_passes(shifts, np, out_ids, ib, MsdRuns{}, false, kbit, vbit, kmin, nullptr);
  return hipGetLastError();
}

}  // namespace ddshe
