// Internal launcher interface between the C-ABI (ddshe_capi.cpp) and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace ddshe {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // 16-byte vector loads

// per-modulus constant block: 5 vectors of S r27 limbs each
enum { kConstN = 0, kConstRmod = 1, kConstR2 = 2, kConstOne = 3, kConstN2x = 4, kConstCount = 5 };

struct Shape {
  int S;    // limbs
  int TPI;  // lanes per bignum
  int W;    // radix bits
};
// Largest column stride (rows, multiple of 64) the Montgomery kernels can address: mul_col reads a
// block of PF limbs through one buffer descriptor with num_records = PF*stride*4 and per-limb
// soffsets q*stride*4, all 32-bit (PF = 4 when S % 4 == 0, else 2). Beyond it the loads would wrap.
inline size_t max_stride(int S) {
  const size_t pf = (S % 4 == 0) ? 4 : 2;
  return (((size_t)1 << 32) / (4 * pf) - 1) / 64 * 64;
}
Shape pick_shape(size_t mod_bits);  // S == 0: unsupported
Shape tail_shape(const Shape& main);  // TPI = 16 shape (more limbs, same W) for tree levels + finalize
size_t max_modulus_bits();

hipError_t launch_ingest_be(const uint8_t* in, size_t width, size_t count, int S, int W, const uint32_t* n2x,
                            uint32_t* X, size_t stride, uint32_t* flags, hipStream_t st,
                            uint8_t* rowflags = nullptr);  // rowflags[i] = 1: row i >= 2N (stored reduced)
// rows [0, count) of an rW matrix (S <= 160 limbs of W bits, value < 2·nmod when nmod != nullptr, else
// canonical) -> width big-endian bytes each (canonical residue when nmod is given), row-major in out
hipError_t launch_egress_be(const uint32_t* X, size_t stride, size_t count, int S, int W, const uint32_t* nmod,
                            size_t width, uint8_t* out, hipStream_t st);
constexpr int kEgressMaxLimbs = 160;
// gate (nullable): the kernel does nothing unless gate[0] & 1 (k_ingest_be's "some row >= 2N" flag)
hipError_t launch_reduce_rows(int S, uint32_t* X, size_t stride, size_t count, const uint32_t* consts, uint32_t n0,
                              hipStream_t st, const uint32_t* gate = nullptr);
// main fold level (throughput shape); partial rows are zero-extended to s_out limbs
// qp_mod (nullable): N~ = N·n0 in main limbs (when W·S >= bits(N~) + 2; see Mont QP)
hipError_t launch_fold(int S, const uint32_t* X, size_t xstride, size_t count, const uint32_t* consts,
                       const uint32_t* qp_mod, uint32_t n0,
                       uint32_t* P, size_t pstride, size_t ngroups, int s_out, hipStream_t st,
                       const uint32_t* ids = nullptr,  // ids: fold rows ids[0..count) (device, u32)
                       int lane1 = 0,  // != 0: one bignum per lane (k_fold1) at lane1 = fold1_limbs(S, bits) limbs
                       size_t inblock_pgs = 0);  // != 0: k_fold InBlock, one row-major leaf of this many words per block
bool fold_qp_enabled();
// k_fold1 (one bignum per lane) exists for S (40, 76) and is worth its longer per-product latency for
// folds of at least fold1_min_rows(S) rows (DDSHE_FOLD1=0 disables it, DDSHE_FOLD1_MIN=<rows> overrides)
bool fold1_shape(int S);
int fold1_limbs(int S, size_t bits);
size_t fold1_min_rows(int S, int cus);
hipError_t fold1_occupancy(int S, int* blocks_per_cu);
// tree levels / finalize in the tail shape (S = tail limb count, consts of the tail shape)
// qp_mod (nullable): N~ = N·n0 in tail limbs, used by the latency-bound levels when tail_qp(S)
bool fold_narrow_shape(int S2);
hipError_t launch_fold_narrow(int S2, const uint32_t* X, size_t xstride, size_t count, int sin, const uint32_t* consts,
                              const uint32_t* qp_mod, uint32_t n0, uint32_t* P, size_t pstride, size_t ngroups,
                              hipStream_t st, size_t pgs = 1);
hipError_t launch_fold_tail(int S, const uint32_t* X, size_t xstride, size_t count, const uint32_t* consts,
                            const uint32_t* qp_mod, uint32_t n0, uint32_t* P, size_t pstride, size_t ngroups,
                            hipStream_t st, size_t pgs = 1);
bool tail_qp(int S);
// Reduction tree (ddshe_tree.hip): S limbs of W bits (Shape.TPI unused) for a main shape of up to
// mod_bits bits; one launch reduces nleaves leaves (limb-major X, Sin limbs of Win bits, stride xstride;
// leaf g is row ids[g] when ids != nullptr) to the canonical result (Y != nullptr: S limbs of W bits,
// times Y R^-1) or a canonical partial (Sout limbs of Wout bits). consts: N | n' | N | 2N | 3N.
// nodes: 4 nleaves + 2 rows of S words (nodes + level buffers), flags: 2 nleaves + 2 words (zeroed here).
// done (nullable; out in host memory): after the root has written out, *done = seq (system scope), so a
// caller can spin on it instead of synchronising the stream.
Shape tree_shape(size_t mod_bits);
hipError_t launch_tree(int S, const uint32_t* X, size_t xstride, int Sin, int Win, size_t nleaves, const uint32_t* ids,
                       const uint32_t* consts, const uint32_t* Y, uint32_t* nodes, uint32_t* flags, uint32_t* out,
                       int Sout, int Wout, hipStream_t st, size_t gstride = 1, uint32_t* done = nullptr,
                       uint32_t seq = 0);
// out[i] = A[i] * B[i] mod N in the tree shape (S limbs of W bits, row-major, operands < N, canonical
// results): one workgroup per pair (k_pairs_sos). consts as launch_tree, R2 = R^2 mod N (R = 2^(W S)).
hipError_t launch_pairs_sos(int S, const uint32_t* A, const uint32_t* B, size_t n, const uint32_t* consts,
                            const uint32_t* R2, uint32_t* out, hipStream_t st);
hipError_t launch_finalize_tail(int S, const uint32_t* P, size_t pstride, const uint32_t* consts, const uint32_t* Y,
                                uint32_t n0, uint32_t* out, hipStream_t st);
hipError_t launch_pairs(int S, const uint32_t* A, const uint32_t* B, size_t stride, size_t count,
                        const uint32_t* consts, uint32_t n0, uint32_t* O, hipStream_t st);
// the same in a tail (latency) shape: S = tail limbs, consts of the tail shape (a few pairs per launch)
hipError_t launch_pairs_tail(int S, const uint32_t* A, const uint32_t* B, size_t stride, size_t count,
                             const uint32_t* consts, uint32_t n0, uint32_t* O, hipStream_t st);
// modexp table: Tab[j] = x^(2j+1)*R mod N (j < nodd), entry j at Tab + j*S*tstride
hipError_t launch_modexp_pre(int S, const uint32_t* Xcol, size_t xstride, size_t count, const uint32_t* consts,
                             const uint32_t* qp_mod, uint32_t n0, int nodd, uint32_t* Tab, size_t tstride,
                             hipStream_t st);
// O = g^m_i * x_i^E mod N (m == nullptr: x_i^E) from the table and the host-built window schedule;
// gR = g*R mod N in rW limbs
hipError_t launch_modexp_ladder(int S, const uint32_t* Tab, size_t tstride, const uint32_t* m, size_t count,
                                const uint32_t* consts, const uint32_t* qp_mod, const uint32_t* gR,
                                const uint32_t* sched, int nsched, uint32_t n0, uint32_t* O, size_t ostride,
                                hipStream_t st);
// CRT encryption pieces (see ddshe_kernels.hip): radix change between rW layouts (flags[0] |= 1 on
// overflow), h = (y_p - y_q)(q^2)^-1 mod p^2 (c12 = c1R | c2R, 2*S limbs), c = h*q^2 + y_q
hipError_t launch_repack(const uint32_t* src, size_t sstride, int Ss, int Ws, uint32_t* dst, size_t dstride, int Sd,
                         int Wd, size_t count, uint32_t* flags, hipStream_t st);
hipError_t launch_crt_h(int S, const uint32_t* Yp, const uint32_t* Yq, size_t stride, size_t count,
                        const uint32_t* consts, const uint32_t* c12, uint32_t n0, uint32_t* H, hipStream_t st);
hipError_t launch_crt_out(int S, const uint32_t* Hn, const uint32_t* Yqn, size_t stride, size_t count,
                          const uint32_t* consts, const uint32_t* q2R, uint32_t n0, uint32_t* O, size_t ostride,
                          hipStream_t st);
hipError_t launch_fill_random(uint32_t* X, size_t stride, int S, int W, uint64_t seed, uint64_t row0, size_t count,
                              int bits, hipStream_t st);
hipError_t launch_gather_rows(const uint32_t* T, size_t tstride, uint32_t tcount, int S, uint64_t seed, uint64_t row0,
                              size_t count, uint32_t* X, size_t xstride, hipStream_t st);
hipError_t launch_synth_rows(int S, const uint32_t* T, size_t tstride, uint32_t tcount, const uint32_t* P,
                             size_t pstride, uint32_t pcount, uint64_t seed, uint64_t row0, size_t count,
                             const uint32_t* consts, uint32_t n0, uint32_t* X, size_t xstride, hipStream_t st,
                             uint32_t shards = 1, uint32_t shard = 0);  // row mapping of a sharded column
size_t ope_blocks(size_t n);
size_t ope_scratch_bytes(size_t n);  // per-tile match counts + per-thread match masks
// rows i with (valid[i] & vmask) != 0 and (valid[i] & vbad) == 0 (valid == nullptr: every row) and
// col[i] <op> bound -> ascending ids in out, count in *total (device)
hipError_t launch_ope_filter(const int64_t* col, const uint8_t* valid, size_t n, int64_t bound, int op, void* scratch,
                             uint64_t* total, uint32_t* out, hipStream_t st, uint32_t vmask = 0xFFu,
                             uint32_t vbad = 0u);
// Search as a row bitmask (no id scatter): after it, ope_mask_words(scratch, n)[w] bit b = row 32w + b
// matches (words in row order; bits past n are 0) and *total (device) the number of matches
// total_zeroed: *total is 0 on entry and the count kernel's tiles add into it (no reduction launch);
// hmask (device pointer of a mapped host buffer of hwords u32 words) with hcounts (device pointer of a
// mapped host array of ope_blocks(n) u32): the mask words and the per-tile match counts are written
// straight into host memory (total unused: the caller adds the counts up)
hipError_t launch_ope_mask(const int64_t* col, const uint8_t* valid, size_t n, int64_t bound, int op, void* scratch,
                           uint64_t* total, hipStream_t st, uint32_t vmask = 0xFFu, uint32_t vbad = 0u,
                           bool total_zeroed = false, uint32_t* hmask = nullptr, size_t hwords = 0,
                           uint32_t* hcounts = nullptr);
uint32_t* ope_mask_words(void* scratch, size_t n);
// rows i with (bytes[i] & vmask) != 0 -> ascending ids in out, count in *total (device); scratch as above.
// rezero: the count pass stores 0 over every non-zero byte it read (a flag buffer kept zeroed between uses)
hipError_t launch_byte_compact(const uint8_t* bytes, size_t n, uint32_t vmask, void* scratch, uint64_t* total,
                               uint32_t* out, hipStream_t st,
                               uint32_t vall = 0, bool rezero = false);
// resident-row mutations (ddshe_mutate.hip): rows ids[i] of dst (S limbs, stride dstride) <- column i of
// src (stride sstride); dst[ids[i]] <- vals[i] for bytes / u64; keep[p] = !dead[perm[p]]; dst[i] = src[idx[i]]
hipError_t launch_scatter_rows(const uint32_t* src, size_t sstride, const uint32_t* ids, size_t n, int S, uint32_t* dst,
                               size_t dstride, hipStream_t st);
hipError_t launch_scatter_bytes(const uint32_t* ids, const uint8_t* vals, size_t n, uint8_t* dst, hipStream_t st);
hipError_t launch_scatter_u64(const uint32_t* ids, const uint64_t* vals, size_t n, uint64_t* dst, hipStream_t st);
hipError_t launch_perm_keep(const uint32_t* perm, const uint8_t* dead, size_t n, uint8_t* keep, hipStream_t st);
hipError_t launch_gather_u32(const uint32_t* src, const uint32_t* idx, size_t n, uint32_t* dst, hipStream_t st);
// OPE ordering (ddshe_sort.hip): stable radix sort of the int64 column -> row ids
size_t rs_scratch_bytes(size_t n);
// ubounds (host, nullable): [lo, hi] of (value ^ 2^63) over a superset of the holders (a resident
// column tracks them on its writes): no min/max pass over the column and no mid-sort host round trip
// hw (nullable): 4 words of coherent, device-mapped host memory (h: host address, d: its device address)
// the ordering stores its small read-backs into (bounds, overflow flag) instead of copying them back; with
// it, a raw call whose previous raw call had a 40..56-bit key span runs the MSD plan without a mid-sort
// host round trip (planned on the device, checked after)
struct MappedWords {
  volatile uint64_t* h;
  uint64_t* d;
};
hipError_t launch_ope_order(const int64_t* col, const uint8_t* valid, size_t n, int desc, void* scratch,
                            uint32_t* out_ids, hipStream_t st, const uint64_t* ubounds = nullptr,
                            const MappedWords* hw = nullptr);
// deterministic-equality scans (ddshe_strscan.hip)
// 64-bit digest of an element string (FNV-1a over the bytes, splitmix finaliser); identical on
// host (needles) and device (table). The table keeps its top 16 bits as a per-element fingerprint
// (str_fp): a scan streams 2 B per element, and a fingerprint hit is always confirmed on the bytes, so
// the wider digest only changes how often that happens (round 5: 32 bits, 4 B per element).
using StrFp = uint16_t;
__host__ __device__ inline uint64_t str_digest(const uint8_t* p, uint64_t len) {
  uint64_t h = 0xcbf29ce484222325ull ^ len;
  for (uint64_t i = 0; i < len; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
  h ^= h >> 30;
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 27;
  h *= 0x94d049bb133111ebull;
  return h ^ (h >> 31);
}
__host__ __device__ inline StrFp str_fp(uint64_t digest) { return (StrFp)(digest >> 48); }
struct StrNeedles {  // up to 3 items (SearchEntryAND/OR triplets), bytes in a device buffer or inline
  uint64_t h[3];
  uint64_t len[3];
  uint64_t off[3];
  int n;
  // needles of up to kStrInline bytes in all travel in the kernel arguments (read from the kernarg
  // segment on a fingerprint hit): no upload before the scan; the kernels get nchars == nullptr then
  static constexpr int kStrInline = 128;
  uint8_t inl[kStrInline];
};
hipError_t launch_str_digest(const uint8_t* chars, const uint64_t* elem_off, size_t nelems, StrFp* fp,
                             hipStream_t st);
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
__device__ __forceinline__ bool str_equal(const uint8_t* __restrict__ x, const uint8_t* __restrict__ y, uint64_t len) {
  for (uint64_t i = 0; i < len; ++i)
    if (x[i] != y[i]) return false;
  return true;
}
// element e equals needle j (its fingerprint already matched): length, then bytes
__device__ __forceinline__ bool str_hit(uint64_t e, int j, const uint64_t* __restrict__ elem_off,
                                        const uint8_t* __restrict__ chars, const uint8_t* __restrict__ nchars,
                                        const StrNeedles& nd) {
  const uint64_t a = elem_off[e], b = elem_off[e + 1];
  const uint8_t* nb = nchars ? nchars : nd.inl;
  return b - a == nd.len[j] && str_equal(chars + a, nb + nd.off[j], nd.len[j]);
}
#endif
constexpr uint32_t kStrDead = 0xFFFFFFFFu;  // elem_row of a superseded element (ddshe_strscan.hip)
// SearchEq/NEq over a position index straight into the compaction masks (k_str_eq_count, the tile
// layout of k_ope_count) + k_ope_scatter: ascending row ids (relative to row0) of the matching rows;
// row_beg[r]: the first heap element of row r's current version
hipError_t launch_str_eq_compact(const StrFp* posfp, const uint64_t* present, size_t row0, size_t nrows,
                                 const uint64_t* row_beg, const uint64_t* elem_off, const uint8_t* chars,
                                 const uint8_t* nchars, const StrNeedles& nd, uint64_t position, int negate,
                                 void* scratch, uint64_t* total, uint32_t* out, hipStream_t st);
// SearchEq's position-major index (ddshe_strscan.hip): per row the fingerprint of element `position`
// and a present bit (live and length - 1 > position) for rows [r_first, r_first + count) (r_first a
// multiple of 64), or patched for the distinct rows ids[0..n)
hipError_t launch_str_posfp(const uint64_t* row_beg, const uint32_t* row_len, const uint8_t* live, size_t r_first,
                            size_t count, const StrFp* fp, uint64_t position, StrFp* posfp, uint64_t* present,
                            hipStream_t st);
hipError_t launch_str_posfp_ids(const uint32_t* ids, size_t n, const uint64_t* row_beg, const uint32_t* row_len,
                                const uint8_t* live, const StrFp* fp, uint64_t position, StrFp* posfp,
                                uint64_t* present, hipStream_t st);
// string-table mutations: row descriptors of distinct rows ids[i] <- (beg[i], len[i]), live; heap
// elements of superseded versions killed; heap compaction into fresh buffers (one wave per row)
hipError_t launch_str_rows_set(const uint32_t* ids, const uint64_t* beg, const uint32_t* len, size_t n,
                               uint64_t* row_beg, uint32_t* row_len, uint8_t* live, hipStream_t st);
hipError_t launch_str_kill(const uint64_t* beg, const uint32_t* len, size_t n, uint32_t* elem_row, hipStream_t st);
hipError_t launch_str_compact(size_t nrows, const uint64_t* old_beg, const uint32_t* len, const uint64_t* new_beg,
                              const uint64_t* new_cbeg, const uint64_t* elem_off, const StrFp* fp,
                              const uint8_t* chars, uint64_t* nelem_off, StrFp* nfp, uint32_t* nelem_row,
                              uint8_t* nchars, hipStream_t st);
// SearchEntry/OR/AND/IsElement: flag byte r - row0 |= bit j for every heap element in [e_first,
// e_first + nelems) equal to needle j whose owner r is live and in [row0, row0 + nrows) (flags zeroed by
// the launcher unless flags_zeroed, 4-byte aligned)
hipError_t launch_str_any(const StrFp* fp, uint64_t e_first, size_t nelems, const uint32_t* elem_row,
                          const uint8_t* live, size_t row0, size_t nrows, const uint64_t* elem_off, const uint8_t* chars,
                          const uint8_t* nchars, const StrNeedles& nd, uint8_t* flags, hipStream_t st,
                          bool flags_zeroed = false);
hipError_t launch_plain_sum(const uint32_t* X, size_t stride, size_t count, int S, size_t nthreads, uint64_t* part,
                            uint64_t* out, hipStream_t st);
// unbounded product tree level: rows (2p, 2p+1) of A[count][len] (radix 2^16 in u32)
// -> V[pairs][2 len] (limbs < 2^18, carries resolved by launch_bigmul_carry passes)
// cap != 0: keep only the low min(2 len, cap) limbs of each product (products mod 2^(16 cap))
hipError_t launch_bigmul_level(const uint32_t* A, size_t count, size_t len, uint64_t* Sk, uint32_t* V, hipStream_t st,
                               size_t cap = 0);
hipError_t launch_bigmul_carry(const uint32_t* V, size_t pairs, size_t outlen, uint32_t* Wout, uint32_t* flag,
                               hipStream_t st);
hipError_t fold_occupancy(int S, int* blocks_per_cu);
// dst[r*drs + c*dcs] = src[r*srs + c*scs] for r < rows, c < cols (u32 words, one device)
hipError_t launch_strided_copy(const uint32_t* src, size_t srs, size_t scs, uint32_t* dst, size_t drs, size_t dcs,
                               size_t rows, size_t cols, hipStream_t st);

// decimal codec (ddshe_codec.hip): per-row status bits
enum : uint32_t { kDecNeg = 1, kDecReduce = 2, kDecWide = 4, kDecFormat = 8 };
// chars4: staged chars, 4-byte aligned, row bytes at [offs[i] - obase + 16, offs[i+1] - obase + 16) with
// at least 16 readable bytes before and after; tab: per-modulus table (ModConsts::dec_table)
hipError_t launch_dec_parse(int S, const uint32_t* chars4, const uint64_t* offs, uint64_t obase, size_t count,
                            const uint32_t* tab, int jfit, int jpad, const uint32_t* consts, uint32_t* X,
                            size_t stride, uint8_t* rowflags, uint32_t* flags, hipStream_t st);
hipError_t launch_dec_fix(int S, uint32_t* X, size_t stride, size_t count, const uint8_t* rowflags,
                          const uint32_t* consts, uint32_t n0, hipStream_t st);

}  // namespace ddshe
