/*
 * ddshe.h — C-ABI of the MI355X homomorphic-aggregation engine.
 *
 * Drop-in boundary for the server-side aggregation path of
 * fmiguelgodinho/dependable-data-storage-csd2017. Every entry point names the
 * reference interface it replaces (paths relative to /root/reference/):
 *
 *   hlib  HomoAdd.sum(c1, c2, nsquare)        src/main/scala/dds/http/DDSRestServer.scala:385, :423
 *   hlib  HomoMult.multiply(c1, c2, pubkey)   src/main/scala/dds/http/DDSRestServer.scala:479, :518
 *   hlib  HomoAdd.encrypt(m, PaillierKey)     src/main/scala/utils/SJHomoLibProvider.scala:58
 *   route SumAll fold loop                    src/main/scala/dds/http/DDSRestServer.scala:397-446
 *   route MultAll fold loop                   src/main/scala/dds/http/DDSRestServer.scala:491-539
 *   route Search{Gt,GtEq,Lt,LtEq} loops       src/main/scala/dds/http/DDSRestServer.scala:682-830
 *
 * Conventions
 *  - Big integers cross the boundary as fixed-width BIG-ENDIAN unsigned
 *    magnitudes (what a JNA shim gets from BigInteger.toByteArray() after
 *    stripping the sign byte and left-padding), `width` bytes per value.
 *  - Every function returns a dds_status; no C++ exception crosses the ABI.
 *    DDS_E_EMPTY maps to the reference's HTTP 404 path, every other non-zero
 *    status to its HTTP 500 path (DDSRestServer.scala:432-442).
 *  - Thread-safe: any number of threads may call into one dds_ctx; each call
 *    runs on its own HIP stream taken from the context's pool.
 *  - The caller owns every host buffer. Device columns (dds_col) are owned by
 *    the library and freed only by dds_col_destroy / dds_ctx_destroy.
 *  - There is NO CPU fallback: every arithmetic entry point runs HIP kernels on
 *    the context's GPU and fails with DDS_E_HIP if it cannot.
 */
#ifndef DDSHE_H
#define DDSHE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum dds_status {
  DDS_OK = 0,
  DDS_E_EMPTY = 1,       /* no operand qualified: reference answers 404      */
  DDS_E_RANGE = 2,       /* operand does not fit the modulus' limb width      */
  DDS_E_HIP = 3,         /* HIP runtime / kernel failure                      */
  DDS_E_ARG = 4,         /* bad argument (NULL, zero width, row id, ...)      */
  DDS_E_NOMEM = 5,       /* device or host allocation failed                  */
  DDS_E_UNSUPPORTED = 6, /* modulus larger than the largest kernel instance   */
  DDS_E_BUFSIZE = 7,     /* output buffer too small (required size returned)  */
  DDS_E_FORMAT = 8       /* NumberFormatException on a decimal operand        */
} dds_status;

typedef struct dds_ctx dds_ctx;
typedef struct dds_col dds_col;
typedef struct dds_strtab dds_strtab;

/* OPE predicates of SearchGt / SearchGtEq / SearchLt / SearchLtEq:
 * keep row iff col <op> bound (DDSRestServer.scala:704, :742, :779, :816). */
typedef enum dds_ope_op { DDS_OPE_GT = 0, DDS_OPE_GE = 1, DDS_OPE_LT = 2, DDS_OPE_LE = 3 } dds_ope_op;

/* ---- context ------------------------------------------------------------- */
int dds_ctx_create(int device, dds_ctx** out);
int dds_ctx_destroy(dds_ctx* ctx);
const char* dds_strerror(int status);
/* last error detail of the calling thread ("" if none) */
const char* dds_last_error(void);
/* largest supported modulus, in bits */
size_t dds_max_modulus_bits(void);
/* Run this context's work on `stream` (a hipStream_t) instead of its pool; NULL restores the pool. */
int dds_ctx_set_stream(dds_ctx* ctx, void* stream);
/* Kernel timing with HIP events on the launch stream (for bench.py's roofline). */
int dds_ctx_set_timing(dds_ctx* ctx, int enable);
/* Accumulated device time (ms) and launch count of the dominant fold kernel
 * (first fold level over the input rows) since the last reset. */
int dds_ctx_get_timing(dds_ctx* ctx, double* fold_ms, uint64_t* fold_launches, double* total_ms);
int dds_ctx_reset_timing(dds_ctx* ctx);
/* Montgomery products issued by the timed fold launches (for algorithmic-work accounting). */
int dds_ctx_get_fold_work(dds_ctx* ctx, uint64_t* modmuls);

/* ---- batched modular products (replace the fold loops) ---------------------
 * dds_modmul_fold: SumAll/MultAll semantics over `count` operands:
 *   count == 0 -> DDS_E_EMPTY (404); count == 1 -> operand copied verbatim
 *   (the reference keeps the first operand unreduced, DDSRestServer.scala:416-417);
 *   count >= 2 -> prod(operands) mod modulus, canonical residue.
 * out receives `*out_len` = byte length of the modulus, big-endian, left-padded
 * (for count == 1: the operand's `width` bytes). out_cap is checked. */
int dds_modmul_fold(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint8_t* operands_be,
                    size_t width, size_t count, uint8_t* out, size_t out_cap, size_t* out_len);
/* Paillier HomoAdd over a column: modulus = nsquare (DDSRestServer.scala:422-423). */
int dds_paillier_sum(dds_ctx* ctx, const uint8_t* nsquare_be, size_t nsq_bytes, const uint8_t* ciphertexts_be,
                     size_t width, size_t count, uint8_t* out, size_t out_cap, size_t* out_len);
/* RSA HomoMult over a column: modulus = n of the X.509 pubkey (DDSRestServer.scala:515-518). */
int dds_rsa_product(dds_ctx* ctx, const uint8_t* n_be, size_t n_bytes, const uint8_t* ciphertexts_be, size_t width,
                    size_t count, uint8_t* out, size_t out_cap, size_t* out_len);
/* Pairwise Sum / Mult routes (DDSRestServer.scala:385, :479), batched over n pairs:
 * out[i] = a[i]*b[i] mod modulus, each mod_bytes wide. */
int dds_modmul_pairs(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint8_t* a_be, const uint8_t* b_be,
                     size_t width, size_t n, uint8_t* out);
/* Pairwise routes with a modulus, one request per call, decimal in and out:
 *   GET /Sum  op1*op2 mod nsquare (HomoAdd.sum, DDSRestServer.scala:385)
 *   GET /Mult op1*op2 mod n of the pubkey (HomoMult.multiply, DDSRestServer.scala:479)
 * BigInteger semantics (signed operands, any modulus > 0; operands parsed before the modulus,
 * malformed -> DDS_E_FORMAT). Concurrent calls on one context under the same modulus are coalesced:
 * the first caller to find the modulus' queue idle runs ONE k_pairs launch over every pair queued
 * until then, the others block until their result is ready. A lone call adds no wait. */
int dds_pair_modmul_dec(dds_ctx* ctx, const char* op1_dec, const char* op2_dec, const char* mod_dec, char* out,
                        size_t out_cap, size_t* out_len);
/* Counters of dds_pair_modmul_dec on this context: calls, and k_pairs launches that served them. */
int dds_pair_stats(dds_ctx* ctx, uint64_t* calls, uint64_t* launches);
/* Where the pairwise batches' time went, cumulative ns on this context: the leaders' time per batch
 * (operand repacking, GPU round trip, results), the GPU round trip alone (H2D + k_pairs + D2H +
 * synchronisation; batches of up to 256 pairs), and the longest batch and the longest GPU round trip
 * since the previous call that asked for them (each such read starts a new window). Against the wall clock of a
 * run, batch_ns / wall is the mean number of batches in flight: near the in-flight limit the engine
 * bounds the rate, well below it the callers' own scheduling does. */
int dds_pair_timing(dds_ctx* ctx, uint64_t* batch_ns, uint64_t* gpu_ns, uint64_t* max_batch_ns,
                    uint64_t* max_gpu_ns);
/* Which engine serves dds_pair_modmul_dec's products on this context (policy < 0: query only; the
 * policy in force before the call goes to *previous when given):
 *   DDS_PAIR_GPU  every request through the coalescing queue (k_pairs batches);
 *   DDS_PAIR_LONE a request that finds its modulus' queue empty, no batch in flight and no other host
 *                 product running is served by the engine's host product (64-bit-limb Comba product +
 *                 Barrett reduction, bn_host.hpp); requests arriving meanwhile queue for a GPU batch;
 *   DDS_PAIR_HOST every request by the host product.
 * Default DDS_PAIR_HOST (measured: it costs the least host CPU per request and the lowest latency at 1, 8
 * and 64 concurrent callers); environment DDSHE_PAIR_POLICY overrides it. Results are
 * identical. */
#define DDS_PAIR_GPU 0
#define DDS_PAIR_LONE 1
#define DDS_PAIR_HOST 2
int dds_pair_set_policy(dds_ctx* ctx, int policy, int* previous);
/* Host CPU of dds_pair_modmul_dec on this context by phase, cumulative thread-CPU ns: decimal codec
 * (operand and modulus parse, reply), limb packing of the GPU batches, the callers' queue and
 * condition-variable time, the batch leaders' wait for the GPU round trip (hipStreamSynchronize), the
 * host products; and the number of requests the host products served. */
int dds_pair_cpu(dds_ctx* ctx, uint64_t* codec_ns, uint64_t* pack_ns, uint64_t* queue_ns, uint64_t* wait_ns,
                 uint64_t* host_ns, uint64_t* host_calls);
/* Sizes of the per-request caches: modulus constants (LRU, at most DDSHE_MAX_MODULI, default 64) and
 * pairwise queues (one per modulus with calls in flight; dropped when idle). */
int dds_ctx_cache_stats(dds_ctx* ctx, size_t* moduli, size_t* pair_queues);
/* Page-lock a caller output buffer the caller reuses across requests (a JNA Memory, a direct
 * ByteBuffer) and map it into the device: results bound for it are then written straight in, without
 * a pinned staging buffer and a second host copy (dds_opecol_search_mask's bitmask by the count kernel
 * itself through the mapping; row-id lists of the searches and orders by one DMA).
 * Registered ranges must not overlap; the buffer must stay allocated until dds_host_unregister (or
 * dds_ctx_destroy, which unregisters every buffer). Like any output buffer, one serves one call at a
 * time (concurrent calls into the same bytes race). */
int dds_host_register(dds_ctx* ctx, void* ptr, size_t bytes);
int dds_host_unregister(dds_ctx* ctx, void* ptr);
/* A reply buffer allocated by the engine: page-locked, mapped into the device and placed by the HIP
 * runtime for the context's device (hipHostMalloc), registered as dds_host_register would. Free it
 * with dds_host_free (dds_ctx_destroy frees any left); dds_host_unregister refuses it. */
int dds_host_alloc(dds_ctx* ctx, size_t bytes, void** out);
int dds_host_free(dds_ctx* ctx, void* ptr);
/* SumAll without nsqr (plain BigInteger add, DDSRestServer.scala:425): sum of count
 * operands; result big-endian in out (min(out_cap) = width + 8 is always enough). */
int dds_bigint_sum(dds_ctx* ctx, const uint8_t* operands_be, size_t width, size_t count, uint8_t* out,
                   size_t out_cap, size_t* out_len);

/* MultAll without pubkey (unbounded BigInteger multiply, DDSRestServer.scala:520):
 * product of count operands on a GPU product tree; result big-endian, minimal length
 * (*out_len), at most count*width bytes. */
int dds_bigint_product(dds_ctx* ctx, const uint8_t* operands_be, size_t width, size_t count, uint8_t* out,
                       size_t out_cap, size_t* out_len);

/* ---- device-resident columns (ciphertexts stay in HBM across requests) ----
 * A column holds `count` residues of one modulus in the engine's resident
 * format (limb-transposed radix-2^W, W = 28 or 27). */
int dds_col_create(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, size_t capacity, dds_col** out);
int dds_col_destroy(dds_col* col);
/* append `count` big-endian operands (validated against the modulus) */
int dds_col_append(dds_col* col, const uint8_t* operands_be, size_t width, size_t count);
/* append `count` decimal rows (BigInteger.toString text, as stored in DDSSet contents) parsed on
 * the GPU. Replaces the per-row new BigInteger(String) of the fold loops
 * (DDSRestServer.scala:417,419,422,513). Rows are an Arrow-style string column: row i is
 * chars[offsets[i] .. offsets[i+1]), offsets has count+1 non-decreasing entries. Syntax is
 * BigInteger(String) radix 10 with ASCII digits: optional '+'/'-', then >= 1 digit.
 * A negative row is stored as its residue (BigInteger.mod). Errors: DDS_E_FORMAT for a malformed
 * row (NumberFormatException), DDS_E_RANGE for |row| >= 2^(W*S) (the column's limb capacity, a
 * few bits above the modulus); the column is unchanged on error. */
int dds_col_append_dec(dds_col* col, const char* chars, const uint64_t* offsets, size_t count);
size_t dds_col_count(const dds_col* col);
/* drop rows [count, dds_col_count) (the storage is kept for later appends) */
int dds_col_truncate(dds_col* col, size_t count);
/* ---- resident rows follow the reference's write routes --------------------------------------
 * The reference changes stored sets in place and re-fetches them on every request
 * (DDSRestServer.scala:401-403): WriteElement overwrites contents(position) (:281-321), AddElement
 * appends an element (:220-255), RemoveSet writes None (:207-218), PutSet of known contents rewrites
 * its key (:170-188). A column row stands for one stored key; these keep it bit-exact without a
 * re-upload:
 *   dds_col_write_rows[_dec]: rows row_ids[0..n) (< dds_col_count) take new operands (validated and
 *     stored exactly as dds_col_append / dds_col_append_dec would; a one-row fold then returns the new
 *     operand unreduced). A repeated id takes its last value. On error the column is unchanged.
 *   dds_col_set_live: live[i] == 0 takes row row_ids[i] out of every fold (a removed set, or a set
 *     whose length no longer passes the route's guard), != 0 puts it back. Appended rows are live.
 *   Every fold (dds_col_fold, _rows, _dec, _partial, _partial_device) folds the LIVE rows of its range
 *   or id list; the 404 / one-operand rules apply to the live rows (a partial reports their number).
 * Mutations wait for folds in flight on the column and folds wait for them (readers/writer lock). */
int dds_col_write_rows(dds_col* col, const uint64_t* row_ids, size_t n, const uint8_t* operands_be, size_t width);
int dds_col_write_rows_dec(dds_col* col, const uint64_t* row_ids, size_t n, const char* chars,
                           const uint64_t* offsets);
int dds_col_set_live(dds_col* col, const uint64_t* row_ids, size_t n, const uint8_t* live);
size_t dds_col_live_count(dds_col* col);
/* download rows [first, first+count) as canonical residues (x mod N), big-endian, mod_bytes each */
int dds_col_read(dds_col* col, size_t first, size_t count, uint8_t* out);
/* fold rows [first, first+count) (SumAll/MultAll semantics as dds_modmul_fold). A one-row fold returns
 * that row's operand as appended, unreduced (DDSRestServer.scala:416-417: the column remembers the
 * operands it had to store as residues); *out_len = max(modulus bytes, operand bytes). A negative
 * operand (decimal rows) has no big-endian magnitude form: DDS_E_RANGE, use dds_col_fold_dec. */
int dds_col_fold(dds_col* col, size_t first, size_t count, uint8_t* out, size_t out_cap, size_t* out_len);
/* Row-subset fold: the rows row_ids[0..n) of the column (ids < dds_col_count; duplicates fold twice),
 * i.e. the sets a SumAll / MultAll route keeps after its dedup and strict guard
 * (DDSRestServer.scala:401-415, 505-509) without re-uploading them. Same result rules as dds_col_fold. */
int dds_col_fold_rows(dds_col* col, const uint64_t* row_ids, size_t n, uint8_t* out, size_t out_cap,
                      size_t* out_len);
/* Same fold with the route's decimal reply (DDSValueResult(acc.toString), :435/:529): rows row_ids[0..n),
 * or rows [0, n) when row_ids is NULL. out receives NUL-terminated text, *out_len its length. */
int dds_col_fold_dec(dds_col* col, const uint64_t* row_ids, size_t n, char* out, size_t out_cap, size_t* out_len);
/* fold rows to one un-finalised partial for multi-GPU combination:
 * partial_r27 receives limbs() words, *rows the row count it covers. */
int dds_col_fold_partial(dds_col* col, size_t first, size_t count, uint32_t* partial_r27, uint64_t* rows);
/* number of 32-bit words in a partial of this column's modulus */
size_t dds_col_partial_words(const dds_col* col);
/* combine partials from several GPUs (same modulus): result = prod of all rows mod N. Each partial must
 * be what dds_col_fold_partial produced (normalised limbs, value in range): DDS_E_RANGE otherwise. */
int dds_combine_partials(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint32_t* partials_r27,
                         const uint64_t* rows, size_t nparts, uint8_t* out, size_t out_cap, size_t* out_len);
/* Device-resident forms for a multi-process (one rank per GPU) gather that never stages the partial
 * limbs through the host: dds_col_fold_partial_device writes the partial (dds_col_partial_words u32,
 * the last two words the exponent) to DEVICE memory of the column's GPU and synchronises before
 * returning; dds_combine_partials_device combines nparts such partials laid out back to back in device
 * memory of ctx's GPU (e.g. the output of an RCCL all_gather). */
int dds_col_fold_partial_device(dds_col* col, size_t first, size_t count, uint32_t* d_partial);
int dds_combine_partials_device(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint32_t* d_partials,
                                const uint64_t* rows, size_t nparts, uint8_t* out, size_t out_cap, size_t* out_len);

/* ---- one caller, several GPUs (SURVEY.md §8b device_mask) ----------------------------------
 * A dds_mctx owns one context per shard; shard 0's device combines. dds_mctx_create takes a device
 * bit mask (bit d = HIP device d); dds_mctx_create_devices an explicit list, where a device may repeat
 * (several shards on one GPU). A dds_mcol spreads its rows over the shards in 64-row blocks,
 * round-robin (global row r on shard (r/64) % G). dds_mcol_fold* fold every shard on its own device
 * concurrently, move the shard partials device-to-device (xGMI peer copies) to the combining device
 * and combine there: same results and result rules as dds_col_fold / dds_col_fold_rows /
 * dds_col_fold_dec, row ids being global. Appends split the batch per shard and upload concurrently;
 * a failed append leaves the column unchanged. */
typedef struct dds_mctx dds_mctx;
typedef struct dds_mcol dds_mcol;
int dds_mctx_create(uint64_t device_mask, dds_mctx** out);
int dds_mctx_create_devices(const int* devices, size_t ndevices, dds_mctx** out);
int dds_mctx_destroy(dds_mctx* m);
size_t dds_mctx_shards(const dds_mctx* m);
int dds_mcol_create(dds_mctx* m, const uint8_t* mod_be, size_t mod_bytes, size_t capacity, dds_mcol** out);
int dds_mcol_destroy(dds_mcol* col);
size_t dds_mcol_count(const dds_mcol* col);
int dds_mcol_append(dds_mcol* col, const uint8_t* operands_be, size_t width, size_t count);
int dds_mcol_append_dec(dds_mcol* col, const char* chars, const uint64_t* offsets, size_t count);
/* synthetic rows as dds_col_fill_paillier_synth with row0 = the current global row count */
int dds_mcol_fill_paillier_synth(dds_mcol* col, const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be,
                                 size_t g_bytes, uint64_t seed, size_t count, uint32_t pool_size);
int dds_mcol_fold(dds_mcol* col, uint8_t* out, size_t out_cap, size_t* out_len);
int dds_mcol_fold_rows(dds_mcol* col, const uint64_t* row_ids, size_t n, uint8_t* out, size_t out_cap,
                       size_t* out_len);
int dds_mcol_fold_dec(dds_mcol* col, const uint64_t* row_ids, size_t n, char* out, size_t out_cap, size_t* out_len);
/* dds_col_write_rows[_dec] / dds_col_set_live / dds_col_live_count on a sharded column (global row ids;
 * a write that fails validation (DDS_E_ARG / DDS_E_RANGE / DDS_E_FORMAT) leaves every shard unchanged;
 * DDS_E_HIP from a write may leave some shards written and is fatal to the column; folds above honour
 * the live mask of every shard) */
int dds_mcol_write_rows(dds_mcol* col, const uint64_t* row_ids, size_t n, const uint8_t* operands_be, size_t width);
int dds_mcol_write_rows_dec(dds_mcol* col, const uint64_t* row_ids, size_t n, const char* chars,
                            const uint64_t* offsets);
int dds_mcol_set_live(dds_mcol* col, const uint64_t* row_ids, size_t n, const uint8_t* live);
size_t dds_mcol_live_count(dds_mcol* col);
/* Synthetic Paillier rows for benchmarks/tests (config 2 of BASELINE.json):
 * c_i = g^m_i * r_a^n * r_b^n mod n^2 with m_i, a, b from splitmix64(seed, row0+i);
 * m_i = splitmix64(seed ^ splitmix64(row0+i)) % 10000 (DDSDataGenerator.scala:274).
 * Needs the Paillier key (n, g) big-endian; pool_size r^n values from seed. */
int dds_col_fill_paillier_synth(dds_col* col, const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be,
                                size_t g_bytes, uint64_t seed, uint64_t row0, size_t count, uint32_t pool_size);

/* ---- OPE range filter (SearchGt/GtEq/Lt/LtEq) ---------------------------
 * Keeps row i iff valid[i] != 0 (reference guard contents.length-1 > position,
 * DDSRestServer.scala:703) and col[i] <op> bound (signed 64-bit: OPE
 * ciphertexts are Java Long, SJHomoLibProvider.scala:55). valid may be NULL.
 * out_idx receives the matching row indices in ascending order. */
int dds_ope_filter(dds_ctx* ctx, const int64_t* col, const uint8_t* valid, size_t n, int64_t bound, int op,
                   uint32_t* out_idx, size_t* out_n);
/* same on device-resident arrays (pointers are device pointers) */
int dds_ope_filter_device(dds_ctx* ctx, const int64_t* d_col, const uint8_t* d_valid, size_t n, int64_t bound, int op,
                          uint32_t* d_out_idx, size_t* out_n);

/* ---- resident OPE column (Search{Gt,GtEq,Lt,LtEq} :682-830, OrderLS/OrderSL :541-606) ----
 * The OPE ciphertexts of one column position stay in HBM across requests. Per row the caller gives
 * the element's text (contents(position).toString, ASCII decimal) and its class:
 *   cls 0: the row lacks the position (contents.length-1 < position)
 *   cls 1: the position is the row's last element (length-1 == position: an Order holder that
 *          Search's strict guard `length-1 > position` skips, :702)
 *   cls 2: elements follow it (both routes read it); cls == NULL: every row is class 2.
 * is_string (NULL: all) flags elements that are Strings: Order reads contents(position).asInstanceOf
 * [String].toLong (:562/:595), which throws on an Int element; Search's BigInteger(toString) does not.
 * Values outside int64 are kept exactly (Search compares BigIntegers); malformed ones are kept as
 * such and fail a request only when the reference's loop would parse them:
 *   dds_opecol_search: the bound (item.value.toString) is parsed only when some row passes the guard
 *     (:702-704): no class-2 row -> 0 matches, any bound; a malformed bound or class-2 element -> 
 *     DDS_E_FORMAT (500). out_idx (capacity dds_opecol_count) receives ascending row ids.
 *   dds_opecol_order: a permutation of the rows, as dds_ope_order with valid = cls != 0; with two or
 *     more holders every holder is parsed by the comparator: a holder that is not a Long String ->
 *     DDS_E_FORMAT; a lone holder is never parsed. */
typedef struct dds_opecol dds_opecol;
int dds_opecol_create(dds_ctx* ctx, size_t capacity, dds_opecol** out);
int dds_opecol_destroy(dds_opecol* col);
size_t dds_opecol_count(const dds_opecol* col);
int dds_opecol_truncate(dds_opecol* col, size_t count);
/* rows already as Java Longs (values) */
int dds_opecol_append(dds_opecol* col, const int64_t* values, const uint8_t* cls, size_t count);
/* rows as the element text the route parses (values[i] may be NULL when cls[i] == 0) */
int dds_opecol_append_dec(dds_opecol* col, const char* const* values, const uint8_t* cls, const uint8_t* is_string,
                          size_t count);
int dds_opecol_search(dds_opecol* col, const char* bound_dec, int op, uint32_t* out_idx, size_t* out_n);
/* The same Search answered as a row bitmask: bit (r % 64) of mask[r / 64] = row r matches (mask_words
 * >= ceil(dds_opecol_count / 64); bits past the last row are 0), *out_n = matches. 1/32 of the bytes of
 * the id list at 50 % selectivity: the form a route holding its keys in row order iterates. */
int dds_opecol_search_mask(dds_opecol* col, const char* bound_dec, int op, uint64_t* mask, size_t mask_words,
                           size_t* out_n);
/* out_idx (capacity dds_opecol_count) receives the permutation of the live rows, *out_n (nullable) its
 * length = dds_opecol_live_count. */
int dds_opecol_order(dds_opecol* col, int descending, uint32_t* out_idx, size_t* out_n);
/* Rows follow the write routes, as dds_col_write_rows / dds_col_set_live: rows row_ids[0..n) take a new
 * element and class (WriteElement :281-321, AddElement :220-255: the class moves when the set grows),
 * as Longs or as the element text (same parsing as dds_opecol_append[_dec]); live[i] == 0 marks the
 * row's set removed (RemoveSet :207-218): no Search matches it and Order leaves it out (filter(nonEmpty),
 * :553/:586/:700); != 0 restores it. Repeated ids: the last entry wins. */
int dds_opecol_write_rows(dds_opecol* col, const uint64_t* row_ids, const int64_t* values, const uint8_t* cls,
                          size_t n);
int dds_opecol_write_rows_dec(dds_opecol* col, const uint64_t* row_ids, const char* const* values,
                              const uint8_t* cls, const uint8_t* is_string, size_t n);
int dds_opecol_set_live(dds_opecol* col, const uint64_t* row_ids, size_t n, const uint8_t* live);
size_t dds_opecol_live_count(dds_opecol* col);

/* ---- OPE ordering (OrderLS / OrderSL, DDSRestServer.scala:541-606) ------------
 * out_idx receives a permutation of [0, n): rows with valid[i] != 0 (the row holds the
 * position: contents.length-1 >= position, :556 / :589) ordered by col (signed 64-bit, the
 * route's `.toLong`) descending (OrderLS, descending != 0) or ascending (OrderSL); rows with
 * valid[i] == 0 go last (OrderLS) or first (OrderSL). Equal keys keep their input order
 * (scala sortWith is stable). valid may be NULL (all rows hold the position). */
int dds_ope_order(dds_ctx* ctx, const int64_t* col, const uint8_t* valid, size_t n, int descending,
                  uint32_t* out_idx);
/* same on device-resident arrays (device pointers) */
int dds_ope_order_device(dds_ctx* ctx, const int64_t* d_col, const uint8_t* d_valid, size_t n, int descending,
                         uint32_t* d_out_idx);

/* ---- deterministic-equality scans ---------------------------
 * HomoDet.compare (hlib, absent) is taken as equality of the ciphertext strings.
 * A string table holds the rows' contents: element e is chars[elem_offsets[e], elem_offsets[e+1]),
 * row r is elements [row_offsets[r], row_offsets[r+1]) (its DDSSet.contents, in column order;
 * DDSSet.scala:3). The table is device-resident with a 32-bit fingerprint per element; results are
 * exact (bytes are compared on a fingerprint hit). out_rows receives ascending ids of live rows
 * (capacity: the table's rows when the scan runs; a caller that appends to the table from another
 * thread sizes it for the rows after those appends).
 *   dds_search_eq     SearchEq / SearchNEq (negate != 0), DDSRestServer.scala:607-681: rows with
 *                     length-1 > position whose element `position` equals / differs from value.
 *   dds_search_entry  SearchEntry (1 value), SearchEntryOR (3, require_all = 0) and
 *                     SearchEntryAND (3, require_all != 0: all three distinct values present),
 *                     DDSRestServer.scala:831-938.
 *   dds_is_element    IsElement, DDSRestServer.scala:322-353 (row out of range: DDS_E_EMPTY, 404). */
int dds_strtab_create(dds_ctx* ctx, const char* chars, const uint64_t* elem_offsets, size_t nelems,
                      const uint64_t* row_offsets, size_t nrows, dds_strtab** out);
int dds_strtab_destroy(dds_strtab* tab);
/* The table follows the write routes in place (DDSRestServer.scala:170-321), as the resident columns
 * do. Batches use the create layout (chars, elem_offsets[nelems+1], row_offsets[nrows+1], both from 0).
 *   dds_strtab_append      PutSet of new keys: rows nrows.. (live)
 *   dds_strtab_write_rows  PutSet of a stored key / AddElement / WriteElement: row row_ids[i] takes the
 *                          contents of batch row i (a repeated id takes its last row) and is live again
 *   dds_strtab_set_live    RemoveSet (live 0: the register holds None, every scan skips the row and
 *                          IsElement answers DDS_E_EMPTY) and its revival (live 1, last contents)
 *   dds_strtab_truncate    drop the rows from `rows` on (a failed batched PutSet rolled back)
 *   dds_strtab_stats       out[0..n) of: rows, live rows, heap elements, elements of the rows' current
 *                          contents, heap bytes, bytes of the current contents, heap compactions,
 *                          cached SearchEq position indexes
 * Scans on one table run concurrently with each other; a write waits for them (and they for it). */
int dds_strtab_append(dds_strtab* tab, const char* chars, const uint64_t* elem_offsets, size_t nelems,
                      const uint64_t* row_offsets, size_t nrows);
int dds_strtab_write_rows(dds_strtab* tab, const uint64_t* row_ids, size_t n, const char* chars,
                          const uint64_t* elem_offsets, size_t nelems, const uint64_t* row_offsets);
int dds_strtab_set_live(dds_strtab* tab, const uint64_t* row_ids, size_t n, const uint8_t* live);
size_t dds_strtab_rows(dds_strtab* tab);
size_t dds_strtab_live_count(dds_strtab* tab);
int dds_strtab_truncate(dds_strtab* tab, size_t rows);
int dds_strtab_stats(dds_strtab* tab, uint64_t* out, size_t n);
int dds_search_eq(dds_strtab* tab, size_t position, const char* value, size_t len, int negate, uint32_t* out_rows,
                  size_t* out_n);
int dds_search_entry(dds_strtab* tab, const char* const* values, const size_t* lens, size_t nvalues, int require_all,
                     uint32_t* out_rows, size_t* out_n);
int dds_is_element(dds_strtab* tab, size_t row, const char* value, size_t len, int* found);

/* ---- batched Paillier encryption (HomoAdd.encrypt, SJHomoLibProvider.scala:58) ----
 * c_i = g^m_i * r_i^n mod n^2 with caller-supplied r_i (big-endian, r_width bytes,
 * values in [1, n^2)). out receives n of nsq_bytes each. */
int dds_paillier_encrypt_batch(dds_ctx* ctx, const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be, size_t g_bytes,
                               const uint32_t* m, const uint8_t* r_be, size_t r_width, size_t count, uint8_t* out,
                               size_t nsq_bytes);

/* HomoAdd.encrypt(m, PaillierKey) with the private factors p, q (the client holds the whole
 * key, SJHomoLibProvider.scala:43-58): bit-identical to dds_paillier_encrypt_batch with n = p*q,
 * computed mod p^2 and q^2 and recombined (Garner) — half-width Montgomery work. r_i in [1, n)
 * (DDS_E_RANGE otherwise); p, q distinct odd primes (DDS_E_ARG otherwise). */
int dds_paillier_encrypt_batch_crt(dds_ctx* ctx, const uint8_t* p_be, size_t p_bytes, const uint8_t* q_be,
                                   size_t q_bytes, const uint8_t* g_be, size_t g_bytes, const uint32_t* m,
                                   const uint8_t* r_be, size_t r_width, size_t count, uint8_t* out, size_t nsq_bytes);

/* Batched modular exponentiation out[i] = base[i]^exp mod modulus (mod_bytes each):
 * HomoMult.encrypt(pk, m) = m^e mod n (SJHomoLibProvider.scala:59) and decrypt-side
 * checks. Bases are validated like fold operands. */
int dds_modexp_batch(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint8_t* exp_be, size_t exp_bytes,
                     const uint8_t* bases_be, size_t width, size_t count, uint8_t* out);

/* ---- device-resident batched encryption (BASELINE.json config 4) --------------
 * dds_col_fill_random: append `count` seeded random rows r < 2^bits (odd, so r != 0):
 *   limb l of row i = splitmix64(splitmix64(seed ^ (row0+i)) + l) in the column's rW layout.
 * dds_col_encrypt_paillier: append Enc(m_i; r_i) = g^m_i r_i^n mod n^2 for the `count` rows of
 *   rcol starting at r_first (r_i in [1, n)), m on the device (d_m, uint32). Both columns are
 *   over n^2. p, q (both or neither): CRT path, same result. */
int dds_col_fill_random(dds_col* col, size_t bits, uint64_t seed, uint64_t row0, size_t count);
/* Table-driven synthetic rows (BASELINE.json config 3): append row i = table[h_i % tcount],
 * h_i = splitmix64(seed ^ splitmix64(row0+i)); table: tcount big-endian values of `width` bytes
 * (e.g. table[j] = (j+1)^e mod n, RSA ciphertexts of the DDSDataGenerator.scala:274 plaintexts). */
int dds_col_fill_table_synth(dds_col* col, const uint8_t* table_be, size_t width, size_t tcount, uint64_t seed,
                             uint64_t row0, size_t count);
int dds_col_encrypt_paillier(dds_col* out, dds_col* rcol, size_t r_first, const uint32_t* d_m, size_t count,
                             const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be, size_t g_bytes,
                             const uint8_t* p_be, size_t p_bytes, const uint8_t* q_be, size_t q_bytes);

/* ---- route-level entry points on decimal strings (what the Scala route holds) ----
 * values: count NUL-terminated decimal strings (contents(position) of the rows that
 * passed the guard). modulus_dec NULL selects the plain add / multiply branch.
 * out receives the decimal result (NUL-terminated) — DDSValueResult(acc.toString). */
int dds_sum_all_dec(dds_ctx* ctx, const char* const* values, size_t count, const char* nsqr_dec, char* out,
                    size_t out_cap, size_t* out_len);
int dds_mult_all_dec(dds_ctx* ctx, const char* const* values, size_t count, const char* n_dec, char* out,
                     size_t out_cap, size_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* DDSHE_H */
