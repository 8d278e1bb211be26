// Host-side internals of the C-ABI (shared by ddshe_capi.cpp, ddshe_opecol.cpp, ddshe_mctx.cpp):
// contexts, stream/buffer pools, per-modulus Montgomery constants, device columns and the
// orchestration helpers around the HIP kernels. Not part of the public ABI (include/ddshe.h).
#pragma once
#include <hip/hip_runtime.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <chrono>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "bn_host.hpp"
#include "ddshe.h"
#include "ddshe_launch.hpp"

namespace ddshe {
namespace host {


extern thread_local std::string g_last_error;
int fail(int code, const std::string& msg);

#define HIP_TRY(expr)                                                                             \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(DDS_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      (void)hipFree(p);
      p = nullptr;
      cap = 0;
    }
    size_t nb = std::max<size_t>(bytes, 256);
    hipError_t e = hipMalloc(&p, nb);
    if (e == hipSuccess) cap = nb;
    return e;
  }
  template <class T>
  T* as() const {
    return (T*)p;
  }
};

struct HostBuf {  // pinned staging (truly asynchronous H2D)
  void* p = nullptr;
  size_t cap = 0;
  unsigned flags = 0;     // hipHostMalloc flags (set before the first ensure)
  void* dptr = nullptr;  // device address when flags map the buffer (hipHostMallocMapped)
  ~HostBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      (void)hipHostFree(p);
      p = nullptr;
      cap = 0;
    }
    dptr = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, flags);
    if (e == hipSuccess) cap = bytes;
    if (e == hipSuccess && (flags & hipHostMallocMapped)) e = hipHostGetDevicePointer(&dptr, p, 0);
    return e;
  }
};

struct Worker {
  hipStream_t stream = nullptr;
  bool timed_fold = false;  // ev[0]/ev[1] bracket a first-level fold launch not yet accounted
  DevBuf in, in2, x, x2, p0, p1, out, flags, y, misc, misc2, tab, ids;
  DevBuf pk, gather;         // multi-device fold: packed partial (shard side), gathered partials (combiner)
  DevBuf tree;               // reduction tree: node values + arrival flags
  hipEvent_t ev_peer = {};   // shard partial copied to the combining device
  // a device counter kept at zero between uses (the Search bitmask's match count: the count kernel's
  // tiles add into it, it is read, then re-zeroed on the stream after the read); ev_done marks the read
  DevBuf ctr;
  bool ctr_zero = false;
  DevBuf sflags;            // string scans' row flags, zero between scans when sflags_zero
  bool sflags_zero = false;
  hipEvent_t ev_done = {};
  DevBuf crt[7];  // CRT encryption scratch (see encrypt_crt_device)
  hipEvent_t ev[4] = {};
  // decimal codec: double-buffered pinned chunks (chars, offsets), their device copies,
  // per-row status bytes, and the event after each slot's last use
  HostBuf hch[2], hoff[2];
  HostBuf hstage;  // fold finalize: Y in, result out (pinned: no staging copies on the latency path)
  uint32_t done_seq = 0;  // fold finalize: the last sequence number the root stored at kStageDoneWord
  HostBuf hcnt;    // coherent + mapped: the Search bitmask's per-tile match counts, stored by the device
  HostBuf hpair;   // pairwise batches: operands and results, coherent + mapped (k_pairs_sos reads and writes it)
  HostBuf hord;    // coherent + mapped: small read-back words stored by kernels (MappedWords)
  HostBuf hscan;   // coherent + mapped: string-table scans' match count, needle bytes and row ids
  HostBuf hbig;    // large read-backs (Search ids / match masks, Order permutations) before the caller's copy
  DevBuf dch[2], doff[2], rflags;
  hipEvent_t ev_dec[2] = {};
  // decimal ingest: H2D copies on their own stream (chunk s + 1 copies while chunk s parses)
  hipStream_t cstream = nullptr;
  hipEvent_t ev_copy[2] = {};
  ~Worker() {
    for (auto e : ev_copy)
      if (e) (void)hipEventDestroy(e);
    if (cstream) (void)hipStreamDestroy(cstream);
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : ev_dec)
      if (e) (void)hipEventDestroy(e);
    if (ev_peer) (void)hipEventDestroy(ev_peer);
    if (ev_done) (void)hipEventDestroy(ev_done);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// Per-modulus constants for the two kernel shapes: the throughput shape (S limbs, TPI
// lanes) of the first fold level, and the latency shape (S2 limbs, 16 lanes) of the
// reduction tree and finalize. Both use radix 2^W, so R = 2^(W*S) and R2 = 2^(W*S2)
// differ only by a power of two: every partial is tracked as prod * 2^E (E signed).
struct ModConsts {
  int S = 0, TPI = 0, W = 0, S2 = 0;
  size_t bits = 0, bytes = 0;
  uint64_t last_use = 0;         // ctx->mods LRU tick (under ctx->mu)
  uint32_t n0 = 0;
  bn::Limbs N, Rmod, half;       // half = (N+1)/2 = 2^-1 mod N
  bn::Limbs qbound;              // partials stay below 2*qbound: N~ = N·n0 when a QP shape is used, else N
  std::vector<uint32_t> host;    // kConstCount * S  (throughput shape)
  std::vector<uint32_t> host2;   // kConstCount * S2 (tail shape)
  uint32_t* d = nullptr;         // device copies
  uint32_t* d2 = nullptr;
  uint32_t* dq = nullptr;        // N~ = N·n0 in tail limbs (tail_qp shapes), else null
  uint32_t* dqm = nullptr;       // N~ in main limbs when R > 4N~ holds for the main shape, else null
  int S3 = 0, W3 = 0;            // reduction-tree shape (ddshe_tree.hip), R3 = 2^(W3*S3)
  bool tree_direct = false;      // raw rows (< 2^(W*S)) may be tree leaves: 2^(2WS) <= R3 * 2^(bits(N)-1)
  uint32_t* d3 = nullptr;        // tree constants: N | n' = -N^-1 mod R3 | N | 2N | 3N | R3^2 mod N
  std::map<int64_t, std::vector<uint32_t>> y3cache;  // E -> 2^(W3*S3 - E) mod N, tree limbs
  std::mutex ymu;
  std::map<int64_t, std::vector<uint32_t>> ycache;  // E -> 2^(W*S2 - E) mod N, tail limbs
  // decimal codec table (k_dec_parse), built on first use: Pt[l*jpad + j] = limb l of 10^(8j)
  // for the jfit powers below 2^(W*S), then jst[i] (first power reaching limb TPI*i, rounded down to 4)
  std::mutex decmu;
  uint32_t* dtab = nullptr;
  int jfit = 0, jpad = 0;
  ~ModConsts() {
    if (d) (void)hipFree(d);
    if (d2) (void)hipFree(d2);
    if (dq) (void)hipFree(dq);
    if (dqm) (void)hipFree(dqm);
    if (d3) (void)hipFree(d3);
    if (y3slab) (void)hipFree(y3slab);
    if (dtab) (void)hipFree(dtab);
  }
  std::vector<uint32_t> rw(const bn::Limbs& v) const { return bn::to_rw(v, S, W); }
  bn::Limbs value(const uint32_t* limbs) const { return bn::from_rw(limbs, S, W); }
  bn::Limbs value2(const uint32_t* limbs) const { return bn::from_rw(limbs, S2, W); }
  // 2^e mod N for a signed e
  bn::Limbs pow2(int64_t e) const {
    return e >= 0 ? bn::powmod_u64(bn::Limbs{2}, (uint64_t)e, N) : bn::powmod_u64(half, (uint64_t)(-e), N);
  }
  // finalize multiplier for a tail-shape partial holding prod * 2^E. Returned BY VALUE: the cache
  // may be cleared by a concurrent caller while this one's async copy still reads its vector.
  std::vector<uint32_t> y_for(int64_t E) {
    std::lock_guard<std::mutex> lk(ymu);
    auto it = ycache.find(E);
    if (it != ycache.end()) return it->second;
    if (ycache.size() >= 64) ycache.clear();
    bn::Limbs y = pow2((int64_t)W * S2 - E);
    return ycache.emplace(E, bn::to_rw(y, S2, W)).first->second;
  }
  // finalize multiplier of the reduction tree for a root holding prod * 2^E (by value, as y_for)
  std::vector<uint32_t> y3_for(int64_t E) {
    std::lock_guard<std::mutex> lk(ymu);
    auto it = y3cache.find(E);
    if (it != y3cache.end()) return it->second;
    if (y3cache.size() >= 64) y3cache.clear();
    bn::Limbs y = pow2((int64_t)W3 * S3 - E);
    return y3cache.emplace(E, bn::to_rw(y, S3, W3)).first->second;
  }
  // device copy of y3_for(E), made on first use and kept until the constants go (a fold's finalize
  // then needs no H2D copy on its critical path): slots of one device block of kYDev * S3 words;
  // nullptr once every slot is taken (the caller then copies Y in its stream)
  static constexpr size_t kYDev = 256;
  uint32_t* y3slab = nullptr;
  std::map<int64_t, uint32_t*> y3dev;
  const uint32_t* y3_device(int64_t E) {
    const std::vector<uint32_t> y = y3_for(E);
    std::lock_guard<std::mutex> lk(ydmu);  // held over the copy: a slot is visible only once filled
    auto it = y3dev.find(E);
    if (it != y3dev.end()) return it->second;
    if (y3dev.size() >= kYDev) return nullptr;
    if (!y3slab && hipMalloc(&y3slab, kYDev * (size_t)S3 * 4) != hipSuccess) {
      y3slab = nullptr;
      return nullptr;
    }
    uint32_t* d = y3slab + y3dev.size() * (size_t)S3;
    if (hipMemcpy(d, y.data(), y.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    y3dev.emplace(E, d);
    return d;
  }
  std::mutex ydmu;
  int64_t wS3() const { return (int64_t)W3 * S3; }
  // bits of 2 contributed by one Montgomery product of the main / tail shape
  int64_t wS() const { return (int64_t)W * S; }
  int64_t wS2() const { return (int64_t)W * S2; }
};

// partial exchanged between GPUs: S2 tail limbs + signed exponent E (two words)
inline size_t partial_words_for(const ModConsts& mc) { return (size_t)mc.S2 + 2; }

struct PairQueue;  // ddshe_pairs.cpp

}  // namespace host
}  // namespace ddshe


struct CrtKey;  // CRT form of a Paillier key (encrypt_crt_device)

struct dds_ctx {
  int device = 0;
  int cus = 0;
  std::mutex mu;
  std::vector<std::unique_ptr<ddshe::host::Worker>> workers;
  std::vector<ddshe::host::Worker*> idle;
  // (modulus, limb count of its shape) -> constants; the shape is normally the narrowest that holds
  // the modulus, a wider one when operands must fit (the odd part of an even modulus)
  std::map<std::pair<ddshe::bn::Limbs, int>, std::shared_ptr<ddshe::host::ModConsts>> mods;
  uint64_t mod_tick = 0;  // LRU clock of mods (under mu)
  std::map<std::pair<ddshe::bn::Limbs, ddshe::bn::Limbs>, std::shared_ptr<CrtKey>> crt_keys;
  hipStream_t ext_stream = nullptr;
  std::atomic<bool> timing{false};
  std::mutex tmu;
  double fold_ms = 0, total_ms = 0;
  uint64_t fold_launches = 0, fold_modmuls = 0, pending_modmuls = 0;
  // pairwise routes (ddshe_pairs.cpp): one coalescing queue per modulus, and its counters
  std::mutex pmu;
  std::map<ddshe::bn::Limbs, std::shared_ptr<ddshe::host::PairQueue>> pair_queues;
  std::atomic<uint64_t> pair_calls{0}, pair_launches{0};
  // where a batch's time goes (dds_pair_timing): leader time per batch (gather, codec, GPU round trip,
  // hand-back), its GPU round trip alone (H2D + k_pairs + D2H + sync), the longest batch
  std::atomic<uint64_t> pair_batch_ns{0}, pair_gpu_ns{0}, pair_max_batch_ns{0}, pair_max_gpu_ns{0};
  // host CPU of the pairwise route by phase (dds_pair_cpu), thread CPU clock ns: decimal codec, limb
  // packing of the batches, queue / condition-variable time of the callers, the leaders' wait for the GPU
  // round trip, the host products (and how many requests they served)
  std::atomic<uint64_t> pair_cpu_ns[5] = {}, pair_host_calls{0};
  std::atomic<int> pair_policy{-1};  // dds_pair_set_policy; -1: DDSHE_PAIR_POLICY / the default
  std::map<ddshe::bn::Limbs, std::shared_ptr<const ddshe::bn::Barrett64>> pair_bar;  // under pmu
  // pairwise batches lease their own workers, at most pair_inflight() of them, made on demand and kept:
  // once a burst has run, no leader creates a stream or pins a buffer again (a queue dropped and
  // recreated under load could otherwise have more leaders than that, each making a worker)
  std::mutex pwmu;
  std::condition_variable pwcv;
  std::vector<ddshe::host::Worker*> pair_free;
  int pair_made = 0;
  // caller output buffers registered with dds_host_register (page-locked): base -> bytes. Results
  // bound for them are DMA'd straight in, with no pinned staging buffer and no second host copy.
  std::mutex regmu;
  struct HostReg {
    size_t bytes;
    void* dptr;          // the range's device address (mapped), or null
    bool owned = false;  // allocated by dds_host_alloc (hipHostFree), else registered caller memory
  };
  std::map<uintptr_t, HostReg> host_regs;
  ~dds_ctx();
};

struct dds_col {
  dds_ctx* ctx = nullptr;
  std::shared_ptr<ddshe::host::ModConsts> mc;
  size_t capacity = 0, count = 0, stride = 0;
  uint32_t* d = nullptr;
  // Folds and reads hold it shared (concurrent SumAll / MultAll requests run side by side); appends,
  // row writes, liveness changes and truncation hold it exclusively, so a fold never sees a half-applied
  // mutation (WriteElement / AddElement / RemoveSet, DDSRestServer.scala:207-321).
  std::shared_mutex mu;
  // Live mask (dds_col_set_live): dlive[r] = 1 when row r takes part in folds (device, capacity bytes,
  // all 1 at creation); hlive its host mirror, allocated when the first row goes dead; ndead the number
  // of dead rows among [0, count). Rows at or past `count` are always 1 (truncate resets them), so an
  // append needs no mask update. With ndead == 0 a fold runs exactly as before (no mask pass).
  uint8_t* dlive = nullptr;
  std::vector<uint8_t> hlive;
  size_t ndead = 0;
  bool live(size_t r) const { return hlive.empty() || hlive[r]; }
  // Rows the column stores as a residue that differs from the operand the caller appended (operands
  // >= 2N, negative decimal rows): their original value. A one-operand fold returns the operand
  // itself, unreduced (DDSRestServer.scala:416-417); rows below 2N are stored verbatim.
  struct Orig {
    ddshe::bn::Limbs mag;
    bool neg = false;
  };
  std::map<size_t, Orig> orig;
  ~dds_col() {
    if (d) (void)hipFree(d);
    if (dlive) (void)hipFree(dlive);
  }
};


namespace ddshe {
namespace host {

// Coalescing queue of the pairwise routes for one modulus: a caller queues its pair; whoever finds
// a batch slot free becomes a leader and runs one k_pairs launch over everything queued so far (group
// commit: no added wait when calls arrive one at a time, one launch per burst under load). Up to
// pair_inflight() batches run at once, each on its own stream, so one batch's host round trip overlaps
// the next; a finished leader wakes exactly the callers it served and the oldest waiter (no herd).
// Default 4 (64 native callers, round 4: 3.13e5 pairs/s, p99 0.45 ms; 2 in flight: 2.46e5, and 8 no
// better); DDSHE_PAIR_INFLIGHT overrides it for A/B runs
inline int pair_inflight() {
  static const int n = [] {
    const char* e = getenv("DDSHE_PAIR_INFLIGHT");
    const int v = e ? atoi(e) : 4;
    return v < 1 ? 1 : v;
  }();
  return n;
}
struct PairReq {
  bn::Limbs a, b;  // magnitudes, already < N
  bn::Limbs r;     // a*b mod N
  int rc = 0;
  std::atomic<bool> done{false};  // release-stored by the leader after r / rc
  bool taken = false;     // in a batch (no longer in pending); under the queue mutex
  bool sleeping = false;  // blocked on cv (else spinning on `done`: the leader must not touch it after)
  std::condition_variable cv;
};
struct PairQueue {
  std::mutex mu;
  std::vector<PairReq*> pending;
  int inflight = 0;
  int host_busy = 0;  // lone requests being served by the host product (policy DDS_PAIR_LONE)
};

// pinned staging of a worker (fixed 16 KiB, allocated once: pointers into it stay valid across a call):
// bytes [0, 64) small readbacks (read_sync), words [16, 4096) the finalize Y and result
constexpr size_t kStageBytes = 16384, kStageWord0 = 16;
constexpr size_t kStageDoneWord = kStageBytes / 4 - 1;  // the finalize's completion word (past Y + result)
inline hipError_t stage_ptr(Worker* w, uint32_t** p) {
  hipError_t e = w->hstage.ensure(kStageBytes);
  *p = e == hipSuccess ? (uint32_t*)w->hstage.p : nullptr;
  return e;
}
// the worker's MappedWords (launch_ope_order's read-back words 0..3; an OPE filter's match count
// at kCountWord), allocated on first use
constexpr size_t kCountWord = 4;
inline hipError_t mapped_words(Worker* w, MappedWords* ow) {
  w->hord.flags = hipHostMallocCoherent | hipHostMallocMapped;
  hipError_t e = w->hord.ensure(64);
  ow->h = (volatile uint64_t*)w->hord.p;
  ow->d = (uint64_t*)w->hord.dptr;
  return e;
}

// copy `bytes` (<= 64) device -> host through the pinned slot and synchronise the stream (a one-wave
// kernel storing them there instead measured the same on the config-1 decimal route)
inline hipError_t read_sync(Worker* w, hipStream_t st, const void* dsrc, void* dst, size_t bytes) {
  uint32_t* h = nullptr;
  hipError_t e = stage_ptr(w, &h);
  if (e != hipSuccess) return e;
  if (bytes > 64) return hipErrorInvalidValue;
  if ((e = hipMemcpyAsync(h, dsrc, bytes, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
  memcpy(dst, h, bytes);
  return hipSuccess;
}

// a new worker (stream, events) owned by ctx->workers and not in ctx->idle; the caller's device must be
// the context's. The HIP calls run outside the context lock, so callers that find an idle worker (and
// get_mod lookups) do not wait behind a creation
inline int new_worker(dds_ctx* ctx, Worker** out) {
  auto nw = std::make_unique<Worker>();
  if (hipStreamCreateWithFlags(&nw->stream, hipStreamNonBlocking) != hipSuccess) return fail(DDS_E_HIP, "hipStreamCreate");
  for (auto& e : nw->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(DDS_E_HIP, "hipEventCreate");
  for (auto& e : nw->ev_dec)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(DDS_E_HIP, "hipEventCreate");
  if (hipEventCreateWithFlags(&nw->ev_peer, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&nw->ev_done, hipEventDisableTiming) != hipSuccess)
    return fail(DDS_E_HIP, "hipEventCreate");
  std::lock_guard<std::mutex> lk(ctx->mu);
  *out = nw.get();
  ctx->workers.push_back(std::move(nw));
  return DDS_OK;
}

struct WorkerLease {
  dds_ctx* ctx;
  Worker* w = nullptr;
  hipStream_t st = nullptr;
  explicit WorkerLease(dds_ctx* c) : ctx(c) {}
  int prev_device = -1;
  int acquire() {
    // every entry point runs on its context's device, whatever the calling thread used before (the
    // caller's current device is restored when the lease ends)
    if (hipGetDevice(&prev_device) != hipSuccess) prev_device = -1;
    if (prev_device != ctx->device && hipSetDevice(ctx->device) != hipSuccess) return fail(DDS_E_HIP, "hipSetDevice");
    {
      std::lock_guard<std::mutex> lk(ctx->mu);
      if (!ctx->idle.empty()) {
        w = ctx->idle.back();
        ctx->idle.pop_back();
      }
    }
    if (!w) {
      const int rc = new_worker(ctx, &w);
      if (rc) return rc;
    }
    st = ctx->ext_stream ? ctx->ext_stream : w->stream;
    return DDS_OK;
  }
  ~WorkerLease() {
    if (w) {
      std::lock_guard<std::mutex> lk(ctx->mu);
      ctx->idle.push_back(w);
    }
    if (prev_device >= 0 && prev_device != ctx->device) (void)hipSetDevice(prev_device);
  }
};


// Upload `count` big-endian operands into an rW column (X, stride) validated against mc.
// Host worker pool for the boundary codecs: parallel copies of caller buffers into pinned staging
// (one thread copies ~10-15 GB/s, below what PCIe moves). parallel_for(n, f) splits [0, n) into
// one contiguous slice per thread, aligned to `align`, and calls f(begin, end) on each.
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool pool;
    return pool;
  }
  template <class F>
  void parallel_for(size_t n, size_t align, F&& f) {
    // a forked child inherits the pool object but not its threads: run on the calling thread
    if (th_.empty() || getpid() != owner_) {
      f((size_t)0, n);
      return;
    }
    std::lock_guard<std::mutex> job(job_mu_);
    const size_t T = th_.size() + 1;
    size_t piece = (n + T - 1) / T;
    piece = (piece + align - 1) / align * align;
    std::function<void(size_t, size_t)> fn = f;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      piece_ = piece;
      pending_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    f((size_t)0, std::min(piece, n));  // slice 0 on the calling thread
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
  }
  void copy(void* dst, const void* src, size_t n) {
    if (n < ((size_t)4 << 20)) {
      memcpy(dst, src, n);
      return;
    }
    parallel_for(n, 4096, [&](size_t a, size_t e) { memcpy((char*)dst + a, (const char*)src + a, e - a); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  CopyPool() : owner_(getpid()) {
    int n = 8;
    if (const char* e = getenv("DDSHE_COPY_THREADS")) n = atoi(e);
    n = std::max(1, std::min(n, 64));
    for (int i = 1; i < n; ++i) th_.emplace_back([this, i] { run(i); });
  }
  void run(int id) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void(size_t, size_t)>* fn = fn_;
      const size_t n = n_, a = (size_t)id * piece_;
      const size_t e = a < n ? std::min(n, a + piece_) : a;
      lk.unlock();
      if (e > a) (*fn)(a, e);
      lk.lock();
      if (--pending_ == 0) done_.notify_one();
    }
  }
  pid_t owner_;
  std::vector<std::thread> th_;
  std::mutex mu_, job_mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t, size_t)>* fn_ = nullptr;
  size_t n_ = 0, piece_ = 0;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};


constexpr size_t kIngestChunkBytes = (size_t)64 << 20;  // binary rows per pinned chunk

// ---- decimal codec (BigInteger.toString rows) ---------------------------------------------
// The rows arrive either Arrow-style (chars + offsets[count+1]) or as NUL-terminated strings
// (the JNA String[] of the route bodies, DDSRestServer.scala:417,419,422,513).
struct DecRows {
  const char* chars = nullptr;
  const uint64_t* offs = nullptr;
  const char* const* strs = nullptr;
  size_t len(size_t i) const { return strs ? strlen(strs[i]) : (size_t)(offs[i + 1] - offs[i]); }
  const char* row(size_t i) const { return strs ? strs[i] : chars + offs[i]; }
};

constexpr size_t kDecChunkBytes = (size_t)64 << 20;  // chars per pinned chunk
constexpr size_t kDecChunkRows = (size_t)1 << 18;
constexpr size_t kDecLenBlock = (size_t)1 << 14;  // String[] rows measured per host-pool pass

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
// rows of one rW matrix of this modulus' shape must stay addressable by the kernels (max_stride)
int check_rows(const ModConsts& mc, size_t rows);
// cap on the per-context modulus-constant cache (DDSHE_MAX_MODULI, default 64; LRU eviction)
size_t max_cached_moduli();
// constants of an odd modulus > 1 in the shape for max(bits(N), min_bits)
int get_mod(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, std::shared_ptr<ModConsts>* out,
            size_t min_bits = 0);
// dds_modmul_fold for an odd modulus, in the shape for max(bits(N), min_bits)
int modmul_fold_be(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, size_t min_bits, const uint8_t* ops,
                   size_t width, size_t count, uint8_t* out, size_t out_cap, size_t* out_len);
int product_tree(dds_ctx* ctx, const std::vector<uint32_t>& h, size_t count, size_t len, size_t cap16, bn::Limbs* out);
bn::Limbs low_bits(const bn::Limbs& x, size_t t);
int fold_even_modulus(dds_ctx* ctx, const bn::Limbs& M, const std::vector<bn::Limbs>& xs, const std::vector<bool>& negs,
                      bn::Limbs* out);
void record_time(dds_ctx* ctx, Worker* w, hipStream_t st, bool begin, int slot);
// [p, p + bytes) lies inside one buffer the caller registered with dds_host_register
bool host_registered(dds_ctx* ctx, const void* p, size_t bytes);
// the device address of p when [p, p + bytes) lies in a registered, device-mapped buffer, else null
void* host_device_ptr(dds_ctx* ctx, const void* p, size_t bytes);
int pick_tpi(int S);
size_t max_fold_groups(dds_ctx* ctx, int S);
// Leaves of the reduction tree: X[l * xs + g * gs] (g = ids[k] when ids), l < Sin limbs of Win bits,
// holding prod * 2^E over n leaves (gs = 1: limb-major, as lane-group launches read them; xs = 1,
// gs = Sin: row-major, written by the launch that hands its partials to the tree)
struct Leaves {
  const uint32_t* X;
  size_t xs;
  int Sin, Win;
  size_t n;
  int64_t E;
  const uint32_t* ids;
  size_t gs = 1;
  size_t rows = 0;  // rows folded into these leaves (finalize: how the host waits for the root)
};
int fold_level1(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint32_t* X, size_t xstride,
                size_t count, const uint32_t* d_ids, Leaves* lv, size_t max_groups = 0);
int reduce_leaves(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const Leaves& lv, bool finalize,
                  bn::Limbs* value, const uint32_t** part, int64_t* Eout);
// canonical product of `count` rows (rows d_ids[0..count) when given); synchronises the stream
int fold_value_device(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint32_t* X, size_t xstride,
                      size_t count, const uint32_t* d_ids, bn::Limbs* value);
// Fold `count` rows of an rW column (rows ids[0..count) when d_ids != nullptr) into one un-finalised
// partial: tail-shape limbs (row 0 of `*part`, stride `*part_stride`) holding prod(rows) * 2^(*E).
int fold_partial_device(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint32_t* X, size_t xstride,
                        size_t count, const uint32_t** part, size_t* part_stride, int64_t* E,
                        const uint32_t* d_ids = nullptr);
void account_fold(dds_ctx* ctx, Worker* w);
int emit_be(const bn::Limbs& v, size_t width, uint8_t* out, size_t out_cap, size_t* out_len);
// Upload `count` big-endian operands into an rW column (X, stride) validated against mc; rows >= 2N
// are reduced on the GPU and, when `reduced` is given, listed there (ascending).
int ingest(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint8_t* ops, size_t width, size_t count,
           DevBuf& raw, uint32_t* X, size_t stride, std::vector<size_t>* reduced = nullptr);
int dec_table(ModConsts& mc);
int ingest_dec(Worker* w, hipStream_t st, ModConsts& mc, const DecRows& src, size_t count, uint32_t* X,
               size_t stride, uint32_t* orflags, std::vector<size_t>* long_rows);
// indices of rows whose status has any bit of `mask` (after ingest_dec)
int dec_rows_with(Worker* w, hipStream_t st, size_t count, uint32_t mask, std::vector<size_t>* rows);
// SumAll/MultAll over the LIVE resident rows among row_ids[0..n) or [first, first+n); value + sign of
// the result. The caller holds col->mu (shared).
int col_fold_value(dds_col* col, const uint64_t* row_ids, size_t first, size_t n, bn::Limbs* v, bool* neg);
// Live rows of [first, first+count) of a column (caller holds col->mu): *d_ids = nullptr and *n = count
// when no row of the column is dead; else the live rows' offsets from `first`, ascending, compacted on
// the GPU into w->ids, and their number (one small read-back).
int col_live_range(dds_col* col, Worker* w, hipStream_t st, size_t first, size_t count, const uint32_t** d_ids,
                   size_t* n);
// Row ids of the list that are live (caller holds col->mu)
std::vector<uint64_t> col_live_ids(const dds_col* col, const uint64_t* ids, size_t n);
// dds_col_write_rows[_dec] in two phases (caller holds col->mu exclusively): prepare ingests and validates
// the new operands into the lease's scratch (the column is untouched, so a failure anywhere — in any
// shard of a dds_mcol — leaves every column unchanged); commit scatters them into the rows.
struct RowWrite {
  std::unique_ptr<WorkerLease> wl;
  std::vector<uint32_t> ids32;                                 // distinct target rows
  std::vector<std::pair<size_t, dds_col::Orig>> origs;         // (index into ids32, appended operand)
  size_t ss = 0;                                               // scratch stride (rows)
};
int col_write_prepare(dds_col* col, const uint64_t* ids, size_t n, const uint8_t* ops, size_t width,
                      const char* chars, const uint64_t* offsets, RowWrite* plan);
int col_write_commit(dds_col* col, RowWrite& plan);
int col_set_live(dds_col* col, const uint64_t* ids, size_t n, const uint8_t* live);
int combine_partials(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint32_t* h_parts,
                     const uint32_t* d_parts, const uint64_t* rows, size_t nparts, uint8_t* out, size_t out_cap,
                     size_t* out_len);
// synthetic Paillier rows (dds_col_fill_paillier_synth); shards/shard: global-row mapping of a
// 64-row-block round-robin sharded column (1, 0: the column's own row numbers)
int col_fill_paillier_synth(dds_col* col, const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be, size_t g_bytes,
                            uint64_t seed, uint64_t row0, size_t count, uint32_t pool_size, uint32_t shards,
                            uint32_t shard);


}  // namespace host
}  // namespace ddshe
