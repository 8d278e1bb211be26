// Pairwise routes with a modulus, coalesced across concurrent callers.
//   GET /Sum  (DDSRestServer.scala:355-395): HomoAdd.sum(op1, op2, nsquare)        (:385)
//   GET /Mult (DDSRestServer.scala:447-490): HomoMult.multiply(op1, op2, pubkey)   (:479)
// Each request is one modular product. Served one by one, a request costs a full GPU round trip for
// one Montgomery product; the proxy runs routes concurrently on its pool (DDSRestServer.scala:21), so
// concurrent requests under one modulus share a queue and the first caller to find it idle runs ONE
// k_pairs launch over every pair queued so far (the others sleep on the queue's condition variable
// and wake with their result). A lone request pays no batching wait. Up to pair_inflight() batches of
// one modulus run at once (own streams): while one waits for its GPU round trip the next gathers and
// launches. A burst of up to kTailPairs
// pairs runs in the latency shape straight from the parsed limbs (one pinned H2D, one k_pairs launch,
// one D2H, one synchronisation); larger ones take the batched dds_modmul_pairs path. A queue lives
// while it has work: the last caller out of an idle queue drops it, so moduli sent once by clients
// leave nothing behind.
// Policy (dds_pair_set_policy): DDS_PAIR_GPU queues every request; DDS_PAIR_LONE serves a request that
// finds its modulus' queue empty, no batch in flight and no other host product running with the
// engine's host product (bn::barrett64_modmul: one 4096-bit product costs less host CPU than a GPU
// round trip's wait), the others queue; DDS_PAIR_HOST serves every request that way.
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <chrono>
#include <condition_variable>
#include <thread>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "ddshe_host.hpp"

using namespace ddshe;
using namespace ddshe::host;

namespace {

constexpr size_t kTailPairs = 256;

void atomic_max(std::atomic<uint64_t>& m, uint64_t v) {
  uint64_t cur = m.load();
  while (v > cur && !m.compare_exchange_weak(cur, v)) {
  }
}

uint64_t since_ns(std::chrono::steady_clock::time_point t0) {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

// thread CPU clock (dds_pair_cpu's phases)
uint64_t cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
enum { kCpuCodec = 0, kCpuPack = 1, kCpuQueue = 2, kCpuWait = 3, kCpuHost = 4 };

int pair_policy(dds_ctx* ctx) {
  const int p = ctx->pair_policy.load(std::memory_order_relaxed);
  if (p >= 0) return p;
  static const int dflt = [] {
    const char* e = getenv("DDSHE_PAIR_POLICY");
    return e ? atoi(e) : DDS_PAIR_HOST;
  }();
  return dflt;
}

// the host product's constants of M (built once per context and modulus; a few dozen moduli at most
// are kept: a client that sends a new modulus per request rebuilds them)
std::shared_ptr<const bn::Barrett64> barrett_of(dds_ctx* ctx, const bn::Limbs& M) {
  {
    std::lock_guard<std::mutex> lk(ctx->pmu);
    auto it = ctx->pair_bar.find(M);
    if (it != ctx->pair_bar.end()) return it->second;
  }
  auto b = std::make_shared<const bn::Barrett64>(bn::barrett64_make(M));
  std::lock_guard<std::mutex> lk(ctx->pmu);
  if (ctx->pair_bar.size() >= 64) ctx->pair_bar.clear();
  ctx->pair_bar.emplace(M, b);
  return b;
}

// never throws: an allocation failure becomes req->rc = DDS_E_NOMEM, so a caller that raised a queue's
// host_busy around it always gets to lower it again
void host_product(dds_ctx* ctx, const bn::Barrett64& bar, PairReq* req) noexcept {
  const uint64_t c0 = cpu_ns();
  try {
    req->r = bn::barrett64_modmul(bar, req->a, req->b);
  } catch (...) {
    req->rc = DDS_E_NOMEM;
  }
  ctx->pair_cpu_ns[kCpuHost].fetch_add(cpu_ns() - c0);
  ctx->pair_host_calls.fetch_add(1);
}

// a worker of the context's pairwise pool (dds_ctx::pair_free): at most pair_inflight() exist; a leader
// that finds none free waits for one (a batch takes tens of µs) instead of making another
struct PairLease {
  dds_ctx* ctx;
  Worker* w = nullptr;
  hipStream_t st = nullptr;
  int prev_device = -1;
  explicit PairLease(dds_ctx* c) : ctx(c) {}
  int acquire() {
    if (hipGetDevice(&prev_device) != hipSuccess) prev_device = -1;
    if (prev_device != ctx->device && hipSetDevice(ctx->device) != hipSuccess) return fail(DDS_E_HIP, "hipSetDevice");
    std::unique_lock<std::mutex> lk(ctx->pwmu);
    while (ctx->pair_free.empty() && ctx->pair_made >= pair_inflight()) ctx->pwcv.wait(lk);
    if (!ctx->pair_free.empty()) {
      w = ctx->pair_free.back();
      ctx->pair_free.pop_back();
    } else {
      ++ctx->pair_made;
      lk.unlock();
      const int rc = new_worker(ctx, &w);
      if (rc) {
        std::lock_guard<std::mutex> g(ctx->pwmu);
        --ctx->pair_made;
        ctx->pwcv.notify_one();
        w = nullptr;
        return rc;
      }
    }
    st = ctx->ext_stream ? ctx->ext_stream : w->stream;
    return DDS_OK;
  }
  ~PairLease() {
    if (w) {
      std::lock_guard<std::mutex> lk(ctx->pwmu);
      ctx->pair_free.push_back(w);
      ctx->pwcv.notify_one();
    }
    if (prev_device >= 0 && prev_device != ctx->device) (void)hipSetDevice(prev_device);
  }
};

// the batch in the tree (latency) shape from limbs already < M: one workgroup product per pair
int tail_batch(dds_ctx* ctx, const bn::Limbs& M, const std::vector<PairReq*>& batch) {
  const size_t mb = bn::byte_length(M), n = batch.size();
  std::vector<uint8_t> mbe(mb);
  bn::to_be(M, mbe.data(), mb);
  std::shared_ptr<ModConsts> mcp;
  int rc = get_mod(ctx, mbe.data(), mb, &mcp);
  if (rc) return rc;
  ModConsts& mc = *mcp;
  PairLease wl(ctx);
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  const int S3 = mc.S3;  // one workgroup per pair in the tree shape (k_pairs_sos)
  const size_t words = (size_t)S3 * n;
  // zero-copy (default): the operands and results live in coherent, device-mapped host memory that
  // k_pairs_sos reads and writes over PCIe (a few hundred bytes per pair), so a batch is one launch and
  // one synchronisation instead of an H2D copy, the launch, a D2H copy and the synchronisation.
  // DDSHE_PAIR_ZEROCOPY=0: the staged copies.
  static const bool zc = [] {
    const char* e = getenv("DDSHE_PAIR_ZEROCOPY");
    return !e || atoi(e) != 0;
  }();
  HostBuf& hb = zc ? w->hpair : w->hch[1];
  if (zc) hb.flags = hipHostMallocCoherent | hipHostMallocMapped;
  // sized once for the largest tail batch: re-pinning a growing buffer (hipHostFree + hipHostMalloc)
  // stalls the leader for tens of ms (max batch 30-34 ms under 64 callers, tools/native/pairs_sweep.sh)
  const size_t cap_bytes = 3 * (size_t)S3 * std::max(n, kTailPairs) * 4;
  HIP_TRY(hb.ensure(cap_bytes));
  uint32_t* h = (uint32_t*)hb.p;
  uint64_t c0 = cpu_ns();
  for (size_t i = 0; i < n; ++i) {
    const std::vector<uint32_t> ra = bn::to_rw(batch[i]->a, S3, mc.W3), rb = bn::to_rw(batch[i]->b, S3, mc.W3);
    std::copy(ra.begin(), ra.end(), h + i * S3);
    std::copy(rb.begin(), rb.end(), h + words + i * S3);
  }
  ctx->pair_cpu_ns[kCpuPack].fetch_add(cpu_ns() - c0);
  const auto g0 = std::chrono::steady_clock::now();
  if (zc) {
    uint32_t* d = (uint32_t*)hb.dptr;
    HIP_TRY(launch_pairs_sos(S3, d, d + words, n, mc.d3, mc.d3 + 5 * (size_t)S3, d + 2 * words, wl.st));
  } else {
    HIP_TRY(w->x2.ensure(cap_bytes));
    uint32_t* d = w->x2.as<uint32_t>();
    HIP_TRY(hipMemcpyAsync(d, h, 2 * words * 4, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(launch_pairs_sos(S3, d, d + words, n, mc.d3, mc.d3 + 5 * (size_t)S3, d + 2 * words, wl.st));
    HIP_TRY(hipMemcpyAsync(h + 2 * words, d + 2 * words, words * 4, hipMemcpyDeviceToHost, wl.st));
  }
  c0 = cpu_ns();
  HIP_TRY(hipStreamSynchronize(wl.st));
  const uint64_t c1 = cpu_ns();
  ctx->pair_cpu_ns[kCpuWait].fetch_add(c1 - c0);
  const uint64_t gns = since_ns(g0);
  ctx->pair_gpu_ns.fetch_add(gns);
  atomic_max(ctx->pair_max_gpu_ns, gns);
  for (size_t i = 0; i < n; ++i) batch[i]->r = bn::from_rw(h + 2 * words + i * S3, S3, mc.W3);
  ctx->pair_cpu_ns[kCpuPack].fetch_add(cpu_ns() - c1);
  return DDS_OK;
}

// one k_pairs launch for the batch: results into each request (rc on failure)
void run_batch_(dds_ctx* ctx, const bn::Limbs& M, const std::vector<PairReq*>& batch) {
  const size_t mb = bn::byte_length(M), n = batch.size();
  if (n <= kTailPairs) {
    const int rc = tail_batch(ctx, M, batch);
    ctx->pair_launches.fetch_add(1);
    for (PairReq* r : batch) r->rc = rc;
    return;
  }
  std::vector<uint8_t> mbe(mb), A(n * mb), B(n * mb), O(n * mb);
  bn::to_be(M, mbe.data(), mb);
  for (size_t i = 0; i < n; ++i) {
    bn::to_be(batch[i]->a, A.data() + i * mb, mb);
    bn::to_be(batch[i]->b, B.data() + i * mb, mb);
  }
  int rc = dds_modmul_pairs(ctx, mbe.data(), mb, A.data(), B.data(), mb, n, O.data());
  ctx->pair_launches.fetch_add(1);
  for (size_t i = 0; i < n; ++i) {
    batch[i]->rc = rc;
    if (!rc) batch[i]->r = bn::from_be(O.data() + i * mb, mb);
  }
}

void run_batch(dds_ctx* ctx, const bn::Limbs& M, const std::vector<PairReq*>& batch) {
  const auto t0 = std::chrono::steady_clock::now();
  run_batch_(ctx, M, batch);
  const uint64_t ns = since_ns(t0);
  ctx->pair_batch_ns.fetch_add(ns);
  atomic_max(ctx->pair_max_batch_ns, ns);
}

// DDSHE_PAIR_SPIN_US (default 0: sleep at once): how long a caller in another leader's batch yields
// before it sleeps on its condition variable. 64 native callers (tools/native/pairs_sweep.sh, round 4,
// warmed up, pre-sized batch buffers): 4 batches in flight 3.13e5 pairs/s at spin 0 against 2.94e5 at
// 100 us (yielding threads take host cores the leaders and the decimal codec need); round 3, at 2 in
// flight: 400 us -> p99 9-19 ms, 100 us -> 0.8-1.0 ms.
int pair_spin_us() {
  static const int us = [] {
    const char* e = getenv("DDSHE_PAIR_SPIN_US");
    return e ? atoi(e) : 0;
  }();
  return us;
}

int modmul_coalesced(dds_ctx* ctx, const bn::Limbs& M, PairReq* req,
                     const std::shared_ptr<const bn::Barrett64>& bar) {
  const int policy = pair_policy(ctx);
  if (policy == DDS_PAIR_HOST) {
    host_product(ctx, *bar, req);
    return req->rc;
  }
  const uint64_t c_in = cpu_ns();
  uint64_t c_batch = 0;  // CPU of the batches this caller led (counted in their own phases)
  std::shared_ptr<PairQueue> q;
  {
    std::lock_guard<std::mutex> lk(ctx->pmu);
    auto& slot = ctx->pair_queues[M];
    if (!slot) slot = std::make_shared<PairQueue>();
    q = slot;
  }
  std::unique_lock<std::mutex> lk(q->mu);
  if (policy == DDS_PAIR_LONE && q->pending.empty() && q->inflight == 0 && q->host_busy == 0) {
    ++q->host_busy;  // lone: the host product, while later callers queue for a GPU batch
    lk.unlock();
    host_product(ctx, *bar, req);
    lk.lock();
    --q->host_busy;
    if (!q->pending.empty() && q->pending.front()->sleeping) q->pending.front()->cv.notify_one();  // a leader
    req->done.store(true, std::memory_order_release);
  } else {
    q->pending.push_back(req);
  }
  while (!req->done.load(std::memory_order_acquire)) {
    if (req->taken) {
      // in another leader's batch: spin briefly without the lock (a batch takes tens of µs), then sleep
      lk.unlock();
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(pair_spin_us());
      while (!req->done.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < until)
        std::this_thread::yield();
      lk.lock();
      if (req->done.load(std::memory_order_acquire)) break;
      req->sleeping = true;
      req->cv.wait(lk);
      req->sleeping = false;
      continue;
    }
    if (q->inflight >= pair_inflight()) {
      req->sleeping = true;
      req->cv.wait(lk);
      req->sleeping = false;
      continue;
    }
    // leader: take everything queued (this request included) and launch once
    ++q->inflight;
    std::vector<PairReq*> batch;
    batch.swap(q->pending);
    for (PairReq* r : batch) r->taken = true;
    lk.unlock();
    const uint64_t b0 = cpu_ns();
    try {
      run_batch(ctx, M, batch);
    } catch (...) {
      for (PairReq* r : batch) r->rc = DDS_E_NOMEM;
    }
    c_batch += cpu_ns() - b0;
    lk.lock();
    --q->inflight;
    if (!q->pending.empty() && q->pending.front()->sleeping) q->pending.front()->cv.notify_one();  // next leader
    for (PairReq* r : batch) {
      if (r == req) continue;
      // a spinning waiter may return (and free r) as soon as `done` is set: read `sleeping` first; a
      // sleeping one cannot return before we release the mutex
      const bool sl = r->sleeping;
      r->done.store(true, std::memory_order_release);
      if (sl) r->cv.notify_one();
    }
    req->done.store(true, std::memory_order_release);
  }
  const bool idle = q->inflight == 0 && q->pending.empty() && q->host_busy == 0;
  lk.unlock();
  if (idle) {  // drop the idle queue (a caller that still holds it just runs as its own leader)
    std::lock_guard<std::mutex> g(ctx->pmu);
    auto it = ctx->pair_queues.find(M);
    if (it != ctx->pair_queues.end() && it->second == q) {
      std::lock_guard<std::mutex> ql(q->mu);
      if (q->inflight == 0 && q->pending.empty() && q->host_busy == 0) ctx->pair_queues.erase(it);
    }
  }
  const uint64_t c_all = cpu_ns() - c_in;
  ctx->pair_cpu_ns[kCpuQueue].fetch_add(c_all > c_batch ? c_all - c_batch : 0);
  return req->rc;
}

}  // namespace

extern "C" {

int dds_pair_modmul_dec(dds_ctx* ctx, const char* a_dec, const char* b_dec, const char* mod_dec, char* out,
                        size_t out_cap, size_t* out_len) {
  try {
    if (!ctx || !a_dec || !b_dec || !mod_dec) return fail(DDS_E_ARG, "bad arguments");
    ctx->pair_calls.fetch_add(1);
    uint64_t c0 = cpu_ns();
    // operands first, then the modulus (:380-383): any of them malformed -> NumberFormatException -> 500
    bn::Limbs a, b, M;
    std::shared_ptr<const bn::Barrett64> bar;
    bool an = false, bneg = false, mneg = false;
    if (!bn::from_dec(a_dec, strlen(a_dec), a, &an)) return fail(DDS_E_FORMAT, "NumberFormatException: operand1");
    if (!bn::from_dec(b_dec, strlen(b_dec), b, &bneg)) return fail(DDS_E_FORMAT, "NumberFormatException: operand2");
    {  // the route passes the same nsqr / pubkey modulus with every request: keep the last parse per thread
      thread_local std::string last_text;
      thread_local bn::Limbs last_mod;
      thread_local bool last_neg = false, last_ok = false;
      thread_local std::shared_ptr<const bn::Barrett64> last_bar;
      thread_local const dds_ctx* last_ctx = nullptr;
      const size_t ml = strlen(mod_dec);
      if (!(last_text.size() == ml && memcmp(last_text.data(), mod_dec, ml) == 0)) {
        last_text.assign(mod_dec, ml);
        last_ok = bn::from_dec(mod_dec, ml, last_mod, &last_neg);
        last_bar.reset();
      }
      if (!last_ok) return fail(DDS_E_FORMAT, "NumberFormatException: modulus");
      M = last_mod;
      mneg = last_neg;
      if (!mneg && !M.empty() && (M[0] & 1u) && bn::bit_length(M) >= 2) {
        if (!last_bar || last_ctx != ctx) last_bar = barrett_of(ctx, M);
        last_ctx = ctx;
        bar = last_bar;
      }
    }
    if (mneg || M.empty()) return fail(DDS_E_FORMAT, "ArithmeticException: BigInteger: modulus not positive");
    if (!(M[0] & 1u) || bn::bit_length(M) < 2) {  // even modulus or 1: the fold's CRT path, uncoalesced
      const char* vals[2] = {a_dec, b_dec};
      return dds_sum_all_dec(ctx, vals, 2, mod_dec, out, out_cap, out_len);
    }
    // BigInteger.mod semantics: |a| |b| mod M on the GPU, the sign applied after
    if (bn::cmp(a, M) >= 0) a = bn::mod(a, M);
    if (bn::cmp(b, M) >= 0) b = bn::mod(b, M);
    PairReq req;
    req.a = std::move(a);
    req.b = std::move(b);
    ctx->pair_cpu_ns[kCpuCodec].fetch_add(cpu_ns() - c0);
    int rc = modmul_coalesced(ctx, M, &req, bar);
    if (rc) return rc;
    c0 = cpu_ns();
    bn::Limbs r = std::move(req.r);
    bn::trim(r);
    if ((an != bneg) && !r.empty()) r = bn::sub(M, r);
    const std::string s = bn::to_dec(r);
    if (out_len) *out_len = s.size();
    if (!out || out_cap < s.size() + 1) return fail(DDS_E_BUFSIZE, "output buffer too small");
    memcpy(out, s.c_str(), s.size() + 1);
    ctx->pair_cpu_ns[kCpuCodec].fetch_add(cpu_ns() - c0);
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_pair_stats(dds_ctx* ctx, uint64_t* calls, uint64_t* launches) {
  if (!ctx) return fail(DDS_E_ARG, "bad arguments");
  if (calls) *calls = ctx->pair_calls.load();
  if (launches) *launches = ctx->pair_launches.load();
  return DDS_OK;
}

int dds_pair_timing(dds_ctx* ctx, uint64_t* batch_ns, uint64_t* gpu_ns, uint64_t* max_batch_ns,
                    uint64_t* max_gpu_ns) {
  if (!ctx) return fail(DDS_E_ARG, "bad arguments");
  if (batch_ns) *batch_ns = ctx->pair_batch_ns.load();
  if (gpu_ns) *gpu_ns = ctx->pair_gpu_ns.load();
  if (max_batch_ns) *max_batch_ns = ctx->pair_max_batch_ns.exchange(0);  // window: since the last read
  if (max_gpu_ns) *max_gpu_ns = ctx->pair_max_gpu_ns.exchange(0);
  return DDS_OK;
}

int dds_pair_set_policy(dds_ctx* ctx, int policy, int* previous) {
  if (!ctx || policy > DDS_PAIR_HOST) return fail(DDS_E_ARG, "bad arguments");
  if (previous) *previous = pair_policy(ctx);
  if (policy >= 0) ctx->pair_policy.store(policy);
  return DDS_OK;
}

int dds_pair_cpu(dds_ctx* ctx, uint64_t* codec_ns, uint64_t* pack_ns, uint64_t* queue_ns, uint64_t* wait_ns,
                 uint64_t* host_ns, uint64_t* host_calls) {
  if (!ctx) return fail(DDS_E_ARG, "bad arguments");
  uint64_t* outs[5] = {codec_ns, pack_ns, queue_ns, wait_ns, host_ns};
  for (int i = 0; i < 5; ++i)
    if (outs[i]) *outs[i] = ctx->pair_cpu_ns[i].load();
  if (host_calls) *host_calls = ctx->pair_host_calls.load();
  return DDS_OK;
}

int dds_ctx_cache_stats(dds_ctx* ctx, size_t* moduli, size_t* pair_queues) {
  if (!ctx) return fail(DDS_E_ARG, "bad arguments");
  if (moduli) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    *moduli = ctx->mods.size();
  }
  if (pair_queues) {
    std::lock_guard<std::mutex> lk(ctx->pmu);
    *pair_queues = ctx->pair_queues.size();
  }
  return DDS_OK;
}

}  // extern "C"
