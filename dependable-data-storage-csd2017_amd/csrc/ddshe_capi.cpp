// C-ABI implementation (include/ddshe.h): contexts, stream/buffer pools, per-modulus
// Montgomery constants, and the host orchestration of the HIP kernels.
//
// The per-row arithmetic of every entry point runs on the GPU; the host only
// parses/serialises the boundary formats and computes O(1) per-call constants.
#include "ddshe.h"

#include <hip/hip_runtime.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "ddshe_host.hpp"

using namespace ddshe;
using namespace ddshe::host;

namespace ddshe {
namespace host {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}




// rows of one rW matrix of this modulus' shape must stay addressable by the kernels (max_stride)
int check_rows(const ModConsts& mc, size_t rows) {
  if (round_up(std::max<size_t>(rows, 1), 64) > max_stride(mc.S))
    return fail(DDS_E_UNSUPPORTED, "row count " + std::to_string(rows) + " exceeds the " +
                                       std::to_string(max_stride(mc.S)) + "-row limit of one column of this modulus");
  return DDS_OK;
}

int get_mod(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, std::shared_ptr<ModConsts>* out,
            size_t min_bits) {
  if (!mod_be || mod_bytes == 0) return fail(DDS_E_ARG, "modulus missing");
  bn::Limbs N = bn::from_be(mod_be, mod_bytes);
  if (N.empty() || (N[0] & 1u) == 0 || bn::bit_length(N) < 2)
    return fail(DDS_E_ARG, "modulus must be odd and > 1 (Montgomery)");
  const Shape sh = pick_shape(std::max(bn::bit_length(N), min_bits));
  if (!sh.S) return fail(DDS_E_UNSUPPORTED, "modulus too large");
  const auto key = std::make_pair(N, sh.S);
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    auto it = ctx->mods.find(key);
    if (it != ctx->mods.end()) {
      it->second->last_use = ++ctx->mod_tick;
      *out = it->second;
      return DDS_OK;
    }
  }
  auto mc = std::make_shared<ModConsts>();
  mc->bits = bn::bit_length(N);
  mc->bytes = (mc->bits + 7) / 8;
  const Shape tail = tail_shape(sh);
  mc->S = sh.S;
  mc->TPI = sh.TPI;
  mc->W = sh.W;
  mc->S2 = tail.S;
  const int S = mc->S;
  mc->N = N;
  mc->half = bn::sub(bn::add(N, bn::Limbs{1}), bn::Limbs{});
  (void)bn::divmod_small(mc->half, 2);
  mc->n0 = bn::mont_n0(N[0], mc->W);
  mc->Rmod = bn::mod(bn::pow2((size_t)mc->W * S), N);
  bn::Limbs R2 = bn::mod(bn::mul(mc->Rmod, mc->Rmod), N);
  bn::Limbs N2 = bn::add(N, N);
  auto fill = [&](std::vector<uint32_t>& dst, int s, const bn::Limbs& rmod, const bn::Limbs& r2) {
    dst.assign((size_t)kConstCount * s + 1, 0);  // +1: ingest reads 2N limb s (always 0 by choice of s)
    auto put = [&](int slot, const bn::Limbs& v) {
      auto r = bn::to_rw(v, s, mc->W);
      std::copy(r.begin(), r.end(), dst.begin() + (size_t)slot * s);
    };
    put(kConstN, N);
    put(kConstRmod, rmod);
    put(kConstR2, r2);
    put(kConstOne, bn::Limbs{1});
    put(kConstN2x, N2);
  };
  fill(mc->host, S, mc->Rmod, R2);
  {
    bn::Limbs rm2 = bn::mod(bn::pow2((size_t)mc->W * mc->S2), N);
    fill(mc->host2, mc->S2, rm2, bn::mod(bn::mul(rm2, rm2), N));
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(DDS_E_HIP, "hipSetDevice");
  if (hipMalloc(&mc->d, mc->host.size() * 4) != hipSuccess || hipMalloc(&mc->d2, mc->host2.size() * 4) != hipSuccess)
    return fail(DDS_E_NOMEM, "const alloc");
  if (hipMemcpy(mc->d, mc->host.data(), mc->host.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(mc->d2, mc->host2.data(), mc->host2.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return fail(DDS_E_HIP, "const upload");
  // N~ = N·n0 ≡ -1 mod 2^W (Mont QP), for the shapes where R = 2^(W·S) > 4N~ holds
  const bn::Limbs nq = bn::mul(N, bn::Limbs{mc->n0});
  auto upload_qp = [&](int s, uint32_t** dst) -> int {
    const std::vector<uint32_t> q = bn::to_rw(nq, s, mc->W);
    if (hipMalloc(dst, q.size() * 4) != hipSuccess) return fail(DDS_E_NOMEM, "const alloc");
    if (hipMemcpy(*dst, q.data(), q.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      return fail(DDS_E_HIP, "const upload");
    return DDS_OK;
  };
  mc->qbound = N;
  if (tail_qp(mc->S2)) {
    if ((size_t)mc->W * mc->S2 < bn::bit_length(nq) + 2) return fail(DDS_E_UNSUPPORTED, "tail shape too narrow");
    if (int rc = upload_qp(mc->S2, &mc->dq)) return rc;
    mc->qbound = nq;
  }
  // reduction-tree constants (ddshe_tree.hip), the class of the main shape's capacity
  {
    const Shape t3 = tree_shape((size_t)mc->W * S - 2);
    if (!t3.S) return fail(DDS_E_UNSUPPORTED, "no tree shape");
    mc->S3 = t3.S;
    mc->W3 = t3.W;
    const size_t k3 = (size_t)mc->W3 * mc->S3;
    // a tree product of raw rows a, b < 2^(W S) stays < 2N when a b / R3 < N (forced-wide shapes fail this)
    mc->tree_direct = k3 + bn::bit_length(N) - 1 >= 2 * (size_t)mc->W * S;
    bn::Limbs inv{1};  // N^-1 mod 2^k3 by Newton: inv <- inv (2 - N inv), doubling the correct bits
    const bn::Limbs two{2};
    for (size_t ok = 1; ok < k3; ok *= 2) {
      const bn::Limbs t = low_bits(bn::mul(N, inv), k3);
      inv = low_bits(bn::mul(inv, low_bits(bn::sub(bn::add(bn::pow2(k3), two), t), k3)), k3);
    }
    bn::trim(inv);
    const bn::Limbs np = bn::sub(bn::pow2(k3), inv);  // -N^-1 mod R3 (inv != 0: N odd)
    std::vector<uint32_t> h3;
    const bn::Limbs r3 = bn::mod(bn::pow2(k3), N);
    for (const bn::Limbs& v : {N, np, N, bn::add(N, N), bn::add(bn::add(N, N), N), bn::mod(bn::mul(r3, r3), N)}) {
      const std::vector<uint32_t> r = bn::to_rw(v, mc->S3, mc->W3);
      h3.insert(h3.end(), r.begin(), r.end());
    }
    if (hipMalloc(&mc->d3, h3.size() * 4) != hipSuccess) return fail(DDS_E_NOMEM, "const alloc");
    if (hipMemcpy(mc->d3, h3.data(), h3.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      return fail(DDS_E_HIP, "const upload");
  }
  if (fold_qp_enabled() && (size_t)mc->W * S >= bn::bit_length(nq) + 2) {
    if (int rc = upload_qp(S, &mc->dqm)) return rc;
    mc->qbound = nq;  // level-1 partials are then < 2N~ too
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  auto it = ctx->mods.find(key);
  if (it != ctx->mods.end()) {
    *out = it->second;
    return DDS_OK;
  }
  // bounded cache: the modulus comes with each request (nsqr / pubkey), so evict the least recently
  // used constants past the cap; columns and calls in flight keep theirs alive (shared_ptr)
  if (ctx->mods.size() >= max_cached_moduli()) {
    auto lru = ctx->mods.begin();
    for (auto i = ctx->mods.begin(); i != ctx->mods.end(); ++i)
      if (i->second->last_use < lru->second->last_use) lru = i;
    ctx->mods.erase(lru);
  }
  mc->last_use = ++ctx->mod_tick;
  ctx->mods.emplace(key, mc);
  *out = mc;
  return DDS_OK;
}

size_t max_cached_moduli() {
  static const size_t n = [] {
    const char* e = getenv("DDSHE_MAX_MODULI");
    return e ? std::max<size_t>(1, (size_t)atoll(e)) : (size_t)64;
  }();
  return n;
}

bool host_registered(dds_ctx* ctx, const void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(ctx->regmu);
  const uintptr_t b = (uintptr_t)p;
  auto it = ctx->host_regs.upper_bound(b);
  if (it == ctx->host_regs.begin()) return false;
  --it;
  return b + bytes <= it->first + it->second.bytes;
}

void* host_device_ptr(dds_ctx* ctx, const void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(ctx->regmu);
  const uintptr_t b = (uintptr_t)p;
  auto it = ctx->host_regs.upper_bound(b);
  if (it == ctx->host_regs.begin()) return nullptr;
  --it;
  if (b + bytes > it->first + it->second.bytes || !it->second.dptr) return nullptr;
  return (char*)it->second.dptr + (b - it->first);
}

void record_time(dds_ctx* ctx, Worker* w, hipStream_t st, bool begin, int slot) {
  if (!ctx->timing.load()) return;
  (void)hipEventRecord(w->ev[slot + (begin ? 0 : 1)], st);
}

int pick_tpi(int S) {
  for (size_t b = 8; b < 1u << 16; b += 8) {
    Shape sh = pick_shape(b);
    if (sh.S == S) return sh.TPI;
    if (!sh.S) break;
  }
  return 1;
}

size_t max_fold_groups(dds_ctx* ctx, int S) {
  int bpc = 0;
  if (fold_occupancy(S, &bpc) != hipSuccess || bpc < 1) bpc = 1;
  return (size_t)ctx->cus * bpc * (256 / pick_tpi(S));
}

// The reduction tree after the first fold level (ddshe_tree.hip: workgroup-cooperative Montgomery
// products, one launch per level). Default on: faster than round 1's per-level lane-group launches at
// every fold size measured (tools/tree_ab.py); DDSHE_TREE=0 selects those (k_fold in the
// tail shape + k_finalize) for A/B runs. DDSHE_TREE_DIRECT (rows, default 2048): folds up to that many
// rows skip the first level and run the tree over the rows themselves (when the tree's R3 covers raw
// rows, ModConsts::tree_direct).
bool use_tree() {
  static const bool on = [] {
    const char* e = getenv("DDSHE_TREE");
    return !(e && e[0] == '0');
  }();
  return on;
}
size_t tree_direct_rows() {
  static const size_t n = [] {
    const char* e = getenv("DDSHE_TREE_DIRECT");
    return e ? (size_t)atoll(e) : (size_t)2048;
  }();
  return n;
}
// DDSHE_TREE_SWITCH (leaves, default 4096): wider levels run as tail-shape lane-group launches (many
// products per launch: throughput), the last log2(switch) levels as tree launches (one workgroup per
// product: latency; the widest of them on 256-thread workgroups, ddshe_tree.hip). Round 3 A/B
// (tools/tree_sweep.sh, profiles/r03_tree_plan_sweep.txt): with the 256-thread wide levels and
// in-kernel hand-offs, 1024 -> 4096 takes a 10k-row fold of the 1024-bit key 0.092 -> 0.088 ms and
// of the 2048-bit key 0.141 -> 0.129 ms; 10M-row folds within noise.
size_t tree_switch_leaves() {
  static const size_t n = [] {
    const char* e = getenv("DDSHE_TREE_SWITCH");
    return e ? (size_t)atoll(e) : (size_t)4096;
  }();
  return n;
}

// DDSHE_NARROW_ROWS (rows, default 65536; 0 disables): folds of up to that many rows run their first
// level in the latency (tail) shape, one product per group, straight from the main-shape rows
size_t narrow_fold_rows() {
  static const size_t n = [] {
    const char* e = getenv("DDSHE_NARROW_ROWS");
    return e ? (size_t)atoll(e) : (size_t)65536;
  }();
  return n;
}

// Level 1 (throughput shape, G groups: group g holds prod_g * R^(1 - c_g)) over `count` rows of X (or
// rows d_ids[0..count)), unless the fold is small enough for the tree alone.
int fold_level1(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint32_t* X, size_t xstride,
                size_t count, const uint32_t* d_ids, Leaves* lv, size_t max_groups) {
  const int S = mc.S, S2 = mc.S2;
  if (use_tree() && mc.tree_direct && count <= tree_direct_rows()) {
    *lv = Leaves{X, xstride, S, mc.W, count, 0, d_ids};
    return DDS_OK;
  }
  // small folds: the first level in the latency shape S2 straight from the rows (one product per group)
  if (!d_ids && S2 > S && S % 4 == 0 && fold_narrow_shape(S2) && count <= narrow_fold_rows()) {
    const size_t G = std::max<size_t>(1, count / 2), ps = round_up(G, 64);
    const bool rowmajor = use_tree() && G <= tree_switch_leaves();  // straight to the tree
    HIP_TRY(w->p0.ensure((size_t)S2 * ps * 4));
    HIP_TRY(launch_fold_narrow(S2, X, xstride, count, S, mc.d2, mc.dq, mc.n0, w->p0.as<uint32_t>(), rowmajor ? 1 : ps,
                               G, st, rowmajor ? (size_t)S2 : 1));
    *lv = Leaves{w->p0.as<uint32_t>(), rowmajor ? 1 : ps, S2, mc.W, G, mc.wS2() * ((int64_t)G - (int64_t)count),
                 nullptr, rowmajor ? (size_t)S2 : 1};
    return DDS_OK;
  }
  // one bignum per lane for long folds of the narrow shapes (k_fold1), lane groups otherwise
  // (k_fold1 may run with fewer limbs than the column's shape: its partials then carry R1 = 2^(W*S1))
  const int S1 = (fold1_shape(S) && count >= fold1_min_rows(S, ctx->cus)) ? fold1_limbs(S, mc.bits) : 0;
  size_t gmax = max_fold_groups(ctx, S);
  if (S1) {
    int bpc = 0;
    if (fold1_occupancy(S1, &bpc) != hipSuccess || bpc < 1) bpc = 1;
    gmax = (size_t)ctx->cus * bpc * 256;
  }
  if (max_groups) gmax = std::min(gmax, max_groups);
  size_t G = std::min(gmax, std::max<size_t>(1, count / 2));
  size_t ps = round_up(G, 64);
  HIP_TRY(w->p0.ensure((size_t)S2 * ps * 4));
  // DDSHE_FOLD_INBLOCK=1 (A/B, off by default): level 1 with the in-block tree (k_fold InBlock), one
  // row-major leaf per block straight to the reduction tree instead of the tail launches that take the
  // G partials down to tree_switch_leaves(). Measured slower (profiles/r06_inblock_ab.txt: headline
  // level 1 14.6 -> 15.7 ms, the strong-split share 1.75 -> 2.11 ms): the in-block products run in the
  // throughput shape (4 lanes per bignum), whose per-product latency is ~4x the tail shape's.
  static const int inblock = [] {
    const char* e = getenv("DDSHE_FOLD_INBLOCK");
    return e ? atoi(e) : 0;
  }();
  const size_t gpb = 256 / (size_t)pick_tpi(S);
  const size_t Gb = G / gpb * gpb;  // whole blocks of live groups
  if (inblock && use_tree() && !S1 && !d_ids && mc.dqm && S2 >= S && Gb > tree_switch_leaves()) {
    G = Gb;
    const size_t B = G / gpb;
    record_time(ctx, w, st, true, 0);
    HIP_TRY(launch_fold(S, X, xstride, count, mc.d, mc.dqm, mc.n0, w->p0.as<uint32_t>(), 1, G, S2, st, nullptr, 0,
                        (size_t)S2));
    record_time(ctx, w, st, false, 0);
    if (ctx->timing.load()) {
      w->timed_fold = true;
      std::lock_guard<std::mutex> lk(ctx->tmu);
      ctx->pending_modmuls = count - B;  // the row products and the in-block ones
    }
    *lv = Leaves{w->p0.as<uint32_t>(), 1, S2, mc.W, B, (int64_t)mc.W * S * ((int64_t)B - (int64_t)count), nullptr,
                 (size_t)S2};
    return DDS_OK;
  }
  record_time(ctx, w, st, true, 0);
  HIP_TRY(launch_fold(S, X, xstride, count, mc.d, mc.dqm, mc.n0, w->p0.as<uint32_t>(), ps, G, S2, st, d_ids, S1));
  record_time(ctx, w, st, false, 0);
  if (ctx->timing.load()) {
    w->timed_fold = true;
    // Montgomery products issued by this launch: every row but each group's first
    std::lock_guard<std::mutex> lk(ctx->tmu);
    ctx->pending_modmuls = count > G ? count - G : 0;
  }
  *lv = Leaves{w->p0.as<uint32_t>(), ps, S2, mc.W, G, (int64_t)mc.W * (S1 ? S1 : S) * ((int64_t)G - (int64_t)count),
               nullptr};
  return DDS_OK;
}

// Reduce n leaves holding prod * 2^Ein to the canonical product (finalize: *value; synchronises the
// stream) or to a canonical partial (S2 limbs of W bits, consecutive, at *part; exponent *Eout).
int reduce_leaves(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const Leaves& lv, bool finalize,
                  bn::Limbs* value, const uint32_t** part, int64_t* Eout) {
  const int S2 = mc.S2;
  if (!use_tree()) {  // round 1: one launch per level in the tail shape, then k_finalize
    if (lv.Sin != S2 || lv.ids) return fail(DDS_E_ARG, "tail levels need leaves in the tail shape");
    HIP_TRY(w->p1.ensure((size_t)S2 * round_up((lv.n + 1) / 2, 64) * 4));
    HIP_TRY(w->x2.ensure((size_t)S2 * round_up((lv.n + 1) / 2, 64) * 4));
    const uint32_t* cur = lv.X;
    uint32_t* bufs[2] = {w->p1.as<uint32_t>(), w->x2.as<uint32_t>()};
    size_t n = lv.n, cs = lv.xs;
    int flip = 0;
    while (n > 1) {
      size_t ng = (n + 1) / 2, ns = round_up(ng, 64);
      HIP_TRY(launch_fold_tail(S2, cur, cs, n, mc.d2, mc.dq, mc.n0, bufs[flip], ns, ng, st));
      cur = bufs[flip];
      flip ^= 1;
      n = ng;
      cs = ns;
    }
    const int64_t E = lv.E - mc.wS2() * ((int64_t)lv.n - 1);
    if (!finalize) {  // partial: S2 limbs at stride cs -> consecutive
      HIP_TRY(w->out.ensure((size_t)S2 * 4));
      HIP_TRY(launch_strided_copy(cur, 0, cs, w->out.as<uint32_t>(), 0, 1, 1, S2, st));
      *part = w->out.as<uint32_t>();
      *Eout = E;
      return DDS_OK;
    }
    uint32_t* hy = nullptr;  // pinned: [0, S2) Y, [S2, 2 S2) result
    HIP_TRY(stage_ptr(w, &hy));
    hy += kStageWord0;
    {
      const std::vector<uint32_t>& y = mc.y_for(E);
      std::copy(y.begin(), y.end(), hy);
    }
    HIP_TRY(w->y.ensure((size_t)S2 * 4));
    HIP_TRY(w->out.ensure((size_t)S2 * 4));
    HIP_TRY(hipMemcpyAsync(w->y.p, hy, (size_t)S2 * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_finalize_tail(S2, cur, cs, mc.d2, w->y.as<uint32_t>(), mc.n0, w->out.as<uint32_t>(), st));
    HIP_TRY(hipMemcpyAsync(hy + S2, w->out.p, (size_t)S2 * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    account_fold(ctx, w);
    *value = mc.value2(hy + S2);
    return DDS_OK;
  }
  Leaves lt = lv;
  if (lv.Sin == S2 && !lv.ids && lv.gs == 1 && lv.n > tree_switch_leaves()) {  // wide levels: tail-shape launches
    HIP_TRY(w->p1.ensure((size_t)S2 * round_up((lv.n + 1) / 2, 64) * 4));
    HIP_TRY(w->x2.ensure((size_t)S2 * round_up((lv.n + 1) / 2, 64) * 4));
    uint32_t* bufs[2] = {w->p1.as<uint32_t>(), w->x2.as<uint32_t>()};
    int flip = 0;
    while (lt.n > tree_switch_leaves()) {
      const size_t ng = (lt.n + 1) / 2, ns = round_up(ng, 64);
      const bool rowmajor = ng <= tree_switch_leaves();  // the last lane-group level: the tree's leaf layout
      HIP_TRY(launch_fold_tail(S2, lt.X, lt.xs, lt.n, mc.d2, mc.dq, mc.n0, bufs[flip], rowmajor ? 1 : ns, ng, st,
                               rowmajor ? (size_t)S2 : 1));
      lt.E -= mc.wS2() * (int64_t)(lt.n - ng);  // n - ng products, R2^-1 each
      lt.X = bufs[flip];
      lt.xs = rowmajor ? 1 : ns;
      lt.gs = rowmajor ? (size_t)S2 : 1;
      lt.n = ng;
      flip ^= 1;
    }
  }
  const int S3 = mc.S3;
  const int64_t E = lt.E - mc.wS3() * ((int64_t)lt.n - 1);  // n-1 tree products, R3^-1 each
  // nodes (2n + 2 rows) + two level buffers (n rows each, multi-launch trees) + flags (2n + 4 words: the
  // final launch may count Y as one more leaf)
  HIP_TRY(w->tree.ensure(((4 * lt.n + 2) * (size_t)S3 + 2 * lt.n + 4) * 4));
  uint32_t* nodes = w->tree.as<uint32_t>();
  uint32_t* tflags = nodes + (4 * lt.n + 2) * (size_t)S3;
  HIP_TRY(w->out.ensure((size_t)std::max(S2, S3) * 4));
  uint32_t* hy = nullptr;  // pinned: [0, S3) Y, [S3, 2 S3) result
  const uint32_t* dY = nullptr;
  if (finalize) {
    HIP_TRY(stage_ptr(w, &hy));
    hy += kStageWord0;
    dY = mc.y3_device(E);  // cached on the device: no copy in the stream
    if (!dY) {
      const std::vector<uint32_t>& y = mc.y3_for(E);
      std::copy(y.begin(), y.end(), hy);
      HIP_TRY(w->y.ensure((size_t)S3 * 4));
      HIP_TRY(hipMemcpyAsync(w->y.p, hy, (size_t)S3 * 4, hipMemcpyHostToDevice, st));
      dY = w->y.as<uint32_t>();
    }
  }
  // finalize: the root block writes the result straight into the pinned stage (no copy launch after it)
  // and then a sequence number the host waits for (the stream's own completion is noticed later by its
  // next user). Short folds spin on it (DDSHE_FOLD_SPIN_ROWS, default 100k rows: ~0.2 ms of device time
  // at 2048-bit keys); a longer fold's caller polls it between 50 us sleeps instead of holding a core of
  // the ForkJoin pool the proxy shares between routes (DDSRestServer.scala:21) for the whole fold (an
  // event made with hipEventBlockingSync measured no different from a spin on ROCm 7: its
  // hipEventSynchronize took the 10M-row fold's 14.5 ms of host CPU). Timing on: hipStreamSynchronize.
  static const size_t spin_rows = [] {
    const char* e = getenv("DDSHE_FOLD_SPIN_ROWS");
    return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)100000;
  }();
  const bool timing = ctx->timing.load();
  const bool spin = finalize && !timing;
  const bool nap = spin && lv.rows > spin_rows;
  volatile uint32_t* dflag = nullptr;
  uint32_t seq = 0;
  if (spin) {
    dflag = reinterpret_cast<volatile uint32_t*>(w->hstage.p) + kStageDoneWord;
    if (++w->done_seq == 0) ++w->done_seq;
    seq = w->done_seq;
    *dflag = 0u;  // whatever the word held, the root's store is the only way it becomes seq (never 0)
  }
  HIP_TRY(launch_tree(S3, lt.X, lt.xs, lt.Sin, lt.Win, lt.n, lt.ids, mc.d3, finalize ? dY : nullptr,
                      nodes, tflags, finalize ? hy + S3 : w->out.as<uint32_t>(), S2, mc.W, st, lt.gs,
                      const_cast<uint32_t*>(dflag), seq));
  if (!finalize) {
    *part = w->out.as<uint32_t>();
    *Eout = E;
    return DDS_OK;
  }
  if (spin) {
    // bounded: past 50 ms of spinning, or 60 s of naps (a loaded GPU, a fault), the stream
    // synchronisation decides
    // synchronisation decides; a napping caller also asks the stream every ~2 ms, so a kernel that
    // failed asynchronously (the word then never changes) is reported at once, not after 60 s
    const auto t0 = std::chrono::steady_clock::now();
    const auto limit = nap ? std::chrono::milliseconds(60000) : std::chrono::milliseconds(50);
    int naps = 0;
    while (*dflag != seq) {
      if (std::chrono::steady_clock::now() - t0 > limit) {
        HIP_TRY(hipStreamSynchronize(st));
        break;
      }
      if (nap) {
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (++naps % 40 == 0 && hipStreamQuery(st) != hipErrorNotReady) {
          HIP_TRY(hipStreamSynchronize(st));  // done (the word is then set too) or an error to report
          break;
        }
      } else {
        __builtin_ia32_pause();
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  } else {
    HIP_TRY(hipStreamSynchronize(st));
  }
  account_fold(ctx, w);
  *value = bn::from_rw(hy + S3, S3, mc.W3);
  return DDS_OK;
}

int fold_partial_device(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint32_t* X, size_t xstride,
                        size_t count, const uint32_t** part, size_t* part_stride, int64_t* E, const uint32_t* d_ids) {
  // DDSHE_PARTIAL_GROUPS (A/B of the strong-split share): cap level 1's groups so the
  // share's partials go straight to the tree (<= 4096) instead of through the tail launches
  static const size_t cap = [] {
    const char* e = getenv("DDSHE_PARTIAL_GROUPS");
    return e ? (size_t)atoll(e) : (size_t)0;
  }();
  Leaves lv;
  int rc = fold_level1(ctx, w, st, mc, X, xstride, count, d_ids, &lv, cap);
  if (rc) return rc;
  *part_stride = 1;
  return reduce_leaves(ctx, w, st, mc, lv, false, nullptr, part, E);
}

int fold_value_device(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint32_t* X, size_t xstride,
                      size_t count, const uint32_t* d_ids, bn::Limbs* value) {
  Leaves lv;
  int rc = fold_level1(ctx, w, st, mc, X, xstride, count, d_ids, &lv);
  if (rc) return rc;
  lv.rows = count;
  return reduce_leaves(ctx, w, st, mc, lv, true, value, nullptr, nullptr);
}

// after the stream has synchronised: account the timed first-level fold launch, if any
void account_fold(dds_ctx* ctx, Worker* w) {
  if (!w->timed_fold) return;
  w->timed_fold = false;
  float ms = 0;
  if (hipEventElapsedTime(&ms, w->ev[0], w->ev[1]) == hipSuccess) {
    std::lock_guard<std::mutex> lk(ctx->tmu);
    ctx->fold_ms += ms;
    ctx->fold_launches += 1;
    ctx->fold_modmuls += ctx->pending_modmuls;
  }
}

int emit_be(const bn::Limbs& v, size_t width, uint8_t* out, size_t out_cap, size_t* out_len) {
  if (out_len) *out_len = width;
  if (!out || out_cap < width) return fail(DDS_E_BUFSIZE, "output buffer too small");
  if (!bn::to_be(v, out, width)) return fail(DDS_E_RANGE, "result does not fit");
  return DDS_OK;
}



int ingest(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint8_t* ops, size_t width, size_t count,
           DevBuf& raw, uint32_t* X, size_t stride, std::vector<size_t>* reduced) {
  (void)ctx;
  if (count == 0) return DDS_OK;
  HIP_TRY(w->flags.ensure(16));
  HIP_TRY(hipMemsetAsync(w->flags.p, 0, 4, st));
  uint8_t* rowflags = nullptr;
  if (reduced) {
    HIP_TRY(w->rflags.ensure(count));
    rowflags = w->rflags.as<uint8_t>();
  }
  const uint32_t* n2x = mc.d + (size_t)kConstN2x * mc.S;
  const size_t crows = std::max<size_t>(1, kIngestChunkBytes / width);
  if (count <= crows) {
    HIP_TRY(raw.ensure(count * width));
    HIP_TRY(hipMemcpyAsync(raw.p, ops, count * width, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_ingest_be(raw.as<uint8_t>(), width, count, mc.S, mc.W, n2x, X, stride, w->flags.as<uint32_t>(), st,
                             rowflags));
  } else {
    // chunked: the pool fills pinned slot s while the DMA + k_ingest_be of slot s^1 run
    bool used[2] = {false, false};
    HIP_TRY(raw.ensure(2 * crows * width));
    for (size_t b = 0, slot = 0; b < count; b += crows, slot ^= 1) {
      const size_t nrows = std::min(crows, count - b), bytes = nrows * width;
      if (used[slot]) HIP_TRY(hipEventSynchronize(w->ev_dec[slot]));
      HIP_TRY(w->hch[slot].ensure(crows * width));
      CopyPool::get().copy(w->hch[slot].p, ops + b * width, bytes);
      uint8_t* d = raw.as<uint8_t>() + slot * crows * width;
      HIP_TRY(hipMemcpyAsync(d, w->hch[slot].p, bytes, hipMemcpyHostToDevice, st));
      HIP_TRY(hipEventRecord(w->ev_dec[slot], st));
      HIP_TRY(launch_ingest_be(d, width, nrows, mc.S, mc.W, n2x, X + b, stride, w->flags.as<uint32_t>(), st,
                               rowflags ? rowflags + b : nullptr));
      used[slot] = true;
    }
  }
  uint32_t flags = 0;
  HIP_TRY(read_sync(w, st, w->flags.p, &flags, 4));
  if (flags & 2u) return fail(DDS_E_RANGE, "operand wider than the modulus limb width");
  if (flags & 1u) {
    HIP_TRY(launch_reduce_rows(mc.S, X, stride, count, mc.d, mc.n0, st));
    if (reduced) {
      std::vector<uint8_t> f(count);
      HIP_TRY(hipMemcpyAsync(f.data(), rowflags, count, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      for (size_t i = 0; i < count; ++i)
        if (f[i]) reduced->push_back(i);
    }
  }
  return DDS_OK;
}



// the worker's copy stream (H2D copies overlapping the compute stream) and its two events
hipError_t copy_stream(Worker* w) {
  if (w->cstream) return hipSuccess;
  hipError_t e = hipStreamCreateWithFlags(&w->cstream, hipStreamNonBlocking);
  for (auto& ev : w->ev_copy)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  return e;
}

// Long folds of host rows (dds_paillier_sum / dds_rsa_product / dds_modmul_fold over millions of rows):
// the rows are folded in pieces as they arrive, so the fold of piece p runs while piece p + 1 crosses
// PCIe instead of after the last chunk. Copy stream: per 64 MiB chunk, the DMA out of the pinned slot the
// host pool filled, then k_ingest_be; compute stream, after a piece's last chunk: k_reduce_rows gated on
// the device by the ingest flags (rows >= 2N), the piece's fold to a partial (fold_partial_device), its
// copy to column p of the partials; then one tree over the pieces' partials. The flags are read after
// the result (a row wider than the limb width fails the call, as ingest() does).
// DDSHE_INGEST_PIECES: pieces (default 8; 1: ingest everything, then fold); from DDSHE_INGEST_PIPE_ROWS
// rows (default 2^21). 10M 512-byte rows, one box: 122.9 ms in one piece, 104.5 in 4, 97.9 in 8.
size_t ingest_pieces(size_t count) {
  static const size_t pieces = [] {
    const char* e = getenv("DDSHE_INGEST_PIECES");
    return e ? (size_t)atoll(e) : (size_t)8;
  }();
  static const size_t min_rows = [] {
    const char* e = getenv("DDSHE_INGEST_PIPE_ROWS");
    return e ? (size_t)atoll(e) : ((size_t)1 << 21);
  }();
  return count >= min_rows ? pieces : 1;
}

int fold_be_pipelined(dds_ctx* ctx, Worker* w, hipStream_t st, ModConsts& mc, const uint8_t* ops, size_t width,
                      size_t count, size_t pieces, bn::Limbs* value) {
  const size_t crows = std::max<size_t>(1, kIngestChunkBytes / width);
  const size_t prow = round_up((count + pieces - 1) / pieces, crows);  // rows per piece: whole chunks
  const size_t np = (count + prow - 1) / prow;
  const size_t stride = round_up(count, 64), S2 = (size_t)mc.S2, pst = round_up(np, 64);
  HIP_TRY(w->x.ensure((size_t)mc.S * stride * 4));
  HIP_TRY(w->in.ensure(2 * crows * width));
  HIP_TRY(w->flags.ensure(16));
  HIP_TRY(w->gather.ensure(S2 * pst * 4));
  HIP_TRY(copy_stream(w));
  uint32_t* X = w->x.as<uint32_t>();
  uint32_t* flags = w->flags.as<uint32_t>();
  uint32_t* parts = w->gather.as<uint32_t>();
  const uint32_t* n2x = mc.d + (size_t)kConstN2x * mc.S;
  hipStream_t cs = w->cstream;
  HIP_TRY(hipMemsetAsync(flags, 0, 4, st));
  HIP_TRY(hipEventRecord(w->ev_copy[1], st));  // the copy stream starts after the clear (and st's earlier work)
  HIP_TRY(hipStreamWaitEvent(cs, w->ev_copy[1], 0));
  int64_t E = 0;
  bool used[2] = {false, false};
  size_t slot = 0;
  for (size_t p = 0; p < np; ++p) {
    const size_t p0 = p * prow, pn = std::min(prow, count - p0);
    for (size_t b = p0; b < p0 + pn; b += crows, slot ^= 1) {
      const size_t nrows = std::min(crows, p0 + pn - b), bytes = nrows * width;
      if (used[slot]) HIP_TRY(hipEventSynchronize(w->ev_dec[slot]));  // the DMA out of this host slot is done
      HIP_TRY(w->hch[slot].ensure(crows * width));
      CopyPool::get().copy(w->hch[slot].p, ops + b * width, bytes);
      uint8_t* d = w->in.as<uint8_t>() + slot * crows * width;  // reused two chunks later, after this ingest (cs)
      HIP_TRY(hipMemcpyAsync(d, w->hch[slot].p, bytes, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipEventRecord(w->ev_dec[slot], cs));
      HIP_TRY(launch_ingest_be(d, width, nrows, mc.S, mc.W, n2x, X + b, stride, flags, cs));
      used[slot] = true;
    }
    HIP_TRY(hipEventRecord(w->ev_copy[0], cs));
    HIP_TRY(hipStreamWaitEvent(st, w->ev_copy[0], 0));
    HIP_TRY(launch_reduce_rows(mc.S, X + p0, stride, pn, mc.d, mc.n0, st, flags));
    const uint32_t* part = nullptr;
    size_t ps = 0;
    int64_t Ep = 0;
    int rc = fold_partial_device(ctx, w, st, mc, X + p0, stride, pn, &part, &ps, &Ep, nullptr);
    if (rc) return rc;
    HIP_TRY(launch_strided_copy(part, 0, 1, parts + p, 0, pst, 1, S2, st));  // S2 limbs -> column p
    E += Ep;
  }
  Leaves lv{parts, pst, (int)S2, mc.W, np, E, nullptr};
  lv.rows = count;
  int rc = reduce_leaves(ctx, w, st, mc, lv, true, value, nullptr, nullptr);
  if (rc) return rc;
  uint32_t fl = 0;
  HIP_TRY(read_sync(w, st, flags, &fl, 4));
  if (fl & 2u) return fail(DDS_E_RANGE, "operand wider than the modulus limb width");
  return DDS_OK;
}

int dec_table(ModConsts& mc) {
  std::lock_guard<std::mutex> lk(mc.decmu);
  if (mc.dtab) return DDS_OK;
  const size_t cap = (size_t)mc.W * mc.S;
  std::vector<bn::Limbs> pw;
  bn::Limbs P{1};
  while (bn::bit_length(P) <= cap) {
    pw.push_back(P);
    P = bn::mul_small_add(P, 100000000u, 0);
  }
  const int jfit = (int)pw.size(), jpad = (jfit + 3) & ~3, L = mc.S / mc.TPI;
  // 64-bit lazy accumulation: jfit * (10^8 - 1) * (2^W - 1) < 2^64
  if ((double)jfit * 1e8 * (double)(1u << mc.W) >= 18446744073709551616.0)
    return fail(DDS_E_UNSUPPORTED, "decimal table bound");
  std::vector<uint32_t> tab((size_t)mc.S * jpad + ((L + 3) & ~3), 0);
  for (int j = 0; j < jfit; ++j) {
    std::vector<uint32_t> rw = mc.rw(pw[j]);
    for (int l = 0; l < mc.S; ++l) tab[(size_t)l * jpad + j] = rw[l];
  }
  for (int i = 0; i < L; ++i) {
    const size_t lbits = (size_t)mc.W * mc.TPI * i;
    int j = 0;
    while (j < jfit && bn::bit_length(pw[j]) <= lbits) ++j;
    tab[(size_t)mc.S * jpad + i] = (uint32_t)(j & ~3);
  }
  uint32_t* d = nullptr;
  HIP_TRY(hipMalloc(&d, tab.size() * 4));
  if (hipMemcpy(d, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return fail(DDS_E_HIP, "decimal table upload");
  }
  mc.dtab = d;
  mc.jfit = jfit;
  mc.jpad = jpad;
  return DDS_OK;
}

// Parse rows [0, count) into X (stride) on the GPU: chunks are packed into pinned buffers
// (host, overlapping the previous chunk's copy + parse), copied, parsed by k_dec_parse, then
// negative / >= 2N rows are fixed by k_dec_fix. *orflags = OR of the row status bits
// (kDecFormat / kDecWide rows hold zeros); w->rflags keeps the per-row bytes. Rows longer than a
// chunk are parsed as "0" and listed in *long_rows for the caller.
int ingest_dec(Worker* w, hipStream_t st, ModConsts& mc, const DecRows& src, size_t count, uint32_t* X,
               size_t stride, uint32_t* orflags, std::vector<size_t>* long_rows) {
  *orflags = 0;
  if (count == 0) return DDS_OK;
  int rc = dec_table(mc);
  if (rc) return rc;
  HIP_TRY(w->rflags.ensure(count));
  HIP_TRY(w->flags.ensure(16));
  HIP_TRY(hipMemsetAsync(w->flags.p, 0, 4, st));
  HIP_TRY(copy_stream(w));
  hipStream_t cs = w->cstream;
  // rows per chunk: a request of fewer than 2 x 2^18 rows still splits into two chunks (>= 4096 rows
  // each), so the second chunk's host and H2D copies overlap the first one's parse (config 1: 10k
  // rows, 6.2 MB of chars). Not more: a small chunk's parse is latency-bound (~46 us whatever its
  // size), and four chunks measured slower (0.43 -> 0.49 ms) than one.
  const size_t crows = std::min(kDecChunkRows, std::max<size_t>(4096, (count + 1) / 2));
  bool used[2] = {false, false};
  int slot = 0;
  std::unique_ptr<uint32_t[]> lens;  // String[] rows: lens[i] valid for i < lens_hi (uninitialised beyond)
  size_t lens_hi = 0;
  for (size_t b = 0; b < count;) {
    if (used[slot]) HIP_TRY(hipEventSynchronize(w->ev_copy[slot]));  // the H2D out of this host slot is done
    HIP_TRY(w->hch[slot].ensure(kDecChunkBytes + 64));
    HIP_TRY(w->hoff[slot].ensure((kDecChunkRows + 1) * 8));
    char* dst = (char*)w->hch[slot].p + 16;
    uint64_t* o = (uint64_t*)w->hoff[slot].p;
    size_t pos = 0, e = b;
    o[0] = 0;
    if (!src.strs) {  // Arrow-style rows: one bulk copy of the chunk's chars, offsets rebased
      const uint64_t base = src.offs[b];
      size_t lo = b, hi = std::min(count, b + crows);  // largest e in [b, hi] with chars <= chunk
      while (lo < hi) {
        const size_t mid = lo + (hi - lo + 1) / 2;
        if (src.offs[mid] - base <= kDecChunkBytes - 64) lo = mid;
        else hi = mid - 1;
      }
      if (lo > b) {
        e = lo;
        pos = (size_t)(src.offs[e] - base);
        CopyPool::get().copy(dst, src.chars + base, pos);
        for (size_t i = b; i <= e; ++i) o[i - b] = src.offs[i] - base;
      }
    }
    if (src.strs && std::min(count - b, crows) >= 1024) {
      // NUL-terminated rows (JNA String[]): lengths and copies spread over the host pool; the
      // chunk cut and the offsets are one sequential pass over the lengths. Lengths are measured
      // in blocks as the cut reaches them and kept for the next chunk (a chunk ends on its byte
      // budget long before crows rows of ciphertext text: measuring [b, b + crows) per chunk read
      // every row ~5 times for 4096-bit rows)
      const size_t hi = std::min(count, b + crows);
      if (!lens) lens.reset(new uint32_t[count]);
      while (e < hi) {
        if (e == lens_hi) {
          const size_t lb = lens_hi, le = std::min(count, lb + kDecLenBlock);
          CopyPool::get().parallel_for(le - lb, 256, [&](size_t x, size_t y) {
            for (size_t i = lb + x; i < lb + y; ++i)  // past the chunk budget: a long row either way
              lens[i] = (uint32_t)std::min<size_t>(strlen(src.strs[i]), kDecChunkBytes);
          });
          lens_hi = le;
        }
        const size_t n = lens[e] > kDecChunkBytes - 64 ? 1 : lens[e];
        if (pos + n > kDecChunkBytes) break;
        if (n != lens[e]) long_rows->push_back(e);
        pos += n;
        o[++e - b] = pos;
      }
      CopyPool::get().parallel_for(e - b, 256, [&](size_t x, size_t y) {
        for (size_t i = x; i < y; ++i)
          memcpy(dst + o[i], o[i + 1] - o[i] == lens[b + i] ? src.strs[b + i] : "0", o[i + 1] - o[i]);
      });
    }
    while (e < count && e - b < crows) {
      size_t n = src.len(e);
      const bool longrow = n > kDecChunkBytes - 64;
      if (longrow) n = 1;
      if (pos + n > kDecChunkBytes) break;
      if (longrow) long_rows->push_back(e);
      memcpy(dst + pos, longrow ? "0" : src.row(e), n);
      pos += n;
      o[++e - b] = pos;
    }
    const size_t nrows = e - b, bytes = (16 + pos + 16 + 3) & ~(size_t)3;
    memset(dst + pos, 0, bytes - 16 - pos);
    // the device slot is free once the parse of its previous chunk has run (a growing buffer is
    // reallocated only after that parse, host-side)
    if (used[slot] && (w->dch[slot].cap < bytes || w->doff[slot].cap < (nrows + 1) * 8))
      HIP_TRY(hipEventSynchronize(w->ev_dec[slot]));
    HIP_TRY(w->dch[slot].ensure(bytes));
    HIP_TRY(w->doff[slot].ensure((nrows + 1) * 8));
    if (used[slot]) HIP_TRY(hipStreamWaitEvent(cs, w->ev_dec[slot], 0));
    HIP_TRY(hipMemcpyAsync(w->dch[slot].p, w->hch[slot].p, bytes, hipMemcpyHostToDevice, cs));
    HIP_TRY(hipMemcpyAsync(w->doff[slot].p, o, (nrows + 1) * 8, hipMemcpyHostToDevice, cs));
    HIP_TRY(hipEventRecord(w->ev_copy[slot], cs));
    HIP_TRY(hipStreamWaitEvent(st, w->ev_copy[slot], 0));
    HIP_TRY(launch_dec_parse(mc.S, w->dch[slot].as<uint32_t>(), w->doff[slot].as<uint64_t>(), 0, nrows, mc.dtab,
                             mc.jfit, mc.jpad, mc.d, X + b, stride, w->rflags.as<uint8_t>() + b,
                             w->flags.as<uint32_t>(), st));
    HIP_TRY(hipEventRecord(w->ev_dec[slot], st));
    used[slot] = true;
    slot ^= 1;
    b = e;
  }
  uint32_t fl = 0;
  HIP_TRY(read_sync(w, st, w->flags.p, &fl, 4));
  if (fl & (kDecNeg | kDecReduce))
    HIP_TRY(launch_dec_fix(mc.S, X, stride, count, w->rflags.as<uint8_t>(), mc.d, mc.n0, st));
  *orflags = fl;
  return DDS_OK;
}

// indices of rows whose status has any bit of `mask` (after ingest_dec)
int dec_rows_with(Worker* w, hipStream_t st, size_t count, uint32_t mask, std::vector<size_t>* rows) {
  std::vector<uint8_t> f(count);
  HIP_TRY(hipMemcpyAsync(f.data(), w->rflags.p, count, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  for (size_t i = 0; i < count; ++i)
    if (f[i] & mask) rows->push_back(i);
  return DDS_OK;
}

int modmul_fold_be(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, size_t min_bits, const uint8_t* ops,
                   size_t width, size_t count, uint8_t* out, size_t out_cap, size_t* out_len) {
  std::shared_ptr<ModConsts> mc;
  int rc = get_mod(ctx, mod_be, mod_bytes, &mc, min_bits);
  if (rc) return rc;
  if ((rc = check_rows(*mc, count))) return rc;
  WorkerLease wl(ctx);
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  bn::Limbs v;
  const size_t pieces = ingest_pieces(count);
  if (pieces > 1) {
    if ((rc = fold_be_pipelined(ctx, w, wl.st, *mc, ops, width, count, pieces, &v))) return rc;
    return emit_be(v, mod_bytes, out, out_cap, out_len);
  }
  const size_t stride = round_up(count, 64);
  HIP_TRY(w->x.ensure((size_t)mc->S * stride * 4));
  if ((rc = ingest(ctx, w, wl.st, *mc, ops, width, count, w->in, w->x.as<uint32_t>(), stride))) return rc;
  if ((rc = fold_value_device(ctx, w, wl.st, *mc, w->x.as<uint32_t>(), stride, count, nullptr, &v))) return rc;
  return emit_be(v, mod_bytes, out, out_cap, out_len);
}

// Product of `count` rows of radix-2^16 limbs (h: count x len u32 words, row-major) on the GPU product
// tree (k_bigmul_*: one level multiplies row pairs, carry passes until every limb is < 2^16).
// cap16 != 0: each level keeps only its low cap16 limbs, i.e. the product mod 2^(16 cap16).
int product_tree(dds_ctx* ctx, const std::vector<uint32_t>& h, size_t count, size_t len, size_t cap16, bn::Limbs* out) {
  WorkerLease wl(ctx);
  int rc;
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  HIP_TRY(w->x.ensure(h.size() * 4));
  HIP_TRY(hipMemcpyAsync(w->x.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(w->flags.ensure(16));
  uint32_t* cur = w->x.as<uint32_t>();
  size_t n = count;
  while (n > 1) {  // one tree level: n rows of len limbs -> ceil(n/2) rows of outlen limbs
    const size_t pairs = (n + 1) / 2, outlen = cap16 ? std::min(2 * len, cap16) : 2 * len;
    HIP_TRY(w->misc.ensure(pairs * outlen * 8));
    HIP_TRY(w->x2.ensure(pairs * outlen * 4));
    HIP_TRY(w->p0.ensure(pairs * outlen * 4));
    HIP_TRY(launch_bigmul_level(cur, n, len, w->misc.as<uint64_t>(), w->x2.as<uint32_t>(), wl.st, cap16));
    uint32_t* v = w->x2.as<uint32_t>();
    uint32_t* u = w->p0.as<uint32_t>();
    for (;;) {  // carry passes until every limb is < 2^16 (ripples are rare and short)
      HIP_TRY(hipMemsetAsync(w->flags.p, 0, 4, wl.st));
      HIP_TRY(launch_bigmul_carry(v, pairs, outlen, u, w->flags.as<uint32_t>(), wl.st));
      uint32_t flag = 0;
      HIP_TRY(read_sync(w, wl.st, w->flags.p, &flag, 4));
      std::swap(u, v);
      if (!flag) break;
    }
    // v holds the normalised level; move it to the level buffer
    HIP_TRY(w->x.ensure(pairs * outlen * 4));
    HIP_TRY(hipMemcpyAsync(w->x.p, v, pairs * outlen * 4, hipMemcpyDeviceToDevice, wl.st));
    cur = w->x.as<uint32_t>();
    n = pairs;
    len = outlen;
  }
  std::vector<uint32_t> res(len);
  HIP_TRY(hipMemcpyAsync(res.data(), cur, len * 4, hipMemcpyDeviceToHost, wl.st));
  HIP_TRY(hipStreamSynchronize(wl.st));
  bn::Limbs v((len + 1) / 2, 0);
  for (size_t i = 0; i < len; ++i) v[i / 2] |= res[i] << (16 * (i % 2));
  bn::trim(v);
  *out = std::move(v);
  return DDS_OK;
}

// x mod 2^t
bn::Limbs low_bits(const bn::Limbs& x, size_t t) {
  bn::Limbs r(x.begin(), x.begin() + std::min(x.size(), (t + 31) / 32));
  if (t % 32 && r.size() == (t + 31) / 32) r.back() &= (1u << (t % 32)) - 1u;
  bn::trim(r);
  return r;
}

// Product of magnitudes xs[i] (signs negs[i]) mod an EVEN modulus M (or M == 1), count >= 2. A
// Montgomery fold needs an odd modulus, so M = 2^t * Q (Q odd) is split: prod mod Q by the
// Montgomery fold (in the shape of M's width, so operands as wide as M's capacity fit), prod mod 2^t
// by the truncated product tree, both on the GPU; then CRT and the sign (-1)^#neg on the host —
// BigInteger.mod semantics (DDSRestServer.scala:422-423, 515-518 send any modulus).
int fold_even_modulus(dds_ctx* ctx, const bn::Limbs& M, const std::vector<bn::Limbs>& xs, const std::vector<bool>& negs,
                      bn::Limbs* out) {
  const size_t count = xs.size();
  size_t t = 0;
  while (!((M[t / 32] >> (t % 32)) & 1u)) ++t;
  bn::Limbs Q = M;
  for (size_t i = 0; i < t; ++i) (void)bn::divmod_small(Q, 2);
  bn::trim(Q);
  const size_t mbits = bn::bit_length(M);
  // rows wider than M's limb capacity: pre-reduce mod M (consistent mod Q and mod 2^t)
  const Shape sh = pick_shape(mbits);
  if (!sh.S) return fail(DDS_E_UNSUPPORTED, "modulus too large");
  const size_t capbits = (size_t)sh.W * sh.S - 2;
  std::vector<bn::Limbs> ys(xs);
  size_t width = 1;
  for (auto& y : ys) {
    if (bn::bit_length(y) > capbits) y = bn::mod(y, M);
    width = std::max(width, bn::byte_length(y));
  }
  bn::Limbs rq;  // prod mod Q
  if (bn::bit_length(Q) >= 2) {
    std::vector<uint8_t> rows(count * width), qbe(bn::byte_length(Q));
    for (size_t i = 0; i < count; ++i) bn::to_be(ys[i], rows.data() + i * width, width);
    bn::to_be(Q, qbe.data(), qbe.size());
    std::vector<uint8_t> r(qbe.size());
    size_t rl = 0;
    int rc = modmul_fold_be(ctx, qbe.data(), qbe.size(), mbits, rows.data(), width, count, r.data(), r.size(), &rl);
    if (rc) return rc;
    rq = bn::from_be(r.data(), rl);
  }
  bn::Limbs r2;  // prod mod 2^t
  if (t > 0) {
    const size_t cap16 = (t + 15) / 16;
    std::vector<uint32_t> h(count * cap16, 0);
    for (size_t i = 0; i < count; ++i) {
      const bn::Limbs lo = low_bits(ys[i], t);
      for (size_t k = 0; k < lo.size() && 2 * k < cap16; ++k) {
        h[i * cap16 + 2 * k] = lo[k] & 0xFFFFu;
        if (2 * k + 1 < cap16) h[i * cap16 + 2 * k + 1] = lo[k] >> 16;
      }
    }
    int rc = product_tree(ctx, h, count, cap16, cap16, &r2);
    if (rc) return rc;
    r2 = low_bits(r2, t);
  }
  // CRT: r = rq + Q * ((r2 - rq) * Q^-1 mod 2^t)
  bn::Limbs r = rq;
  if (t > 0) {
    const bn::Limbs two_t = bn::pow2(t);
    bn::Limbs qinv{1};  // Newton: qinv <- qinv (2 - Q qinv) mod 2^t, doubling the correct bits
    for (size_t bits = 1; bits < t; bits *= 2) {
      const bn::Limbs qq = low_bits(bn::mul(Q, qinv), t);
      qinv = low_bits(bn::mul(qinv, bn::sub(bn::add(two_t, bn::Limbs{2}), qq)), t);
    }
    const bn::Limbs rqt = low_bits(rq, t);
    const bn::Limbs d = bn::cmp(r2, rqt) >= 0 ? bn::sub(r2, rqt) : bn::sub(bn::add(r2, two_t), rqt);
    r = bn::add(rq, bn::mul(Q, low_bits(bn::mul(d, qinv), t)));
  }
  size_t nneg = 0;
  for (bool b : negs) nneg += b;
  bn::trim(r);
  if ((nneg & 1) && !r.empty()) r = bn::sub(M, r);
  *out = r;
  return DDS_OK;
}

// Combine partials (dds_col_fold_partial layout: S2 limbs + exponent, back to back) given in host
// memory (h_parts) or device memory of ctx's GPU (d_parts): validate them, one more tree, finalize.
int combine_partials(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint32_t* h_parts,
                     const uint32_t* d_parts, const uint64_t* rows, size_t nparts, uint8_t* out, size_t out_cap,
                     size_t* out_len) {
  std::shared_ptr<ModConsts> mc;
  int rc = get_mod(ctx, mod_be, mod_bytes, &mc);
  if (rc) return rc;
  uint64_t k = 0;
  for (size_t i = 0; i < nparts; ++i) k += rows[i];
  if (k == 0) return fail(DDS_E_EMPTY, "no operand");
  const size_t S2 = (size_t)mc->S2, pw = partial_words_for(*mc);
  WorkerLease wl(ctx);
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  std::vector<uint32_t> hp;
  if (d_parts) {  // limbs + exponents are a few hundred bytes per partial: read them back to check
    hp.resize(nparts * pw);
    HIP_TRY(hipMemcpyAsync(hp.data(), d_parts, hp.size() * 4, hipMemcpyDeviceToHost, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    h_parts = hp.data();
  }
  // the tree kernels' lazy-accumulation bound needs fully normalised limbs and a value below the
  // bound the fold leaves its partials under (2N~ when a QP shape is used, else 2N): reject the rest
  const bn::Limbs bound = bn::add(mc->qbound, mc->qbound);
  int64_t E = 0;  // sum of the partials' exponents (reduce_leaves accounts for its own products)
  for (size_t i = 0; i < nparts; ++i) {
    const uint32_t* pl = h_parts + i * pw;
    for (size_t l = 0; l < S2; ++l)
      if (pl[l] >> mc->W) return fail(DDS_E_RANGE, "partial " + std::to_string(i) + ": limb not normalised");
    if (bn::cmp(mc->value2(pl), bound) >= 0) return fail(DDS_E_RANGE, "partial " + std::to_string(i) + " out of range");
    E += (int64_t)((uint64_t)pl[S2] | ((uint64_t)pl[S2 + 1] << 32));
  }
  const size_t stride = round_up(nparts, 64);
  HIP_TRY(w->x.ensure(S2 * stride * 4));
  std::vector<uint32_t> h;
  if (d_parts) {
    HIP_TRY(launch_strided_copy(d_parts, pw, 1, w->x.as<uint32_t>(), 1, stride, nparts, S2, wl.st));
  } else {
    h.assign(S2 * stride, 0);
    for (size_t i = 0; i < nparts; ++i)
      for (size_t l = 0; l < S2; ++l) h[l * stride + i] = h_parts[i * pw + l];
    HIP_TRY(hipMemcpyAsync(w->x.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, wl.st));
  }
  bn::Limbs v;
  const Leaves lv{w->x.as<uint32_t>(), stride, (int)S2, mc->W, nparts, E, nullptr};
  if ((rc = reduce_leaves(ctx, w, wl.st, *mc, lv, true, &v, nullptr, nullptr))) return rc;  // syncs: h may go
  return emit_be(v, mod_bytes, out, out_cap, out_len);
}

// SumAll/MultAll over rows of a resident column (DDSRestServer.scala:412-430, 506-524): the live rows
// among row_ids[0..n) (nullptr: rows [first, first+n)). No live row -> DDS_E_EMPTY (404); one -> the
// operand as appended, unreduced (:416-417); else the canonical product mod N. Caller holds col->mu.
int col_fold_value(dds_col* col, const uint64_t* row_ids, size_t first, size_t n, bn::Limbs* v, bool* neg) {
  *neg = false;
  ModConsts& mc = *col->mc;
  const size_t rows = col->count;
  if (row_ids) {
    for (size_t i = 0; i < n; ++i)
      if (row_ids[i] >= rows) return fail(DDS_E_ARG, "row id " + std::to_string(row_ids[i]) + " out of range");
  } else if (first + n > rows) {
    return fail(DDS_E_ARG, "rows out of range");
  }
  std::vector<uint64_t> kept;  // removed sets never fold (RemoveSet, DDSRestServer.scala:207-218)
  if (row_ids && col->ndead) {
    kept = col_live_ids(col, row_ids, n);
    row_ids = kept.data();
    n = kept.size();
  }
  WorkerLease wl(col->ctx);
  int rc;
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  const uint32_t* d_ids = nullptr;
  const uint32_t* X = col->d;
  size_t r1 = first;  // the row of a one-operand fold
  if (!row_ids) {
    size_t nl = n;
    if ((rc = col_live_range(col, w, wl.st, first, n, &d_ids, &nl))) return rc;
    if (d_ids && nl == 1) {
      uint32_t off = 0;
      HIP_TRY(read_sync(w, wl.st, d_ids, &off, 4));
      r1 = first + off;
    }
    n = nl;
    X = col->d + first;
  } else if (n) {
    r1 = (size_t)row_ids[0];
  }
  if (n == 0) return fail(DDS_E_EMPTY, "no operand");
  if (n == 1) {
    auto it = col->orig.find(r1);
    if (it != col->orig.end()) {
      *v = it->second.mag;
      *neg = it->second.neg;
      return DDS_OK;
    }
    std::vector<uint32_t> h((size_t)mc.S);  // stored verbatim (< 2N): the raw limbs
    HIP_TRY(hipMemcpy2DAsync(h.data(), 4, col->d + r1, col->stride * 4, 4, (size_t)mc.S, hipMemcpyDeviceToHost, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    *v = mc.value(h.data());
    return DDS_OK;
  }
  std::vector<uint32_t> ids32;
  if (row_ids) {
    ids32.assign(row_ids, row_ids + n);  // < count <= max_stride < 2^32
    HIP_TRY(w->ids.ensure(n * 4));
    HIP_TRY(hipMemcpyAsync(w->ids.p, ids32.data(), n * 4, hipMemcpyHostToDevice, wl.st));
    d_ids = w->ids.as<uint32_t>();
  }
  // synchronises: ids32 may go afterwards
  return fold_value_device(col->ctx, w, wl.st, mc, X, col->stride, n, d_ids, v);
}

int col_live_range(dds_col* col, Worker* w, hipStream_t st, size_t first, size_t count, const uint32_t** d_ids,
                   size_t* n) {
  *d_ids = nullptr;
  *n = count;
  if (col->ndead == 0 || count == 0) return DDS_OK;
  HIP_TRY(w->misc.ensure(ope_scratch_bytes(count)));
  HIP_TRY(w->ids.ensure(count * 4));
  HIP_TRY(w->flags.ensure(16));
  HIP_TRY(launch_byte_compact(col->dlive + first, count, 1u, w->misc.p, w->flags.as<uint64_t>(), w->ids.as<uint32_t>(),
                              st));
  uint64_t total = 0;
  HIP_TRY(read_sync(w, st, w->flags.p, &total, 8));
  *n = (size_t)total;
  *d_ids = w->ids.as<uint32_t>();
  return DDS_OK;
}

std::vector<uint64_t> col_live_ids(const dds_col* col, const uint64_t* ids, size_t n) {
  std::vector<uint64_t> out;
  out.reserve(n);
  for (size_t i = 0; i < n; ++i)
    if (col->live((size_t)ids[i])) out.push_back(ids[i]);
  return out;
}

// Overwrite rows ids[0..n) with new operands: big-endian (ops, width) or decimal (chars, offsets). The
// new values are ingested into scratch exactly as an append would (validation, >= 2N rows reduced and
// their originals kept for a one-operand fold), then scattered into the column. A repeated id takes
// its last value.
int col_write_prepare(dds_col* col, const uint64_t* ids, size_t n, const uint8_t* ops, size_t width,
                      const char* chars, const uint64_t* offsets, RowWrite* plan) {
  for (size_t i = 0; i < n; ++i)
    if (ids[i] >= col->count) return fail(DDS_E_ARG, "row id " + std::to_string(ids[i]) + " out of range");
  if (n == 0) return DDS_OK;
  // last occurrence of each id wins (a scatter of duplicates would race)
  std::vector<size_t> pick;
  {
    std::map<uint64_t, size_t> last;
    for (size_t i = 0; i < n; ++i) last[ids[i]] = i;
    if (last.size() == n) {
      pick.resize(n);
      for (size_t i = 0; i < n; ++i) pick[i] = i;
    } else {
      for (auto& kv : last) pick.push_back(kv.second);
    }
  }
  const size_t m = pick.size();
  ModConsts& mc = *col->mc;
  plan->wl.reset(new WorkerLease(col->ctx));
  int rc;
  if ((rc = plan->wl->acquire())) return rc;
  Worker* w = plan->wl->w;
  hipStream_t st = plan->wl->st;
  const size_t ss = round_up(m, 64);
  plan->ss = ss;
  HIP_TRY(w->x2.ensure((size_t)mc.S * ss * 4));
  std::vector<size_t> changed;
  if (ops) {
    std::vector<uint8_t> packed;
    const uint8_t* src = ops;
    if (m != n) {
      packed.resize(m * width);
      for (size_t j = 0; j < m; ++j) memcpy(packed.data() + j * width, ops + pick[j] * width, width);
      src = packed.data();
    }
    if ((rc = ingest(col->ctx, w, st, mc, src, width, m, w->in, w->x2.as<uint32_t>(), ss, &changed))) return rc;
    for (size_t j : changed) plan->origs.emplace_back(j, dds_col::Orig{bn::from_be(src + j * width, width), false});
  } else {
    std::vector<char> ch;
    std::vector<uint64_t> of(1, 0);
    for (size_t j = 0; j < m; ++j) {
      const size_t i = pick[j];
      if (offsets[i + 1] < offsets[i]) return fail(DDS_E_ARG, "offsets must be non-decreasing");
      ch.insert(ch.end(), chars + offsets[i], chars + offsets[i + 1]);
      of.push_back(ch.size());
    }
    ch.push_back('\0');
    DecRows rows;
    rows.chars = ch.data();
    rows.offs = of.data();
    uint32_t fl = 0;
    std::vector<size_t> longr;
    if ((rc = ingest_dec(w, st, mc, rows, m, w->x2.as<uint32_t>(), ss, &fl, &longr))) return rc;
    if (fl & (kDecFormat | kDecWide)) {
      std::vector<size_t> bad;
      if ((rc = dec_rows_with(w, st, m, kDecFormat, &bad))) return rc;
      if (!bad.empty()) return fail(DDS_E_FORMAT, "row " + std::to_string(ids[pick[bad[0]]]) + ": NumberFormatException");
      return fail(DDS_E_RANGE, "decimal row wider than the column limb capacity");
    }
    if (!longr.empty()) return fail(DDS_E_RANGE, "decimal row wider than the column limb capacity");
    if (fl & (kDecNeg | kDecReduce))
      if ((rc = dec_rows_with(w, st, m, kDecNeg | kDecReduce, &changed))) return rc;
    for (size_t j : changed) {
      dds_col::Orig o;
      if (!bn::from_dec(ch.data() + of[j], (size_t)(of[j + 1] - of[j]), o.mag, &o.neg))
        return fail(DDS_E_FORMAT, "row " + std::to_string(ids[pick[j]]) + ": NumberFormatException");
      plan->origs.emplace_back(j, std::move(o));
    }
  }
  plan->ids32.resize(m);
  for (size_t j = 0; j < m; ++j) plan->ids32[j] = (uint32_t)ids[pick[j]];
  return DDS_OK;
}

int col_write_commit(dds_col* col, RowWrite& plan) {
  const size_t m = plan.ids32.size();
  if (m == 0) return DDS_OK;
  Worker* w = plan.wl->w;
  hipStream_t st = plan.wl->st;
  // a multi-device write prepares every shard before committing any, so the current device is the last
  // prepared shard's: the worker's buffers must be (re)allocated on this column's device
  if (hipSetDevice(col->ctx->device) != hipSuccess) return fail(DDS_E_HIP, "hipSetDevice");
  HIP_TRY(w->ids.ensure(m * 4));
  HIP_TRY(hipMemcpyAsync(w->ids.p, plan.ids32.data(), m * 4, hipMemcpyHostToDevice, st));
  HIP_TRY(launch_scatter_rows(w->x2.as<uint32_t>(), plan.ss, w->ids.as<uint32_t>(), m, col->mc->S, col->d, col->stride,
                              st));
  HIP_TRY(hipStreamSynchronize(st));
  for (size_t j = 0; j < m; ++j) col->orig.erase((size_t)plan.ids32[j]);
  for (auto& o : plan.origs) col->orig[(size_t)plan.ids32[o.first]] = std::move(o.second);
  return DDS_OK;
}

int col_set_live(dds_col* col, const uint64_t* ids, size_t n, const uint8_t* live) {
  for (size_t i = 0; i < n; ++i)
    if (ids[i] >= col->count) return fail(DDS_E_ARG, "row id " + std::to_string(ids[i]) + " out of range");
  if (n == 0) return DDS_OK;
  std::map<uint64_t, uint8_t> last;  // last flag of each id wins
  for (size_t i = 0; i < n; ++i) last[ids[i]] = live[i] ? 1 : 0;
  std::vector<uint32_t> ids32;
  std::vector<uint8_t> vals;
  for (auto& kv : last)
    if (col->live((size_t)kv.first) != (kv.second != 0)) {
      ids32.push_back((uint32_t)kv.first);
      vals.push_back(kv.second);
    }
  if (ids32.empty()) return DDS_OK;
  WorkerLease wl(col->ctx);
  int rc;
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  const size_t m = ids32.size();
  HIP_TRY(w->ids.ensure(m * 4));
  HIP_TRY(w->in2.ensure(m));
  HIP_TRY(hipMemcpyAsync(w->ids.p, ids32.data(), m * 4, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(hipMemcpyAsync(w->in2.p, vals.data(), m, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(launch_scatter_bytes(w->ids.as<uint32_t>(), w->in2.as<uint8_t>(), m, col->dlive, wl.st));
  HIP_TRY(hipStreamSynchronize(wl.st));
  if (col->hlive.empty()) col->hlive.assign(col->capacity, 1);
  for (size_t j = 0; j < m; ++j) {
    col->hlive[ids32[j]] = vals[j];
    col->ndead = vals[j] ? col->ndead - 1 : col->ndead + 1;
  }
  return DDS_OK;
}

}  // namespace host
}  // namespace ddshe

// =============================================================================
dds_ctx::~dds_ctx() {
  for (auto& kv : host_regs) {
    void* p = reinterpret_cast<void*>(kv.first);
    if (kv.second.owned)
      (void)hipHostFree(p);
    else
      (void)hipHostUnregister(p);
  }
}

extern "C" {

const char* dds_strerror(int s) {
  switch (s) {
    case DDS_OK: return "ok";
    case DDS_E_EMPTY: return "no operand (404)";
    case DDS_E_RANGE: return "operand out of range";
    case DDS_E_HIP: return "HIP error";
    case DDS_E_ARG: return "invalid argument";
    case DDS_E_NOMEM: return "out of memory";
    case DDS_E_UNSUPPORTED: return "unsupported";
    case DDS_E_BUFSIZE: return "buffer too small";
    case DDS_E_FORMAT: return "number format";
    default: return "unknown";
  }
}

const char* dds_last_error(void) { return g_last_error.c_str(); }

size_t dds_max_modulus_bits(void) { return max_modulus_bits(); }

int dds_ctx_create(int device, dds_ctx** out) {
  if (!out) return fail(DDS_E_ARG, "out");
  *out = nullptr;
  try {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(DDS_E_HIP, "no HIP device");
    if (device < 0 || device >= n) return fail(DDS_E_ARG, "device index");
    if (hipSetDevice(device) != hipSuccess) return fail(DDS_E_HIP, "hipSetDevice");
    auto* c = new dds_ctx();
    c->device = device;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) {
      delete c;
      return fail(DDS_E_HIP, "hipGetDeviceProperties");
    }
    c->cus = p.multiProcessorCount;
    *out = c;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  } catch (...) {
    return fail(DDS_E_HIP, "unexpected exception");
  }
}

int dds_ctx_destroy(dds_ctx* ctx) {
  if (!ctx) return DDS_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  delete ctx;
  return DDS_OK;
}

int dds_host_register(dds_ctx* ctx, void* ptr, size_t bytes) {
  if (!ctx || !ptr || !bytes) return fail(DDS_E_ARG, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->regmu);
  const uintptr_t b = (uintptr_t)ptr;
  auto it = ctx->host_regs.upper_bound(b);
  if (it != ctx->host_regs.begin()) {
    auto pv = std::prev(it);
    if (pv->first == b && pv->second.bytes == bytes) return DDS_OK;  // already registered
    if (pv->first + pv->second.bytes > b) return fail(DDS_E_ARG, "overlaps a registered buffer");
  }
  if (it != ctx->host_regs.end() && it->first < b + bytes) return fail(DDS_E_ARG, "overlaps a registered buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterMapped));
  void* dptr = nullptr;
  if (hipHostGetDevicePointer(&dptr, ptr, 0) != hipSuccess) dptr = nullptr;  // DMA copies still work
  (void)hipGetLastError();
  ctx->host_regs[b] = dds_ctx::HostReg{bytes, dptr, false};
  return DDS_OK;
}

int dds_host_unregister(dds_ctx* ctx, void* ptr) {
  if (!ctx || !ptr) return fail(DDS_E_ARG, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->regmu);
  auto it = ctx->host_regs.find((uintptr_t)ptr);
  if (it == ctx->host_regs.end()) return fail(DDS_E_ARG, "not a registered buffer");
  if (it->second.owned) return fail(DDS_E_ARG, "allocated by dds_host_alloc: release it with dds_host_free");
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();  // no copy into it is still in flight
  hipError_t e = hipHostUnregister(ptr);
  ctx->host_regs.erase(it);
  return e == hipSuccess ? DDS_OK : fail(DDS_E_HIP, "hipHostUnregister");
}

int dds_host_alloc(dds_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !bytes || !out) return fail(DDS_E_ARG, "bad arguments");
  *out = nullptr;
  std::lock_guard<std::mutex> lk(ctx->regmu);
  HIP_TRY(hipSetDevice(ctx->device));
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocMapped) != hipSuccess || !p) {
    (void)hipGetLastError();
    return fail(DDS_E_NOMEM, "hipHostMalloc");
  }
  void* dptr = nullptr;
  if (hipHostGetDevicePointer(&dptr, p, 0) != hipSuccess) dptr = nullptr;
  (void)hipGetLastError();
  ctx->host_regs[(uintptr_t)p] = dds_ctx::HostReg{bytes, dptr, true};
  *out = p;
  return DDS_OK;
}

int dds_host_free(dds_ctx* ctx, void* ptr) {
  if (!ctx || !ptr) return fail(DDS_E_ARG, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->regmu);
  auto it = ctx->host_regs.find((uintptr_t)ptr);
  if (it == ctx->host_regs.end() || !it->second.owned) return fail(DDS_E_ARG, "not a dds_host_alloc buffer");
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();  // nothing still writes into it
  hipError_t e = hipHostFree(ptr);
  ctx->host_regs.erase(it);
  return e == hipSuccess ? DDS_OK : fail(DDS_E_HIP, "hipHostFree");
}

int dds_ctx_set_stream(dds_ctx* ctx, void* stream) {
  if (!ctx) return fail(DDS_E_ARG, "ctx");
  ctx->ext_stream = (hipStream_t)stream;
  return DDS_OK;
}

int dds_ctx_set_timing(dds_ctx* ctx, int enable) {
  if (!ctx) return fail(DDS_E_ARG, "ctx");
  ctx->timing.store(enable != 0);
  return DDS_OK;
}

int dds_ctx_get_timing(dds_ctx* ctx, double* fold_ms, uint64_t* fold_launches, double* total_ms) {
  if (!ctx) return fail(DDS_E_ARG, "ctx");
  std::lock_guard<std::mutex> lk(ctx->tmu);
  if (fold_ms) *fold_ms = ctx->fold_ms;
  if (fold_launches) *fold_launches = ctx->fold_launches;
  if (total_ms) *total_ms = ctx->total_ms;
  return DDS_OK;
}

int dds_ctx_reset_timing(dds_ctx* ctx) {
  if (!ctx) return fail(DDS_E_ARG, "ctx");
  std::lock_guard<std::mutex> lk(ctx->tmu);
  ctx->fold_ms = ctx->total_ms = 0;
  ctx->fold_launches = ctx->fold_modmuls = 0;
  return DDS_OK;
}

int dds_ctx_get_fold_work(dds_ctx* ctx, uint64_t* modmuls) {
  if (!ctx || !modmuls) return fail(DDS_E_ARG, "ctx");
  std::lock_guard<std::mutex> lk(ctx->tmu);
  *modmuls = ctx->fold_modmuls;
  return DDS_OK;
}

int dds_modmul_fold(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint8_t* ops, size_t width,
                    size_t count, uint8_t* out, size_t out_cap, size_t* out_len) {
  try {
    if (!ctx || (!ops && count) || width == 0) return fail(DDS_E_ARG, "bad arguments");
    if (count == 0) return fail(DDS_E_EMPTY, "no operand");
    if (count == 1) {  // DDSRestServer.scala:416-417: first operand is kept unreduced
      if (out_len) *out_len = width;
      if (!out || out_cap < width) return fail(DDS_E_BUFSIZE, "output buffer too small");
      memcpy(out, ops, width);
      return DDS_OK;
    }
    if (!mod_be || mod_bytes == 0) return fail(DDS_E_ARG, "modulus missing");
    const bn::Limbs M = bn::from_be(mod_be, mod_bytes);
    if (M.empty()) return fail(DDS_E_ARG, "modulus must be positive (BigInteger.mod)");
    if (!(M[0] & 1u) || bn::bit_length(M) < 2) {  // even modulus or 1: CRT split (fold_even_modulus)
      std::vector<bn::Limbs> xs(count);
      for (size_t i = 0; i < count; ++i) xs[i] = bn::from_be(ops + i * width, width);
      bn::Limbs r;
      int rc = fold_even_modulus(ctx, M, xs, std::vector<bool>(count, false), &r);
      if (rc) return rc;
      return emit_be(r, mod_bytes, out, out_cap, out_len);
    }
    return modmul_fold_be(ctx, mod_be, mod_bytes, 0, ops, width, count, out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  } catch (...) {
    return fail(DDS_E_HIP, "unexpected exception");
  }
}

int dds_paillier_sum(dds_ctx* ctx, const uint8_t* nsq, size_t nsq_bytes, const uint8_t* c, size_t width, size_t count,
                     uint8_t* out, size_t out_cap, size_t* out_len) {
  return dds_modmul_fold(ctx, nsq, nsq_bytes, c, width, count, out, out_cap, out_len);
}

int dds_rsa_product(dds_ctx* ctx, const uint8_t* n, size_t n_bytes, const uint8_t* c, size_t width, size_t count,
                    uint8_t* out, size_t out_cap, size_t* out_len) {
  return dds_modmul_fold(ctx, n, n_bytes, c, width, count, out, out_cap, out_len);
}

// A few pairs (one /Sum or /Mult request, or a small burst of them, DDSRestServer.scala:385,479) are
// latency-bound: operands go to the tail (latency) shape on the host (limb split; an operand >= 2N is
// reduced first, as BigInteger.multiply(..).mod would), one pinned H2D copy, one k_pairs launch at 16-32
// lanes per bignum, one D2H copy: one stream synchronisation instead of three (two ingest range checks
// and the readback), and two Montgomery products of ~14 us instead of ~30 us at the throughput shape.
constexpr size_t kSmallPairs = 8;
int small_pairs(Worker* w, hipStream_t st, ModConsts& mc, const uint8_t* a, const uint8_t* b, size_t width, size_t n,
                size_t mod_bytes, uint8_t* out) {
  const int S3 = mc.S3;  // one workgroup per pair in the tree shape (k_pairs_sos)
  const size_t words = (size_t)S3 * n;
  HIP_TRY(w->hch[0].ensure(3 * words * 4));
  HIP_TRY(w->x.ensure(3 * words * 4));
  uint32_t* h = (uint32_t*)w->hch[0].p;
  for (int k = 0; k < 2; ++k) {
    const uint8_t* src = k ? b : a;
    for (size_t i = 0; i < n; ++i) {
      bn::Limbs v = bn::from_be(src + i * width, width);
      if (bn::bit_length(v) > (size_t)mc.W * mc.S)  // as the lane-group path's ingest (k_ingest_be flag 2)
        return fail(DDS_E_RANGE, "operand wider than the modulus limb width");
      if (bn::cmp(v, mc.N) >= 0) v = bn::mod(v, mc.N);
      const std::vector<uint32_t> rw = bn::to_rw(v, S3, mc.W3);
      std::copy(rw.begin(), rw.end(), h + k * words + i * S3);
    }
  }
  uint32_t* d = w->x.as<uint32_t>();
  HIP_TRY(hipMemcpyAsync(d, h, 2 * words * 4, hipMemcpyHostToDevice, st));
  HIP_TRY(launch_pairs_sos(S3, d, d + words, n, mc.d3, mc.d3 + 5 * (size_t)S3, d + 2 * words, st));
  HIP_TRY(hipMemcpyAsync(h + 2 * words, d + 2 * words, words * 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  for (size_t i = 0; i < n; ++i)
    if (!bn::to_be(bn::from_rw(h + 2 * words + i * S3, S3, mc.W3), out + i * mod_bytes, mod_bytes))
      return fail(DDS_E_RANGE, "result does not fit");
  return DDS_OK;
}

int dds_modmul_pairs(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint8_t* a, const uint8_t* b,
                     size_t width, size_t n, uint8_t* out) {
  try {
    if (!ctx || width == 0 || (n && (!a || !b || !out))) return fail(DDS_E_ARG, "bad arguments");
    if (n == 0) return DDS_OK;
    std::shared_ptr<ModConsts> mc;
    int rc = get_mod(ctx, mod_be, mod_bytes, &mc);
    if (rc) return rc;
    if ((rc = check_rows(*mc, n))) return rc;
    WorkerLease wl(ctx);
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    if (n <= kSmallPairs) return small_pairs(w, wl.st, *mc, a, b, width, n, mod_bytes, out);
    const int S = mc->S;
    const size_t stride = round_up(n, 64);
    HIP_TRY(w->x.ensure((size_t)S * stride * 4));
    HIP_TRY(w->x2.ensure((size_t)S * stride * 4));
    HIP_TRY(w->p0.ensure((size_t)S * stride * 4));
    if ((rc = ingest(ctx, w, wl.st, *mc, a, width, n, w->in, w->x.as<uint32_t>(), stride))) return rc;
    if ((rc = ingest(ctx, w, wl.st, *mc, b, width, n, w->in2, w->x2.as<uint32_t>(), stride))) return rc;
    HIP_TRY(launch_pairs(S, w->x.as<uint32_t>(), w->x2.as<uint32_t>(), stride, n, mc->d, mc->n0,
                         w->p0.as<uint32_t>(), wl.st));
    if (S <= kEgressMaxLimbs) {  // canonical products -> big-endian bytes on the GPU, one copy out
      HIP_TRY(w->misc.ensure(n * mod_bytes));
      HIP_TRY(launch_egress_be(w->p0.as<uint32_t>(), stride, n, S, mc->W, nullptr, mod_bytes, w->misc.as<uint8_t>(),
                               wl.st));
      HIP_TRY(hipMemcpyAsync(out, w->misc.p, n * mod_bytes, hipMemcpyDeviceToHost, wl.st));
      HIP_TRY(hipStreamSynchronize(wl.st));
      return DDS_OK;
    }
    std::vector<uint32_t> h((size_t)S * stride);
    HIP_TRY(hipMemcpyAsync(h.data(), w->p0.p, h.size() * 4, hipMemcpyDeviceToHost, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    std::vector<uint32_t> limbs(S);
    for (size_t i = 0; i < n; ++i) {
      for (int l = 0; l < S; ++l) limbs[l] = h[(size_t)l * stride + i];
      if (!bn::to_be(mc->value(limbs.data()), out + i * mod_bytes, mod_bytes))
        return fail(DDS_E_RANGE, "result does not fit");
    }
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  } catch (...) {
    return fail(DDS_E_HIP, "unexpected exception");
  }
}

int dds_bigint_sum(dds_ctx* ctx, const uint8_t* ops, size_t width, size_t count, uint8_t* out, size_t out_cap,
                   size_t* out_len) {
  try {
    if (!ctx || width == 0 || (count && !ops)) return fail(DDS_E_ARG, "bad arguments");
    if (count == 0) return fail(DDS_E_EMPTY, "no operand");
    WorkerLease wl(ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    const int S = (int)((width * 8 + 26) / 27);
    const size_t stride = round_up(count, 64);
    HIP_TRY(w->x.ensure((size_t)S * stride * 4));
    HIP_TRY(w->in.ensure(count * width));
    HIP_TRY(w->flags.ensure(16));
    // 2N sentinel with limb S set: every row compares below it (no range check for plain sums)
    std::vector<uint32_t> sentinel((size_t)S + 1, 0);
    sentinel[S] = 1;
    constexpr int kPlainW = 27;
    HIP_TRY(w->misc2.ensure(sentinel.size() * 4));
    HIP_TRY(hipMemcpyAsync(w->misc2.p, sentinel.data(), sentinel.size() * 4, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(hipMemcpyAsync(w->in.p, ops, count * width, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(hipMemsetAsync(w->flags.p, 0, 4, wl.st));
    HIP_TRY(launch_ingest_be(w->in.as<uint8_t>(), width, count, S, kPlainW, w->misc2.as<uint32_t>(), w->x.as<uint32_t>(),
                             stride, w->flags.as<uint32_t>(), wl.st));
    const size_t nthreads = std::min<size_t>(count, (size_t)ctx->cus * 1024);
    HIP_TRY(w->misc.ensure((size_t)S * nthreads * 8));
    HIP_TRY(w->out.ensure((size_t)S * 8));
    HIP_TRY(launch_plain_sum(w->x.as<uint32_t>(), stride, count, S, nthreads, w->misc.as<uint64_t>(),
                             w->out.as<uint64_t>(), wl.st));
    std::vector<uint64_t> sums(S);
    HIP_TRY(hipMemcpyAsync(sums.data(), w->out.p, (size_t)S * 8, hipMemcpyDeviceToHost, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    // combine 64-bit limb sums: value = sum_l sums[l] * 2^(27 l)
    bn::Limbs acc;
    for (int l = S - 1; l >= 0; --l) {
      // acc = acc * 2^27 + sums[l]
      bn::Limbs sh = bn::mul(acc, bn::Limbs{1u << 27});
      acc = bn::add(sh, bn::from_u64(sums[l]));
    }
    const size_t need = std::max<size_t>(1, bn::byte_length(acc));
    const size_t w_out = std::max(width, need);
    return emit_be(acc, w_out, out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  } catch (...) {
    return fail(DDS_E_HIP, "unexpected exception");
  }
}

int dds_bigint_product(dds_ctx* ctx, const uint8_t* ops, size_t width, size_t count, uint8_t* out, size_t out_cap,
                       size_t* out_len) {
  try {
    if (!ctx || width == 0 || (count && !ops)) return fail(DDS_E_ARG, "bad arguments");
    if (count == 0) return fail(DDS_E_EMPTY, "no operand");
    // boundary format: big-endian bytes -> radix-2^16 limbs (one per u32 word), row-major
    size_t len = (width + 1) / 2;
    std::vector<uint32_t> h(count * len, 0);
    for (size_t r = 0; r < count; ++r)
      for (size_t i = 0; i < width; ++i) {
        const size_t bit = 8 * (width - 1 - i);
        h[r * len + bit / 16] |= (uint32_t)ops[r * width + i] << (bit % 16);
      }
    bn::Limbs v;
    int rc = product_tree(ctx, h, count, len, 0, &v);
    if (rc) return rc;
    return emit_be(v, std::max<size_t>(1, bn::byte_length(v)), out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

// ---- device columns -----------------------------------------------------------
int dds_col_create(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, size_t capacity, dds_col** out) {
  try {
    if (!ctx || !out || capacity == 0) return fail(DDS_E_ARG, "bad arguments");
    *out = nullptr;
    std::shared_ptr<ModConsts> mc;
    int rc = get_mod(ctx, mod_be, mod_bytes, &mc);
    if (rc) return rc;
    if ((rc = check_rows(*mc, capacity))) return rc;
    auto* c = new dds_col();
    c->ctx = ctx;
    c->mc = mc;
    c->capacity = capacity;
    c->stride = round_up(capacity, 64);
    if (hipSetDevice(ctx->device) != hipSuccess || hipMalloc(&c->d, (size_t)mc->S * c->stride * 4) != hipSuccess ||
        hipMalloc(&c->dlive, c->stride + 16) != hipSuccess) {
      delete c;
      return fail(DDS_E_NOMEM, "column allocation");
    }
    if (hipMemset(c->dlive, 1, c->stride + 16) != hipSuccess) {
      delete c;
      return fail(DDS_E_HIP, "live mask initialisation");
    }
    *out = c;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_destroy(dds_col* col) {
  delete col;
  return DDS_OK;
}

size_t dds_col_count(const dds_col* col) { return col ? col->count : 0; }

int dds_col_truncate(dds_col* col, size_t count) {
  if (!col) return fail(DDS_E_ARG, "bad arguments");
  std::unique_lock<std::shared_mutex> lk(col->mu);
  if (count > col->count) return fail(DDS_E_ARG, "truncate beyond the row count");
  if (col->ndead) {  // dropped rows come back live (rows past `count` always are)
    size_t dropped = 0;
    for (size_t r = count; r < col->count; ++r) {
      dropped += !col->hlive[r];
      col->hlive[r] = 1;
    }
    if (dropped) {
      HIP_TRY(hipSetDevice(col->ctx->device));
      HIP_TRY(hipMemset(col->dlive + count, 1, col->count - count));
      col->ndead -= dropped;
    }
  }
  col->count = count;
  col->orig.erase(col->orig.lower_bound(count), col->orig.end());
  return DDS_OK;
}

int dds_col_write_rows(dds_col* col, const uint64_t* row_ids, size_t n, const uint8_t* operands_be, size_t width) {
  try {
    if (!col || (n && (!row_ids || !operands_be || width == 0))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    RowWrite plan;
    int rc = col_write_prepare(col, row_ids, n, operands_be, width, nullptr, nullptr, &plan);
    return rc ? rc : col_write_commit(col, plan);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_write_rows_dec(dds_col* col, const uint64_t* row_ids, size_t n, const char* chars,
                           const uint64_t* offsets) {
  try {
    if (!col || (n && (!row_ids || !chars || !offsets))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    RowWrite plan;
    int rc = col_write_prepare(col, row_ids, n, nullptr, 0, chars, offsets, &plan);
    return rc ? rc : col_write_commit(col, plan);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_set_live(dds_col* col, const uint64_t* row_ids, size_t n, const uint8_t* live) {
  try {
    if (!col || (n && (!row_ids || !live))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    return col_set_live(col, row_ids, n, live);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

size_t dds_col_live_count(dds_col* col) {
  if (!col) return 0;
  std::shared_lock<std::shared_mutex> lk(col->mu);
  return col->count - col->ndead;
}

size_t dds_col_partial_words(const dds_col* col) { return col ? partial_words_for(*col->mc) : 0; }

int dds_col_append(dds_col* col, const uint8_t* ops, size_t width, size_t count) {
  try {
    if (!col || width == 0 || (count && !ops)) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    if (col->count + count > col->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    if (count == 0) return DDS_OK;
    WorkerLease wl(col->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    // ingest writes with the column's stride starting at row `count`
    std::vector<size_t> reduced;
    if ((rc = ingest(col->ctx, wl.w, wl.st, *col->mc, ops, width, count, wl.w->in, col->d + col->count, col->stride,
                     &reduced)))
      return rc;
    HIP_TRY(hipStreamSynchronize(wl.st));
    for (size_t i : reduced) col->orig[col->count + i] = dds_col::Orig{bn::from_be(ops + i * width, width), false};
    col->count += count;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_append_dec(dds_col* col, const char* chars, const uint64_t* offsets, size_t count) {
  try {
    if (!col || (count && (!chars || !offsets))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    if (col->count + count > col->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    if (count == 0) return DDS_OK;
    for (size_t i = 0; i < count; ++i)
      if (offsets[i + 1] < offsets[i]) return fail(DDS_E_ARG, "offsets must be non-decreasing");
    WorkerLease wl(col->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    DecRows src;
    src.chars = chars;
    src.offs = offsets;
    uint32_t fl = 0;
    std::vector<size_t> longr;
    if ((rc = ingest_dec(wl.w, wl.st, *col->mc, src, count, col->d + col->count, col->stride, &fl, &longr)))
      return rc;
    if (fl & (kDecFormat | kDecWide)) {
      std::vector<size_t> bad;
      if ((rc = dec_rows_with(wl.w, wl.st, count, kDecFormat, &bad))) return rc;
      if (!bad.empty()) return fail(DDS_E_FORMAT, "row " + std::to_string(bad[0]) + ": NumberFormatException");
      return fail(DDS_E_RANGE, "decimal row wider than the column limb capacity");
    }
    if (!longr.empty()) return fail(DDS_E_RANGE, "decimal row wider than the column limb capacity");
    std::vector<size_t> changed;
    if (fl & (kDecNeg | kDecReduce))
      if ((rc = dec_rows_with(wl.w, wl.st, count, kDecNeg | kDecReduce, &changed))) return rc;
    HIP_TRY(hipStreamSynchronize(wl.st));
    for (size_t i : changed) {
      dds_col::Orig o;
      if (!bn::from_dec(chars + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), o.mag, &o.neg))
        return fail(DDS_E_FORMAT, "row " + std::to_string(i) + ": NumberFormatException");
      col->orig[col->count + i] = std::move(o);
    }
    col->count += count;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_read(dds_col* col, size_t first, size_t count, uint8_t* out) {
  try {
    if (!col) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(col->mu);
    if ((count && !out) || first + count > col->count) return fail(DDS_E_ARG, "bad arguments");
    const int S = col->mc->S;
    if (count && S <= kEgressMaxLimbs) {  // rows (< 2N) -> canonical big-endian bytes on the GPU
      WorkerLease wl(col->ctx);
      int rc;
      if ((rc = wl.acquire())) return rc;
      Worker* w = wl.w;
      const size_t bytes = col->mc->bytes;
      for (size_t b = 0; b < count;) {  // bounded device staging: chunks of <= 256 MiB of bytes
        const size_t n = std::min(count - b, std::max<size_t>(1, ((size_t)256 << 20) / bytes));
        HIP_TRY(w->misc.ensure(n * bytes));
        HIP_TRY(launch_egress_be(col->d + first + b, col->stride, n, S, col->mc->W, col->mc->d + (size_t)kConstN * S,
                                 bytes, w->misc.as<uint8_t>(), wl.st));
        HIP_TRY(hipMemcpyAsync(out + b * bytes, w->misc.p, n * bytes, hipMemcpyDeviceToHost, wl.st));
        HIP_TRY(hipStreamSynchronize(wl.st));
        b += n;
      }
      return DDS_OK;
    }
    std::vector<uint32_t> h((size_t)S * count);
    if (count)
      HIP_TRY(hipMemcpy2D(h.data(), count * 4, col->d + first, col->stride * 4, count * 4, (size_t)S,
                          hipMemcpyDeviceToHost));
    std::vector<uint32_t> limbs(S);
    for (size_t i = 0; i < count; ++i) {
      for (int l = 0; l < S; ++l) limbs[l] = h[(size_t)l * count + i];
      bn::Limbs v = col->mc->value(limbs.data());
      if (bn::cmp(v, col->mc->N) >= 0) v = bn::mod(v, col->mc->N);  // rows are kept < 2N
      if (!bn::to_be(v, out + i * col->mc->bytes, col->mc->bytes))
        return fail(DDS_E_RANGE, "row does not fit");
    }
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_fold_partial(dds_col* col, size_t first, size_t count, uint32_t* partial, uint64_t* rows) {
  try {
    if (!col || !partial) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(col->mu);
    if (first + count > col->count) return fail(DDS_E_ARG, "bad arguments");
    ModConsts& mc = *col->mc;
    const size_t S2 = (size_t)mc.S2;
    int64_t E = 0;
    WorkerLease wl(col->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    const uint32_t* d_ids = nullptr;
    if ((rc = col_live_range(col, wl.w, wl.st, first, count, &d_ids, &count))) return rc;  // live rows only
    if (count == 0) {  // empty partial: prod = 1, E = 0
      std::fill(partial, partial + S2, 0u);
      partial[0] = 1;
    } else {
      const uint32_t* part;
      size_t ps;
      if ((rc = fold_partial_device(col->ctx, wl.w, wl.st, mc, col->d + first, col->stride, count, &part, &ps, &E,
                                    d_ids)))
        return rc;
      HIP_TRY(hipMemcpy2DAsync(partial, 4, part, ps * 4, 4, S2, hipMemcpyDeviceToHost, wl.st));
      HIP_TRY(hipStreamSynchronize(wl.st));
      account_fold(col->ctx, wl.w);
    }
    partial[S2] = (uint32_t)(uint64_t)E;
    partial[S2 + 1] = (uint32_t)((uint64_t)E >> 32);
    if (rows) *rows = count;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_fold(dds_col* col, size_t first, size_t count, uint8_t* out, size_t out_cap, size_t* out_len) {
  try {
    if (!col) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(col->mu);
    if (first + count > col->count) return fail(DDS_E_ARG, "bad arguments");
    bn::Limbs v;
    bool neg = false;
    int rc = col_fold_value(col, nullptr, first, count, &v, &neg);
    if (rc) return rc;
    if (neg) return fail(DDS_E_RANGE, "the single operand is negative: use dds_col_fold_dec");
    return emit_be(v, std::max(col->mc->bytes, bn::byte_length(v)), out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_fold_rows(dds_col* col, const uint64_t* row_ids, size_t n, uint8_t* out, size_t out_cap,
                      size_t* out_len) {
  try {
    if (!col || (n && !row_ids)) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(col->mu);
    bn::Limbs v;
    bool neg = false;
    int rc = col_fold_value(col, row_ids, 0, n, &v, &neg);
    if (rc) return rc;
    if (neg) return fail(DDS_E_RANGE, "the single operand is negative: use dds_col_fold_dec");
    return emit_be(v, std::max(col->mc->bytes, bn::byte_length(v)), out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_fold_dec(dds_col* col, const uint64_t* row_ids, size_t n, char* out, size_t out_cap, size_t* out_len) {
  try {
    if (!col) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(col->mu);
    if (!row_ids && n > col->count) return fail(DDS_E_ARG, "bad arguments");
    bn::Limbs v;
    bool neg = false;
    int rc = col_fold_value(col, row_ids, 0, n, &v, &neg);
    if (rc) return rc;
    const std::string t = bn::to_dec(v, neg);
    if (out_len) *out_len = t.size();
    if (!out || out_cap < t.size() + 1) return fail(DDS_E_BUFSIZE, "output buffer too small");
    memcpy(out, t.c_str(), t.size() + 1);
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_combine_partials(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint32_t* partials,
                         const uint64_t* rows, size_t nparts, uint8_t* out, size_t out_cap, size_t* out_len) {
  try {
    if (!ctx || !partials || !rows || nparts == 0) return fail(DDS_E_ARG, "bad arguments");
    return combine_partials(ctx, mod_be, mod_bytes, partials, nullptr, rows, nparts, out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_combine_partials_device(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint32_t* d_partials,
                                const uint64_t* rows, size_t nparts, uint8_t* out, size_t out_cap, size_t* out_len) {
  try {
    if (!ctx || !d_partials || !rows || nparts == 0) return fail(DDS_E_ARG, "bad arguments");
    return combine_partials(ctx, mod_be, mod_bytes, nullptr, d_partials, rows, nparts, out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_fold_partial_device(dds_col* col, size_t first, size_t count, uint32_t* d_partial) {
  try {
    if (!col || !d_partial) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(col->mu);
    if (first + count > col->count) return fail(DDS_E_ARG, "bad arguments");
    ModConsts& mc = *col->mc;
    const size_t S2 = (size_t)mc.S2;
    WorkerLease wl(col->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    int64_t E = 0;
    const uint32_t* d_ids = nullptr;
    if ((rc = col_live_range(col, wl.w, wl.st, first, count, &d_ids, &count))) return rc;  // live rows only
    if (count == 0) {  // empty partial: prod = 1, E = 0
      HIP_TRY(hipMemsetAsync(d_partial, 0, S2 * 4, wl.st));
      const uint32_t one = 1;
      HIP_TRY(hipMemcpyAsync(d_partial, &one, 4, hipMemcpyHostToDevice, wl.st));
    } else {
      const uint32_t* part;
      size_t ps;
      if ((rc = fold_partial_device(col->ctx, wl.w, wl.st, mc, col->d + first, col->stride, count, &part, &ps, &E,
                                    d_ids)))
        return rc;
      HIP_TRY(launch_strided_copy(part, 0, ps, d_partial, 0, 1, 1, S2, wl.st));
    }
    const uint32_t ew[2] = {(uint32_t)(uint64_t)E, (uint32_t)((uint64_t)E >> 32)};
    HIP_TRY(hipMemcpyAsync(d_partial + S2, ew, 8, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    account_fold(col->ctx, wl.w);
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

// ---- modular exponentiation / Paillier encryption --------------------------------
namespace {
// Sliding-window schedule of a uniform exponent E (left to right): sched[0] = index of the
// leading window's odd power, then (nsq << 16) | (idx + 1) per later window (idx + 1 == 0:
// trailing squarings only). Returns the number of odd powers the table must hold.
int window_schedule(const bn::Limbs& E, std::vector<uint32_t>* sched) {
  sched->clear();
  const int nb = (int)bn::bit_length(E);
  if (nb == 0) return 1;
  auto bit = [&](int i) { return (E[(size_t)i >> 5] >> (i & 31)) & 1u; };
  // window width minimising table + multiplies (table of 2^(w-1) odd powers per row)
  const int w = nb <= 24 ? 1 : nb <= 80 ? 3 : nb <= 240 ? 4 : 5;
  int i = nb - 1;
  uint32_t pending_sq = 0;
  bool first = true;
  while (i >= 0) {
    if (!bit(i)) {
      ++pending_sq;
      --i;
      continue;
    }
    int j = std::max(i - w + 1, 0);
    while (!bit(j)) ++j;  // window [i..j] ends on a set bit
    uint32_t v = 0;
    for (int k = i; k >= j; --k) v = (v << 1) | bit(k);
    const uint32_t idx = (v - 1) / 2;
    if (first) {
      sched->push_back(idx);
      first = false;
    } else {
      pending_sq += (uint32_t)(i - j + 1);
      sched->push_back((pending_sq << 16) | (idx + 1));
    }
    pending_sq = 0;
    i = j - 1;
  }
  while (pending_sq > 0) {  // trailing zero bits: squarings only, <= 0xFFFF per entry
    const uint32_t c = std::min<uint32_t>(pending_sq, 0xFFFF);
    sched->push_back(c << 16);
    pending_sq -= c;
  }
  return 1 << (w - 1);
}

// out[i] = g^m[i] * x[i]^E mod N on the device (d_m == nullptr: x[i]^E). x rows are rW,
// fully normalised, < 2N. Processes the batch in equal chunks so the per-row window table
// (nodd * S words per row) stays within kModexpTabBytes of HBM.
constexpr size_t kModexpTabBytes = (size_t)8 << 30;
int modexp_device(Worker* w, hipStream_t st, ModConsts& mc, const bn::Limbs& E, const bn::Limbs* g,
                  const uint32_t* d_x, size_t xstride, const uint32_t* d_m, size_t count, uint32_t* d_out,
                  size_t ostride) {
  if (count == 0) return DDS_OK;
  const int S = mc.S;
  std::vector<uint32_t> sched;
  const int nodd = window_schedule(E, &sched);
  std::vector<uint32_t> gr;
  if (d_m) gr = mc.rw(bn::mod(bn::mul(bn::mod(*g, mc.N), mc.Rmod), mc.N));
  else gr.assign((size_t)S, 0);
  const size_t sched_words = std::max<size_t>(sched.size(), 1);
  HIP_TRY(w->y.ensure((gr.size() + sched_words) * 4));
  uint32_t* d_gr = w->y.as<uint32_t>();
  uint32_t* d_sched = d_gr + gr.size();
  HIP_TRY(hipMemcpyAsync(d_gr, gr.data(), gr.size() * 4, hipMemcpyHostToDevice, st));
  if (!sched.empty())
    HIP_TRY(hipMemcpyAsync(d_sched, sched.data(), sched.size() * 4, hipMemcpyHostToDevice, st));
  const size_t row_bytes = (size_t)nodd * S * 4;
  // equal chunks (a short last chunk would leave most CUs idle for a whole ladder)
  const size_t cap = std::max<size_t>(64, kModexpTabBytes / row_bytes / 64 * 64);
  const size_t nch = (count + cap - 1) / cap;
  const size_t chunk = round_up((count + nch - 1) / nch, 64);
  HIP_TRY(w->tab.ensure((size_t)nodd * S * chunk * 4));
  for (size_t c0 = 0; c0 < count; c0 += chunk) {
    const size_t cc = std::min(chunk, count - c0);
    HIP_TRY(launch_modexp_pre(S, d_x + c0, xstride, cc, mc.d, mc.dqm, mc.n0, nodd, w->tab.as<uint32_t>(), chunk, st));
    HIP_TRY(launch_modexp_ladder(S, w->tab.as<uint32_t>(), chunk, d_m ? d_m + c0 : nullptr, cc, mc.d, mc.dqm, d_gr, d_sched,
                                 (int)sched.size(), mc.n0, d_out + c0, ostride, st));
  }
  HIP_TRY(hipStreamSynchronize(st));  // host vectors above must outlive the async copies
  return DDS_OK;
}

int encrypt_device(Worker* w, hipStream_t st, ModConsts& mc, const bn::Limbs& n, const bn::Limbs& g,
                   const uint32_t* d_m, const uint32_t* d_rcol, size_t rstride, size_t count, uint32_t* d_out,
                   size_t ostride, bool use_n_exponent) {
  return modexp_device(w, st, mc, use_n_exponent ? n : bn::Limbs{}, &g, d_rcol, rstride, d_m, count, d_out, ostride);
}
}  // namespace

// CRT form of a Paillier key (p, q): per-modulus constants of p^2, q^2, n^2 and the Garner
// constants c1R = (q^2)^-1 R_p, c2R = -(q^2)^-1 R_p (mod p^2), q2R = q^2 R_n (mod n^2).
struct CrtKey {
  std::shared_ptr<ModConsts> mp, mq, mn;
  bn::Limbs n;
  uint32_t* d = nullptr;  // c1R | c2R (2 Sp limbs) | q2R (Sn limbs)
  ~CrtKey() {
    if (d) (void)hipFree(d);
  }
};

namespace {
int get_crt_key(dds_ctx* ctx, const bn::Limbs& p, const bn::Limbs& q, std::shared_ptr<CrtKey>* out) {
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    auto it = ctx->crt_keys.find({p, q});
    if (it != ctx->crt_keys.end()) {
      *out = it->second;
      return DDS_OK;
    }
  }
  if (p.empty() || q.empty() || !(p[0] & 1u) || !(q[0] & 1u) || bn::cmp(p, q) == 0 || bn::bit_length(p) < 2 ||
      bn::bit_length(q) < 2)
    return fail(DDS_E_ARG, "p, q must be distinct odd primes");
  auto k = std::make_shared<CrtKey>();
  k->n = bn::mul(p, q);
  const bn::Limbs p2 = bn::mul(p, p), q2 = bn::mul(q, q), n2 = bn::mul(k->n, k->n);
  auto be = [](const bn::Limbs& v) {
    std::vector<uint8_t> b(bn::byte_length(v));
    bn::to_be(v, b.data(), b.size());
    return b;
  };
  int rc;
  auto bp = be(p2), bq = be(q2), bn2 = be(n2);
  if ((rc = get_mod(ctx, bp.data(), bp.size(), &k->mp)) || (rc = get_mod(ctx, bq.data(), bq.size(), &k->mq)) ||
      (rc = get_mod(ctx, bn2.data(), bn2.size(), &k->mn)))
    return rc;
  // (q^2)^-1 mod p^2 = (q^2)^(p(p-1)-1) (Euler, p prime); verified below
  const bn::Limbs phi = bn::mul(p, bn::sub(p, bn::Limbs{1}));
  const bn::Limbs qinv = bn::powmod(bn::mod(q2, p2), bn::sub(phi, bn::Limbs{1}), p2);
  if (bn::cmp(bn::mod(bn::mul(qinv, q2), p2), bn::Limbs{1}) != 0) return fail(DDS_E_ARG, "p, q must be distinct primes");
  const ModConsts &mp = *k->mp, &mn = *k->mn;
  std::vector<uint32_t> host;
  auto put = [&](const std::vector<uint32_t>& v) { host.insert(host.end(), v.begin(), v.end()); };
  put(mp.rw(bn::mulmod(qinv, mp.Rmod, p2)));
  put(mp.rw(bn::mulmod(bn::sub(p2, qinv), mp.Rmod, p2)));
  put(mn.rw(bn::mulmod(q2, mn.Rmod, n2)));
  if (hipSetDevice(ctx->device) != hipSuccess || hipMalloc(&k->d, host.size() * 4) != hipSuccess)
    return fail(DDS_E_NOMEM, "crt const alloc");
  HIP_TRY(hipMemcpy(k->d, host.data(), host.size() * 4, hipMemcpyHostToDevice));
  std::lock_guard<std::mutex> lk(ctx->mu);
  auto it = ctx->crt_keys.find({p, q});
  if (it != ctx->crt_keys.end()) {
    *out = it->second;
    return DDS_OK;
  }
  if (ctx->crt_keys.size() > 16) ctx->crt_keys.clear();
  ctx->crt_keys.emplace(std::make_pair(p, q), k);
  *out = k;
  return DDS_OK;
}

// The CRT halves need r < R_p, R_q (r fits the half-width limb layout) and y_q < R_p.
bool crt_fits(const CrtKey& k) {
  const size_t cap_p = (size_t)k.mp->S * k.mp->W - 2, cap_q = (size_t)k.mq->S * k.mq->W - 2;
  const size_t nb = bn::bit_length(k.n);
  return nb <= cap_p && nb <= cap_q && k.mq->bits <= cap_p;
}

// out = g^m r^n mod n^2 for rows of r (n^2 layout, values < 2^bits(n)) through the CRT halves
int encrypt_crt_device(Worker* w, hipStream_t st, CrtKey& k, const bn::Limbs& g, const uint32_t* d_m,
                       const uint32_t* d_r, size_t rstride, size_t count, uint32_t* d_out, size_t ostride) {
  ModConsts &mp = *k.mp, &mq = *k.mq, &mn = *k.mn;
  const size_t chunk = std::min<size_t>(round_up(count, 64), (size_t)1 << 20);
  const size_t sp = (size_t)mp.S * chunk * 4, sq = (size_t)mq.S * chunk * 4, sn = (size_t)mn.S * chunk * 4;
  const size_t sizes[7] = {sp, sq, sp, sq, sp, sn, sn};
  for (int i = 0; i < 7; ++i) HIP_TRY(w->crt[i].ensure(sizes[i]));
  HIP_TRY(w->flags.ensure(16));
  HIP_TRY(hipMemsetAsync(w->flags.as<uint32_t>() + 1, 0, 4, st));
  uint32_t* fl = w->flags.as<uint32_t>() + 1;
  uint32_t *A = w->crt[0].as<uint32_t>(), *B = w->crt[1].as<uint32_t>(), *C = w->crt[2].as<uint32_t>(),
           *D = w->crt[3].as<uint32_t>(), *E = w->crt[4].as<uint32_t>(), *F = w->crt[5].as<uint32_t>(),
           *Gq = w->crt[6].as<uint32_t>();
  int rc;
  for (size_t c0 = 0; c0 < count; c0 += chunk) {
    const size_t cc = std::min(chunk, count - c0);
    HIP_TRY(launch_repack(d_r + c0, rstride, mn.S, mn.W, A, chunk, mp.S, mp.W, cc, fl, st));
    HIP_TRY(launch_repack(d_r + c0, rstride, mn.S, mn.W, B, chunk, mq.S, mq.W, cc, fl, st));
    if ((rc = modexp_device(w, st, mp, k.n, &g, A, chunk, d_m + c0, cc, C, chunk))) return rc;
    if ((rc = modexp_device(w, st, mq, k.n, &g, B, chunk, d_m + c0, cc, D, chunk))) return rc;
    HIP_TRY(launch_repack(D, chunk, mq.S, mq.W, E, chunk, mp.S, mp.W, cc, fl, st));
    HIP_TRY(launch_crt_h(mp.S, C, E, chunk, cc, mp.d, k.d, mp.n0, A, st));
    HIP_TRY(launch_repack(A, chunk, mp.S, mp.W, F, chunk, mn.S, mn.W, cc, fl, st));
    HIP_TRY(launch_repack(D, chunk, mq.S, mq.W, Gq, chunk, mn.S, mn.W, cc, fl, st));
    HIP_TRY(launch_crt_out(mn.S, F, Gq, chunk, cc, mn.d, k.d + 2 * (size_t)mp.S, mn.n0, d_out + c0, ostride, st));
  }
  uint32_t flags = 0;
  HIP_TRY(read_sync(w, st, fl, &flags, 4));
  if (flags) return fail(DDS_E_RANGE, "r does not fit below 2^bits(n)");
  return DDS_OK;
}
}  // namespace

int dds_paillier_encrypt_batch(dds_ctx* ctx, const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be, size_t g_bytes,
                               const uint32_t* m, const uint8_t* r_be, size_t r_width, size_t count, uint8_t* out,
                               size_t nsq_bytes) {
  try {
    if (!ctx || !n_be || !g_be || r_width == 0 || (count && (!m || !r_be || !out))) return fail(DDS_E_ARG, "bad args");
    if (count == 0) return DDS_OK;
    bn::Limbs n = bn::from_be(n_be, n_bytes);
    bn::Limbs nsq = bn::mul(n, n);
    if (nsq_bytes < bn::byte_length(nsq)) return fail(DDS_E_BUFSIZE, "nsq_bytes too small");
    std::vector<uint8_t> nsq_be(bn::byte_length(nsq));
    bn::to_be(nsq, nsq_be.data(), nsq_be.size());
    std::shared_ptr<ModConsts> mc;
    int rc = get_mod(ctx, nsq_be.data(), nsq_be.size(), &mc);
    if (rc) return rc;
    bn::Limbs g = bn::from_be(g_be, g_bytes);
    if ((rc = check_rows(*mc, count))) return rc;
    WorkerLease wl(ctx);
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    const int S = mc->S;
    const size_t stride = round_up(count, 64);
    HIP_TRY(w->x.ensure((size_t)S * stride * 4));
    HIP_TRY(w->x2.ensure((size_t)S * stride * 4));
    HIP_TRY(w->misc.ensure(count * 4));
    if ((rc = ingest(ctx, w, wl.st, *mc, r_be, r_width, count, w->in, w->x.as<uint32_t>(), stride))) return rc;
    HIP_TRY(hipMemcpyAsync(w->misc.p, m, count * 4, hipMemcpyHostToDevice, wl.st));
    if ((rc = encrypt_device(w, wl.st, *mc, n, g, w->misc.as<uint32_t>(), w->x.as<uint32_t>(), stride, count,
                             w->x2.as<uint32_t>(), stride, true)))
      return rc;
    std::vector<uint32_t> h((size_t)S * stride);
    HIP_TRY(hipMemcpy(h.data(), w->x2.p, h.size() * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> limbs(S);
    for (size_t i = 0; i < count; ++i) {
      for (int l = 0; l < S; ++l) limbs[l] = h[(size_t)l * stride + i];
      if (!bn::to_be(mc->value(limbs.data()), out + i * nsq_bytes, nsq_bytes))
        return fail(DDS_E_RANGE, "result does not fit");
    }
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_modexp_batch(dds_ctx* ctx, const uint8_t* mod_be, size_t mod_bytes, const uint8_t* exp_be, size_t exp_bytes,
                     const uint8_t* bases_be, size_t width, size_t count, uint8_t* out) {
  try {
    if (!ctx || !exp_be || width == 0 || (count && (!bases_be || !out))) return fail(DDS_E_ARG, "bad arguments");
    if (count == 0) return DDS_OK;
    std::shared_ptr<ModConsts> mc;
    int rc = get_mod(ctx, mod_be, mod_bytes, &mc);
    if (rc) return rc;
    bn::Limbs e = bn::from_be(exp_be, exp_bytes);
    if ((rc = check_rows(*mc, count))) return rc;
    WorkerLease wl(ctx);
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    const int S = mc->S;
    const size_t stride = round_up(count, 64);
    HIP_TRY(w->x.ensure((size_t)S * stride * 4));
    HIP_TRY(w->x2.ensure((size_t)S * stride * 4));
    if ((rc = ingest(ctx, w, wl.st, *mc, bases_be, width, count, w->in, w->x.as<uint32_t>(), stride))) return rc;
    if ((rc = modexp_device(w, wl.st, *mc, e, nullptr, w->x.as<uint32_t>(), stride, nullptr, count,
                            w->x2.as<uint32_t>(), stride)))
      return rc;
    std::vector<uint32_t> h((size_t)S * stride);
    HIP_TRY(hipMemcpyAsync(h.data(), w->x2.p, h.size() * 4, hipMemcpyDeviceToHost, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    std::vector<uint32_t> limbs(S);
    for (size_t i = 0; i < count; ++i) {
      for (int l = 0; l < S; ++l) limbs[l] = h[(size_t)l * stride + i];
      if (!bn::to_be(mc->value(limbs.data()), out + i * mod_bytes, mod_bytes))
        return fail(DDS_E_RANGE, "result does not fit");
    }
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

static uint64_t splitmix64_host(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

int dds_col_fill_paillier_synth(dds_col* col, const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be,
                                size_t g_bytes, uint64_t seed, uint64_t row0, size_t count, uint32_t pool_size) {
  return ddshe::host::col_fill_paillier_synth(col, n_be, n_bytes, g_be, g_bytes, seed, row0, count, pool_size, 1, 0);
}

}  // extern "C"

namespace ddshe {
namespace host {
int col_fill_paillier_synth(dds_col* col, const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be, size_t g_bytes,
                            uint64_t seed, uint64_t row0, size_t count, uint32_t pool_size, uint32_t shards,
                            uint32_t shard) {
  try {
    if (!col || !n_be || !g_be || pool_size == 0 || shards == 0 || shard >= shards) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    if (col->count + count > col->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    ModConsts& mc = *col->mc;
    bn::Limbs n = bn::from_be(n_be, n_bytes), g = bn::from_be(g_be, g_bytes);
    if (bn::cmp(bn::mul(n, n), mc.N) != 0) return fail(DDS_E_ARG, "column modulus is not n^2");
    const int S = mc.S;
    const uint32_t tcount = 10000;  // DDSDataGenerator.scala:274 Random.nextInt(10000)
    WorkerLease wl(col->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    hipStream_t st = wl.st;
    // table T[m] = g^m (encrypt kernel with r = 1 and exponent n disabled)
    const size_t ts = round_up(tcount, 64), ps = round_up(pool_size, 64);
    HIP_TRY(w->misc.ensure((size_t)S * ts * 4));                      // T
    HIP_TRY(w->misc2.ensure((size_t)S * ps * 4 * 2));                 // pool (plain) + pool (Montgomery)
    HIP_TRY(w->x.ensure((size_t)S * std::max(ts, ps) * 4));           // r column
    HIP_TRY(w->in2.ensure((size_t)std::max(ts, ps) * 4));             // exponents m
    std::vector<uint32_t> ones((size_t)S * ts, 0), ms(ts, 0);
    for (size_t i = 0; i < ts; ++i) ones[i] = 1;  // limb 0 = 1
    for (uint32_t i = 0; i < tcount; ++i) ms[i] = i;
    HIP_TRY(hipMemcpyAsync(w->x.p, ones.data(), ones.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(w->in2.p, ms.data(), ms.size() * 4, hipMemcpyHostToDevice, st));
    if ((rc = encrypt_device(w, st, mc, n, g, w->in2.as<uint32_t>(), w->x.as<uint32_t>(), ts, tcount,
                             w->misc.as<uint32_t>(), ts, false)))
      return rc;
    // pool P_j = r_j^n (encrypt with m = 0), r_j from seed
    std::vector<uint32_t> rcol((size_t)S * ps, 0), zeros(ps, 0);
    for (uint32_t j = 0; j < pool_size; ++j) {
      bn::Limbs r(n.size(), 0);
      for (size_t q = 0; q < r.size(); ++q)
        r[q] = (uint32_t)splitmix64_host(seed * 0x100000001B3ull + ((uint64_t)j << 20) + q);
      bn::trim(r);
      r = bn::mod(r, n);
      if (r.empty()) r = bn::Limbs{1};
      auto rl = mc.rw(r);
      for (int l = 0; l < S; ++l) rcol[(size_t)l * ps + j] = rl[l];
    }
    HIP_TRY(hipMemcpyAsync(w->x.p, rcol.data(), rcol.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(w->in2.p, zeros.data(), zeros.size() * 4, hipMemcpyHostToDevice, st));
    uint32_t* pool_plain = w->misc2.as<uint32_t>();
    uint32_t* pool_mont = pool_plain + (size_t)S * ps;
    if ((rc = encrypt_device(w, st, mc, n, g, w->in2.as<uint32_t>(), w->x.as<uint32_t>(), ps, pool_size,
                             pool_plain, ps, true)))
      return rc;
    // Montgomery form P*R mod N = pairs(P, R mod N)
    std::vector<uint32_t> rmod_col((size_t)S * ps, 0);
    for (int l = 0; l < S; ++l)
      for (size_t j = 0; j < ps; ++j) rmod_col[(size_t)l * ps + j] = mc.host[(size_t)kConstRmod * S + l];
    HIP_TRY(hipMemcpyAsync(w->x.p, rmod_col.data(), rmod_col.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_pairs(S, pool_plain, w->x.as<uint32_t>(), ps, pool_size, mc.d, mc.n0, pool_mont, st));
    HIP_TRY(launch_synth_rows(S, w->misc.as<uint32_t>(), ts, tcount, pool_mont, ps, pool_size, seed, row0, count, mc.d,
                              mc.n0, col->d + col->count, col->stride, st, shards, shard));
    HIP_TRY(hipStreamSynchronize(st));
    col->count += count;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}
}  // namespace host
}  // namespace ddshe

extern "C" {

int dds_paillier_encrypt_batch_crt(dds_ctx* ctx, const uint8_t* p_be, size_t p_bytes, const uint8_t* q_be,
                                   size_t q_bytes, const uint8_t* g_be, size_t g_bytes, const uint32_t* m,
                                   const uint8_t* r_be, size_t r_width, size_t count, uint8_t* out, size_t nsq_bytes) {
  try {
    if (!ctx || !p_be || !q_be || !g_be || r_width == 0 || (count && (!m || !r_be || !out)))
      return fail(DDS_E_ARG, "bad args");
    if (count == 0) return DDS_OK;
    std::shared_ptr<CrtKey> k;
    int rc = get_crt_key(ctx, bn::from_be(p_be, p_bytes), bn::from_be(q_be, q_bytes), &k);
    if (rc) return rc;
    ModConsts& mn = *k->mn;
    if (nsq_bytes < mn.bytes) return fail(DDS_E_BUFSIZE, "nsq_bytes too small");
    for (size_t i = 0; i < count; ++i) {  // r in [1, n): the CRT halves need r < 2^bits(n)
      bn::Limbs r = bn::from_be(r_be + i * r_width, r_width);
      if (r.empty() || bn::cmp(r, k->n) >= 0) return fail(DDS_E_RANGE, "r must be in [1, n)");
    }
    const bn::Limbs g = bn::from_be(g_be, g_bytes);
    if ((rc = check_rows(mn, count))) return rc;
    WorkerLease wl(ctx);
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    const int S = mn.S;
    const size_t stride = round_up(count, 64);
    HIP_TRY(w->x.ensure((size_t)S * stride * 4));
    HIP_TRY(w->x2.ensure((size_t)S * stride * 4));
    HIP_TRY(w->misc.ensure(count * 4));
    if ((rc = ingest(ctx, w, wl.st, mn, r_be, r_width, count, w->in, w->x.as<uint32_t>(), stride))) return rc;
    HIP_TRY(hipMemcpyAsync(w->misc.p, m, count * 4, hipMemcpyHostToDevice, wl.st));
    if (crt_fits(*k))
      rc = encrypt_crt_device(w, wl.st, *k, g, w->misc.as<uint32_t>(), w->x.as<uint32_t>(), stride, count,
                              w->x2.as<uint32_t>(), stride);
    else  // unbalanced factors: public-key path (same result)
      rc = encrypt_device(w, wl.st, mn, k->n, g, w->misc.as<uint32_t>(), w->x.as<uint32_t>(), stride, count,
                          w->x2.as<uint32_t>(), stride, true);
    if (rc) return rc;
    std::vector<uint32_t> h((size_t)S * stride);
    HIP_TRY(hipMemcpy(h.data(), w->x2.p, h.size() * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> limbs(S);
    for (size_t i = 0; i < count; ++i) {
      for (int l = 0; l < S; ++l) limbs[l] = h[(size_t)l * stride + i];
      if (!bn::to_be(mn.value(limbs.data()), out + i * nsq_bytes, nsq_bytes))
        return fail(DDS_E_RANGE, "result does not fit");
    }
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_fill_table_synth(dds_col* col, const uint8_t* table_be, size_t width, size_t tcount, uint64_t seed,
                             uint64_t row0, size_t count) {
  try {
    if (!col || !table_be || width == 0 || tcount == 0 || tcount > 0xFFFFFFFFu) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    if (col->count + count > col->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    WorkerLease wl(col->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    ModConsts& mc = *col->mc;
    const size_t ts = round_up(tcount, 64);
    HIP_TRY(w->misc.ensure((size_t)mc.S * ts * 4));
    if ((rc = ingest(col->ctx, w, wl.st, mc, table_be, width, tcount, w->in, w->misc.as<uint32_t>(), ts))) return rc;
    HIP_TRY(launch_gather_rows(w->misc.as<uint32_t>(), ts, (uint32_t)tcount, mc.S, seed, row0, count,
                               col->d + col->count, col->stride, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    col->count += count;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_fill_random(dds_col* col, size_t bits, uint64_t seed, uint64_t row0, size_t count) {
  try {
    if (!col || bits == 0) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    if (col->count + count > col->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    if (bits >= col->mc->bits) return fail(DDS_E_RANGE, "random rows must stay below the modulus");
    WorkerLease wl(col->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    HIP_TRY(launch_fill_random(col->d + col->count, col->stride, col->mc->S, col->mc->W, seed, row0, count, (int)bits,
                               wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    col->count += count;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_col_encrypt_paillier(dds_col* out, dds_col* rcol, size_t r_first, const uint32_t* d_m, size_t count,
                             const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be, size_t g_bytes,
                             const uint8_t* p_be, size_t p_bytes, const uint8_t* q_be, size_t q_bytes) {
  try {
    if (!out || !rcol || !n_be || !g_be || (count && !d_m) || (!p_be) != (!q_be)) return fail(DDS_E_ARG, "bad args");
    if (count == 0) return DDS_OK;
    if (r_first + count > rcol->count) return fail(DDS_E_ARG, "r rows out of range");
    std::unique_lock<std::shared_mutex> lk(out->mu, std::defer_lock);
    std::unique_lock<std::shared_mutex> lr(rcol->mu, std::defer_lock);
    if (out == rcol) return fail(DDS_E_ARG, "out and r columns must differ");
    std::lock(lk, lr);
    if (out->count + count > out->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    const bn::Limbs n = bn::from_be(n_be, n_bytes), g = bn::from_be(g_be, g_bytes);
    const bn::Limbs nsq = bn::mul(n, n);
    if (bn::cmp(nsq, out->mc->N) != 0 || bn::cmp(nsq, rcol->mc->N) != 0)
      return fail(DDS_E_ARG, "columns must be over n^2");
    std::shared_ptr<CrtKey> k;
    int rc;
    if (p_be) {
      if ((rc = get_crt_key(out->ctx, bn::from_be(p_be, p_bytes), bn::from_be(q_be, q_bytes), &k))) return rc;
      if (bn::cmp(k->n, n) != 0) return fail(DDS_E_ARG, "p*q != n");
    }
    WorkerLease wl(out->ctx);
    if ((rc = wl.acquire())) return rc;
    uint32_t* dst = out->d + out->count;
    const uint32_t* r = rcol->d + r_first;
    if (k && crt_fits(*k))
      rc = encrypt_crt_device(wl.w, wl.st, *k, g, d_m, r, rcol->stride, count, dst, out->stride);
    else
      rc = encrypt_device(wl.w, wl.st, *out->mc, n, g, d_m, r, rcol->stride, count, dst, out->stride, true);
    if (rc) return rc;
    out->count += count;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

// ---- OPE filter ------------------------------------------------------------------
int dds_ope_filter_device(dds_ctx* ctx, const int64_t* d_col, const uint8_t* d_valid, size_t n, int64_t bound, int op,
                          uint32_t* d_out, size_t* out_n) {
  try {
    if (!ctx || !out_n || op < 0 || op > 3 || (n && (!d_col || !d_out))) return fail(DDS_E_ARG, "bad arguments");
    if (n > 0xFFFFFFFFull) return fail(DDS_E_ARG, "row index exceeds 32 bits");
    *out_n = 0;
    if (n == 0) return DDS_OK;
    WorkerLease wl(ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    HIP_TRY(w->misc.ensure(ope_scratch_bytes(n)));
    MappedWords hw;  // the match count is stored by the scatter into coherent mapped host memory: no copy
    HIP_TRY(mapped_words(w, &hw));
    hw.h[kCountWord] = 0;  // no rows: no scatter block stores it
    record_time(ctx, w, wl.st, true, 2);
    HIP_TRY(launch_ope_filter(d_col, d_valid, n, bound, op, w->misc.p, hw.d + kCountWord, d_out, wl.st));
    record_time(ctx, w, wl.st, false, 2);
    HIP_TRY(hipStreamSynchronize(wl.st));
    const uint64_t total = hw.h[kCountWord];
    if (ctx->timing.load()) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, w->ev[2], w->ev[3]) == hipSuccess) {
        std::lock_guard<std::mutex> lk(ctx->tmu);
        ctx->total_ms += ms;
      }
    }
    *out_n = (size_t)total;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_ope_filter(dds_ctx* ctx, const int64_t* col, const uint8_t* valid, size_t n, int64_t bound, int op,
                   uint32_t* out_idx, size_t* out_n) {
  try {
    if (!ctx || !out_n || op < 0 || op > 3 || (n && (!col || !out_idx))) return fail(DDS_E_ARG, "bad arguments");
    *out_n = 0;
    if (n == 0) return DDS_OK;
    WorkerLease wl(ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    HIP_TRY(w->in.ensure(n * 8));
    HIP_TRY(w->in2.ensure(n));
    HIP_TRY(w->out.ensure(n * 4));
    HIP_TRY(hipMemcpyAsync(w->in.p, col, n * 8, hipMemcpyHostToDevice, wl.st));
    if (valid) HIP_TRY(hipMemcpyAsync(w->in2.p, valid, n, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    // run on the same worker's buffers through the device entry point
    const int64_t* dcol = w->in.as<int64_t>();
    const uint8_t* dvalid = valid ? w->in2.as<uint8_t>() : nullptr;
    uint32_t* dout = w->out.as<uint32_t>();
    size_t got = 0;
    if ((rc = dds_ope_filter_device(ctx, dcol, dvalid, n, bound, op, dout, &got))) return rc;
    if (got) HIP_TRY(hipMemcpy(out_idx, dout, got * 4, hipMemcpyDeviceToHost));
    *out_n = got;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

// ---- OPE ordering (OrderLS / OrderSL) ---------------------------------------------
int dds_ope_order_device(dds_ctx* ctx, const int64_t* d_col, const uint8_t* d_valid, size_t n, int descending,
                         uint32_t* d_out_idx) {
  try {
    if (!ctx || (n && (!d_col || !d_out_idx))) return fail(DDS_E_ARG, "bad arguments");
    if (n > 0xFFFFFFFFull) return fail(DDS_E_ARG, "row index exceeds 32 bits");
    if (n == 0) return DDS_OK;
    WorkerLease wl(ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    HIP_TRY(w->tab.ensure(rs_scratch_bytes(n)));
    MappedWords ow;
    HIP_TRY(mapped_words(w, &ow));
    HIP_TRY(launch_ope_order(d_col, d_valid, n, descending ? 1 : 0, w->tab.p, d_out_idx, wl.st, nullptr, &ow));
    HIP_TRY(hipStreamSynchronize(wl.st));
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_ope_order(dds_ctx* ctx, const int64_t* col, const uint8_t* valid, size_t n, int descending,
                  uint32_t* out_idx) {
  try {
    if (!ctx || (n && (!col || !out_idx))) return fail(DDS_E_ARG, "bad arguments");
    if (n == 0) return DDS_OK;
    WorkerLease wl(ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    HIP_TRY(w->in.ensure(n * 8));
    HIP_TRY(w->in2.ensure(n));
    HIP_TRY(w->out.ensure(n * 4));
    HIP_TRY(hipMemcpyAsync(w->in.p, col, n * 8, hipMemcpyHostToDevice, wl.st));
    if (valid) HIP_TRY(hipMemcpyAsync(w->in2.p, valid, n, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(w->tab.ensure(rs_scratch_bytes(n)));
    MappedWords ow;
    HIP_TRY(mapped_words(w, &ow));
    HIP_TRY(launch_ope_order(w->in.as<int64_t>(), valid ? w->in2.as<uint8_t>() : nullptr, n, descending ? 1 : 0,
                             w->tab.p, w->out.as<uint32_t>(), wl.st, nullptr, &ow));
    HIP_TRY(hipMemcpyAsync(out_idx, w->out.p, n * 4, hipMemcpyDeviceToHost, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

// ---- deterministic-equality scans: ddshe_strtab.cpp -------------------------------------

// ---- decimal route entry points ----------------------------------------------------
namespace {
int parse_values(const char* const* values, size_t count, std::vector<bn::Limbs>* mags, std::vector<bool>* negs) {
  mags->resize(count);
  negs->assign(count, false);
  for (size_t i = 0; i < count; ++i) {
    if (!values[i]) return fail(DDS_E_ARG, "NULL operand");
    bool neg = false;
    if (!bn::from_dec(values[i], strlen(values[i]), (*mags)[i], &neg))
      return fail(DDS_E_FORMAT, std::string("NumberFormatException: ") + values[i]);
    (*negs)[i] = neg;
  }
  return DDS_OK;
}

int write_dec(const std::string& s, char* out, size_t out_cap, size_t* out_len) {
  if (out_len) *out_len = s.size();
  if (!out || out_cap < s.size() + 1) return fail(DDS_E_BUFSIZE, "output buffer too small");
  memcpy(out, s.c_str(), s.size() + 1);
  return DDS_OK;
}

// shared by SumAll (nsqr) and MultAll (pubkey modulus): acc = prod mod M over decimal operands
// Modular SumAll / MultAll over decimal rows (DDSRestServer.scala:412-430, 506-524): rows are
// parsed on the GPU (ingest_dec) straight into a device column, then folded. Rows the column
// cannot hold (|x| >= 2^(W*S): never a well-formed ciphertext) are reduced exactly on the host
// at the boundary so the result keeps BigInteger semantics.
int fold_dec_mod(dds_ctx* ctx, const char* const* values, size_t count, const char* mod_dec, char* out,
                 size_t out_cap, size_t* out_len) {
  bn::Limbs M;
  bool mneg = false;
  if (!bn::from_dec(mod_dec, strlen(mod_dec), M, &mneg) || mneg || M.empty())
    return fail(DDS_E_FORMAT, "modulus: NumberFormatException / non-positive");
  if (!(M[0] & 1u) || bn::bit_length(M) < 2) {  // even modulus or 1 (BigInteger.mod accepts any m > 0)
    std::vector<bn::Limbs> mags;
    std::vector<bool> negs;
    int rc = parse_values(values, count, &mags, &negs);
    if (rc) return rc;
    bn::Limbs r;
    if ((rc = fold_even_modulus(ctx, M, mags, negs, &r))) return rc;
    return write_dec(bn::to_dec(r), out, out_cap, out_len);
  }
  const size_t mb = bn::byte_length(M);
  std::vector<uint8_t> mbe(mb);
  bn::to_be(M, mbe.data(), mb);
  std::shared_ptr<ModConsts> mc;
  int rc = get_mod(ctx, mbe.data(), mb, &mc);
  if (rc) return rc;
  if ((rc = check_rows(*mc, count))) return rc;
  WorkerLease wl(ctx);
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  const size_t stride = round_up(count, 64);
  HIP_TRY(w->x.ensure((size_t)mc->S * stride * 4));
  uint32_t* X = w->x.as<uint32_t>();
  DecRows src;
  src.strs = values;
  uint32_t fl = 0;
  std::vector<size_t> host_rows;
  if ((rc = ingest_dec(w, wl.st, *mc, src, count, X, stride, &fl, &host_rows))) return rc;
  if (fl & kDecFormat) {
    std::vector<size_t> bad;
    if ((rc = dec_rows_with(w, wl.st, count, kDecFormat, &bad))) return rc;
    return fail(DDS_E_FORMAT, std::string("NumberFormatException: row ") + std::to_string(bad.empty() ? 0 : bad[0]));
  }
  if (fl & kDecWide)
    if ((rc = dec_rows_with(w, wl.st, count, kDecWide, &host_rows))) return rc;
  std::vector<uint32_t> fixed;  // limbs of the host-reduced rows; alive until the copies complete
  fixed.reserve(host_rows.size() * mc->S);
  for (size_t i : host_rows) {
    bn::Limbs x;
    bool neg = false;
    if (!bn::from_dec(values[i], strlen(values[i]), x, &neg))
      return fail(DDS_E_FORMAT, std::string("NumberFormatException: row ") + std::to_string(i));
    x = bn::mod(x, M);
    if (neg && !x.empty()) x = bn::sub(M, x);
    std::vector<uint32_t> rw = mc->rw(x);
    fixed.insert(fixed.end(), rw.begin(), rw.end());
  }
  for (size_t k = 0; k < host_rows.size(); ++k)
    HIP_TRY(hipMemcpy2DAsync(X + host_rows[k], stride * 4, fixed.data() + k * mc->S, 4, 4, (size_t)mc->S,
                             hipMemcpyHostToDevice, wl.st));
  if (!host_rows.empty()) HIP_TRY(hipStreamSynchronize(wl.st));
  bn::Limbs v;
  if ((rc = fold_value_device(ctx, w, wl.st, *mc, X, stride, count, nullptr, &v))) return rc;
  return write_dec(bn::to_dec(v), out, out_cap, out_len);
}

int fold_dec(dds_ctx* ctx, const char* const* values, size_t count, const char* mod_dec, bool additive, char* out,
             size_t out_cap, size_t* out_len) {
  if (!ctx || (count && !values)) return fail(DDS_E_ARG, "bad arguments");
  if (count == 0) return fail(DDS_E_EMPTY, "no operand");
  for (size_t i = 0; i < count; ++i)
    if (!values[i]) return fail(DDS_E_ARG, "NULL operand");
  if (mod_dec && count > 1) return fold_dec_mod(ctx, values, count, mod_dec, out, out_cap, out_len);
  std::vector<bn::Limbs> mags;
  std::vector<bool> negs;
  int rc = parse_values(values, count, &mags, &negs);
  if (rc) return rc;
  if (count == 1) return write_dec(bn::to_dec(mags[0], negs[0]), out, out_cap, out_len);  // unreduced (:416-417)
  if (!mod_dec && !additive) {  // unbounded product (DDSRestServer.scala:520) on the GPU product tree
    size_t width = 1;
    bool neg = false;
    for (size_t i = 0; i < count; ++i) {
      width = std::max(width, bn::byte_length(mags[i]));
      neg ^= (bool)negs[i];
    }
    std::vector<uint8_t> ops(count * width);
    for (size_t i = 0; i < count; ++i) bn::to_be(mags[i], ops.data() + i * width, width);
    std::vector<uint8_t> buf(count * width + 8);
    size_t len = 0;
    if ((rc = dds_bigint_product(ctx, ops.data(), width, count, buf.data(), buf.size(), &len))) return rc;
    bn::Limbs r = bn::from_be(buf.data(), len);
    return write_dec(bn::to_dec(r, neg && !r.empty()), out, out_cap, out_len);
  }
  if (!mod_dec) {
    // plain sum: positives and negatives summed separately on the GPU
    size_t width = 1;
    for (auto& m : mags) width = std::max(width, bn::byte_length(m));
    std::vector<uint8_t> pos, neg;
    size_t npos = 0, nneg = 0;
    for (size_t i = 0; i < count; ++i) {
      auto& dst = negs[i] ? neg : pos;
      size_t off = dst.size();
      dst.resize(off + width);
      bn::to_be(mags[i], dst.data() + off, width);
      (negs[i] ? nneg : npos)++;
    }
    bn::Limbs sp, sn;
    std::vector<uint8_t> buf(width + 16);
    size_t len = 0;
    if (npos) {
      if ((rc = dds_bigint_sum(ctx, pos.data(), width, npos, buf.data(), buf.size(), &len))) return rc;
      sp = bn::from_be(buf.data(), len);
    }
    if (nneg) {
      if ((rc = dds_bigint_sum(ctx, neg.data(), width, nneg, buf.data(), buf.size(), &len))) return rc;
      sn = bn::from_be(buf.data(), len);
    }
    const bool rneg = bn::cmp(sp, sn) < 0;
    bn::Limbs r = rneg ? bn::sub(sn, sp) : bn::sub(sp, sn);
    return write_dec(bn::to_dec(r, rneg), out, out_cap, out_len);
  }
  return fold_dec_mod(ctx, values, count, mod_dec, out, out_cap, out_len);
}
}  // namespace

int dds_sum_all_dec(dds_ctx* ctx, const char* const* values, size_t count, const char* nsqr_dec, char* out,
                    size_t out_cap, size_t* out_len) {
  try {
    return fold_dec(ctx, values, count, nsqr_dec, true, out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mult_all_dec(dds_ctx* ctx, const char* const* values, size_t count, const char* n_dec, char* out,
                     size_t out_cap, size_t* out_len) {
  try {
    return fold_dec(ctx, values, count, n_dec, false, out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

}  // extern "C"
