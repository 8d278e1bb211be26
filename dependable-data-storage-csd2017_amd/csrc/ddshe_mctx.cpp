// Multi-device context (include/ddshe.h, dds_mctx_* / dds_mcol_*): one C-ABI caller — the JVM proxy
// process whose routes run on a ForkJoin pool (DDSRestServer.scala:21) — drives every GPU of a node.
//
// A sharded column (dds_mcol) spreads its rows over the shards in 64-row blocks, round-robin:
// global row r lives on shard (r/64) % G at local row ((r/64)/G)*64 + r%64, so every shard holds a
// contiguous key range per block and incremental appends stay balanced. (A column created whole and
// never appended to could be cut into G contiguous ranges instead; the reference's PutSet arrives one
// set at a time (DDSRestServer.scala:170-188), and contiguous ranges would put every new row on the
// last shard until it fills, so the fold would run on one GPU. The 64-row blocks keep each shard's
// reads of a block one 256-byte line per limb, the same coalescing a contiguous range gives.)
// A fold (SumAll / MultAll, :412-430, :506-524) runs each shard's first level + tree on its own device
// and stream — from one host thread per shard when the fold is large enough for the thread start to
// be noise — packs the shard's partial, copies it device-to-device into the combining device
// (hipMemcpyPeerAsync over xGMI between distinct GPUs), and the combining device's stream waits on one
// event per shard before the last tree over the G partials and the finalize. The only host round trip
// is the result (plus one count read-back per shard holding removed rows, dds_mcol_set_live).
#include "ddshe_host.hpp"

using namespace ddshe;
using namespace ddshe::host;

struct dds_mctx {
  std::vector<dds_ctx*> shards;  // owned; shards[0] combines
  std::vector<int> devices;
  ~dds_mctx() {
    for (auto c : shards) dds_ctx_destroy(c);
  }
};

struct dds_mcol {
  dds_mctx* m = nullptr;
  std::vector<dds_col*> cols;  // one per shard, owned
  size_t capacity = 0, count = 0;
  size_t mod_bytes = 0;
  // shared by folds, exclusive for appends / writes / liveness; taken before any shard column's lock
  std::shared_mutex mu;
  ~dds_mcol() {
    for (auto c : cols) dds_col_destroy(c);
  }
};

namespace {

struct DeviceGuard {  // the caller's current device survives a multi-device call
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

inline size_t shard_of(size_t r, size_t G) { return (r >> 6) % G; }
inline size_t local_of(size_t r, size_t G) { return (((r >> 6) / G) << 6) | (r & 63); }
// rows of shard s among global rows [0, n)
inline size_t rows_on(size_t n, size_t G, size_t s) {
  const size_t cyc = 64 * G, full = n / cyc, rem = n % cyc;
  const size_t lo = 64 * s;
  return full * 64 + (rem > lo ? std::min<size_t>(64, rem - lo) : 0);
}

// run fn(s) for every shard on its own host thread; the first failure's status and message win
template <class F>
int for_shards(size_t G, F&& fn) {
  std::vector<int> rc(G, DDS_OK);
  std::vector<std::string> msg(G);
  std::vector<std::thread> th;
  for (size_t s = 0; s < G; ++s)
    th.emplace_back([&, s] {
      rc[s] = fn(s);
      if (rc[s]) msg[s] = dds_last_error();
    });
  for (auto& t : th) t.join();
  for (size_t s = 0; s < G; ++s)
    if (rc[s]) return fail(rc[s], "shard " + std::to_string(s) + ": " + msg[s]);
  return DDS_OK;
}

// Undo a partially applied append: every shard back to the row count it had before.
void rollback(dds_mcol* mc, const std::vector<size_t>& before) {
  for (size_t s = 0; s < mc->cols.size(); ++s) (void)dds_col_truncate(mc->cols[s], before[s]);
}

constexpr size_t kPackBytes = (size_t)64 << 20;  // host staging per shard append call
// folds of at least this many rows set up their shards from one host thread each (a thread start costs
// tens of µs, a shard's host-side set-up — occupancy queries, buffers, a count read-back per shard
// with removed rows — about as much; below it the shards are issued from the calling thread)
constexpr size_t kThreadedFoldRows = (size_t)1 << 16;

// SumAll / MultAll over a sharded column: the live rows among ids[0..n) (global ids) or of all rows.
// Caller holds mcol->mu (shared).
int mcol_fold(dds_mcol* mcol, const uint64_t* ids, size_t n, bn::Limbs* v, bool* neg) {
  *neg = false;
  const size_t G = mcol->cols.size();
  std::vector<std::shared_lock<std::shared_mutex>> locks;  // shard rows stay put during the fold
  for (auto c : mcol->cols) locks.emplace_back(c->mu);
  std::vector<std::vector<uint64_t>> lids(G);
  std::vector<size_t> cnt(G, 0);
  if (ids) {
    for (size_t i = 0; i < n; ++i) {
      if (ids[i] >= mcol->count) return fail(DDS_E_ARG, "row id " + std::to_string(ids[i]) + " out of range");
      lids[shard_of(ids[i], G)].push_back(local_of(ids[i], G));
    }
    for (size_t s = 0; s < G; ++s) {
      if (mcol->cols[s]->ndead) lids[s] = col_live_ids(mcol->cols[s], lids[s].data(), lids[s].size());
      cnt[s] = lids[s].size();
    }
  } else {
    for (size_t s = 0; s < G; ++s) cnt[s] = mcol->cols[s]->count - mcol->cols[s]->ndead;
  }
  size_t k = 0;
  std::vector<size_t> act;
  for (size_t s = 0; s < G; ++s) {
    k += cnt[s];
    if (cnt[s]) act.push_back(s);
  }
  if (k == 0) return fail(DDS_E_EMPTY, "no operand");
  if (act.size() == 1) {  // one shard holds every live operand (k == 1: the original operand)
    const size_t s = act[0];
    dds_col* col = mcol->cols[s];
    return ids ? col_fold_value(col, lids[s].data(), 0, cnt[s], v, neg) : col_fold_value(col, nullptr, 0, col->count, v, neg);
  }
  DeviceGuard dg;
  ModConsts& mc0 = *mcol->cols[0]->mc;
  const size_t S2 = (size_t)mc0.S2, na = act.size();
  dds_ctx* c0 = mcol->m->shards[0];
  WorkerLease l0(c0);
  int rc;
  if ((rc = l0.acquire())) return rc;
  HIP_TRY(l0.w->gather.ensure(na * S2 * 4));
  uint32_t* gather = l0.w->gather.as<uint32_t>();
  std::vector<std::unique_ptr<WorkerLease>> ls(na);
  std::vector<std::vector<uint32_t>> ids32(na);  // alive until the final synchronisation
  std::vector<int64_t> Es(na, 0);
  auto shard_part = [&](size_t j) -> int {
    const size_t s = act[j];
    dds_col* col = mcol->cols[s];
    dds_ctx* cs = col->ctx;
    ls[j].reset(new WorkerLease(cs));
    WorkerLease& l = *ls[j];
    int r;
    if ((r = l.acquire())) return r;
    const uint32_t* d_ids = nullptr;
    size_t rows = cnt[s];
    if (ids) {
      ids32[j].assign(lids[s].begin(), lids[s].end());
      HIP_TRY(l.w->ids.ensure(rows * 4));
      HIP_TRY(hipMemcpyAsync(l.w->ids.p, ids32[j].data(), rows * 4, hipMemcpyHostToDevice, l.st));
      d_ids = l.w->ids.as<uint32_t>();
    } else if ((r = col_live_range(col, l.w, l.st, 0, col->count, &d_ids, &rows))) {
      return r;
    }
    const uint32_t* part;
    size_t ps;
    if ((r = fold_partial_device(cs, l.w, l.st, *col->mc, col->d, col->stride, rows, &part, &ps, &Es[j], d_ids)))
      return r;
    // pack the partial (S2 limbs at stride ps) into S2 consecutive words, then device-to-device
    HIP_TRY(l.w->pk.ensure(S2 * 4));
    HIP_TRY(launch_strided_copy(part, 0, ps, l.w->pk.as<uint32_t>(), 0, 1, 1, S2, l.st));
    HIP_TRY(hipMemcpyPeerAsync(gather + j * S2, c0->device, l.w->pk.p, cs->device, S2 * 4, l.st));
    HIP_TRY(hipEventRecord(l.w->ev_peer, l.st));
    return DDS_OK;
  };
  if (k >= kThreadedFoldRows) {
    rc = for_shards(na, shard_part);
  } else {
    for (size_t j = 0; j < na && !rc; ++j) rc = shard_part(j);
  }
  if (rc) return rc;
  int64_t E = 0;  // sum of the shard exponents (reduce_leaves accounts for its own products)
  for (int64_t e : Es) E += e;
  HIP_TRY(hipSetDevice(c0->device));
  for (auto& l : ls) HIP_TRY(hipStreamWaitEvent(l0.st, l->w->ev_peer, 0));
  // rows of packed partials -> the limb-major layout of the tree levels
  const size_t stride = round_up(na, 64);
  Worker* w0 = l0.w;
  HIP_TRY(w0->x.ensure(S2 * stride * 4));
  HIP_TRY(launch_strided_copy(gather, S2, 1, w0->x.as<uint32_t>(), 1, stride, na, S2, l0.st));
  const Leaves lv{w0->x.as<uint32_t>(), stride, (int)S2, mc0.W, na, E, nullptr};
  if ((rc = reduce_leaves(c0, w0, l0.st, mc0, lv, true, v, nullptr, nullptr))) return rc;
  for (auto& l : ls) account_fold(l->ctx, l->w);
  return DDS_OK;
}

// Global row ids -> per-shard local ids (validated against the row count)
int split_ids(dds_mcol* c, const uint64_t* ids, size_t n, std::vector<std::vector<uint64_t>>* lids,
              std::vector<std::vector<size_t>>* pos) {
  const size_t G = c->cols.size();
  lids->assign(G, {});
  pos->assign(G, {});
  for (size_t i = 0; i < n; ++i) {
    if (ids[i] >= c->count) return fail(DDS_E_ARG, "row id " + std::to_string(ids[i]) + " out of range");
    const size_t s = shard_of(ids[i], G);
    (*lids)[s].push_back(local_of(ids[i], G));
    (*pos)[s].push_back(i);
  }
  return DDS_OK;
}

// dds_mcol_write_rows[_dec]: every shard's new rows are prepared (ingested, validated) before any is
// committed, so a validation error (range, format, row id) leaves the whole column unchanged. A HIP
// error during a commit (scatter / sync) can leave earlier shards committed: the column is then in an
// undefined state and the caller must treat DDS_E_HIP from here as fatal to it.
int mcol_write(dds_mcol* c, const uint64_t* ids, size_t n, const uint8_t* ops, size_t width, const char* chars,
               const uint64_t* offsets) {
  std::unique_lock<std::shared_mutex> lk(c->mu);
  std::vector<std::vector<uint64_t>> lids;
  std::vector<std::vector<size_t>> pos;
  int rc = split_ids(c, ids, n, &lids, &pos);
  if (rc) return rc;
  DeviceGuard dg;
  const size_t G = c->cols.size();
  std::vector<std::unique_lock<std::shared_mutex>> locks;
  for (auto col : c->cols) locks.emplace_back(col->mu);
  std::vector<RowWrite> plans(G);
  for (size_t s = 0; s < G; ++s) {
    if (lids[s].empty()) continue;
    const size_t m = lids[s].size();
    if (ops) {
      std::vector<uint8_t> buf(m * width);
      for (size_t j = 0; j < m; ++j) memcpy(buf.data() + j * width, ops + pos[s][j] * width, width);
      rc = col_write_prepare(c->cols[s], lids[s].data(), m, buf.data(), width, nullptr, nullptr, &plans[s]);
    } else {
      std::vector<char> ch;
      std::vector<uint64_t> of(1, 0);
      for (size_t j = 0; j < m; ++j) {
        const size_t i = pos[s][j];
        if (offsets[i + 1] < offsets[i]) return fail(DDS_E_ARG, "offsets must be non-decreasing");
        ch.insert(ch.end(), chars + offsets[i], chars + offsets[i + 1]);
        of.push_back(ch.size());
      }
      ch.push_back('\0');
      rc = col_write_prepare(c->cols[s], lids[s].data(), m, nullptr, 0, ch.data(), of.data(), &plans[s]);
    }
    if (rc) return rc;
  }
  for (size_t s = 0; s < G; ++s)
    if ((rc = col_write_commit(c->cols[s], plans[s]))) return rc;
  return DDS_OK;
}

}  // namespace

extern "C" {

int dds_mctx_create_devices(const int* devices, size_t ndevices, dds_mctx** out) {
  try {
    if (!out || !devices || ndevices == 0 || ndevices > 64) return fail(DDS_E_ARG, "bad arguments");
    *out = nullptr;
    DeviceGuard dg;
    std::unique_ptr<dds_mctx> m(new dds_mctx());
    for (size_t i = 0; i < ndevices; ++i) {
      dds_ctx* c = nullptr;
      int rc = dds_ctx_create(devices[i], &c);
      if (rc) return rc;
      m->shards.push_back(c);
      m->devices.push_back(devices[i]);
    }
    // direct xGMI copies between the combining device and every other one (both directions)
    const int d0 = devices[0];
    for (size_t i = 1; i < ndevices; ++i) {
      const int d = devices[i];
      if (d == d0) continue;
      int ok = 0;
      if (hipDeviceCanAccessPeer(&ok, d, d0) == hipSuccess && ok) {
        HIP_TRY(hipSetDevice(d));
        hipError_t e = hipDeviceEnablePeerAccess(d0, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(DDS_E_HIP, "hipDeviceEnablePeerAccess");
        (void)hipGetLastError();
      }
      if (hipDeviceCanAccessPeer(&ok, d0, d) == hipSuccess && ok) {
        HIP_TRY(hipSetDevice(d0));
        hipError_t e = hipDeviceEnablePeerAccess(d, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(DDS_E_HIP, "hipDeviceEnablePeerAccess");
        (void)hipGetLastError();
      }
    }
    *out = m.release();
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mctx_create(uint64_t device_mask, dds_mctx** out) {
  std::vector<int> devs;
  for (int d = 0; d < 64; ++d)
    if ((device_mask >> d) & 1u) devs.push_back(d);
  if (devs.empty()) return fail(DDS_E_ARG, "empty device mask");
  return dds_mctx_create_devices(devs.data(), devs.size(), out);
}

int dds_mctx_destroy(dds_mctx* m) {
  delete m;
  return DDS_OK;
}

size_t dds_mctx_shards(const dds_mctx* m) { return m ? m->shards.size() : 0; }

int dds_mcol_create(dds_mctx* m, const uint8_t* mod_be, size_t mod_bytes, size_t capacity, dds_mcol** out) {
  try {
    if (!m || !out || capacity == 0) return fail(DDS_E_ARG, "bad arguments");
    *out = nullptr;
    DeviceGuard dg;
    std::unique_ptr<dds_mcol> c(new dds_mcol());
    c->m = m;
    c->capacity = capacity;
    const size_t G = m->shards.size();
    for (size_t s = 0; s < G; ++s) {
      dds_col* col = nullptr;
      int rc = dds_col_create(m->shards[s], mod_be, mod_bytes, std::max<size_t>(64, rows_on(capacity, G, s)), &col);
      if (rc) return rc;
      c->cols.push_back(col);
    }
    c->mod_bytes = c->cols[0]->mc->bytes;
    *out = c.release();
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mcol_destroy(dds_mcol* c) {
  DeviceGuard dg;
  delete c;
  return DDS_OK;
}

size_t dds_mcol_count(const dds_mcol* c) { return c ? c->count : 0; }

size_t dds_mcol_live_count(dds_mcol* c) {
  if (!c) return 0;
  std::shared_lock<std::shared_mutex> lk(c->mu);
  size_t n = 0;
  for (auto col : c->cols) n += dds_col_live_count(col);
  return n;
}

int dds_mcol_write_rows(dds_mcol* c, const uint64_t* row_ids, size_t n, const uint8_t* operands_be, size_t width) {
  try {
    if (!c || (n && (!row_ids || !operands_be || width == 0))) return fail(DDS_E_ARG, "bad arguments");
    return mcol_write(c, row_ids, n, operands_be, width, nullptr, nullptr);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mcol_write_rows_dec(dds_mcol* c, const uint64_t* row_ids, size_t n, const char* chars,
                            const uint64_t* offsets) {
  try {
    if (!c || (n && (!row_ids || !chars || !offsets))) return fail(DDS_E_ARG, "bad arguments");
    return mcol_write(c, row_ids, n, nullptr, 0, chars, offsets);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mcol_set_live(dds_mcol* c, const uint64_t* row_ids, size_t n, const uint8_t* live) {
  try {
    if (!c || (n && (!row_ids || !live))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(c->mu);
    std::vector<std::vector<uint64_t>> lids;
    std::vector<std::vector<size_t>> pos;
    int rc = split_ids(c, row_ids, n, &lids, &pos);
    if (rc) return rc;
    DeviceGuard dg;
    for (size_t s = 0; s < c->cols.size(); ++s) {
      if (lids[s].empty()) continue;
      std::vector<uint8_t> f(lids[s].size());
      for (size_t j = 0; j < f.size(); ++j) f[j] = live[pos[s][j]];
      std::unique_lock<std::shared_mutex> lc(c->cols[s]->mu);
      if ((rc = col_set_live(c->cols[s], lids[s].data(), f.size(), f.data()))) return rc;
    }
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mcol_append(dds_mcol* c, const uint8_t* ops, size_t width, size_t count) {
  try {
    if (!c || width == 0 || (count && !ops)) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(c->mu);
    if (c->count + count > c->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    if (count == 0) return DDS_OK;
    DeviceGuard dg;
    const size_t G = c->cols.size(), c0 = c->count, c1 = c0 + count;
    std::vector<size_t> before(G);
    for (size_t s = 0; s < G; ++s) before[s] = dds_col_count(c->cols[s]);
    const size_t per = std::max<size_t>(64, kPackBytes / width / 64 * 64);
    int rc = for_shards(G, [&](size_t s) -> int {
      std::vector<uint8_t> buf;
      buf.reserve(std::min(per, count) * width);
      size_t rows = 0;
      for (size_t q = c0 >> 6; (q << 6) < c1; ++q) {  // the 64-row blocks of [c0, c1) on shard s
        if (q % G != s) continue;
        const size_t a = std::max(c0, q << 6), b = std::min(c1, (q + 1) << 6);
        buf.insert(buf.end(), ops + (a - c0) * width, ops + (b - c0) * width);
        rows += b - a;
        if (rows >= per) {
          if (int r = dds_col_append(c->cols[s], buf.data(), width, rows)) return r;
          buf.clear();
          rows = 0;
        }
      }
      return rows ? dds_col_append(c->cols[s], buf.data(), width, rows) : DDS_OK;
    });
    if (rc) {
      rollback(c, before);
      return rc;
    }
    c->count = c1;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mcol_append_dec(dds_mcol* c, const char* chars, const uint64_t* offsets, size_t count) {
  try {
    if (!c || (count && (!chars || !offsets))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(c->mu);
    if (c->count + count > c->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    if (count == 0) return DDS_OK;
    for (size_t i = 0; i < count; ++i)
      if (offsets[i + 1] < offsets[i]) return fail(DDS_E_ARG, "offsets must be non-decreasing");
    DeviceGuard dg;
    const size_t G = c->cols.size(), c0 = c->count, c1 = c0 + count;
    std::vector<size_t> before(G);
    for (size_t s = 0; s < G; ++s) before[s] = dds_col_count(c->cols[s]);
    int rc = for_shards(G, [&](size_t s) -> int {
      std::vector<char> ch;
      std::vector<uint64_t> of{0};
      auto flush = [&]() -> int {
        const size_t rows = of.size() - 1;
        int r = rows ? dds_col_append_dec(c->cols[s], ch.data(), of.data(), rows) : DDS_OK;
        ch.clear();
        of.assign(1, 0);
        return r;
      };
      for (size_t q = c0 >> 6; (q << 6) < c1; ++q) {
        if (q % G != s) continue;
        const size_t a = std::max(c0, q << 6), b = std::min(c1, (q + 1) << 6);
        for (size_t r = a; r < b; ++r) {
          const size_t i = r - c0;
          ch.insert(ch.end(), chars + offsets[i], chars + offsets[i + 1]);
          of.push_back(ch.size());
        }
        if (ch.size() >= kPackBytes)
          if (int r = flush()) return r;
      }
      return flush();
    });
    if (rc) {
      rollback(c, before);
      return rc;
    }
    c->count = c1;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mcol_fill_paillier_synth(dds_mcol* c, const uint8_t* n_be, size_t n_bytes, const uint8_t* g_be, size_t g_bytes,
                                 uint64_t seed, size_t count, uint32_t pool_size) {
  try {
    if (!c) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(c->mu);
    if (c->count + count > c->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    DeviceGuard dg;
    const size_t G = c->cols.size(), c0 = c->count, c1 = c0 + count;
    std::vector<size_t> before(G);
    for (size_t s = 0; s < G; ++s) before[s] = dds_col_count(c->cols[s]);
    int rc = for_shards(G, [&](size_t s) -> int {
      const size_t a = rows_on(c0, G, s), b = rows_on(c1, G, s);
      if (b == a) return DDS_OK;
      return col_fill_paillier_synth(c->cols[s], n_be, n_bytes, g_be, g_bytes, seed, a, b - a, pool_size,
                                     (uint32_t)G, (uint32_t)s);
    });
    if (rc) {
      rollback(c, before);
      return rc;
    }
    c->count = c1;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mcol_fold(dds_mcol* c, uint8_t* out, size_t out_cap, size_t* out_len) {
  return dds_mcol_fold_rows(c, nullptr, 0, out, out_cap, out_len);
}

int dds_mcol_fold_rows(dds_mcol* c, const uint64_t* row_ids, size_t n, uint8_t* out, size_t out_cap, size_t* out_len) {
  try {
    if (!c) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(c->mu);
    bn::Limbs v;
    bool neg = false;
    int rc = mcol_fold(c, row_ids, n, &v, &neg);
    if (rc) return rc;
    if (neg) return fail(DDS_E_RANGE, "the single operand is negative: use dds_mcol_fold_dec");
    return emit_be(v, std::max(c->mod_bytes, bn::byte_length(v)), out, out_cap, out_len);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_mcol_fold_dec(dds_mcol* c, const uint64_t* row_ids, size_t n, char* out, size_t out_cap, size_t* out_len) {
  try {
    if (!c) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(c->mu);
    bn::Limbs v;
    bool neg = false;
    int rc = mcol_fold(c, row_ids, n, &v, &neg);
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

}  // extern "C"
