// Resident string table (include/ddshe.h, dds_strtab_*): the contents of the stored sets kept in HBM
// across requests for the deterministic-equality scans
//   SearchEq / SearchNEq   DDSRestServer.scala:607-681
//   SearchEntry / OR / AND DDSRestServer.scala:831-938
//   IsElement              DDSRestServer.scala:322-353
// and following the write routes (PutSet :170-205, AddElement :220-255, WriteElement :281-321, RemoveSet
// :207-218) in place, as the resident ciphertext and OPE columns do: a write gives its row a new
// version of the set's contents, RemoveSet clears the row's live byte (the register holds None, which
// every route filters out, filter(nonEmpty) :619, :843) and a later PutSet of the same key revives it.
//
// Layout (ddshe_strscan.hip): an element heap (chars, elem_off, a fingerprint and the owning row per
// element) and per row its current version (row_beg, row_len) and live byte. A write appends the new
// versions to the heap and kills the old ones (their elements' owner becomes kStrDead, so a scan skips
// them); when the heap is out of room, the current versions are compacted into fresh buffers sized
// 1.5x what they hold, so scans stream at most about 1.5x the live elements. SearchEq's position
// indexes (one per recently queried position) are patched by every write rather than rebuilt.
//
// Concurrency: scans share the table lock (std::shared_mutex) and run on their own worker streams;
// writes take it exclusively and synchronise before returning. The position-index cache has its own
// mutex; an index in use stays alive (shared_ptr) until its query has synchronised.
#include <shared_mutex>

#include "ddshe_host.hpp"

using namespace ddshe;
using namespace ddshe::host;

namespace {
template <class T>
hipError_t dalloc(T** p, size_t n) {
  *p = nullptr;
  return hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(n, 1) * sizeof(T));
}
template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

struct PosIdx {
  uint64_t position = 0;
  StrFp* fp = nullptr;
  uint64_t* present = nullptr;
  ~PosIdx() {
    dfree(fp);
    dfree(present);
  }
};
}  // namespace

struct dds_strtab {
  dds_ctx* ctx = nullptr;
  // rows
  size_t nrows = 0, rcap = 0, nlive = 0;
  uint64_t* row_beg = nullptr;
  uint32_t* row_len = nullptr;
  uint8_t* live = nullptr;
  std::vector<uint64_t> h_beg, h_bytes;  // host mirror: first heap element, bytes of the current version
  std::vector<uint32_t> h_len;
  std::vector<uint8_t> h_live;
  // element heap
  size_t nheap = 0, ecap = 0, nchars = 0, ccap = 0;
  size_t vel = 0, vch = 0;  // elements / bytes of the rows' current versions (dead rows' included)
  uint8_t* chars = nullptr;
  uint64_t* elem_off = nullptr;  // nheap + 1 entries in use (elem_off[nheap] == nchars)
  StrFp* fp = nullptr;
  uint32_t* elem_row = nullptr;
  uint64_t compactions = 0;
  // SearchEq position indexes, most recent last (sized rcap)
  static constexpr size_t kPosIdx = 8;
  std::vector<std::shared_ptr<PosIdx>> pos;
  std::mutex posmu;
  std::shared_mutex mu;
  ~dds_strtab() {
    dfree(row_beg);
    dfree(row_len);
    dfree(live);
    dfree(chars);
    dfree(elem_off);
    dfree(fp);
    dfree(elem_row);
  }
};

namespace {
constexpr size_t kStrMinCap = 1024;

// Grow the row arrays to hold `need` rows (copying the rows in use); position indexes are sized to the
// row capacity, so they are dropped (rebuilt on their next query).
int grow_rows(dds_strtab* t, size_t need, hipStream_t st) {
  if (need <= t->rcap) return DDS_OK;
  const size_t cap = std::max({need, t->rcap + t->rcap / 2, kStrMinCap});
  uint64_t* b = nullptr;
  uint32_t* l = nullptr;
  uint8_t* v = nullptr;
  if (dalloc(&b, cap) != hipSuccess || dalloc(&l, cap) != hipSuccess || dalloc(&v, cap) != hipSuccess) {
    dfree(b);
    dfree(l);
    dfree(v);
    return fail(DDS_E_NOMEM, "string table rows");
  }
  if (t->nrows) {
    HIP_TRY(hipMemcpyAsync(b, t->row_beg, t->nrows * 8, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(l, t->row_len, t->nrows * 4, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(v, t->live, t->nrows, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  dfree(t->row_beg);
  dfree(t->row_len);
  dfree(t->live);
  t->row_beg = b;
  t->row_len = l;
  t->live = v;
  t->rcap = cap;
  std::lock_guard<std::mutex> lk(t->posmu);
  t->pos.clear();
  return DDS_OK;
}

// Move every row's current version into fresh heap buffers with room for `ecap` elements and `ccap`
// bytes; superseded versions are dropped.
int compact(dds_strtab* t, size_t ecap, size_t ccap, Worker* w, hipStream_t st) {
  uint8_t* ch = nullptr;
  uint64_t* eo = nullptr;
  StrFp* f = nullptr;
  uint32_t* er = nullptr;
  if (dalloc(&ch, ccap) != hipSuccess || dalloc(&eo, ecap + 1) != hipSuccess || dalloc(&f, ecap) != hipSuccess ||
      dalloc(&er, ecap) != hipSuccess) {
    dfree(ch);
    dfree(eo);
    dfree(f);
    dfree(er);
    return fail(DDS_E_NOMEM, "string table heap");
  }
  const size_t n = t->nrows;
  std::vector<uint64_t> nb(n), ncb(n);
  uint64_t e = 0, c = 0;
  for (size_t r = 0; r < n; ++r) {
    nb[r] = e;
    ncb[r] = c;
    e += t->h_len[r];
    c += t->h_bytes[r];
  }
  if (n) {
    // the host's lengths: a row being rewritten already counts as empty (its device length is stale)
    HIP_TRY(w->misc2.ensure(2 * n * 8 + n * 4));
    uint64_t* d_nb = w->misc2.as<uint64_t>();
    uint32_t* d_len = reinterpret_cast<uint32_t*>(d_nb + 2 * n);
    HIP_TRY(hipMemcpyAsync(d_nb, nb.data(), n * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_nb + n, ncb.data(), n * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_len, t->h_len.data(), n * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_str_compact(n, t->row_beg, d_len, d_nb, d_nb + n, t->elem_off, t->fp, t->chars, eo, f, er, ch, st));
    HIP_TRY(hipMemcpyAsync(t->row_beg, d_nb, n * 8, hipMemcpyDeviceToDevice, st));
  }
  HIP_TRY(hipMemcpyAsync(eo + e, &c, 8, hipMemcpyHostToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));
  dfree(t->chars);
  dfree(t->elem_off);
  dfree(t->fp);
  dfree(t->elem_row);
  t->chars = ch;
  t->elem_off = eo;
  t->fp = f;
  t->elem_row = er;
  t->ecap = ecap;
  t->ccap = ccap;
  t->nheap = e;
  t->nchars = c;
  t->h_beg = std::move(nb);
  ++t->compactions;
  return DDS_OK;
}

// Patch every cached position index for the distinct rows d_ids[0..n) (device u32), or for the rows
// [r_first, nrows) when d_ids is null.
int patch_indexes(dds_strtab* t, const uint32_t* d_ids, size_t n, size_t r_first, hipStream_t st) {
  std::lock_guard<std::mutex> lk(t->posmu);
  for (auto& x : t->pos) {
    if (d_ids)
      HIP_TRY(launch_str_posfp_ids(d_ids, n, t->row_beg, t->row_len, t->live, t->fp, x->position, x->fp, x->present,
                                   st));
    else {
      const size_t r0 = r_first & ~(size_t)63;
      HIP_TRY(launch_str_posfp(t->row_beg, t->row_len, t->live, r0, t->nrows - r0, t->fp, x->position, x->fp,
                               x->present, st));
    }
  }
  return DDS_OK;
}

bool check_batch(const uint64_t* eoff, size_t ne, const uint64_t* roff, size_t nb, const char* chars) {
  if (!eoff || !roff || (eoff[ne] && !chars)) return false;
  if (eoff[0] != 0 || roff[0] != 0 || roff[nb] != ne) return false;
  for (size_t e = 0; e < ne; ++e)
    if (eoff[e + 1] < eoff[e]) return false;
  for (size_t r = 0; r < nb; ++r)
    if (roff[r + 1] < roff[r] || roff[r + 1] - roff[r] > 0xFFFFFFFFull) return false;
  return true;
}

// New versions for the batch's rows (chars, eoff[ne + 1], roff[nb + 1]): appended as rows nrows.. when
// ids is null, else row ids[i] (distinct, < nrows) takes batch row i. Caller holds the table exclusively.
int put_rows(dds_strtab* t, const uint32_t* ids, size_t nb, const char* chars, const uint64_t* eoff, size_t ne,
             const uint64_t* roff) {
  WorkerLease wl(t->ctx);
  int rc;
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  hipStream_t st = wl.st;
  const size_t nc = eoff[ne];
  const size_t r_first = t->nrows;
  if (!ids && (rc = grow_rows(t, t->nrows + nb, st))) return rc;
  // room for the new elements first (a compaction that fails leaves the table as it was; it still
  // copies the versions this write replaces, so it is sized for them too)
  if (t->nheap + ne > t->ecap || t->nchars + nc > t->ccap) {
    // a fresh table is sized to its first batch (+1/16); later growth leaves half the live size free
    const bool first = t->nheap == 0 && t->ecap == 0;
    const size_t le = t->vel + ne, lc = t->vch + nc;
    const size_t ecap = std::max(kStrMinCap, first ? le + le / 16 : le + le / 2);
    const size_t ccap = std::max(kStrMinCap, first ? lc + lc / 16 : lc + lc / 2);
    if ((rc = compact(t, ecap, ccap, w, st))) return rc;
  }
  if (ids) {  // the rows' current versions become garbage
    std::vector<uint64_t> ob(nb);
    std::vector<uint32_t> ol(nb);
    for (size_t i = 0; i < nb; ++i) {
      ob[i] = t->h_beg[ids[i]];
      ol[i] = t->h_len[ids[i]];
    }
    HIP_TRY(w->misc.ensure(nb * 12));
    HIP_TRY(hipMemcpyAsync(w->misc.p, ob.data(), nb * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(w->misc.as<uint8_t>() + nb * 8, ol.data(), nb * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_str_kill(w->misc.as<uint64_t>(), reinterpret_cast<const uint32_t*>(w->misc.as<uint8_t>() + nb * 8),
                            nb, t->elem_row, st));
    HIP_TRY(hipStreamSynchronize(st));  // staged from host vectors (misc is reused below)
    for (size_t i = 0; i < nb; ++i) {
      const uint32_t r = ids[i];
      t->vel -= t->h_len[r];
      t->vch -= t->h_bytes[r];
    }
  }
  // bytes, rebased element offsets, fingerprints and owners of the new elements
  const uint64_t e0 = t->nheap, c0 = t->nchars;
  std::vector<uint64_t> off(ne);
  std::vector<uint32_t> owner(ne);
  for (size_t e = 0; e < ne; ++e) off[e] = c0 + eoff[e + 1];
  for (size_t i = 0; i < nb; ++i) {
    const uint32_t r = ids ? ids[i] : (uint32_t)(r_first + i);
    for (uint64_t e = roff[i]; e < roff[i + 1]; ++e) owner[e] = r;
  }
  if (nc) HIP_TRY(hipMemcpyAsync(t->chars + c0, chars, nc, hipMemcpyHostToDevice, st));
  if (ne) {
    HIP_TRY(hipMemcpyAsync(t->elem_off + e0 + 1, off.data(), ne * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(t->elem_row + e0, owner.data(), ne * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_str_digest(t->chars, t->elem_off + e0, ne, t->fp + e0, st));
  }
  // row descriptors (host mirror + device)
  std::vector<uint64_t> beg(nb);
  std::vector<uint32_t> len(nb);
  if (!ids) {
    t->h_beg.resize(t->nrows + nb);
    t->h_len.resize(t->nrows + nb);
    t->h_bytes.resize(t->nrows + nb);
    t->h_live.resize(t->nrows + nb, 0);
  }
  for (size_t i = 0; i < nb; ++i) {
    const size_t r = ids ? ids[i] : r_first + i;
    beg[i] = e0 + roff[i];
    len[i] = (uint32_t)(roff[i + 1] - roff[i]);
    t->h_beg[r] = beg[i];
    t->h_len[r] = len[i];
    t->h_bytes[r] = eoff[roff[i + 1]] - eoff[roff[i]];
    if (!t->h_live[r]) ++t->nlive;
    t->h_live[r] = 1;
  }
  if (!ids) {
    if (nb) {
      HIP_TRY(hipMemcpyAsync(t->row_beg + r_first, beg.data(), nb * 8, hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemcpyAsync(t->row_len + r_first, len.data(), nb * 4, hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemsetAsync(t->live + r_first, 1, nb, st));
    }
  } else {
    HIP_TRY(w->ids.ensure(nb * 4));
    HIP_TRY(w->misc.ensure(nb * 12));
    HIP_TRY(hipMemcpyAsync(w->ids.p, ids, nb * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(w->misc.p, beg.data(), nb * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(w->misc.as<uint8_t>() + nb * 8, len.data(), nb * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_str_rows_set(w->ids.as<uint32_t>(), w->misc.as<uint64_t>(),
                                reinterpret_cast<const uint32_t*>(w->misc.as<uint8_t>() + nb * 8), nb, t->row_beg,
                                t->row_len, t->live, st));
  }
  t->nheap += ne;
  t->nchars += nc;
  t->vel += ne;
  t->vch += nc;
  if (!ids) t->nrows += nb;
  if ((rc = ids ? patch_indexes(t, w->ids.as<uint32_t>(), nb, 0, st) : patch_indexes(t, nullptr, 0, r_first, st)))
    return rc;
  HIP_TRY(hipStreamSynchronize(st));
  return DDS_OK;
}

// the distinct ids (last occurrence wins) and, per id, the batch row it takes: one pass from the end over
// a bitmap of the table's rows (a std::map of 100k ids cost ~15 ms of a 100k-row write)
void last_wins(const uint64_t* ids, size_t n, size_t nrows, std::vector<uint32_t>* out, std::vector<size_t>* pick) {
  std::vector<uint64_t> seen((nrows + 63) / 64, 0);
  out->clear();
  pick->clear();
  for (size_t i = n; i-- > 0;) {
    const uint64_t r = ids[i], bit = 1ull << (r & 63);
    if (seen[r >> 6] & bit) continue;
    seen[r >> 6] |= bit;
    out->push_back((uint32_t)r);
    pick->push_back(i);
  }
}

// the position index of `position` (built on first use; the kPosIdx most recent are kept)
int pos_index(dds_strtab* t, uint64_t position, hipStream_t st, std::shared_ptr<PosIdx>* out) {
  std::lock_guard<std::mutex> lk(t->posmu);
  for (auto it = t->pos.begin(); it != t->pos.end(); ++it)
    if ((*it)->position == position) {
      auto x = *it;  // most recent last
      t->pos.erase(it);
      t->pos.push_back(x);
      *out = x;
      return DDS_OK;
    }
  auto x = std::make_shared<PosIdx>();
  x->position = position;
  if (dalloc(&x->fp, t->rcap) != hipSuccess || dalloc(&x->present, t->rcap / 64 + 1) != hipSuccess)
    return fail(DDS_E_NOMEM, "position index");
  HIP_TRY(launch_str_posfp(t->row_beg, t->row_len, t->live, 0, t->nrows, t->fp, position, x->fp, x->present, st));
  // other queries may take the index from the cache right away: it is complete before it is shared
  HIP_TRY(hipStreamSynchronize(st));
  if (t->pos.size() >= dds_strtab::kPosIdx) t->pos.erase(t->pos.begin());  // in-flight users hold their own ref
  t->pos.push_back(x);
  *out = x;
  return DDS_OK;
}

// scan -> row flags / position-index masks -> stable compaction into ascending row ids
// mode 0: SearchEq/NEq at `position`; 1: any element equals a needle; 2: every needle present
int str_scan(dds_strtab* t, size_t row0, size_t nrows, const char* const* values, const size_t* lens, int nvalues,
             int mode, uint64_t position, int negate, uint32_t* out_rows, size_t* out_n) {
  StrNeedles nd{};
  nd.n = nvalues;
  std::vector<uint8_t> nb;
  for (int j = 0; j < nvalues; ++j) {
    if (!values[j] && lens[j]) return fail(DDS_E_ARG, "NULL value");
    nd.off[j] = nb.size();
    nd.len[j] = lens[j];
    nd.h[j] = str_digest((const uint8_t*)values[j], lens[j]);
    nb.insert(nb.end(), (const uint8_t*)values[j], (const uint8_t*)values[j] + lens[j]);
  }
  dds_ctx* ctx = t->ctx;
  WorkerLease wl(ctx);
  int rc;
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  HIP_TRY(w->in2.ensure(std::max<size_t>(nb.size(), 1)));
  HIP_TRY(w->misc.ensure(ope_scratch_bytes(nrows)));
  // the worker's coherent, device-mapped scan buffer: [0, 8) the match count, then the needle bytes
  // (DMA'd from there: pinned, no staging), then the row ids. The compaction stores the count and the
  // ids over PCIe straight into it, so a scan is its launches and one stream synchronisation (no copy
  // launch and no second round trip for the ids)
  const size_t nbal = round_up(std::max<size_t>(nb.size(), 1), 64);
  w->hscan.flags = hipHostMallocCoherent | hipHostMallocMapped;
  HIP_TRY(w->hscan.ensure(64 + nbal + std::max<size_t>(nrows, 1) * 4));
  uint8_t* hs = (uint8_t*)w->hscan.p;
  uint8_t* ds = (uint8_t*)w->hscan.dptr;
  if (!ds) return fail(DDS_E_HIP, "scan buffer has no device mapping");
  uint64_t* d_total = (uint64_t*)ds;
  *(volatile uint64_t*)hs = 0;  // no rows: no scatter block stores the count
  uint32_t* dst = (uint32_t*)(ds + 64 + nbal);
  // short needles ride in the kernel arguments (no upload); longer ones are DMA'd from pinned memory
  const bool inl = nb.size() <= (size_t)StrNeedles::kStrInline;
  if (inl) {
    if (!nb.empty()) memcpy(nd.inl, nb.data(), nb.size());
  } else {
    memcpy(hs + 64, nb.data(), nb.size());
    HIP_TRY(hipMemcpyAsync(w->in2.p, hs + 64, nb.size(), hipMemcpyHostToDevice, wl.st));
  }
  const uint8_t* d_needles = inl ? nullptr : w->in2.as<uint8_t>();
  std::shared_ptr<PosIdx> px;
  if (mode == 0 && (rc = pos_index(t, position, wl.st, &px))) return rc;
  record_time(ctx, w, wl.st, true, 2);
  if (mode == 0) {  // SearchEq / NEq over the position index, straight into the compaction masks
    HIP_TRY(launch_str_eq_compact(px->fp, px->present, row0, nrows, t->row_beg, t->elem_off, t->chars,
                                  d_needles, nd, position, negate, w->misc.p, d_total, dst, wl.st));
  } else {
    // row flags: the worker's own buffer, kept zeroed between scans (the count pass re-zeroes what the
    // scan set); a fresh or possibly dirty buffer (an earlier scan that failed mid-way) is cleared first
    const size_t fbytes = round_up(std::max<size_t>(nrows, 1), 4);
    if (w->sflags.cap < fbytes) w->sflags_zero = false;
    HIP_TRY(w->sflags.ensure(fbytes));
    uint8_t* flags = w->sflags.as<uint8_t>();
    if (!w->sflags_zero) HIP_TRY(hipMemsetAsync(flags, 0, w->sflags.cap, wl.st));  // the whole buffer
    w->sflags_zero = false;
    // the whole heap, or one row's current version (IsElement)
    const uint64_t e_first = nrows == 1 ? t->h_beg[row0] : 0;
    const uint64_t ne = nrows == 1 ? t->h_len[row0] : t->nheap;
    HIP_TRY(launch_str_any(t->fp, e_first, ne, t->elem_row, t->live, row0, nrows, t->elem_off, t->chars,
                           d_needles, nd, flags, wl.st, true));
    const uint32_t req = mode == 2 ? (1u << nvalues) - 1u : 0u;  // AND: every needle's bit
    HIP_TRY(launch_byte_compact(flags, nrows, 0xFFu, w->misc.p, d_total, dst, wl.st, req, true));
  }
  record_time(ctx, w, wl.st, false, 2);
  HIP_TRY(hipStreamSynchronize(wl.st));
  const uint64_t total = *(volatile uint64_t*)hs;
  if (total > nrows) return fail(DDS_E_HIP, "scan count out of range");
  // the count pass re-zeroed the flags it read: clean only once the stream finished and the count is sane
  if (mode != 0) w->sflags_zero = true;
  if (total) memcpy(out_rows, hs + 64 + nbal, total * 4);
  if (ctx->timing.load()) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, w->ev[2], w->ev[3]) == hipSuccess) {
      std::lock_guard<std::mutex> lk(ctx->tmu);
      ctx->total_ms += ms;
    }
  }
  *out_n = (size_t)total;
  return DDS_OK;
}
}  // namespace

extern "C" {

int dds_strtab_create(dds_ctx* ctx, const char* chars, const uint64_t* elem_offsets, size_t nelems,
                      const uint64_t* row_offsets, size_t nrows, dds_strtab** out) {
  try {
    if (!ctx || !out) return fail(DDS_E_ARG, "bad arguments");
    *out = nullptr;
    if (!check_batch(elem_offsets, nelems, row_offsets, nrows, chars))
      return fail(DDS_E_ARG, "offsets must start at 0, be monotone and cover every element");
    if (nrows >= kStrDead) return fail(DDS_E_ARG, "too many rows");
    std::unique_ptr<dds_strtab> t(new dds_strtab());
    t->ctx = ctx;
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = put_rows(t.get(), nullptr, nrows, chars, elem_offsets, nelems, row_offsets);
    if (rc) return rc;
    *out = t.release();
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_strtab_destroy(dds_strtab* tab) {
  delete tab;
  return DDS_OK;
}

size_t dds_strtab_rows(dds_strtab* tab) {
  if (!tab) return 0;
  std::shared_lock<std::shared_mutex> lk(tab->mu);
  return tab->nrows;
}

size_t dds_strtab_live_count(dds_strtab* tab) {
  if (!tab) return 0;
  std::shared_lock<std::shared_mutex> lk(tab->mu);
  return tab->nlive;
}

int dds_strtab_append(dds_strtab* tab, const char* chars, const uint64_t* elem_offsets, size_t nelems,
                      const uint64_t* row_offsets, size_t nrows) {
  try {
    if (!tab) return fail(DDS_E_ARG, "bad arguments");
    if (!check_batch(elem_offsets, nelems, row_offsets, nrows, chars))
      return fail(DDS_E_ARG, "offsets must start at 0, be monotone and cover every element");
    std::unique_lock<std::shared_mutex> lk(tab->mu);
    if (tab->nrows + nrows >= kStrDead) return fail(DDS_E_ARG, "too many rows");
    return put_rows(tab, nullptr, nrows, chars, elem_offsets, nelems, row_offsets);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_strtab_write_rows(dds_strtab* tab, const uint64_t* row_ids, size_t n, const char* chars,
                          const uint64_t* elem_offsets, size_t nelems, const uint64_t* row_offsets) {
  try {
    if (!tab || (n && !row_ids)) return fail(DDS_E_ARG, "bad arguments");
    if (!check_batch(elem_offsets, nelems, row_offsets, n, chars))
      return fail(DDS_E_ARG, "offsets must start at 0, be monotone and cover every element");
    std::unique_lock<std::shared_mutex> lk(tab->mu);
    for (size_t i = 0; i < n; ++i)
      if (row_ids[i] >= tab->nrows) return fail(DDS_E_ARG, "row id " + std::to_string(row_ids[i]) + " out of range");
    if (n == 0) return DDS_OK;
    std::vector<uint32_t> ids;
    std::vector<size_t> pick;
    last_wins(row_ids, n, tab->nrows, &ids, &pick);
    if (ids.size() == n) {  // no repeated id: the batch as given, in its own order
      for (size_t i = 0; i < n; ++i) ids[i] = (uint32_t)row_ids[i];
      return put_rows(tab, ids.data(), n, chars, elem_offsets, nelems, row_offsets);
    }
    // repeated ids: only the last version of each row goes to the heap
    std::vector<uint64_t> eo(1, 0), ro(1, 0);
    std::string ch;
    for (size_t i : pick) {
      for (uint64_t e = row_offsets[i]; e < row_offsets[i + 1]; ++e) {
        ch.append(chars + elem_offsets[e], elem_offsets[e + 1] - elem_offsets[e]);
        eo.push_back(ch.size());
      }
      ro.push_back(eo.size() - 1);
    }
    return put_rows(tab, ids.data(), ids.size(), ch.data(), eo.data(), eo.size() - 1, ro.data());
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_strtab_set_live(dds_strtab* tab, const uint64_t* row_ids, size_t n, const uint8_t* live) {
  try {
    if (!tab || (n && (!row_ids || !live))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(tab->mu);
    for (size_t i = 0; i < n; ++i)
      if (row_ids[i] >= tab->nrows) return fail(DDS_E_ARG, "row id " + std::to_string(row_ids[i]) + " out of range");
    std::vector<uint32_t> uniq;  // last flag of each id wins
    std::vector<size_t> pick;
    last_wins(row_ids, n, tab->nrows, &uniq, &pick);
    std::vector<uint32_t> ids;
    std::vector<uint8_t> vals;
    for (size_t j = 0; j < uniq.size(); ++j) {
      const uint8_t v = live[pick[j]] ? 1 : 0;
      if (tab->h_live[uniq[j]] != v) {
        ids.push_back(uniq[j]);
        vals.push_back(v);
      }
    }
    if (ids.empty()) return DDS_OK;
    WorkerLease wl(tab->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    const size_t m = ids.size();
    HIP_TRY(w->ids.ensure(m * 4));
    HIP_TRY(w->in2.ensure(m));
    HIP_TRY(hipMemcpyAsync(w->ids.p, ids.data(), m * 4, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(hipMemcpyAsync(w->in2.p, vals.data(), m, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(launch_scatter_bytes(w->ids.as<uint32_t>(), w->in2.as<uint8_t>(), m, tab->live, wl.st));
    if ((rc = patch_indexes(tab, w->ids.as<uint32_t>(), m, 0, wl.st))) return rc;
    HIP_TRY(hipStreamSynchronize(wl.st));
    for (size_t i = 0; i < m; ++i) {
      tab->h_live[ids[i]] = vals[i];
      tab->nlive += vals[i] ? 1 : (size_t)-1;
    }
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_strtab_truncate(dds_strtab* tab, size_t rows) {
  try {
    if (!tab) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(tab->mu);
    if (rows >= tab->nrows) return DDS_OK;
    const size_t m = tab->nrows - rows;
    std::vector<uint64_t> ob(tab->h_beg.begin() + rows, tab->h_beg.end());
    std::vector<uint32_t> ol(tab->h_len.begin() + rows, tab->h_len.end());
    WorkerLease wl(tab->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    HIP_TRY(w->misc.ensure(m * 12));
    HIP_TRY(hipMemcpyAsync(w->misc.p, ob.data(), m * 8, hipMemcpyHostToDevice, wl.st));
    HIP_TRY(hipMemcpyAsync(w->misc.as<uint8_t>() + m * 8, ol.data(), m * 4, hipMemcpyHostToDevice, wl.st));
    // the dropped rows' elements must not match rows appended later under the same ids
    HIP_TRY(launch_str_kill(w->misc.as<uint64_t>(), reinterpret_cast<const uint32_t*>(w->misc.as<uint8_t>() + m * 8), m,
                            tab->elem_row, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    for (size_t r = rows; r < tab->nrows; ++r) {
      tab->vel -= tab->h_len[r];
      tab->vch -= tab->h_bytes[r];
      tab->nlive -= tab->h_live[r];
    }
    tab->h_beg.resize(rows);
    tab->h_len.resize(rows);
    tab->h_bytes.resize(rows);
    tab->h_live.resize(rows);
    tab->nrows = rows;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_strtab_stats(dds_strtab* tab, uint64_t* out, size_t n) {
  if (!tab || (n && !out)) return fail(DDS_E_ARG, "bad arguments");
  std::shared_lock<std::shared_mutex> lk(tab->mu);
  size_t npos = 0;
  {
    std::lock_guard<std::mutex> pl(tab->posmu);
    npos = tab->pos.size();
  }
  const uint64_t v[] = {tab->nrows, tab->nlive, tab->nheap, tab->vel, tab->nchars, tab->vch, tab->compactions, npos};
  for (size_t i = 0; i < n && i < sizeof(v) / sizeof(v[0]); ++i) out[i] = v[i];
  return DDS_OK;
}

int dds_search_eq(dds_strtab* tab, size_t position, const char* value, size_t len, int negate, uint32_t* out_rows,
                  size_t* out_n) {
  try {
    if (!tab || !out_n || (len && !value)) return fail(DDS_E_ARG, "bad arguments");
    *out_n = 0;
    std::shared_lock<std::shared_mutex> lk(tab->mu);
    if (tab->nrows == 0) return DDS_OK;
    if (!out_rows) return fail(DDS_E_ARG, "bad arguments");
    const char* v[1] = {value};
    size_t l[1] = {len};
    return str_scan(tab, 0, tab->nrows, v, l, 1, 0, position, negate, out_rows, out_n);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_search_entry(dds_strtab* tab, const char* const* values, const size_t* lens, size_t nvalues, int require_all,
                     uint32_t* out_rows, size_t* out_n) {
  try {
    if (!tab || !out_n || !values || !lens || nvalues == 0 || nvalues > 3) return fail(DDS_E_ARG, "bad arguments");
    *out_n = 0;
    if (require_all) {  // SearchEntryAND needs 3 distinct matched strings (DDSRestServer.scala:924)
      for (size_t i = 0; i < nvalues; ++i)
        for (size_t j = i + 1; j < nvalues; ++j)
          if (lens[i] == lens[j] && memcmp(values[i], values[j], lens[i]) == 0) return DDS_OK;
      if (nvalues != 3) return fail(DDS_E_ARG, "SearchEntryAND takes three values");
    }
    std::shared_lock<std::shared_mutex> lk(tab->mu);
    if (tab->nrows == 0) return DDS_OK;
    if (!out_rows) return fail(DDS_E_ARG, "bad arguments");
    return str_scan(tab, 0, tab->nrows, values, lens, (int)nvalues, require_all ? 2 : 1, 0, 0, out_rows, out_n);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_is_element(dds_strtab* tab, size_t row, const char* value, size_t len, int* found) {
  try {
    if (!tab || !found || (len && !value)) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(tab->mu);
    if (row >= tab->nrows || !tab->h_live[row]) return fail(DDS_E_EMPTY, "no such row");  // None: 404 (:348)
    const char* v[1] = {value};
    size_t l[1] = {len};
    uint32_t id = 0;
    size_t n = 0;
    int rc = str_scan(tab, row, 1, v, l, 1, 1, 0, 0, &id, &n);
    if (rc) return rc;
    *found = n ? 1 : 0;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

}  // extern "C"
