// Resident OPE column (include/ddshe.h, dds_opecol_*): the int64 OPE ciphertexts of one column
// position kept in HBM across requests, for the range predicates SearchGt/GtEq/Lt/LtEq
// (DDSRestServer.scala:682-830) and the orderings OrderLS/OrderSL (:541-606).
//
// Per row the device holds the value (int64, as the GPU compares it) and a class byte:
//   kHold   the row holds the position (contents.length-1 >= position: Order's holders, :557/:590)
//   kSearch elements follow it (contents.length-1 > position: Search's strict guard, :702)
//   kBad    the element is not a decimal integer (new BigInteger / String.toLong would throw)
//   kWide   a decimal integer outside int64 (Search compares BigIntegers exactly: host-side rows)
//   kNotStr the element is not a String (Order's asInstanceOf[String] throws; Search's toString does not)
// The reference throws lazily, inside the loop, only for rows the loop reaches; the column keeps the
// counts needed to reproduce exactly when a request answers 500 instead of a key list.
//
// Rows follow the write routes (dds_opecol_write_rows*, dds_opecol_set_live): WriteElement / AddElement
// change a row's element or class (:220-321), RemoveSet makes its set None (:207-218), which every
// route filters out before its loop (filter(nonEmpty), :553, :586, :700). A dead row's device class
// byte is 0 (no Search match, an Order non-holder) and d_dead marks it, so Order drops it from the
// permutation; its host class stays in hflg for a later revival. The counts cover live rows only.
#include "ddshe_host.hpp"

using namespace ddshe;
using namespace ddshe::host;

namespace {
enum : uint8_t { kHold = 1, kSearch = 2, kBad = 4, kWide = 8, kNotStr = 16 };
}

struct dds_opecol {
  dds_ctx* ctx = nullptr;
  size_t capacity = 0, count = 0;
  int64_t* d_val = nullptr;
  uint8_t* d_flg = nullptr;
  uint8_t* d_dead = nullptr;                            // 1 = removed set (allocated with the first one)
  // Search / Order / live_count hold it shared (concurrent requests on one column run side by side on
  // their own worker streams, as the reference's routes do on the ForkJoin pool, DDSRestServer.scala:21);
  // appends, row writes, liveness changes and truncation hold it exclusively
  std::shared_mutex mu;
  std::vector<uint8_t> hflg;                            // host mirror of the class bytes (dead rows too)
  std::vector<uint8_t> hdead;                           // host mirror of d_dead (empty: none dead yet)
  size_t ndead = 0;
  std::map<size_t, std::pair<bn::Limbs, bool>> wide;  // kWide rows: exact value (magnitude, negative)
  // [ulo, uhi]: bounds of every value ever stored in d_val, in unsigned order (v ^ 2^63); a superset
  // of the holders' keys, kept on writes so Order starts its passes without a min/max pass over the
  // column and its host round trip (only the pass count depends on how tight the bounds are)
  uint64_t ulo = ~0ull, uhi = 0;
  void widen(const int64_t* v, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      const uint64_t u = (uint64_t)v[i] ^ 0x8000000000000000ull;
      ulo = std::min(ulo, u);
      uhi = std::max(uhi, u);
    }
  }
  size_t n_search = 0, n_hold = 0;
  size_t n_search_bad = 0;  // kSearch rows that Search's BigInteger parse rejects
  size_t n_hold_bad = 0;    // kHold rows that Order's asInstanceOf[String].toLong rejects
  ~dds_opecol() {
    if (d_val) (void)hipFree(d_val);
    if (d_flg) (void)hipFree(d_flg);
    if (d_dead) (void)hipFree(d_dead);
  }
  bool dead(size_t r) const { return !hdead.empty() && hdead[r]; }
  void account(uint8_t f, int sign) {
    const size_t d = (size_t)1;
    auto upd = [&](size_t& c, bool on) {
      if (on) c = sign > 0 ? c + d : c - d;
    };
    upd(n_search, f & kSearch);
    upd(n_hold, f & kHold);
    upd(n_search_bad, (f & kSearch) && (f & kBad));
    upd(n_hold_bad, (f & kHold) && (f & (kBad | kWide | kNotStr)));
  }
};

namespace {

// java.lang.Long.parseLong / new BigInteger(String) on ASCII text: optional sign, >= 1 digit.
// Returns 0: int64 in *v; 1: outside int64 (magnitude in *mag, sign in *neg); -1: malformed.
int parse_ope(const char* s, int64_t* v, bn::Limbs* mag, bool* neg) {
  const size_t len = strlen(s);
  size_t i = 0;
  bool ng = false;
  if (i < len && (s[i] == '+' || s[i] == '-')) ng = s[i++] == '-';
  if (i == len) return -1;
  for (size_t k = i; k < len; ++k)
    if (s[k] < '0' || s[k] > '9') return -1;
  while (i + 1 < len && s[i] == '0') ++i;  // leading zeros
  if (len - i <= 18) {
    int64_t x = 0;
    for (size_t k = i; k < len; ++k) x = x * 10 + (s[k] - '0');
    *v = ng ? -x : x;
    return 0;
  }
  if (!bn::from_dec(s, len, *mag, neg)) return -1;
  // |x| <= 2^63 - 1, or x == -2^63
  const size_t bl = bn::bit_length(*mag);
  if (bl <= 63) {
    const uint64_t u = (uint64_t)(*mag)[0] | ((mag->size() > 1 ? (uint64_t)(*mag)[1] : 0ull) << 32);
    *v = *neg ? -(int64_t)u : (int64_t)u;
    return 0;
  }
  if (bl == 64 && *neg && (*mag)[0] == 0 && (*mag)[1] == 0x80000000u) {
    *v = INT64_MIN;
    return 0;
  }
  return 1;
}

// signed compare of (neg_a, a) with (neg_b, b)
int scmp(bool na, const bn::Limbs& a, bool nb, const bn::Limbs& b) {
  if (a.empty()) na = false;
  if (b.empty()) nb = false;
  if (na != nb) return na ? -1 : 1;
  const int c = bn::cmp(a, b);
  return na ? -c : c;
}

bool ope_pred(int c, int op) {
  switch (op) {
    case DDS_OPE_GT: return c > 0;
    case DDS_OPE_GE: return c >= 0;
    case DDS_OPE_LT: return c < 0;
    default: return c <= 0;
  }
}

int append_rows(dds_opecol* col, const int64_t* vals, const uint8_t* flg, size_t count) {
  WorkerLease wl(col->ctx);
  int rc;
  if ((rc = wl.acquire())) return rc;
  HIP_TRY(hipMemcpyAsync(col->d_val + col->count, vals, count * 8, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(hipMemcpyAsync(col->d_flg + col->count, flg, count, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(hipStreamSynchronize(wl.st));
  col->widen(vals, count);
  col->hflg.insert(col->hflg.end(), flg, flg + count);
  for (size_t i = 0; i < count; ++i) col->account(flg[i], +1);
  col->count += count;
  return DDS_OK;
}

uint8_t class_bits(uint8_t cls) { return cls == 0 ? 0 : (cls == 1 ? kHold : (uint8_t)(kHold | kSearch)); }

// Rows given as element text (append_dec / write_rows_dec): value, class byte, exact value if wide
struct OpeRows {
  std::vector<int64_t> v;
  std::vector<uint8_t> f;
  std::vector<std::pair<size_t, std::pair<bn::Limbs, bool>>> wide;  // (index in the batch, value)
};
int parse_rows(const char* const* values, const uint8_t* cls, const uint8_t* is_string, size_t count, OpeRows* out) {
  out->v.assign(count, 0);
  out->f.assign(count, 0);
  for (size_t i = 0; i < count; ++i) {
    const uint8_t c = cls ? cls[i] : 2;
    if (c > 2) return fail(DDS_E_ARG, "row class must be 0, 1 or 2");
    out->f[i] = class_bits(c);
    if (!out->f[i]) continue;  // the row lacks the position: its element is never read
    if (!values[i]) return fail(DDS_E_ARG, "NULL element for a row that holds the position");
    if (is_string && !is_string[i]) out->f[i] |= kNotStr;
    bn::Limbs mag;
    bool neg = false;
    const int k = parse_ope(values[i], &out->v[i], &mag, &neg);
    if (k < 0) {
      out->f[i] |= kBad;
    } else if (k > 0) {
      out->f[i] |= kWide;
      out->wide.emplace_back(i, std::make_pair(std::move(mag), neg));
    }
  }
  return DDS_OK;
}

int class_rows(const uint8_t* cls, size_t count, std::vector<uint8_t>* f) {
  f->resize(count);
  for (size_t i = 0; i < count; ++i) {
    const uint8_t c = cls ? cls[i] : 2;
    if (c > 2) return fail(DDS_E_ARG, "row class must be 0, 1 or 2");
    (*f)[i] = class_bits(c);
  }
  return DDS_OK;
}

int check_ids(const dds_opecol* col, const uint64_t* ids, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (ids[i] >= col->count) return fail(DDS_E_ARG, "row id " + std::to_string(ids[i]) + " out of range");
  return DDS_OK;
}

// Rows ids[i] take (vals[i], flg[i]); repeated ids: the last entry wins. Counts, wide values and the
// device copies follow; a dead row keeps class byte 0 on the device.
int write_rows(dds_opecol* col, const uint64_t* ids, const int64_t* vals, const uint8_t* flg, size_t n,
               const std::map<size_t, std::pair<bn::Limbs, bool>>& wide_in) {
  std::map<uint64_t, size_t> last;
  for (size_t i = 0; i < n; ++i) last[ids[i]] = i;
  const size_t m = last.size();
  std::vector<uint32_t> id32;
  std::vector<int64_t> v;
  std::vector<uint8_t> df;
  id32.reserve(m);
  v.reserve(m);
  df.reserve(m);
  for (auto& kv : last) {
    id32.push_back((uint32_t)kv.first);
    v.push_back(vals[kv.second]);
    df.push_back(col->dead(kv.first) ? 0 : flg[kv.second]);
  }
  WorkerLease wl(col->ctx);
  int rc;
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  HIP_TRY(w->ids.ensure(m * 4));
  HIP_TRY(w->in.ensure(m * 8));
  HIP_TRY(w->in2.ensure(m));
  HIP_TRY(hipMemcpyAsync(w->ids.p, id32.data(), m * 4, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(hipMemcpyAsync(w->in.p, v.data(), m * 8, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(hipMemcpyAsync(w->in2.p, df.data(), m, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(launch_scatter_u64(w->ids.as<uint32_t>(), w->in.as<uint64_t>(), m, (uint64_t*)col->d_val, wl.st));
  HIP_TRY(launch_scatter_bytes(w->ids.as<uint32_t>(), w->in2.as<uint8_t>(), m, col->d_flg, wl.st));
  HIP_TRY(hipStreamSynchronize(wl.st));
  col->widen(v.data(), m);
  for (auto& kv : last) {
    const size_t r = (size_t)kv.first, i = kv.second;
    if (!col->dead(r)) {
      col->account(col->hflg[r], -1);
      col->account(flg[i], +1);
    }
    col->hflg[r] = flg[i];
    col->wide.erase(r);
    auto it = wide_in.find(i);
    if (it != wide_in.end()) col->wide.emplace(r, it->second);
  }
  return DDS_OK;
}

}  // namespace

extern "C" {

int dds_opecol_create(dds_ctx* ctx, size_t capacity, dds_opecol** out) {
  try {
    if (!ctx || !out || capacity == 0) return fail(DDS_E_ARG, "bad arguments");
    if (capacity > 0xFFFFFFFFull) return fail(DDS_E_ARG, "row index exceeds 32 bits");
    *out = nullptr;
    std::unique_ptr<dds_opecol> c(new dds_opecol());
    c->ctx = ctx;
    c->capacity = capacity;
    HIP_TRY(hipSetDevice(ctx->device));
    // +16: the filter's 16-byte vector loads may touch the padding after the last row
    if (hipMalloc(&c->d_val, capacity * 8 + 16) != hipSuccess || hipMalloc(&c->d_flg, capacity + 16) != hipSuccess)
      return fail(DDS_E_NOMEM, "OPE column allocation");
    c->hflg.reserve(std::min<size_t>(capacity, (size_t)1 << 24));
    *out = c.release();
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_opecol_destroy(dds_opecol* col) {
  delete col;
  return DDS_OK;
}

size_t dds_opecol_count(const dds_opecol* col) { return col ? col->count : 0; }

int dds_opecol_truncate(dds_opecol* col, size_t count) {
  if (!col) return fail(DDS_E_ARG, "bad arguments");
  std::unique_lock<std::shared_mutex> lk(col->mu);
  if (count > col->count) return fail(DDS_E_ARG, "truncate beyond the row count");
  size_t undead = 0;
  for (size_t i = count; i < col->count; ++i) {
    if (!col->dead(i)) {
      col->account(col->hflg[i], -1);
    } else {
      col->hdead[i] = 0;
      ++undead;
    }
  }
  if (undead) {  // rows past the count are never dead
    HIP_TRY(hipSetDevice(col->ctx->device));
    HIP_TRY(hipMemset(col->d_dead + count, 0, col->count - count));
    col->ndead -= undead;
  }
  col->hflg.resize(count);
  col->wide.erase(col->wide.lower_bound(count), col->wide.end());
  col->count = count;
  return DDS_OK;
}

int dds_opecol_append(dds_opecol* col, const int64_t* values, const uint8_t* cls, size_t count) {
  try {
    if (!col || (count && !values)) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    if (col->count + count > col->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    if (count == 0) return DDS_OK;
    std::vector<uint8_t> f(count);
    for (size_t i = 0; i < count; ++i) {
      const uint8_t c = cls ? cls[i] : 2;
      if (c > 2) return fail(DDS_E_ARG, "row class must be 0, 1 or 2");
      f[i] = class_bits(c);
    }
    return append_rows(col, values, f.data(), count);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_opecol_append_dec(dds_opecol* col, const char* const* values, const uint8_t* cls, const uint8_t* is_string,
                          size_t count) {
  try {
    if (!col || (count && !values)) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    if (col->count + count > col->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    if (count == 0) return DDS_OK;
    OpeRows rows;
    int rc = parse_rows(values, cls, is_string, count, &rows);
    if (rc) return rc;
    const size_t base = col->count;
    if ((rc = append_rows(col, rows.v.data(), rows.f.data(), count))) return rc;
    for (auto& e : rows.wide) col->wide.emplace(base + e.first, std::move(e.second));
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

}  // extern "C"

namespace {

// Search prelude (:702-704): the bound is parsed inside the per-row condition, after the guard, i.e.
// only if some live row passes the guard; any qualifying row the parse rejects fails the request
// (500). *none: no row qualifies (no match, any bound). Else the GPU predicate: int64 rows against
// the bound clamped to int64 (an equivalent predicate there), *b / *gop.
struct SearchBound {
  bool none = false;
  bn::Limbs bmag;
  bool bneg = false;
  int64_t b = 0;
  int gop = 0;
};
int search_bound(const dds_opecol* col, const char* bound_dec, int op, SearchBound* sb) {
  if (col->n_search == 0) {
    sb->none = true;
    return DDS_OK;
  }
  if (!bound_dec) return fail(DDS_E_ARG, "bound missing");
  if (!bn::from_dec(bound_dec, strlen(bound_dec), sb->bmag, &sb->bneg))
    return fail(DDS_E_FORMAT, std::string("NumberFormatException: bound ") + bound_dec);
  if (col->n_search_bad) return fail(DDS_E_FORMAT, "NumberFormatException: a qualifying row is not an integer");
  sb->gop = op;
  int64_t bv;
  bn::Limbs m2;
  bool n2;
  const std::string bt = bn::to_dec(sb->bmag, sb->bneg);
  if (parse_ope(bt.c_str(), &bv, &m2, &n2) == 0) {
    sb->b = bv;
  } else if (!sb->bneg) {  // bound > INT64_MAX: col > / >= bound never, col < / <= bound always
    sb->gop = (op == DDS_OPE_GT || op == DDS_OPE_GE) ? DDS_OPE_GT : DDS_OPE_LE;
    sb->b = INT64_MAX;
  } else {                 // bound < INT64_MIN: col > / >= bound always, col < / <= bound never
    sb->gop = (op == DDS_OPE_GT || op == DDS_OPE_GE) ? DDS_OPE_GE : DDS_OPE_LT;
    sb->b = INT64_MIN;
  }
  return DDS_OK;
}

// live rows outside int64 that match: exact BigInteger compare on the host, ascending
std::vector<uint32_t> wide_matches(const dds_opecol* col, const SearchBound& sb, int op) {
  std::vector<uint32_t> extra;
  for (const auto& e : col->wide)
    if (!col->dead(e.first) && (col->hflg[e.first] & kSearch) &&
        ope_pred(scmp(e.second.second, e.second.first, sb.bneg, sb.bmag), op))
      extra.push_back((uint32_t)e.first);
  return extra;
}

void add_filter_time(dds_ctx* ctx, Worker* w) {
  if (!ctx->timing.load()) return;
  float ms = 0;
  if (hipEventElapsedTime(&ms, w->ev[2], w->ev[3]) == hipSuccess) {
    std::lock_guard<std::mutex> tk(ctx->tmu);
    ctx->total_ms += ms;
  }
}

int set_dead(dds_opecol* col, const uint64_t* ids, size_t n, const uint8_t* live) {
  std::map<uint64_t, uint8_t> last;  // last flag of each id wins
  for (size_t i = 0; i < n; ++i) last[ids[i]] = live[i] ? 0 : 1;
  std::vector<uint32_t> id32;
  std::vector<uint8_t> dead, flg;
  for (auto& kv : last)
    if (col->dead(kv.first) != (kv.second != 0)) {
      id32.push_back((uint32_t)kv.first);
      dead.push_back(kv.second);
      flg.push_back(kv.second ? 0 : col->hflg[kv.first]);
    }
  if (id32.empty()) return DDS_OK;
  if (!col->d_dead) {
    HIP_TRY(hipSetDevice(col->ctx->device));
    if (hipMalloc(&col->d_dead, col->capacity + 16) != hipSuccess) return fail(DDS_E_NOMEM, "OPE dead mask");
    HIP_TRY(hipMemset(col->d_dead, 0, col->capacity + 16));
  }
  WorkerLease wl(col->ctx);
  int rc;
  if ((rc = wl.acquire())) return rc;
  Worker* w = wl.w;
  const size_t m = id32.size();
  HIP_TRY(w->ids.ensure(m * 4));
  HIP_TRY(w->in.ensure(m));
  HIP_TRY(w->in2.ensure(m));
  HIP_TRY(hipMemcpyAsync(w->ids.p, id32.data(), m * 4, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(hipMemcpyAsync(w->in.p, dead.data(), m, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(hipMemcpyAsync(w->in2.p, flg.data(), m, hipMemcpyHostToDevice, wl.st));
  HIP_TRY(launch_scatter_bytes(w->ids.as<uint32_t>(), w->in.as<uint8_t>(), m, col->d_dead, wl.st));
  HIP_TRY(launch_scatter_bytes(w->ids.as<uint32_t>(), w->in2.as<uint8_t>(), m, col->d_flg, wl.st));
  HIP_TRY(hipStreamSynchronize(wl.st));
  if (col->hdead.empty()) col->hdead.assign(col->capacity, 0);
  for (size_t j = 0; j < m; ++j) {
    const size_t r = id32[j];
    col->account(col->hflg[r], dead[j] ? -1 : +1);
    col->hdead[r] = dead[j];
    col->ndead = dead[j] ? col->ndead + 1 : col->ndead - 1;
  }
  return DDS_OK;
}

}  // namespace

extern "C" {

int dds_opecol_write_rows(dds_opecol* col, const uint64_t* row_ids, const int64_t* values, const uint8_t* cls,
                          size_t n) {
  try {
    if (!col || (n && (!row_ids || !values))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    int rc = check_ids(col, row_ids, n);
    if (rc || n == 0) return rc;
    std::vector<uint8_t> f;
    if ((rc = class_rows(cls, n, &f))) return rc;
    return write_rows(col, row_ids, values, f.data(), n, {});
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_opecol_write_rows_dec(dds_opecol* col, const uint64_t* row_ids, const char* const* values,
                              const uint8_t* cls, const uint8_t* is_string, size_t n) {
  try {
    if (!col || (n && (!row_ids || !values))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    int rc = check_ids(col, row_ids, n);
    if (rc || n == 0) return rc;
    OpeRows rows;
    if ((rc = parse_rows(values, cls, is_string, n, &rows))) return rc;
    std::map<size_t, std::pair<bn::Limbs, bool>> wide;
    for (auto& e : rows.wide) wide.emplace(e.first, std::move(e.second));
    return write_rows(col, row_ids, rows.v.data(), rows.f.data(), n, wide);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_opecol_set_live(dds_opecol* col, const uint64_t* row_ids, size_t n, const uint8_t* live) {
  try {
    if (!col || (n && (!row_ids || !live))) return fail(DDS_E_ARG, "bad arguments");
    std::unique_lock<std::shared_mutex> lk(col->mu);
    int rc = check_ids(col, row_ids, n);
    if (rc || n == 0) return rc;
    return set_dead(col, row_ids, n, live);
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

size_t dds_opecol_live_count(dds_opecol* col) {
  if (!col) return 0;
  std::shared_lock<std::shared_mutex> lk(col->mu);
  return col->count - col->ndead;
}

int dds_opecol_search(dds_opecol* col, const char* bound_dec, int op, uint32_t* out_idx, size_t* out_n) {
  try {
    if (!col || !out_n || op < 0 || op > 3 || (col->count && !out_idx)) return fail(DDS_E_ARG, "bad arguments");
    *out_n = 0;
    std::shared_lock<std::shared_mutex> lk(col->mu);
    SearchBound sb;
    int rc = search_bound(col, bound_dec, op, &sb);
    if (rc || sb.none) return rc;
    dds_ctx* ctx = col->ctx;
    WorkerLease wl(ctx);
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    const size_t n = col->count;
    HIP_TRY(w->misc.ensure(ope_scratch_bytes(n)));
    HIP_TRY(w->out.ensure(n * 4));
    MappedWords hw;  // the match count is stored by the scatter into coherent mapped host memory: no copy
    HIP_TRY(mapped_words(w, &hw));
    hw.h[kCountWord] = 0;  // no rows: no scatter block stores it
    record_time(ctx, w, wl.st, true, 2);
    HIP_TRY(launch_ope_filter(col->d_val, col->d_flg, n, sb.b, sb.gop, w->misc.p, hw.d + kCountWord,
                              w->out.as<uint32_t>(), wl.st, kSearch, kWide));
    record_time(ctx, w, wl.st, false, 2);
    HIP_TRY(hipStreamSynchronize(wl.st));
    const uint64_t total = hw.h[kCountWord];
    // straight into the caller's buffer (measured: a pinned stage + host copy was slower at 20 MB; a
    // page-locked reply buffer takes one DMA); the route-shaped answer is dds_opecol_search_mask (n/8
    // bytes instead of 4 bytes per match)
    if (total && host_registered(ctx, out_idx, total * 4)) {
      HIP_TRY(hipMemcpyAsync(out_idx, w->out.p, total * 4, hipMemcpyDeviceToHost, wl.st));
      HIP_TRY(hipStreamSynchronize(wl.st));
    } else if (total) {
      HIP_TRY(hipMemcpy(out_idx, w->out.p, total * 4, hipMemcpyDeviceToHost));
    }
    add_filter_time(ctx, w);
    size_t got = (size_t)total;
    const std::vector<uint32_t> extra = wide_matches(col, sb, op);  // merged in row order
    if (!extra.empty()) {
      std::vector<uint32_t> merged(got + extra.size());
      std::merge(out_idx, out_idx + got, extra.begin(), extra.end(), merged.begin());
      std::copy(merged.begin(), merged.end(), out_idx);
      got = merged.size();
    }
    *out_n = got;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_opecol_search_mask(dds_opecol* col, const char* bound_dec, int op, uint64_t* mask, size_t mask_words,
                           size_t* out_n) {
  try {
    if (!col || !out_n || op < 0 || op > 3) return fail(DDS_E_ARG, "bad arguments");
    *out_n = 0;
    std::shared_lock<std::shared_mutex> lk(col->mu);
    const size_t n = col->count, words = (n + 63) / 64;
    if (mask_words < words || (words && !mask)) return fail(DDS_E_BUFSIZE, "mask needs ceil(count / 64) words");
    SearchBound sb;
    int rc = search_bound(col, bound_dec, op, &sb);
    if (rc) return rc;
    if (sb.none || n == 0) {
      if (words) memset(mask, 0, words * 8);
      return DDS_OK;
    }
    dds_ctx* ctx = col->ctx;
    WorkerLease wl(ctx);
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    const size_t bytes = words * 8;
    // a registered caller buffer is written by the count kernel itself through its device mapping, and
    // the per-tile counts go to a mapped host array the host adds up: one launch, no copies at all.
    // DDSHE_MASK_ZEROCOPY=0 keeps one DMA into it instead
    static const bool zc = [] {
      const char* e = getenv("DDSHE_MASK_ZEROCOPY");
      return !(e && e[0] == '0');
    }();
    uint32_t* hm = zc ? (uint32_t*)host_device_ptr(ctx, mask, bytes) : nullptr;
    uint64_t total = 0;
    if (hm) {
      const size_t nb = ope_blocks(n);
      w->hcnt.flags = hipHostMallocCoherent | hipHostMallocMapped;
      HIP_TRY(w->hcnt.ensure(std::max<size_t>(nb * 4, 64)));
      void* dp = w->hcnt.dptr;
      record_time(ctx, w, wl.st, true, 2);
      HIP_TRY(launch_ope_mask(col->d_val, col->d_flg, n, sb.b, sb.gop, w->misc.p, nullptr, wl.st, kSearch, kWide,
                              false, hm, 2 * words, (uint32_t*)dp));
      record_time(ctx, w, wl.st, false, 2);
      HIP_TRY(hipStreamSynchronize(wl.st));
      const uint32_t* c = (const uint32_t*)w->hcnt.p;
      for (size_t t = 0; t < nb; ++t) total += c[t];
    } else {
      // match words in row order (u32 word k = rows [32k, 32k + 32), little-endian: two of them are the
      // u64 word of the caller's layout). The match count: the count kernel's tiles add into the
      // worker's zeroed counter (no reduction launch), re-zeroed on the stream after it is read.
      HIP_TRY(w->misc.ensure(ope_scratch_bytes(n) + 64));
      HIP_TRY(w->ctr.ensure(64));
      uint32_t* mw = ope_mask_words(w->misc.p, n);
      uint64_t* dtotal = w->ctr.as<uint64_t>();
      if (!w->ctr_zero) HIP_TRY(hipMemsetAsync(dtotal, 0, 8, wl.st));
      w->ctr_zero = false;
      uint32_t* stg = nullptr;
      HIP_TRY(stage_ptr(w, &stg));
      const bool direct = host_registered(ctx, mask, bytes);  // page-locked caller buffer: one DMA
      record_time(ctx, w, wl.st, true, 2);
      HIP_TRY(launch_ope_mask(col->d_val, col->d_flg, n, sb.b, sb.gop, w->misc.p, dtotal, wl.st, kSearch, kWide, true));
      record_time(ctx, w, wl.st, false, 2);
      uint8_t* h = nullptr;
      if (!direct) {
        HIP_TRY(w->hbig.ensure(bytes));
        h = (uint8_t*)w->hbig.p;
      }
      HIP_TRY(hipMemcpyAsync(stg, dtotal, 8, hipMemcpyDeviceToHost, wl.st));
      HIP_TRY(hipMemcpyAsync(direct ? (void*)mask : (void*)h, mw, bytes, hipMemcpyDeviceToHost, wl.st));
      HIP_TRY(hipEventRecord(w->ev_done, wl.st));
      HIP_TRY(hipMemsetAsync(dtotal, 0, 8, wl.st));  // off the reply's path: the caller waits for ev_done only
      w->ctr_zero = true;
      HIP_TRY(hipEventSynchronize(w->ev_done));
      memcpy(&total, stg, 8);
      if (!direct) {
        if (bytes >= ((size_t)1 << 20)) {
          CopyPool::get().parallel_for(bytes, 4096, [&](size_t a, size_t e) { memcpy((char*)mask + a, h + a, e - a); });
        } else {
          memcpy(mask, h, bytes);
        }
      }
    }
    add_filter_time(ctx, w);
    for (uint32_t r : wide_matches(col, sb, op)) {
      mask[r / 64] |= 1ull << (r % 64);
      ++total;
    }
    *out_n = (size_t)total;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_opecol_order(dds_opecol* col, int descending, uint32_t* out_idx, size_t* out_n) {
  try {
    if (!col || (col->count && !out_idx)) return fail(DDS_E_ARG, "bad arguments");
    std::shared_lock<std::shared_mutex> lk(col->mu);
    const size_t n = col->count;
    if (out_n) *out_n = 0;
    if (n == 0) return DDS_OK;
    // sortWith parses only when comparing two holders, and every holder meets another one when there
    // are two or more: then one element that is not a String holding a Long fails the request
    if (col->n_hold >= 2 && col->n_hold_bad)
      return fail(DDS_E_FORMAT, "NumberFormatException / ClassCastException: a holder is not a Long string");
    WorkerLease wl(col->ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    HIP_TRY(w->tab.ensure(rs_scratch_bytes(n)));
    HIP_TRY(w->out.ensure(n * 4));
    // the sort's valid test is flag != 0, i.e. kHold (rows lacking the position have no other bit; a
    // removed set's device byte is 0, so it sorts with them)
    const uint64_t ub[2] = {col->ulo, col->uhi};
    record_time(col->ctx, w, wl.st, true, 2);
    MappedWords ow;
    HIP_TRY(mapped_words(w, &ow));
    HIP_TRY(launch_ope_order(col->d_val, col->d_flg, n, descending ? 1 : 0, w->tab.p, w->out.as<uint32_t>(), wl.st,
                             ub, &ow));
    const uint32_t* res = w->out.as<uint32_t>();
    size_t m = n;
    if (col->ndead) {  // drop removed sets from the permutation, order kept (filter(nonEmpty), :553, :586)
      m = n - col->ndead;
      HIP_TRY(w->in2.ensure(n));
      HIP_TRY(w->misc.ensure(ope_scratch_bytes(n)));
      HIP_TRY(w->ids.ensure(n * 4));
      HIP_TRY(w->flags.ensure(16));
      HIP_TRY(w->p1.ensure(n * 4));
      HIP_TRY(launch_perm_keep(res, col->d_dead, n, w->in2.as<uint8_t>(), wl.st));
      HIP_TRY(launch_byte_compact(w->in2.as<uint8_t>(), n, 1u, w->misc.p, w->flags.as<uint64_t>(),
                                  w->ids.as<uint32_t>(), wl.st));
      HIP_TRY(launch_gather_u32(res, w->ids.as<uint32_t>(), m, w->p1.as<uint32_t>(), wl.st));
      res = w->p1.as<uint32_t>();
    }
    record_time(col->ctx, w, wl.st, false, 2);
    const bool direct = m && host_registered(col->ctx, out_idx, m * 4);  // page-locked reply buffer: one DMA
    if (m) {
      if (!direct) HIP_TRY(w->hbig.ensure(m * 4));
      HIP_TRY(hipMemcpyAsync(direct ? (void*)out_idx : w->hbig.p, res, m * 4, hipMemcpyDeviceToHost, wl.st));
    }
    HIP_TRY(hipStreamSynchronize(wl.st));
    add_filter_time(col->ctx, w);  // device time of the ordering (HIP events), for dds_ctx_get_timing
    if (m && !direct) CopyPool::get().copy(out_idx, w->hbig.p, m * 4);
    if (out_n) *out_n = m;
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

}  // extern "C"
