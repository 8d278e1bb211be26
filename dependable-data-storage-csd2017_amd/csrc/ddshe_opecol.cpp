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
  std::mutex mu;
  std::vector<uint8_t> hflg;                            // host mirror of the class bytes
  std::map<size_t, std::pair<bn::Limbs, bool>> wide;  // kWide rows: exact value (magnitude, negative)
  size_t n_search = 0, n_hold = 0;
  size_t n_search_bad = 0;  // kSearch rows that Search's BigInteger parse rejects
  size_t n_hold_bad = 0;    // kHold rows that Order's asInstanceOf[String].toLong rejects
  ~dds_opecol() {
    if (d_val) (void)hipFree(d_val);
    if (d_flg) (void)hipFree(d_flg);
  }
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
  col->hflg.insert(col->hflg.end(), flg, flg + count);
  for (size_t i = 0; i < count; ++i) col->account(flg[i], +1);
  col->count += count;
  return DDS_OK;
}

uint8_t class_bits(uint8_t cls) { return cls == 0 ? 0 : (cls == 1 ? kHold : (uint8_t)(kHold | kSearch)); }

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
  std::lock_guard<std::mutex> lk(col->mu);
  if (count > col->count) return fail(DDS_E_ARG, "truncate beyond the row count");
  for (size_t i = count; i < col->count; ++i) col->account(col->hflg[i], -1);
  col->hflg.resize(count);
  col->wide.erase(col->wide.lower_bound(count), col->wide.end());
  col->count = count;
  return DDS_OK;
}

int dds_opecol_append(dds_opecol* col, const int64_t* values, const uint8_t* cls, size_t count) {
  try {
    if (!col || (count && !values)) return fail(DDS_E_ARG, "bad arguments");
    std::lock_guard<std::mutex> lk(col->mu);
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
    std::lock_guard<std::mutex> lk(col->mu);
    if (col->count + count > col->capacity) return fail(DDS_E_ARG, "column capacity exceeded");
    if (count == 0) return DDS_OK;
    std::vector<int64_t> v(count, 0);
    std::vector<uint8_t> f(count);
    std::vector<std::pair<size_t, std::pair<bn::Limbs, bool>>> wide;
    for (size_t i = 0; i < count; ++i) {
      const uint8_t c = cls ? cls[i] : 2;
      if (c > 2) return fail(DDS_E_ARG, "row class must be 0, 1 or 2");
      f[i] = class_bits(c);
      if (!f[i]) continue;  // the row lacks the position: its element is never read
      if (!values[i]) return fail(DDS_E_ARG, "NULL element for a row that holds the position");
      if (is_string && !is_string[i]) f[i] |= kNotStr;
      bn::Limbs mag;
      bool neg = false;
      const int k = parse_ope(values[i], &v[i], &mag, &neg);
      if (k < 0) {
        f[i] |= kBad;
      } else if (k > 0) {
        f[i] |= kWide;
        wide.emplace_back(col->count + i, std::make_pair(std::move(mag), neg));
      }
    }
    int rc = append_rows(col, v.data(), f.data(), count);
    if (rc) return rc;
    for (auto& e : wide) col->wide.emplace(e.first, std::move(e.second));
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

int dds_opecol_search(dds_opecol* col, const char* bound_dec, int op, uint32_t* out_idx, size_t* out_n) {
  try {
    if (!col || !out_n || op < 0 || op > 3 || (col->count && !out_idx)) return fail(DDS_E_ARG, "bad arguments");
    *out_n = 0;
    std::lock_guard<std::mutex> lk(col->mu);
    // the bound is parsed inside the per-row condition, after the guard (:702-704): only if some row
    // passes the guard; any qualifying row the parse rejects fails the whole request (500)
    if (col->n_search == 0) return DDS_OK;
    if (!bound_dec) return fail(DDS_E_ARG, "bound missing");
    bn::Limbs bmag;
    bool bneg = false;
    if (!bn::from_dec(bound_dec, strlen(bound_dec), bmag, &bneg))
      return fail(DDS_E_FORMAT, std::string("NumberFormatException: bound ") + bound_dec);
    if (col->n_search_bad) return fail(DDS_E_FORMAT, "NumberFormatException: a qualifying row is not an integer");
    // int64 rows on the GPU against the bound clamped to int64 (an equivalent predicate there)
    int64_t b = 0;
    int gop = op;
    {
      int64_t bv;
      bn::Limbs m2;
      bool n2;
      const std::string bt = bn::to_dec(bmag, bneg);
      if (parse_ope(bt.c_str(), &bv, &m2, &n2) == 0) {
        b = bv;
      } else if (!bneg) {  // bound > INT64_MAX: col > / >= bound never, col < / <= bound always
        gop = (op == DDS_OPE_GT || op == DDS_OPE_GE) ? DDS_OPE_GT : DDS_OPE_LE;
        b = INT64_MAX;
      } else {             // bound < INT64_MIN: col > / >= bound always, col < / <= bound never
        gop = (op == DDS_OPE_GT || op == DDS_OPE_GE) ? DDS_OPE_GE : DDS_OPE_LT;
        b = INT64_MIN;
      }
    }
    dds_ctx* ctx = col->ctx;
    WorkerLease wl(ctx);
    int rc;
    if ((rc = wl.acquire())) return rc;
    Worker* w = wl.w;
    const size_t n = col->count;
    HIP_TRY(w->misc.ensure(ope_scratch_bytes(n)));
    HIP_TRY(w->flags.ensure(16));
    HIP_TRY(w->out.ensure(n * 4));
    record_time(ctx, w, wl.st, true, 2);
    HIP_TRY(launch_ope_filter(col->d_val, col->d_flg, n, b, gop, w->misc.p, w->flags.as<uint64_t>(),
                              w->out.as<uint32_t>(), wl.st, kSearch, kWide));
    record_time(ctx, w, wl.st, false, 2);
    uint64_t total = 0;
    HIP_TRY(read_sync(w, wl.st, w->flags.p, &total, 8));
    if (total) HIP_TRY(hipMemcpy(out_idx, w->out.p, total * 4, hipMemcpyDeviceToHost));
    if (ctx->timing.load()) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, w->ev[2], w->ev[3]) == hipSuccess) {
        std::lock_guard<std::mutex> tk(ctx->tmu);
        ctx->total_ms += ms;
      }
    }
    size_t got = (size_t)total;
    // rows outside int64: exact BigInteger compare here, merged in row order
    std::vector<uint32_t> extra;
    for (const auto& e : col->wide)
      if ((col->hflg[e.first] & kSearch) && ope_pred(scmp(e.second.second, e.second.first, bneg, bmag), op))
        extra.push_back((uint32_t)e.first);
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

int dds_opecol_order(dds_opecol* col, int descending, uint32_t* out_idx) {
  try {
    if (!col || (col->count && !out_idx)) return fail(DDS_E_ARG, "bad arguments");
    std::lock_guard<std::mutex> lk(col->mu);
    const size_t n = col->count;
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
    // the sort's valid test is flag != 0, i.e. kHold (rows lacking the position have no other bit)
    HIP_TRY(launch_ope_order(col->d_val, col->d_flg, n, descending ? 1 : 0, w->tab.p, w->out.as<uint32_t>(), wl.st));
    HIP_TRY(hipMemcpyAsync(out_idx, w->out.p, n * 4, hipMemcpyDeviceToHost, wl.st));
    HIP_TRY(hipStreamSynchronize(wl.st));
    return DDS_OK;
  } catch (const std::bad_alloc&) {
    return fail(DDS_E_NOMEM, "host allocation");
  }
}

}  // extern "C"
