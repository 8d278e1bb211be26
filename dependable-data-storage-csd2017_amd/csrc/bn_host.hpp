// Host-side multiprecision helpers for the C-ABI boundary.
//
// Used for per-modulus constants (n', R mod N, R^2 mod N, R^k mod N, Barrett mu), for
// the boundary codecs the JVM side would otherwise do (BigInteger.toByteArray /
// new BigInteger(String), DDSRestServer.scala:417,419,422), and for the single product
// of a pairwise /Sum or /Mult request (barrett64_modmul, ddshe_pairs.cpp).
// No per-row arithmetic of the folds, filters, encryption or ordering runs here: that is on
// the GPU.
#pragma once
#include <cstdio>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

namespace ddshe {
namespace bn {

using Limbs = std::vector<uint32_t>;  // little-endian 32-bit words, trimmed (no leading zeros)

inline void trim(Limbs& a) {
  while (!a.empty() && a.back() == 0) a.pop_back();
}

inline Limbs from_u64(uint64_t v) {
  Limbs r;
  while (v) {
    r.push_back((uint32_t)v);
    v >>= 32;
  }
  return r;
}

inline int cmp(const Limbs& a, const Limbs& b) {
  if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
  for (size_t i = a.size(); i-- > 0;)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}

inline bool is_zero(const Limbs& a) { return a.empty(); }

inline size_t bit_length(const Limbs& a) {
  if (a.empty()) return 0;
  return 32 * (a.size() - 1) + (32 - __builtin_clz(a.back()));
}

inline bool test_bit(const Limbs& a, size_t i) {
  return (i / 32) < a.size() && ((a[i / 32] >> (i % 32)) & 1u);
}

// a - b, requires a >= b
inline Limbs sub(const Limbs& a, const Limbs& b) {
  Limbs r(a.size());
  int64_t br = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    int64_t d = (int64_t)a[i] - (i < b.size() ? (int64_t)b[i] : 0) - br;
    br = d < 0;
    r[i] = (uint32_t)(d + (br ? (int64_t)1 << 32 : 0));
  }
  trim(r);
  return r;
}

inline Limbs add(const Limbs& a, const Limbs& b) {
  Limbs r(std::max(a.size(), b.size()) + 1);
  uint64_t c = 0;
  for (size_t i = 0; i < r.size(); ++i) {
    c += (i < a.size() ? a[i] : 0ull) + (i < b.size() ? b[i] : 0ull);
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  trim(r);
  return r;
}

inline Limbs mul(const Limbs& a, const Limbs& b) {
  if (a.empty() || b.empty()) return {};
  Limbs r(a.size() + b.size(), 0);
  for (size_t i = 0; i < a.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.size(); ++j) {
      uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + c;
      r[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    r[i + b.size()] = (uint32_t)c;
  }
  trim(r);
  return r;
}

inline Limbs mul_small_add(const Limbs& a, uint32_t m, uint32_t add) {
  Limbs r(a.size() + 1);
  uint64_t c = add;
  for (size_t i = 0; i < a.size(); ++i) {
    c += (uint64_t)a[i] * m;
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  r[a.size()] = (uint32_t)c;
  trim(r);
  return r;
}

// a / d (d small), returns remainder
inline uint32_t divmod_small(Limbs& a, uint32_t d) {
  uint64_t rem = 0;
  for (size_t i = a.size(); i-- > 0;) {
    uint64_t cur = (rem << 32) | a[i];
    a[i] = (uint32_t)(cur / d);
    rem = cur % d;
  }
  trim(a);
  return (uint32_t)rem;
}

// Knuth algorithm D: returns a mod m (m non-zero); the quotient into *quot when given.
inline Limbs mod(const Limbs& a, const Limbs& m, Limbs* quot = nullptr) {
  if (cmp(a, m) < 0) {
    if (quot) quot->clear();
    return a;
  }
  if (m.size() == 1) {
    Limbs t = a;
    const Limbs r = from_u64(divmod_small(t, m[0]));
    if (quot) quot->swap(t);
    return r;
  }
  const int s = __builtin_clz(m.back());
  const size_t n = m.size(), mm = a.size() - n;
  Limbs v(n), u(a.size() + 1);
  for (size_t i = n; i-- > 0;) v[i] = (m[i] << s) | (s && i ? (uint32_t)((uint64_t)m[i - 1] >> (32 - s)) : 0);
  u[a.size()] = s ? (uint32_t)((uint64_t)a.back() >> (32 - s)) : 0;
  for (size_t i = a.size(); i-- > 0;) u[i] = (a[i] << s) | (s && i ? (uint32_t)((uint64_t)a[i - 1] >> (32 - s)) : 0);
  if (quot) quot->assign(mm + 1, 0);
  for (size_t j = mm + 1; j-- > 0;) {
    uint64_t num = ((uint64_t)u[j + n] << 32) | u[j + n - 1];
    uint64_t qhat = num / v[n - 1], rhat = num % v[n - 1];
    while (qhat >> 32 || qhat * v[n - 2] > ((rhat << 32) | u[j + n - 2])) {
      --qhat;
      rhat += v[n - 1];
      if (rhat >> 32) break;
    }
    int64_t borrow = 0;
    uint64_t carry = 0;
    for (size_t i = 0; i < n; ++i) {
      uint64_t p = qhat * v[i] + carry;
      carry = p >> 32;
      int64_t t = (int64_t)u[i + j] - (int64_t)(uint32_t)p - borrow;
      u[i + j] = (uint32_t)t;
      borrow = t < 0;
    }
    int64_t t = (int64_t)u[j + n] - (int64_t)carry - borrow;
    u[j + n] = (uint32_t)t;
    if (t < 0) {  // add back
      uint64_t c = 0;
      for (size_t i = 0; i < n; ++i) {
        c += (uint64_t)u[i + j] + v[i];
        u[i + j] = (uint32_t)c;
        c >>= 32;
      }
      u[j + n] += (uint32_t)c;
      --qhat;
    }
    if (quot) (*quot)[j] = (uint32_t)qhat;
  }
  if (quot) trim(*quot);
  Limbs r(n);
  for (size_t i = 0; i < n; ++i) r[i] = (u[i] >> s) | (s && i + 1 < u.size() ? (uint32_t)((uint64_t)u[i + 1] << (32 - s)) : 0);
  trim(r);
  return r;
}

inline Limbs mulmod(const Limbs& a, const Limbs& b, const Limbs& m) { return mod(mul(a, b), m); }

inline Limbs pow2(size_t e) {
  Limbs r(e / 32 + 1, 0);
  r[e / 32] = 1u << (e % 32);
  return r;
}

inline Limbs powmod(Limbs base, const Limbs& e, const Limbs& m) {
  Limbs r = mod(Limbs{1}, m);
  base = mod(base, m);
  for (size_t i = bit_length(e); i-- > 0;) {
    r = mulmod(r, r, m);
    if (test_bit(e, i)) r = mulmod(r, base, m);
  }
  return r;
}

inline Limbs powmod_u64(const Limbs& base, uint64_t e, const Limbs& m) { return powmod(base, from_u64(e), m); }

// ---- codecs --------------------------------------------------------------------
inline Limbs from_be(const uint8_t* p, size_t n) {
  Limbs r((n + 3) / 4, 0);
  for (size_t i = 0; i < n; ++i) {
    size_t bit = 8 * (n - 1 - i);
    r[bit / 32] |= (uint32_t)p[i] << (bit % 32);
  }
  trim(r);
  return r;
}

// writes exactly `width` bytes big-endian; returns false if the value does not fit
inline bool to_be(const Limbs& a, uint8_t* out, size_t width) {
  if (bit_length(a) > 8 * width) return false;
  for (size_t i = 0; i < width; ++i) {
    size_t bit = 8 * (width - 1 - i);
    out[i] = bit / 32 < a.size() ? (uint8_t)(a[bit / 32] >> (bit % 32)) : 0;
  }
  return true;
}

inline size_t byte_length(const Limbs& a) { return (bit_length(a) + 7) / 8; }

// new BigInteger(String) magnitude; sets *neg. Returns false on NumberFormatException.
// 19-digit chunks into 64-bit words (w = w * 10^k + chunk with 128-bit products): a 1233-digit value
// (the /Sum operands of the committed key) in 65 chunk steps instead of 137 steps over 32-bit limbs.
inline bool from_dec(const char* s, size_t len, Limbs& out, bool* neg) {
  size_t i = 0;
  *neg = false;
  if (i < len && (s[i] == '+' || s[i] == '-')) {
    *neg = s[i] == '-';
    ++i;
  }
  if (i == len) return false;
  static constexpr uint64_t kPow10[20] = {1ull,
                                          10ull,
                                          100ull,
                                          1000ull,
                                          10000ull,
                                          100000ull,
                                          1000000ull,
                                          10000000ull,
                                          100000000ull,
                                          1000000000ull,
                                          10000000000ull,
                                          100000000000ull,
                                          1000000000000ull,
                                          10000000000000ull,
                                          100000000000000ull,
                                          1000000000000000ull,
                                          10000000000000000ull,
                                          100000000000000000ull,
                                          1000000000000000000ull,
                                          10000000000000000000ull};
  const size_t nd = len - i;
  std::vector<uint64_t> w;
  w.reserve(nd / 19 + 2);
  size_t k = nd % 19 ? nd % 19 : 19;  // the first chunk takes the odd digits
  while (i < len) {
    uint64_t chunk = 0;
    for (size_t e = i + k; i < e; ++i) {
      const unsigned d = (unsigned)(unsigned char)s[i] - (unsigned)'0';
      if (d > 9) return false;
      chunk = chunk * 10 + d;
    }
    const uint64_t mulv = kPow10[k];
    uint64_t c = chunk;
    for (auto& x : w) {  // w = w * mulv + chunk, in place
      const unsigned __int128 p = (unsigned __int128)x * mulv + c;
      x = (uint64_t)p;
      c = (uint64_t)(p >> 64);
    }
    if (c) w.push_back(c);
    k = 19;
  }
  Limbs r(2 * w.size());
  for (size_t j = 0; j < w.size(); ++j) {
    r[2 * j] = (uint32_t)w[j];
    r[2 * j + 1] = (uint32_t)(w[j] >> 32);
  }
  trim(r);
  if (r.empty()) *neg = false;
  out.swap(r);
  return true;
}

// BigInteger.toString: repeated division by 10^18 over 64-bit words, each step a two-word by one-word
// division with a precomputed reciprocal (Moller-Granlund, divisor normalised to 2^63..2^64). Four
// division passes run interleaved in one top-down sweep (pass p + 1 divides the quotient words pass p
// has just produced), so four independent remainder chains fill the multiplier's pipeline instead of
// one; the 10^18 digits are printed two decimal digits at a time from a table. The /Sum reply
// (DDSRestServer.scala:385-387) is a 1233-digit number for the committed key.
inline std::string to_dec(const Limbs& a32, bool neg = false) {
  if (a32.empty()) return "0";
  constexpr uint64_t D = 1000000000000000000ull;  // 10^18 < 2^60
  constexpr int SH = 4;                            // D << 4 in [2^63, 2^64)
  constexpr uint64_t DN = D << SH;
  constexpr uint64_t DINV = (uint64_t)((~(unsigned __int128)0) / DN - ((unsigned __int128)1 << 64));
  // one step: (rem, x) / D -> quotient word, rem updated (rem < D)
  auto step = [](uint64_t& rem, uint64_t x) -> uint64_t {
    const uint64_t nh = (rem << SH) | (x >> (64 - SH)), nl = x << SH;  // nh < DN since rem < D
    const unsigned __int128 p = (unsigned __int128)nh * DINV + (((unsigned __int128)(nh + 1) << 64) | nl);
    uint64_t q = (uint64_t)(p >> 64);
    uint64_t r = nl - q * DN;
    if (r > (uint64_t)p) {
      --q;
      r += DN;
    }
    if (r >= DN) {
      ++q;
      r -= DN;
    }
    rem = r >> SH;
    return q;
  };
  std::vector<uint64_t> w((a32.size() + 1) / 2);
  for (size_t i = 0; i < a32.size(); ++i) w[i / 2] |= (uint64_t)a32[i] << (32 * (i % 2));
  while (!w.empty() && w.back() == 0) w.pop_back();
  constexpr int kPasses = 4;  // 2, 6 and 8 measured no faster
  std::vector<uint64_t> chunks;  // base-10^18 digits, least significant first
  chunks.reserve(w.size() * 64 / 59 + 2 * kPasses);
  while (!w.empty()) {
    uint64_t r[kPasses] = {};
    for (size_t i = w.size(); i-- > 0;) {
      uint64_t q = w[i];
#pragma GCC unroll 8
      for (int p = 0; p < kPasses; ++p) q = step(r[p], q);
      w[i] = q;
    }
    for (int p = 0; p < kPasses; ++p) chunks.push_back(r[p]);
    while (!w.empty() && w.back() == 0) w.pop_back();
  }
  while (chunks.size() > 1 && chunks.back() == 0) chunks.pop_back();  // zero chunks above the value
  static const char kPairs[] =
      "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
      "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
      "8081828384858687888990919293949596979899";
  std::string s;
  s.reserve(1 + 18 * chunks.size());
  if (neg) s.push_back('-');
  {
    char buf[24];
    int n = 0;
    uint64_t v = chunks.back();
    do {
      buf[n++] = (char)('0' + v % 10);
      v /= 10;
    } while (v);
    while (n) s.push_back(buf[--n]);
  }
  const size_t head = s.size();
  s.resize(head + 18 * (chunks.size() - 1));
  char* p = &s[head];
  for (size_t i = chunks.size() - 1; i-- > 0; p += 18) {
    uint64_t v = chunks[i];
    for (int k = 16; k >= 0; k -= 2) {
      const uint64_t q = v / 100;
      const unsigned r = (unsigned)(v - q * 100);
      p[k] = kPairs[2 * r];
      p[k + 1] = kPairs[2 * r + 1];
      v = q;
    }
  }
  return s;
}

// radix-2^W limbs (S of them, zero-padded); requires value < 2^(W*S)
inline std::vector<uint32_t> to_rw(const Limbs& a, int S, int W) {
  std::vector<uint32_t> r(S, 0);
  for (int l = 0; l < S; ++l) {
    size_t bit = (size_t)W * l;
    uint64_t w = 0;
    size_t wi = bit / 32, sh = bit % 32;
    if (wi < a.size()) w = a[wi];
    if (wi + 1 < a.size()) w |= (uint64_t)a[wi + 1] << 32;
    r[l] = (uint32_t)(w >> sh) & ((1u << W) - 1);
  }
  return r;
}

// radix-2^W limbs (possibly unnormalised, each < 2^32) -> value
inline Limbs from_rw(const uint32_t* r, int S, int W) {
  Limbs acc(((size_t)W * S + 64) / 32 + 2, 0);
  for (int l = 0; l < S; ++l) {
    size_t bit = (size_t)W * l;
    uint64_t v = (uint64_t)r[l] << (bit % 32);
    size_t wi = bit / 32;
    uint64_t c = 0;
    for (size_t k = wi; k < acc.size() && (v || c); ++k) {
      c += (uint64_t)acc[k] + (uint32_t)v;
      acc[k] = (uint32_t)c;
      c >>= 32;
      v >>= 32;
    }
  }
  trim(acc);
  return acc;
}

// -N^{-1} mod 2^W (N odd)
inline uint32_t mont_n0(uint32_t n_low, int W) {
  uint32_t inv = n_low;  // Newton: inv = inv*(2 - n*inv), 5 iterations for 32 bits
  for (int i = 0; i < 5; ++i) inv *= 2u - n_low * inv;
  return (0u - inv) & ((1u << W) - 1);
}

// ---- host modular product (the pairwise routes' lone requests) -----------------------------------
// /Sum and /Mult (DDSRestServer.scala:385,479) are ONE modular product per request: a request with no
// batch partner queued is served here rather than by a GPU round trip (ddshe_pairs.cpp). 64-bit limbs,
// base B = 2^64, N of k limbs: the product by column sums (Comba: a 3-word accumulator per column, no
// carry chain through memory), then Barrett (HAC 14.42) with mu = floor(B^(2k) / N) precomputed per
// modulus: q = floor(floor(x / B^(k-1)) * mu / B^(k+1)), r = x - q N (mod B^(k+1)), at most two
// subtractions of N. About 2.5 k^2 multiplies (k = 64 at the committed 4096-bit n^2).
struct Barrett64 {
  size_t k = 0;
  std::vector<uint64_t> n;   // N, k limbs
  std::vector<uint64_t> mu;  // floor(B^(2k) / N), k + 1 limbs
};

inline std::vector<uint64_t> to_u64(const Limbs& a, size_t k) {
  std::vector<uint64_t> r(k, 0);
  for (size_t i = 0; i < a.size() && i / 2 < k; ++i) r[i / 2] |= (uint64_t)a[i] << (32 * (i & 1));
  return r;
}

inline Limbs from_u64v(const uint64_t* a, size_t k) {
  Limbs r(2 * k);
  for (size_t i = 0; i < k; ++i) {
    r[2 * i] = (uint32_t)a[i];
    r[2 * i + 1] = (uint32_t)(a[i] >> 32);
  }
  trim(r);
  return r;
}

inline Barrett64 barrett64_make(const Limbs& N) {
  Barrett64 m;
  m.k = (bit_length(N) + 63) / 64;
  m.n = to_u64(N, m.k);
  Limbs mu;
  (void)mod(pow2(128 * m.k), N, &mu);
  m.mu = to_u64(mu, m.k + 1);
  return m;
}

// column sums: out[c] = column c of a * b for c in [c0, c1) (out must not alias; c1 <= na + nb). c0 > 0
// drops the carries of the lower columns (Barrett's truncated product: the quotient estimate is then at
// most a few units low); c1 < na + nb gives the product mod B^c1.
inline void mul_u64(const uint64_t* a, size_t na, const uint64_t* b, size_t nb, uint64_t* out, size_t c0 = 0,
                    size_t c1 = ~(size_t)0) {
  typedef unsigned __int128 u128;
  u128 acc = 0;
  uint64_t top = 0;
  c1 = std::min(c1, na + nb);
  for (size_t c = c0; c < c1 && c + 1 < na + nb; ++c) {
    const size_t i0 = c >= nb ? c - nb + 1 : 0, i1 = std::min(c, na - 1);
    for (size_t i = i0; i <= i1; ++i) {
      const u128 p = (u128)a[i] * b[c - i];
      acc += p;
      top += acc < p;
    }
    out[c] = (uint64_t)acc;
    acc = (acc >> 64) | ((u128)top << 64);
    top = 0;
  }
  if (c1 == na + nb) out[na + nb - 1] = (uint64_t)acc;
}

// a * b mod N for a, b < N (reduced operands), as a trimmed value
inline Limbs barrett64_modmul(const Barrett64& m, const Limbs& a, const Limbs& b) {
  typedef unsigned __int128 u128;
  const size_t k = m.k;
  std::vector<uint64_t> buf(2 * k + 2 * (k + 2) + (2 * k + 2) + (k + 1) + (k + 1) + 2 * (k + 1), 0);
  uint64_t* x = buf.data();         // 2k: a b
  uint64_t* q2 = x + 2 * k;         // 2k + 2: q1 mu
  uint64_t* r2 = q2 + 2 * k + 2;    // 2k + 1: q3 N
  const std::vector<uint64_t> av = to_u64(a, k), bv = to_u64(b, k);
  mul_u64(av.data(), k, bv.data(), k, x);
  // q1 = x / B^(k-1): k + 1 limbs; q3 = q1 mu / B^(k+1) from the columns >= k - 1 only
  mul_u64(x + k - 1, k + 1, m.mu.data(), k + 1, q2, k - 1);
  const uint64_t* q3 = q2 + k + 1;  // k + 1 limbs
  mul_u64(q3, k + 1, m.n.data(), k, r2, 0, k + 1);  // q3 N mod B^(k+1)
  // r = x - q3 N mod B^(k+1)
  std::vector<uint64_t> r(k + 1);
  uint64_t br = 0;
  for (size_t j = 0; j <= k; ++j) {
    const u128 d = (u128)x[j] - r2[j] - br;
    r[j] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1u;
  }
  for (int it = 0; it < 8; ++it) {  // r < 5N: Barrett's 2 plus the truncated product's few
    bool ge = r[k] != 0;
    if (!ge) {
      ge = true;
      for (size_t j = k; j-- > 0;)
        if (r[j] != m.n[j]) {
          ge = r[j] > m.n[j];
          break;
        }
    }
    if (!ge) break;
    br = 0;
    for (size_t j = 0; j <= k; ++j) {
      const u128 d = (u128)r[j] - (j < k ? m.n[j] : 0) - br;
      r[j] = (uint64_t)d;
      br = (uint64_t)(d >> 64) & 1u;
    }
  }
  return from_u64v(r.data(), k);
}

}  // namespace bn
}  // namespace ddshe
