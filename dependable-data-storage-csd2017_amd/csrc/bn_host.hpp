// Host-side multiprecision helpers for the C-ABI boundary.
//
// Used only for per-modulus constants (n', R mod N, R^2 mod N, R^k mod N) and for
// the boundary codecs the JVM side would otherwise do (BigInteger.toByteArray /
// new BigInteger(String), DDSRestServer.scala:417,419,422). No per-row
// arithmetic of the hot path runs here: that is on the GPU.
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

// Knuth algorithm D: returns a mod m (m non-zero).
inline Limbs mod(const Limbs& a, const Limbs& m) {
  if (cmp(a, m) < 0) return a;
  if (m.size() == 1) {
    Limbs t = a;
    return from_u64(divmod_small(t, m[0]));
  }
  const int s = __builtin_clz(m.back());
  const size_t n = m.size(), mm = a.size() - n;
  Limbs v(n), u(a.size() + 1);
  for (size_t i = n; i-- > 0;) v[i] = (m[i] << s) | (s && i ? (uint32_t)((uint64_t)m[i - 1] >> (32 - s)) : 0);
  u[a.size()] = s ? (uint32_t)((uint64_t)a.back() >> (32 - s)) : 0;
  for (size_t i = a.size(); i-- > 0;) u[i] = (a[i] << s) | (s && i ? (uint32_t)((uint64_t)a[i - 1] >> (32 - s)) : 0);
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
    }
  }
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
inline bool from_dec(const char* s, size_t len, Limbs& out, bool* neg) {
  size_t i = 0;
  *neg = false;
  if (i < len && (s[i] == '+' || s[i] == '-')) {
    *neg = s[i] == '-';
    ++i;
  }
  if (i == len) return false;
  Limbs r;
  r.reserve((len - i) / 9 + 2);  // > log2(10^9)/32 limbs per 9 digits: no reallocation below
  while (i < len) {
    uint32_t chunk = 0, mulv = 1;
    int k = 0;
    for (; k < 9 && i < len; ++k, ++i) {
      if (s[i] < '0' || s[i] > '9') return false;
      chunk = chunk * 10 + (uint32_t)(s[i] - '0');
      mulv *= 10;
    }
    uint64_t c = chunk;  // r = r * mulv + chunk, in place
    for (auto& x : r) {
      c += (uint64_t)x * mulv;
      x = (uint32_t)c;
      c >>= 32;
    }
    if (c) r.push_back((uint32_t)c);
  }
  trim(r);
  if (r.empty()) *neg = false;
  out = r;
  return true;
}

// BigInteger.toString: repeated division by 10^18 over 64-bit words, each step a two-word by one-word
// division with a precomputed reciprocal (Moller-Granlund, divisor normalised to 2^63..2^64): about a
// quarter of the steps of dividing 32-bit limbs by 10^9 (the /Sum reply, DDSRestServer.scala:385-387,
// is a 1233-digit number for the committed key).
inline std::string to_dec(const Limbs& a32, bool neg = false) {
  if (a32.empty()) return "0";
  constexpr uint64_t D = 1000000000000000000ull;  // 10^18 < 2^60
  constexpr int SH = 4;                            // D << 4 in [2^63, 2^64)
  constexpr uint64_t DN = D << SH;
  const uint64_t DINV = (uint64_t)((~(unsigned __int128)0) / DN - ((unsigned __int128)1 << 64));
  std::vector<uint64_t> w((a32.size() + 1) / 2);
  for (size_t i = 0; i < a32.size(); ++i) w[i / 2] |= (uint64_t)a32[i] << (32 * (i % 2));
  while (!w.empty() && w.back() == 0) w.pop_back();
  std::vector<uint64_t> chunks;  // base-10^18 digits, least significant first
  while (!w.empty()) {
    uint64_t rem = 0;
    for (size_t i = w.size(); i-- > 0;) {
      const uint64_t x = w[i];
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
      w[i] = q;
      rem = r >> SH;
    }
    chunks.push_back(rem);
    while (!w.empty() && w.back() == 0) w.pop_back();
  }
  std::string s;
  if (neg) s.push_back('-');
  s += std::to_string(chunks.back());
  char buf[24];
  for (size_t i = chunks.size() - 1; i-- > 0;) {
    snprintf(buf, sizeof(buf), "%018llu", (unsigned long long)chunks[i]);
    s += buf;
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

}  // namespace bn
}  // namespace ddshe
