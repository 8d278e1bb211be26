/*
 * fold_ref.c — plain-C CPU restatement of the reference fold (TEST INFRASTRUCTURE / CPU BASELINE ONLY).
 *
 * Restates the SumAll / MultAll hot loop of the reference REST proxy
 *   /root/reference/src/main/scala/dds/http/DDSRestServer.scala:412-430 (SumAll) and :506-524 (MultAll):
 *     acc = new BigInteger(x0)                       (first operand unreduced, :416-417)
 *     acc = HomoAdd.sum(acc, x, nsquare)             (= acc.multiply(x).mod(nsquare), :423)
 * as java.math.BigInteger computes it: full schoolbook product of 32-bit limbs, then a
 * Knuth algorithm-D remainder. Single-threaded like the reference's onComplete callback.
 * Used by tests/ (parity at medium sizes) and by bench.py's cpu_baseline leg; never by
 * the product path. "port" baseline: the reference itself (Scala + absent hlib jar) is
 * unbuildable here.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint32_t* w; size_t n; } bn_t; /* little-endian limbs, n used */

static size_t trim(const uint32_t* w, size_t n) { while (n && !w[n - 1]) --n; return n; }

static void from_be(const uint8_t* p, size_t bytes, uint32_t* w, size_t nw) {
  memset(w, 0, nw * 4);
  for (size_t i = 0; i < bytes; ++i) {
    size_t bit = 8 * (bytes - 1 - i);
    if (bit / 32 < nw) w[bit / 32] |= (uint32_t)p[i] << (bit % 32);
  }
}

static void to_be(const uint32_t* w, size_t nw, uint8_t* p, size_t bytes) {
  for (size_t i = 0; i < bytes; ++i) {
    size_t bit = 8 * (bytes - 1 - i);
    p[i] = bit / 32 < nw ? (uint8_t)(w[bit / 32] >> (bit % 32)) : 0;
  }
}

/* r[0..an+bn) = a*b */
static void mul(const uint32_t* a, size_t an, const uint32_t* b, size_t bn, uint32_t* r) {
  memset(r, 0, (an + bn) * 4);
  for (size_t i = 0; i < an; ++i) {
    uint64_t c = 0, ai = a[i];
    for (size_t j = 0; j < bn; ++j) {
      uint64_t t = ai * b[j] + r[i + j] + c;
      r[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    r[i + bn] = (uint32_t)c;
  }
}

/* u (un limbs, destroyed) mod v (vn >= 2 limbs, normalised copy vs given) -> rem (vn limbs) */
static void knuth_mod(uint32_t* u, size_t un, const uint32_t* v_in, size_t vn, uint32_t* rem, uint32_t* scratch) {
  uint32_t* v = scratch;           /* vn */
  uint32_t* un_ = scratch + vn;    /* un + 1 */
  int s = __builtin_clz(v_in[vn - 1]);
  for (size_t i = vn; i-- > 0;) v[i] = (v_in[i] << s) | (s && i ? (uint32_t)((uint64_t)v_in[i - 1] >> (32 - s)) : 0);
  un_[un] = s ? (uint32_t)((uint64_t)u[un - 1] >> (32 - s)) : 0;
  for (size_t i = un; i-- > 0;) un_[i] = (u[i] << s) | (s && i ? (uint32_t)((uint64_t)u[i - 1] >> (32 - s)) : 0);
  for (size_t jj = un - vn + 1; jj-- > 0;) {
    size_t j = jj;
    uint64_t num = ((uint64_t)un_[j + vn] << 32) | un_[j + vn - 1];
    uint64_t qhat = num / v[vn - 1], rhat = num % v[vn - 1];
    while (qhat >> 32 || qhat * v[vn - 2] > ((rhat << 32) | un_[j + vn - 2])) {
      --qhat;
      rhat += v[vn - 1];
      if (rhat >> 32) break;
    }
    int64_t borrow = 0;
    uint64_t carry = 0;
    for (size_t i = 0; i < vn; ++i) {
      uint64_t p = qhat * v[i] + carry;
      carry = p >> 32;
      int64_t t = (int64_t)un_[i + j] - (int64_t)(uint32_t)p - borrow;
      un_[i + j] = (uint32_t)t;
      borrow = t < 0;
    }
    int64_t t = (int64_t)un_[j + vn] - (int64_t)carry - borrow;
    un_[j + vn] = (uint32_t)t;
    if (t < 0) {
      uint64_t c = 0;
      for (size_t i = 0; i < vn; ++i) {
        c += (uint64_t)un_[i + j] + v[i];
        un_[i + j] = (uint32_t)c;
        c >>= 32;
      }
      un_[j + vn] += (uint32_t)c;
    }
  }
  for (size_t i = 0; i < vn; ++i) rem[i] = (un_[i] >> s) | (s ? (uint32_t)((uint64_t)un_[i + 1] << (32 - s)) : 0);
}

/*
 * Fold `count` big-endian operands of `width` bytes modulo N (mod_bytes, big-endian, N > 2^32).
 * Writes mod_bytes bytes (count >= 2) or width bytes verbatim (count == 1). Returns 0, or
 * 1 for count == 0 (404), 2 for bad arguments.
 */
int ddsref_fold(const uint8_t* mod_be, size_t mod_bytes, const uint8_t* ops, size_t width, size_t count,
                uint8_t* out) {
  if (count == 0) return 1;
  if (count == 1) { memcpy(out, ops, width); return 0; }
  size_t nw = (mod_bytes + 3) / 4, xw = (width + 3) / 4;
  uint32_t* N = calloc(nw, 4);
  from_be(mod_be, mod_bytes, N, nw);
  size_t nn = trim(N, nw);
  if (nn < 2) { free(N); return 2; }
  size_t cap = (nn > xw ? nn : xw);
  uint32_t* acc = calloc(cap, 4);
  uint32_t* x = calloc(xw, 4);
  uint32_t* prod = calloc(2 * cap + 2, 4);
  uint32_t* scratch = calloc(nn + 2 * cap + 4, 4);
  from_be(ops, width, acc, xw);
  size_t an = trim(acc, xw);
  for (size_t k = 1; k < count; ++k) {
    from_be(ops + k * width, width, x, xw);
    size_t xn = trim(x, xw);
    if (!an || !xn) { an = 0; continue; }
    mul(acc, an, x, xn, prod);                       /* acc.multiply(x) */
    size_t pn = trim(prod, an + xn);
    int lt = pn < nn;
    if (pn == nn) {
      lt = 0;
      for (size_t i = pn; i-- > 0;) if (prod[i] != N[i]) { lt = prod[i] < N[i]; break; }
    }
    if (lt) { memcpy(acc, prod, pn * 4); an = pn; continue; }
    knuth_mod(prod, pn, N, nn, acc, scratch);         /* .mod(nsquare) */
    an = trim(acc, nn);
  }
  memset(out, 0, mod_bytes);
  to_be(acc, an, out, mod_bytes);
  free(N); free(acc); free(x); free(prod); free(scratch);
  return 0;
}
