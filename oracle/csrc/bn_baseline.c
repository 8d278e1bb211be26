/*
 * bn_baseline.c — OpenSSL BIGNUM CPU baselines (TEST INFRASTRUCTURE / CPU BASELINE ONLY).
 *
 * "a C++ OpenSSL BN_mod_mul fold, 1 thread (faithful) and nproc threads (slice
 * fold + combine)". Restates
 *   SumAll / MultAll fold  /root/reference/src/main/scala/dds/http/DDSRestServer.scala:412-430, :506-524
 *     acc = x0 (unreduced); acc = acc * x mod N     (HomoAdd.sum / HomoMult.multiply, :423, :518)
 *   HomoAdd.encrypt(m, key) = g^m * r^n mod n^2    (utils/SJHomoLibProvider.scala:58; hlib absent,
 *                                                   textbook Paillier with the key's random g)
 * with OpenSSL's BN_mod_mul / BN_mod_exp (Montgomery + sliding window for odd moduli, the same
 * algorithm family as java.math.BigInteger.modPow). Used only by bench.py's cpu_baseline leg and
 * tests; never by the product path.
 */
#include <openssl/bn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const uint8_t* mod;
  size_t mod_bytes;
  const uint8_t* ops;
  size_t width, first, count;
  uint8_t* out; /* mod_bytes */
  int rc;
} fold_job;

static void* fold_worker(void* arg) {
  fold_job* j = (fold_job*)arg;
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *N = BN_bin2bn(j->mod, (int)j->mod_bytes, NULL), *acc = BN_new(), *x = BN_new();
  j->rc = 1;
  if (!ctx || !N || !acc || !x) goto done;
  BN_bin2bn(j->ops + j->first * j->width, (int)j->width, acc);
  for (size_t i = 1; i < j->count; ++i) {
    BN_bin2bn(j->ops + (j->first + i) * j->width, (int)j->width, x);
    if (!BN_mod_mul(acc, acc, x, N, ctx)) goto done;
  }
  if (j->count > 1 || BN_num_bytes(acc) <= (int)j->mod_bytes) {
    if (!BN_mod(acc, acc, N, ctx)) goto done;  /* slice partials are combined mod N */
    BN_bn2binpad(acc, j->out, (int)j->mod_bytes);
    j->rc = 0;
  }
done:
  BN_free(N);
  BN_free(acc);
  BN_free(x);
  BN_CTX_free(ctx);
  return NULL;
}

/* prod(ops) mod N over count >= 2 operands with `threads` contiguous slices (1 = the faithful
 * single-threaded loop). out: mod_bytes big-endian. Returns 0 on success. */
int bnref_fold(const uint8_t* mod, size_t mod_bytes, const uint8_t* ops, size_t width, size_t count, int threads,
               uint8_t* out) {
  if (count < 2 || threads < 1) return 2;
  if ((size_t)threads > count / 2) threads = (int)(count / 2);
  fold_job* jobs = calloc((size_t)threads, sizeof(fold_job));
  pthread_t* tid = calloc((size_t)threads, sizeof(pthread_t));
  uint8_t* parts = calloc((size_t)threads, mod_bytes);
  int rc = 0;
  for (int t = 0; t < threads; ++t) {
    const size_t a = count * (size_t)t / (size_t)threads, b = count * (size_t)(t + 1) / (size_t)threads;
    jobs[t] = (fold_job){mod, mod_bytes, ops, width, a, b - a, parts + (size_t)t * mod_bytes, 0};
    if (threads == 1) fold_worker(&jobs[t]);
    else pthread_create(&tid[t], NULL, fold_worker, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  for (int t = 0; t < threads; ++t) rc |= jobs[t].rc;
  if (!rc) {
    if (threads == 1) {
      memcpy(out, parts, mod_bytes);
    } else {
      fold_job c = {mod, mod_bytes, parts, mod_bytes, 0, (size_t)threads, out, 0};
      fold_worker(&c);
      rc = c.rc;
    }
  }
  free(jobs);
  free(tid);
  free(parts);
  return rc;
}

typedef struct {
  const uint8_t *n, *g;
  size_t n_bytes, g_bytes;
  const uint32_t* m;
  const uint8_t* r;
  size_t r_width, first, count, nsq_bytes;
  uint8_t* out;
  int rc;
} enc_job;

static void* enc_worker(void* arg) {
  enc_job* j = (enc_job*)arg;
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *n = BN_bin2bn(j->n, (int)j->n_bytes, NULL), *g = BN_bin2bn(j->g, (int)j->g_bytes, NULL);
  BIGNUM *nsq = BN_new(), *a = BN_new(), *b = BN_new(), *r = BN_new(), *m = BN_new();
  BN_MONT_CTX* mont = BN_MONT_CTX_new();
  j->rc = 1;
  if (!ctx || !n || !g || !nsq || !a || !b || !r || !m || !mont) goto done;
  if (!BN_sqr(nsq, n, ctx) || !BN_MONT_CTX_set(mont, nsq, ctx)) goto done;
  for (size_t i = j->first; i < j->first + j->count; ++i) {
    BN_set_word(m, j->m[i]);
    BN_bin2bn(j->r + i * j->r_width, (int)j->r_width, r);
    if (!BN_mod_exp_mont(a, g, m, nsq, ctx, mont) || !BN_mod_exp_mont(b, r, n, nsq, ctx, mont) ||
        !BN_mod_mul(a, a, b, nsq, ctx))
      goto done;
    BN_bn2binpad(a, j->out + i * j->nsq_bytes, (int)j->nsq_bytes);
  }
  j->rc = 0;
done:
  BN_free(n); BN_free(g); BN_free(nsq); BN_free(a); BN_free(b); BN_free(r); BN_free(m);
  BN_MONT_CTX_free(mont);
  BN_CTX_free(ctx);
  return NULL;
}

/* out[i] = g^m[i] * r[i]^n mod n^2 (public-key Paillier encryption), `threads` workers. */
int bnref_paillier_encrypt(const uint8_t* n, size_t n_bytes, const uint8_t* g, size_t g_bytes, const uint32_t* m,
                           const uint8_t* r, size_t r_width, size_t count, int threads, uint8_t* out,
                           size_t nsq_bytes) {
  if (threads < 1) return 2;
  if ((size_t)threads > count) threads = count ? (int)count : 1;
  enc_job* jobs = calloc((size_t)threads, sizeof(enc_job));
  pthread_t* tid = calloc((size_t)threads, sizeof(pthread_t));
  int rc = 0;
  for (int t = 0; t < threads; ++t) {
    const size_t a = count * (size_t)t / (size_t)threads, b = count * (size_t)(t + 1) / (size_t)threads;
    jobs[t] = (enc_job){n, g, n_bytes, g_bytes, m, r, r_width, a, b - a, nsq_bytes, out, 0};
    if (threads == 1) enc_worker(&jobs[t]);
    else pthread_create(&tid[t], NULL, enc_worker, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  for (int t = 0; t < threads; ++t) rc |= jobs[t].rc;
  free(jobs);
  free(tid);
  return rc;
}
