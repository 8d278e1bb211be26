// /Sum coalescing under native threads (VERDICT r02 "next" 5): T threads call dds_pair_modmul_dec
// concurrently on one context, as the proxy's ForkJoin pool runs /Sum routes (DDSRestServer.scala:21,
// 355-395), with no interpreter lock between them. Reports calls per k_pairs launch, pairs/s and the
// per-call latency distribution as one JSON line, plus a few (a, b, result) samples for the caller to
// check (bench.py verifies them with Python ints). The serving policy is the context default
// (DDSHE_PAIR_POLICY; dds_pair_set_policy); the line carries the host CPU per call, whole process and by
// phase (dds_pair_cpu).
//
//   pair_bench <modulus_dec> <threads> <calls_per_thread> [seed] [warmup_calls_per_thread=20]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>
#include <atomic>
#include <sys/resource.h>

#include "ddshe.h"

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <modulus_dec> <threads> <calls_per_thread> [seed] [warmup]\n", argv[0]);
    return 2;
  }
  const std::string mod = argv[1];
  const int T = atoi(argv[2]), K = atoi(argv[3]);
  const unsigned seed = argc > 4 ? (unsigned)atoi(argv[4]) : 7u;
  const int WU = argc > 5 ? atoi(argv[5]) : 20;  // warm-up calls per thread, not timed
  dds_ctx* ctx = nullptr;
  if (dds_ctx_create(0, &ctx)) {
    fprintf(stderr, "dds_ctx_create: %s\n", dds_last_error());
    return 1;
  }
  // operands: random decimals one digit shorter than the modulus (so below it), per thread
  std::vector<std::vector<std::string>> A(T), B(T), R(T);
  std::mt19937_64 rng(seed);
  auto rnd = [&](size_t digits) {
    std::string s(digits, '0');
    s[0] = (char)('1' + rng() % 9);
    for (size_t i = 1; i < digits; ++i) s[i] = (char)('0' + rng() % 10);
    return s;
  };
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < K + 1; ++i) {
      A[t].push_back(rnd(mod.size() - 1));
      B[t].push_back(rnd(mod.size() - 1));
    }
  const size_t cap = 2 * mod.size() + 64;
  // warm-up (modulus constants, streams, pinned buffers), then a barrier and the timed phase
  {
    std::vector<char> out(cap);
    size_t len = 0;
    if (dds_pair_modmul_dec(ctx, A[0][K].c_str(), B[0][K].c_str(), mod.c_str(), out.data(), cap, &len)) {
      fprintf(stderr, "warm-up: %s\n", dds_last_error());
      return 1;
    }
  }
  uint64_t c0 = 0, l0 = 0, c1 = 0, l1 = 0, b0 = 0, g0 = 0, b1 = 0, g1 = 0, mx = 0, mg = 0;
  std::vector<std::vector<double>> lat(T);
  std::atomic<int> ready{0}, errors{0};
  std::atomic<bool> go{false};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      std::vector<char> out(cap);
      size_t len = 0;
      // warm-up under load: every caller's first calls (the workers, streams and pinned batch buffers
      // the concurrent leaders need are set up here, as in a server that has been running)
      for (int i = 0; i < WU; ++i)
        if (dds_pair_modmul_dec(ctx, A[t][K].c_str(), B[t][K].c_str(), mod.c_str(), out.data(), cap, &len))
          errors.fetch_add(1);
      ready.fetch_add(1);
      while (!go.load()) std::this_thread::yield();
      for (int i = 0; i < K; ++i) {
        const auto s = std::chrono::steady_clock::now();
        const int rc = dds_pair_modmul_dec(ctx, A[t][i].c_str(), B[t][i].c_str(), mod.c_str(), out.data(), cap, &len);
        const auto e = std::chrono::steady_clock::now();
        if (rc) {
          errors.fetch_add(1);
          continue;
        }
        lat[t].push_back(std::chrono::duration<double, std::milli>(e - s).count());
        if (i < 2) R[t].push_back(std::string(out.data(), len));
      }
    });
  while (ready.load() < T) std::this_thread::yield();
  dds_pair_stats(ctx, &c0, &l0);
  dds_pair_timing(ctx, &b0, &g0, &mx, &mg);  // also restarts the longest-batch windows
  uint64_t p0[6], p1[6];  // host CPU by phase (dds_pair_cpu)
  dds_pair_cpu(ctx, &p0[0], &p0[1], &p0[2], &p0[3], &p0[4], &p0[5]);
  struct rusage ru0, ru1;
  getrusage(RUSAGE_SELF, &ru0);
  const auto t0 = std::chrono::steady_clock::now();
  go.store(true);
  for (auto& x : th) x.join();
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  getrusage(RUSAGE_SELF, &ru1);
  auto tv = [](const timeval& a, const timeval& b) { return (double)(b.tv_sec - a.tv_sec) + 1e-6 * (double)(b.tv_usec - a.tv_usec); };
  const double cpu_s = tv(ru0.ru_utime, ru1.ru_utime) + tv(ru0.ru_stime, ru1.ru_stime);
  dds_pair_stats(ctx, &c1, &l1);
  dds_pair_timing(ctx, &b1, &g1, &mx, &mg);
  dds_pair_cpu(ctx, &p1[0], &p1[1], &p1[2], &p1[3], &p1[4], &p1[5]);
  int policy = -1;
  dds_pair_set_policy(ctx, -1, &policy);
  const double ncalls = c1 > c0 ? (double)(c1 - c0) : 1.0;
  auto per_call_us = [&](int i) { return (double)(p1[i] - p0[i]) / ncalls * 1e-3; };
  const double nl = l1 > l0 ? (double)(l1 - l0) : 1.0;
  std::vector<double> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, (size_t)(p * all.size()))]; };
  size_t moduli = 0, queues = 0;
  dds_ctx_cache_stats(ctx, &moduli, &queues);
  printf("{\"threads\": %d, \"calls\": %llu, \"launches\": %llu, \"calls_per_launch\": %.2f, \"pairs_per_s\": %.1f, "
         "\"p50_ms\": %.4f, \"p99_ms\": %.4f, \"max_ms\": %.4f, \"errors\": %d, \"modulus_digits\": %zu, "
         "\"cached_moduli\": %zu, \"pair_queues_after\": %zu, \"hw_threads\": %u, "
         "\"batch_us_per_launch\": %.2f, \"gpu_round_trip_us_per_launch\": %.2f, \"wall_us_per_launch\": %.2f, "
         "\"mean_batches_in_flight\": %.3f, \"max_batch_ms\": %.3f, \"max_gpu_round_trip_ms\": %.3f, \"cpu_cores_busy\": %.2f, "
         "\"involuntary_switches\": %ld, \"voluntary_switches\": %ld, \"policy\": %d, \"cpu_us_per_call\": %.2f, "
         "\"phase_cpu_us_per_call\": {\"codec\": %.2f, \"pack\": %.2f, \"queue\": %.2f, \"gpu_wait\": %.2f, "
         "\"host_product\": %.2f}, \"host_served\": %llu, \"samples\": [",
         T, (unsigned long long)(c1 - c0), (unsigned long long)(l1 - l0),
         (l1 > l0) ? (double)(c1 - c0) / (double)(l1 - l0) : 0.0, (double)all.size() / secs, pct(0.5), pct(0.99),
         all.empty() ? 0.0 : all.back(), errors.load(), mod.size(), moduli, queues, std::thread::hardware_concurrency(),
         (double)(b1 - b0) / nl * 1e-3, (double)(g1 - g0) / nl * 1e-3, secs / nl * 1e6, (double)(b1 - b0) * 1e-9 / secs,
         (double)mx * 1e-6, (double)mg * 1e-6, cpu_s / secs, ru1.ru_nivcsw - ru0.ru_nivcsw, ru1.ru_nvcsw - ru0.ru_nvcsw,
         policy, cpu_s / ncalls * 1e6, per_call_us(0), per_call_us(1), per_call_us(2), per_call_us(3), per_call_us(4),
         (unsigned long long)(p1[5] - p0[5]));
  bool first = true;
  for (int t = 0; t < std::min(T, 4); ++t)
    for (size_t i = 0; i < R[t].size(); ++i) {
      printf("%s[\"%s\", \"%s\", \"%s\"]", first ? "" : ", ", A[t][i].c_str(), B[t][i].c_str(), R[t][i].c_str());
      first = false;
    }
  printf("]}\n");
  dds_ctx_destroy(ctx);
  return errors.load() ? 1 : 0;
}
