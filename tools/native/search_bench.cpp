// The Search route from native code (the call a JNA binding makes, without the Python binding's
// marshalling): T repetitions of dds_opecol_search_mask over a resident 10M-row OPE column into an
// engine-allocated reply buffer (dds_host_alloc), each op of SearchGt/GtEq/Lt/LtEq at the median bound.
// Checks every reply against a host count of the same predicate, prints one JSON line.
//
//   search_bench [rows=10000000] [reps=25] [seed=3]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "ddshe.h"

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 25;
  const unsigned seed = argc > 3 ? (unsigned)atoi(argv[3]) : 3u;
  dds_ctx* ctx = nullptr;
  if (dds_ctx_create(0, &ctx)) {
    fprintf(stderr, "dds_ctx_create: %s\n", dds_last_error());
    return 1;
  }
  // an OPE-shaped column: a seeded increasing map of 10^4 plaintexts, rows drawing from it; 5 % of the
  // rows lack the position (class 0), the rest hold a Long (class 2)
  std::mt19937_64 rng(seed);
  std::vector<int64_t> map(10000);
  int64_t acc = -(int64_t(1) << 52);
  for (auto& m : map) m = (acc += 1 + (int64_t)(rng() % (uint64_t(1) << 40)));
  std::vector<int64_t> col(n);
  std::vector<uint8_t> cls(n);
  for (size_t i = 0; i < n; ++i) {
    col[i] = map[rng() % map.size()];
    cls[i] = (rng() % 100) < 95 ? 2 : 0;
  }
  const int64_t bound = map[map.size() / 2];
  dds_opecol* oc = nullptr;
  if (dds_opecol_create(ctx, n, &oc) || dds_opecol_append(oc, col.data(), cls.data(), n)) {
    fprintf(stderr, "opecol: %s\n", dds_last_error());
    return 1;
  }
  const size_t words = (n + 63) / 64;
  void* buf = nullptr;
  if (dds_host_alloc(ctx, words * 8, &buf)) {
    fprintf(stderr, "dds_host_alloc: %s\n", dds_last_error());
    return 1;
  }
  uint64_t* mask = (uint64_t*)buf;
  const std::string b = std::to_string(bound);
  std::vector<double> ms;
  int bad = 0;
  for (int op = 0; op < 4; ++op) {
    size_t want = 0;
    for (size_t i = 0; i < n; ++i) {
      if (!cls[i]) continue;
      const int64_t v = col[i];
      want += op == 0 ? v > bound : op == 1 ? v >= bound : op == 2 ? v < bound : v <= bound;
    }
    for (int r = 0; r < reps + 2; ++r) {
      size_t got = 0;
      const auto t0 = std::chrono::steady_clock::now();
      const int rc = dds_opecol_search_mask(oc, b.c_str(), op, mask, words, &got);
      const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (rc) {
        fprintf(stderr, "search_mask: %s\n", dds_last_error());
        return 1;
      }
      if (r >= 2) ms.push_back(t);  // the first two calls size the worker's buffers
      size_t pop = 0;
      for (size_t w = 0; w < words; ++w) pop += (size_t)__builtin_popcountll(mask[w]);
      if (got != want || pop != want) ++bad;
    }
  }
  std::sort(ms.begin(), ms.end());
  const double med = ms[ms.size() / 2];
  const double gbps = 9.0 * (double)n / (med * 1e-3) / 1e9;  // int64 + class byte per row, as the bench
  printf("{\"rows\": %zu, \"calls\": %zu, \"median_ms\": %.4f, \"p10_ms\": %.4f, \"p90_ms\": %.4f, "
         "\"route_GBps\": %.1f, \"route_frac_of_8TBps\": %.4f, \"mismatches\": %d, "
         "\"path\": \"dds_opecol_search_mask from C++ into a dds_host_alloc buffer\"}\n",
         n, ms.size(), med, ms[ms.size() / 10], ms[ms.size() * 9 / 10], gbps, gbps / 8000.0, bad);
  dds_host_free(ctx, buf);
  dds_opecol_destroy(oc);
  dds_ctx_destroy(ctx);
  return bad ? 1 : 0;
}
