// The deterministic-equality routes from native code (the calls a JNA binding makes, without the Python
// binding's marshalling): T repetitions of SearchEntryOR (dds_search_entry, 3 values) and SearchEq at
// position 3 (dds_search_eq) over a resident string table of `rows` rows x 8 elements, each a 32-hex-char
// value drawn from a seeded vocabulary of 100k (the shape of bench.py's entry_search workload).
// Every reply is checked against a host scan of the same rows; prints one JSON line.
//
//   scan_bench [rows=10000000] [reps=25] [seed=3]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "ddshe.h"

namespace {
constexpr int kElems = 8, kWidth = 32, kVocab = 100000;

double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
}
}  // namespace

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 25;
  const unsigned seed = argc > 3 ? (unsigned)atoi(argv[3]) : 3u;
  dds_ctx* ctx = nullptr;
  if (dds_ctx_create(0, &ctx)) {
    fprintf(stderr, "dds_ctx_create: %s\n", dds_last_error());
    return 1;
  }
  std::mt19937_64 rng(seed);
  std::vector<char> vocab((size_t)kVocab * kWidth);
  for (auto& c : vocab) {
    const int d = (int)(rng() % 16);
    c = (char)(d < 10 ? '0' + d : 'a' + d - 10);
  }
  const size_t nel = n * kElems;
  std::vector<uint32_t> pick(nel);
  for (auto& p : pick) p = (uint32_t)(rng() % kVocab);
  std::vector<char> chars(nel * kWidth);
  for (size_t e = 0; e < nel; ++e) memcpy(chars.data() + e * kWidth, vocab.data() + (size_t)pick[e] * kWidth, kWidth);
  std::vector<uint64_t> eoff(nel + 1), roff(n + 1);
  for (size_t e = 0; e <= nel; ++e) eoff[e] = e * kWidth;
  for (size_t r = 0; r <= n; ++r) roff[r] = r * kElems;
  dds_strtab* tab = nullptr;
  if (dds_strtab_create(ctx, chars.data(), eoff.data(), nel, roff.data(), n, &tab)) {
    fprintf(stderr, "dds_strtab_create: %s\n", dds_last_error());
    return 1;
  }
  std::vector<char>().swap(chars);
  const uint32_t nid[3] = {11, 222, 3333};
  std::string needles[3];
  const char* vals[3];
  size_t lens[3];
  for (int j = 0; j < 3; ++j) {
    needles[j].assign(vocab.data() + (size_t)nid[j] * kWidth, kWidth);
    vals[j] = needles[j].c_str();
    lens[j] = kWidth;
  }
  // host answers (vocabulary index equality = string equality: the vocabulary may repeat a value, so
  // compare the strings of the picks, as the route does)
  std::vector<uint32_t> want_or, want_eq;
  for (size_t r = 0; r < n; ++r) {
    bool any = false;
    for (int k = 0; k < kElems && !any; ++k)
      for (int j = 0; j < 3 && !any; ++j)
        any = memcmp(vocab.data() + (size_t)pick[r * kElems + k] * kWidth, vals[j], kWidth) == 0;
    if (any) want_or.push_back((uint32_t)r);
    if (memcmp(vocab.data() + (size_t)pick[r * kElems + 3] * kWidth, vals[0], kWidth) == 0)
      want_eq.push_back((uint32_t)r);
  }
  std::vector<uint32_t> out(n);
  std::vector<double> t_or, t_eq;
  int bad = 0;
  for (int r = 0; r < reps + 2; ++r) {  // the first two rounds size the workers' buffers
    size_t got = 0;
    auto t0 = std::chrono::steady_clock::now();
    if (dds_search_entry(tab, vals, lens, 3, 0, out.data(), &got)) {
      fprintf(stderr, "dds_search_entry: %s\n", dds_last_error());
      return 1;
    }
    const double a = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (got != want_or.size() || !std::equal(want_or.begin(), want_or.end(), out.begin())) ++bad;
    t0 = std::chrono::steady_clock::now();
    if (dds_search_eq(tab, 3, vals[0], lens[0], 0, out.data(), &got)) {
      fprintf(stderr, "dds_search_eq: %s\n", dds_last_error());
      return 1;
    }
    const double b = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (got != want_eq.size() || !std::equal(want_eq.begin(), want_eq.end(), out.begin())) ++bad;
    if (r >= 2) {
      t_or.push_back(a);
      t_eq.push_back(b);
    }
  }
  printf("{\"rows\": %zu, \"elements_per_row\": %d, \"calls_each\": %zu, \"or_median_ms\": %.4f, \"or_p90_ms\": %.4f, "
         "\"eq_median_ms\": %.4f, \"eq_p90_ms\": %.4f, \"or_matches\": %zu, \"eq_matches\": %zu, \"mismatches\": %d, "
         "\"path\": \"dds_search_entry (SearchEntryOR, 3 values) + dds_search_eq (position 3) from C++\"}\n",
         n, kElems, t_or.size(), pct(t_or, 0.5), pct(t_or, 0.9), pct(t_eq, 0.5), pct(t_eq, 0.9), want_or.size(),
         want_eq.size(), bad);
  dds_strtab_destroy(tab);
  dds_ctx_destroy(ctx);
  return bad ? 1 : 0;
}
