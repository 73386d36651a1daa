// Standalone stress test of the host runtime core, built with -fsanitize=address,undefined by
// tests/test_native_sanitizers.py (race/memory checking of native host code; GPU
// sanitizers are not available on the test pool).  Random allocate / cache / prefix-hit / free
// sequences against a shadow model, plus indexer churn; exits non-zero on the first mismatch.
#include <cstdio>
#include <random>
#include <set>

#include "kv_runtime.h"

using mxs_rt::BlockPool;
using mxs_rt::KvIndexer;

#define REQUIRE(c)                                                     \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "FAILED %s at line %d\n", #c, __LINE__);   \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  std::mt19937_64 rng(12345);
  // ---- block pool vs a shadow reference count
  BlockPool p(257, true);
  std::vector<int> shadow(257, 0);
  std::vector<std::vector<int>> held;
  for (int step = 0; step < 200000; ++step) {
    const int op = static_cast<int>(rng() % 10);
    if (op < 4 && p.num_free() > 0) {
      const int n = 1 + static_cast<int>(rng() % std::min(8, p.num_free()));
      auto b = p.allocate(n);
      std::vector<uint64_t> hs;
      for (int x : b) {
        REQUIRE(shadow[x] == 0);
        shadow[x] = 1;
        hs.push_back(1 + rng() % 500);
      }
      p.cache_blocks(b, hs);
      held.push_back(b);
    } else if (op < 7 && !held.empty()) {
      const size_t i = rng() % held.size();
      std::vector<int> b = held[i];
      held.erase(held.begin() + static_cast<long>(i));
      for (int x : b) --shadow[x];
      p.free(std::vector<int>(b.rbegin(), b.rend()));
    } else {
      std::vector<uint64_t> q;
      for (int k = 0; k < 4; ++k) q.push_back(1 + rng() % 500);
      auto hit = p.get_cached_prefix(q);
      for (int x : hit) ++shadow[x];
      if (!hit.empty()) held.push_back(hit);
    }
    if (step % 1000 == 0) {
      REQUIRE(p.check_invariants());
      for (int b = 0; b < 257; ++b) REQUIRE(p.ref_count(b) == shadow[b]);
      auto ev = p.take_events();
      (void)ev;
    }
  }
  // double free must be rejected, not corrupt the pool
  {
    BlockPool q(4, true);
    auto b = q.allocate(1);
    q.free(b);
    bool threw = false;
    try {
      q.free(b);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    REQUIRE(threw && q.check_invariants());
  }
  // ---- hashing: prefix property
  std::vector<int64_t> toks(1000);
  for (auto& t : toks) t = static_cast<int64_t>(rng() % 128000);
  auto h = mxs_rt::block_hashes(toks, 16, 0, 0);
  auto h2 = mxs_rt::block_hashes(std::vector<int64_t>(toks.begin(), toks.begin() + 160), 16, 0, 0);
  REQUIRE(h.size() == 62 && h2.size() == 10);
  for (size_t i = 0; i < h2.size(); ++i) REQUIRE(h[i] == h2[i]);
  // ---- indexer churn vs a shadow set per worker
  KvIndexer ix;
  std::vector<std::set<uint64_t>> sh(64);
  for (int step = 0; step < 100000; ++step) {
    const int w = static_cast<int>(rng() % 64);
    std::vector<uint64_t> hs;
    for (int k = 0; k < 8; ++k) hs.push_back(h[rng() % h.size()]);
    if (rng() % 3) {
      ix.apply_stored(w, hs);
      sh[w].insert(hs.begin(), hs.end());
    } else {
      ix.apply_removed(w, hs);
      for (auto x : hs) sh[w].erase(x);
    }
    if (step % 997 == 0) {
      const int v = static_cast<int>(rng() % 64);
      ix.remove_worker(v);
      sh[v].clear();
    }
    if (step % 500 == 0) {
      for (int x = 0; x < 64; ++x) REQUIRE(ix.num_blocks(x) == static_cast<int>(sh[x].size()));
      auto m = ix.find_matches(h, 64);
      for (int x = 0; x < 64; ++x) {
        int want = 0;
        while (want < static_cast<int>(h.size()) && sh[x].count(h[want])) ++want;
        REQUIRE(m[x] == want);
      }
    }
  }
  std::printf("kv_runtime stress: OK\n");
  return 0;
}
