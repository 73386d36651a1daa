// Core of the native host runtime (no Python): block pool, block hashing, KV indexer.
// Bound to Python by block_pool.cpp (module mxserve._rt); exercised standalone under ASan/UBSan by
// test_kv_runtime.cpp (tests/test_native_sanitizers.py).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace mxs_rt {
namespace detail {

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// 64-bit mixing in the spirit of xxh64's avalanche; deterministic across processes and platforms.
constexpr uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL, P3 = 0x165667B19E3779F9ULL;
inline uint64_t mix(uint64_t h) {
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

inline uint64_t hash_block(uint64_t parent, const int64_t* tok, int n, uint64_t extra) {
  uint64_t h = parent * P1 + extra + 0x27D4EB2F165667C5ULL + static_cast<uint64_t>(n);
  for (int i = 0; i < n; ++i) {
    h ^= mix(static_cast<uint64_t>(tok[i]) * P2);
    h = rotl(h, 27) * P1 + P3;
  }
  h = mix(h);
  return h == 0 ? 1 : h;  // 0 is reserved for "no hash"
}

}  // namespace detail
using detail::hash_block;

inline std::vector<uint64_t> block_hashes(const std::vector<int64_t>& tokens, int block_size, uint64_t extra,
                                   uint64_t parent) {
  std::vector<uint64_t> out;
  const int nfull = static_cast<int>(tokens.size()) / block_size;
  out.reserve(nfull);
  for (int b = 0; b < nfull; ++b) {
    parent = hash_block(parent, tokens.data() + static_cast<size_t>(b) * block_size, block_size, extra);
    out.push_back(parent);
  }
  return out;
}

class BlockPool {
 public:
  BlockPool(int num_blocks, bool prefix_caching)
      : n_(num_blocks), caching_(prefix_caching), ref_(num_blocks, 0), hash_(num_blocks, 0),
        prev_(num_blocks, -1), next_(num_blocks, -1) {
    if (num_blocks <= 0) throw std::invalid_argument("num_blocks must be > 0");
    for (int b = 0; b < n_; ++b) push_back(b);
  }

  int num_blocks() const { return n_; }
  int num_free() const { return nfree_; }
  double usage() const { return 1.0 - static_cast<double>(nfree_) / n_; }
  int num_cached() const { return static_cast<int>(map_.size()); }

  std::vector<int> allocate(int n) {
    if (n > nfree_) throw std::runtime_error("BlockPool: out of blocks");
    std::vector<int> out;
    out.reserve(n);
    for (int i = 0; i < n; ++i) {
      int b = head_;
      unlink(b);
      evict_hash(b);
      ref_[b] = 1;
      out.push_back(b);
    }
    return out;
  }

  // Free in the given order; callers pass a sequence's blocks tail-first so that the blocks least
  // likely to be shared are evicted first.
  void free(const std::vector<int>& blocks) {
    for (int b : blocks) {
      check(b);
      if (ref_[b] <= 0) throw std::runtime_error("BlockPool: double free of block " + std::to_string(b));
      if (--ref_[b] == 0) push_back(b);
    }
  }

  // Longest prefix of `hashes` present in the cache; takes a reference on every hit.
  std::vector<int> get_cached_prefix(const std::vector<uint64_t>& hashes) {
    std::vector<int> out;
    if (!caching_) return out;
    for (uint64_t h : hashes) {
      auto it = map_.find(h);
      if (it == map_.end()) break;
      int b = it->second;
      if (ref_[b] == 0) unlink(b);
      ++ref_[b];
      out.push_back(b);
    }
    hits_ += out.size();
    queries_ += hashes.size();
    return out;
  }

  // Count (without referencing) how many leading hashes are cached.
  int count_cached_prefix(const std::vector<uint64_t>& hashes) const {
    int n = 0;
    if (!caching_) return 0;
    for (uint64_t h : hashes) {
      if (map_.find(h) == map_.end()) break;
      ++n;
    }
    return n;
  }

  void cache_blocks(const std::vector<int>& blocks, const std::vector<uint64_t>& hashes) {
    if (!caching_) return;
    if (blocks.size() != hashes.size()) throw std::invalid_argument("blocks/hashes size mismatch");
    for (size_t i = 0; i < blocks.size(); ++i) {
      int b = blocks[i];
      check(b);
      uint64_t h = hashes[i];
      if (hash_[b] == h) continue;
      if (hash_[b] != 0) evict_hash(b);
      if (map_.count(h)) continue;  // another block already holds this content
      hash_[b] = h;
      map_.emplace(h, b);
      stored_.push_back(h);
    }
  }

  void reset_prefix_cache() {
    for (int b = 0; b < n_; ++b) evict_hash(b);
  }

  // (stored, removed) hashes since the last call -- the KV events a worker publishes
  std::pair<std::vector<uint64_t>, std::vector<uint64_t>> take_events() {
    std::pair<std::vector<uint64_t>, std::vector<uint64_t>> t{std::move(stored_), std::move(removed_)};
    stored_.clear();
    removed_.clear();
    return t;
  }

  double hit_rate() const { return queries_ ? static_cast<double>(hits_) / queries_ : 0.0; }
  int ref_count(int b) const { check(b); return ref_[b]; }

  // Invariants (SURVEY.md §5.2 block-manager checker): free-queue membership <=> ref == 0,
  // no negative refs, hash map and per-block hashes agree, nfree matches the queue length.
  bool check_invariants() const {
    int cnt = 0;
    std::vector<char> inq(n_, 0);
    for (int b = head_; b != -1; b = next_[b]) {
      if (b < 0 || b >= n_ || inq[b]) return false;
      inq[b] = 1;
      ++cnt;
      if (cnt > n_) return false;
    }
    if (cnt != nfree_) return false;
    for (int b = 0; b < n_; ++b) {
      if (ref_[b] < 0) return false;
      if ((ref_[b] == 0) != static_cast<bool>(inq[b])) return false;
      if (hash_[b] != 0) {
        auto it = map_.find(hash_[b]);
        if (it == map_.end() || it->second != b) return false;
      }
    }
    for (auto& kv : map_)
      if (hash_[kv.second] != kv.first) return false;
    return true;
  }

 private:
  void check(int b) const {
    if (b < 0 || b >= n_) throw std::out_of_range("block id " + std::to_string(b));
  }
  void push_back(int b) {
    prev_[b] = tail_;
    next_[b] = -1;
    if (tail_ != -1) next_[tail_] = b; else head_ = b;
    tail_ = b;
    ++nfree_;
  }
  void unlink(int b) {
    if (prev_[b] != -1) next_[prev_[b]] = next_[b]; else head_ = next_[b];
    if (next_[b] != -1) prev_[next_[b]] = prev_[b]; else tail_ = prev_[b];
    prev_[b] = next_[b] = -1;
    --nfree_;
  }
  void evict_hash(int b) {
    if (hash_[b] == 0) return;
    auto it = map_.find(hash_[b]);
    if (it != map_.end() && it->second == b) {
      map_.erase(it);
      removed_.push_back(hash_[b]);
    }
    hash_[b] = 0;
  }

  int n_;
  bool caching_;
  std::vector<int> ref_;
  std::vector<uint64_t> hash_;
  std::vector<int> prev_, next_;
  int head_ = -1, tail_ = -1, nfree_ = 0;
  std::unordered_map<uint64_t, int> map_;
  std::vector<uint64_t> stored_, removed_;
  uint64_t hits_ = 0, queries_ = 0;
};

// Router-side global index.  Workers are small integers (< 64) assigned by the router.
class KvIndexer {
 public:
  void apply_stored(int worker, const std::vector<uint64_t>& hashes) {
    uint64_t bit = wbit(worker);
    for (uint64_t h : hashes) {
      uint64_t& m = map_[h];
      if (!(m & bit)) ++count_[worker];
      m |= bit;
    }
  }
  void apply_removed(int worker, const std::vector<uint64_t>& hashes) {
    uint64_t bit = wbit(worker);
    for (uint64_t h : hashes) {
      auto it = map_.find(h);
      if (it == map_.end() || !(it->second & bit)) continue;
      it->second &= ~bit;
      --count_[worker];
      if (it->second == 0) map_.erase(it);
    }
  }
  void remove_worker(int worker) {
    uint64_t bit = wbit(worker);
    for (auto it = map_.begin(); it != map_.end();) {
      it->second &= ~bit;
      if (it->second == 0) it = map_.erase(it); else ++it;
    }
    count_[worker] = 0;
  }
  // Overlap (number of leading blocks cached) for each worker in [0, num_workers).
  std::vector<int> find_matches(const std::vector<uint64_t>& hashes, int num_workers) const {
    std::vector<int> out(num_workers, 0);
    uint64_t alive = num_workers >= 64 ? ~0ULL : ((1ULL << num_workers) - 1);
    for (size_t i = 0; i < hashes.size() && alive; ++i) {
      auto it = map_.find(hashes[i]);
      uint64_t m = it == map_.end() ? 0 : it->second;
      uint64_t still = alive & m;
      for (int w = 0; w < num_workers; ++w)
        if (still >> w & 1ULL) out[w] = static_cast<int>(i) + 1;
      alive = still;
    }
    return out;
  }
  int num_blocks(int worker) const { return worker >= 0 && worker < 64 ? count_[worker] : 0; }
  size_t size() const { return map_.size(); }

 private:
  static uint64_t wbit(int w) {
    if (w < 0 || w >= 64) throw std::out_of_range("worker index must be in [0, 64)");
    return 1ULL << w;
  }
  std::unordered_map<uint64_t, uint64_t> map_;
  int count_[64] = {0};
};

}  // namespace mxs_rt
