// Host-side presence filter over the digests a GPU cache tier holds (Bloom filter, k = 4,
// double hashing on the 128-bit MurmurHash3 digest). A GET whose digest the filter has
// never seen is answered "miss" on the host without a GPU batch; a cold-key miss then
// costs what a DRAM-cache miss costs instead of a kernel round trip.
//
// Only false positives are possible for keys added before the lookup: evictions and
// deletes never clear bits (a stale bit just sends that GET to the GPU, which misses).
// The owner rebuilds the filter from the tier's live keys when it fills up.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>

#include "digest.h"

namespace shellac {

class PresenceFilter {
 public:
  static constexpr int kHashes = 4;

  explicit PresenceFilter(uint64_t min_bits) {
    uint64_t bits = 1 << 16;
    while (bits < min_bits) bits <<= 1;
    mask_ = bits - 1;
    words_ = bits / 64;
    w_.reset(new std::atomic<uint64_t>[words_]);
    clear();
  }

  void add(const Digest& d) {
    const uint64_t h2 = d.hi | 1;
    for (int i = 0; i < kHashes; ++i) {
      const uint64_t b = (d.lo + (uint64_t)i * h2) & mask_;
      w_[b >> 6].fetch_or(1ull << (b & 63), std::memory_order_relaxed);
    }
    adds_.fetch_add(1, std::memory_order_relaxed);
  }

  bool maybe(const Digest& d) const {
    const uint64_t h2 = d.hi | 1;
    for (int i = 0; i < kHashes; ++i) {
      const uint64_t b = (d.lo + (uint64_t)i * h2) & mask_;
      if (!(w_[b >> 6].load(std::memory_order_relaxed) & (1ull << (b & 63)))) return false;
    }
    return true;
  }

  void clear() {
    for (uint64_t i = 0; i < words_; ++i) w_[i].store(0, std::memory_order_relaxed);
    adds_.store(0, std::memory_order_relaxed);
  }

  uint64_t bits() const { return mask_ + 1; }
  uint64_t adds() const { return adds_.load(std::memory_order_relaxed); }
  // Expected fraction of set bits after adds() insertions: 1 - e^(-k n / m).
  double fill() const;

 private:
  std::unique_ptr<std::atomic<uint64_t>[]> w_;
  uint64_t mask_ = 0, words_ = 0;
  std::atomic<uint64_t> adds_{0};
};

inline double PresenceFilter::fill() const {
  const double x = (double)kHashes * (double)adds() / (double)bits();
  // 1 - e^-x without <cmath> in every includer
  double term = 1, sum = 1;
  for (int i = 1; i < 30; ++i) {
    term *= -x / i;
    sum += term;
  }
  return x > 20 ? 1.0 : 1.0 - sum;
}

}  // namespace shellac
