// Host request router of the host-routed multi-GPU topology: ketama ownership plus
// hot-object spreading.
//
// Reference: the cache client picks the memcached node owning a key by ketama
// (src/python/shellac/server/Server.py:81-83), so a node receives its keys' true share
// of the traffic, hot keys included (README.md:30 sells ketama for node loss, not for
// load). Here each GPU of a node is a ketama node (DigestRing points), and the router
// adds what a Zipf workload needs on top: the hottest objects are replicated on every
// GPU (SURVEY.md §5.8 hot-object replication), a GET of one goes to a GPU chosen to
// even out the load, and a SET of one is written through to every GPU.
//
// Decisions are a pure function of (digest, position in the stream), identical to the
// tensor version in shellac_amd/parallel/hotspread.py (tests check both agree):
//   owner(d)   first ring point >= ring_position(d) (wrapping), DigestRing's rule. A
//              65536-entry table answers a 2^16-wide span no point splits directly and
//              names the first point of a split span otherwise, from which a short scan
//              (~1 point) finds the owner: no binary search on the request path.
//   GET i      a hot object's GETs go to its designated rank (chosen at the hot set's
//              refresh to even out the load; every rank holds a replica), or, for the few
//              objects too hot for one rank, to spray(seq0 + i): rank r with probability w_r
//              from a Weyl sequence, u = frac(j * 0x9E3779B97F4A7C15 / 2^64) (top 53 bits),
//              r = #{cumulative weight <= u}. Every other GET to owner(d).
//   SET        hot(d) ? every rank (dest -1) : owner(d).
//
// Throughput: a batch is split over a persistent worker pool (threads created once, not
// per call); a request costs a table load (cold) or a filter word and a hot-table slot
// (hot). Software prefetching of the slots measured no faster (they are cache-resident).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "digest.h"

namespace shellac {

class HostRouter {
 public:
  explicit HostRouter(int nshards, int points_per_shard = 160);
  ~HostRouter();
  HostRouter(const HostRouter&) = delete;
  HostRouter& operator=(const HostRouter&) = delete;
  int nshards() const { return n_; }
  int owner(const Digest& d) const {
    const uint32_t p = ring_position(d);
    const int32_t t = tab_[p >> 16];
    if (t >= 0) return t;
    size_t i = (size_t)(-(int64_t)t - 1);  // the span's first point; the owner is at or after it
    const size_t np = pts_.size();
    while (i < np && pts_[i] < p) ++i;
    return own_[i == np ? 0 : i];
  }
  // The replicated hot set (n digests, any order), each object's designated GET rank
  // (`rank`: n values, -1 = sprayed; null = all sprayed) and the spray weights (`w`:
  // nshards non-negative weights, normalised here). n = 0: no spreading.
  void set_hot(const Digest* hot, int64_t n, const int32_t* rank, const double* w);
  int64_t nhot() const { return nhot_; }
  // kNotHot, kSpray, or the object's designated rank
  static constexpr int kNotHot = -2, kSpray = -1;
  int hot_rank(const Digest& d) const {
    if (!nhot_) return kNotHot;
    const uint64_t b = (d.lo >> 20) & bits_mask_;
    if (!((hot_bits_[b >> 6] >> (b & 63)) & 1)) return kNotHot;
    for (uint64_t s = d.lo & hot_mask_;; s = (s + 1) & hot_mask_) {
      const HotSlot& e = hot_tab_[s];
      if (e.lo == d.lo && e.hi == d.hi) return e.rank;
      if (!e.lo && !e.hi) return kNotHot;
    }
  }
  bool is_hot(const Digest& d) const { return hot_rank(d) != kNotHot; }
  // dest[i] for a GET stream whose first request has stream position seq0; counts[r] +=
  // requests sent to r. `threads` <= 0: one.
  void route_gets(const Digest* keys, int64_t n, uint64_t seq0, int32_t* dest, int64_t* counts,
                  int threads) const;
  // dest[i] = owner, or -1 (a hot object: every rank); counts[r] += rows rank r stores.
  void route_sets(const Digest* keys, int64_t n, int32_t* dest, int64_t* counts,
                  int threads) const;
  // Cumulative spray weights (nshards doubles, the last exactly 1).
  const std::vector<double>& cumulative() const { return cw_; }

 private:
  // one slot of the hot table: the digest and its designated rank in one 32-B line half
  struct alignas(32) HotSlot {
    uint64_t lo = 0, hi = 0;
    int32_t rank = kSpray;
  };
  int search(uint32_t p) const;
  int spray(uint64_t j) const;
  template <bool kSets>
  void route_range(const Digest* keys, int64_t a, int64_t b, uint64_t seq0, int32_t* dest,
                   int64_t* counts) const;
  // f(a, b, counts) over `threads` slices of [0, n) on the worker pool; counts summed
  void parallel(int64_t n, int threads, int64_t* counts,
                const std::function<void(int64_t, int64_t, int64_t*)>& f) const;
  void worker(int id);
  int n_;
  std::vector<uint32_t> pts_;
  std::vector<int32_t> own_;
  std::vector<int32_t> tab_;      // 65536: owner of a span no point splits, else -(first point + 1)
  std::vector<HotSlot> hot_tab_;  // open addressing on lo (a hash already), {0, 0} = empty
  uint64_t hot_mask_ = 0;
  // a one-hash filter in front of it, 16 bits per hot object (~6 % of cold digests pass):
  // a cold request then costs no table line
  std::vector<uint64_t> hot_bits_;
  uint64_t bits_mask_ = 0;
  int64_t nhot_ = 0;
  std::vector<double> cw_;
  // the worker pool (grown on demand; one job at a time: callers serialise on call_mu_)
  mutable std::mutex call_mu_, mu_;
  mutable std::condition_variable cv_, done_cv_;
  mutable std::vector<std::thread> pool_;
  mutable const std::function<void(int)>* job_ = nullptr;
  mutable uint64_t gen_ = 0;
  mutable int want_ = 0, left_ = 0;
  mutable bool stop_ = false;
};

}  // namespace shellac
