// Host request router of the multi-GPU cache: ketama ownership plus hot-object spreading.
// Used by the proxy's HBM tier (HbmBackend routes every GET / SET / DELETE through it)
// and by the bench's host-routed job (parallel/hotspread.py HotSpread).
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
//              65536-entry span table answers it with one 8-byte load and two compares: each
//              2^16-wide span stores the (at most two) points inside it and the owners on
//              either side of them; the rare span with more points falls back to a search.
//   GET i      a hot object's GETs go to its designated rank (chosen at the hot set's
//              refresh to even out the load; every rank holds a replica), or, for the few
//              objects too hot for one rank, to spray(seq0 + i): rank r with probability w_r
//              from a Weyl sequence, u = frac(j * 0x9E3779B97F4A7C15 / 2^64) (top 53 bits),
//              r = #{cumulative weight <= u}. Every other GET to owner(d).
//   SET        hot(d) ? every rank (dest -1) : owner(d).
//
// Concurrency: the hot set is an immutable HotTable. set_hot builds the next one aside,
// publishes it with one pointer store and then waits until no reader can still hold the
// previous one (a sleepable-RCU grace period: readers count themselves in one of two
// per-slot counters picked by the current phase; the writer flips the phase twice and
// waits for the old phase's counters to drain) before freeing it. Readers (route_gets /
// route_sets per call, a Read guard per request in the proxy) take no lock and touch
// only a counter line of their own thread slot. When set_hot returns, every routing
// decision made under an older table has finished — the hot-set refresh protocol of
// HbmBackend (write-through first, designation second) relies on exactly that.
//
// Throughput: a batch is split over a persistent worker pool (threads created once, not
// per call). Requests go eight at a time through 512-bit lanes where the CPU has AVX-512
// (route_x8): the span entry, filter word and hot-table slots are gathered and owner,
// hot code and spray rank computed and selected under lane masks; a lane needing more (a
// span with more than two points, a digest past its second probe slot, a spray over more
// than 64 ranks) is redone by the scalar rule. The scalar rule (CPUs without
// AVX-512) selects by masks too: branching on hot vs cold mispredicted on a large share of
// a Zipf stream's requests. The hot set must arrive hottest first (HotSpread passes plan's
// order): inserted in digest order, displaced hot objects sent a quarter of the 8-lane
// groups down the second probe and 4.6 % of the lanes to the scalar redo. Per thread on a
// Xeon core (scripts/router_micro.py, 8 GPUs, 1024 hot objects, Zipf 0.99): 45-63 M
// requests/s scalar, 165-190 M in lanes; 174 and ~260 M without a hot set.
// The hot table matches a digest on its low word and the top 48 bits of its high word (the
// low 16 bits hold the rank): a cold digest agreeing on those 112 bits would be treated as
// hot — consistently for its GETs and SETs, so it would still be served correctly.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
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
    const uint64_t e = span_[p >> 16];
    if (e >> 63) return search(p);  // a span with more than two points
    const uint32_t t = p & 0xFFFFu, c1 = e & 0xFFFFu, c2 = (e >> 16) & 0xFFFFu;
    const int o1 = (int)((e >> 32) & 1023), o2 = (int)((e >> 42) & 1023),
              o3 = (int)((e >> 52) & 1023);
    return t <= c1 ? o1 : (t <= c2 ? o2 : o3);
  }
  // kNotHot, kSpray, or the object's designated rank
  static constexpr int kNotHot = -2, kSpray = -1;

  // hot table: open addressing on lo (linear probing, at most a quarter full), slots
  // {lo, (hi & ~0xFFFF) | code}, code = designated rank + 2 (1: sprayed, 0: empty). The hot
  // set is inserted hottest first, so the objects that carry most requests sit in their
  // home slot; a one-hash filter (16 bits per object) answers most cold digests.
  struct HotSlot {
    uint64_t lo = 0, tag = 0;
  };
  struct HotTable {
    std::vector<HotSlot> tab = std::vector<HotSlot>(1);  // one empty slot: no hot set
    uint64_t mask = 0;
    std::vector<uint64_t> bits = std::vector<uint64_t>(1, 0);
    uint64_t bits_mask = 0;
    int64_t nhot = 0;
    std::vector<double> cw;         // cumulative spray weights (the last exactly 1)
    std::vector<uint64_t> spray_t;  // ceil(cw * 2^53): spray() on integers (the lane path)
    static bool match(const HotSlot& e, const Digest& d) {
      return (e.lo == d.lo) & (((e.tag ^ d.hi) >> 16) == 0) & ((e.tag & 0xFFFFu) != 0);
    }
    // 0: not hot; 1: sprayed; r + 2: designated rank r. The common cases (a cold digest the
    // filter rejects, a hot one in its home slot) take no data-dependent branch: a rejected
    // digest reads slot 0 instead of its home slot (a cached line), and the code is masked.
    uint32_t code(const Digest& d) const {
      const uint64_t fb = (d.lo >> 20) & bits_mask;
      const uint64_t pass = (bits[fb >> 6] >> (fb & 63)) & 1;
      const HotSlot& e = tab[d.lo & mask];  // the home slot, read either way
      const uint64_t hit = pass & (uint64_t)match(e, d);
      if (__builtin_expect(pass & (hit ^ 1), 0)) return code_slow(d);  // probe further
      return (uint32_t)(e.tag & 0xFFFFu & ((uint64_t)0 - hit));
    }
    uint32_t code_slow(const Digest& d) const;
    int spray(uint64_t j) const;  // the Weyl rank of stream position j
  };

  // A reader's hold on the current table (no lock; see the header comment). Keep it for
  // the whole decision, including whatever the decision queues.
  class Read {
   public:
    explicit Read(const HostRouter& r);
    ~Read();
    Read(const Read&) = delete;
    Read& operator=(const Read&) = delete;
    const HotTable& table() const { return *t_; }
    int hot_rank(const Digest& d) const {
      const uint32_t c = t_->nhot ? t_->code(d) : 0;
      return c == 0 ? kNotHot : (int)c - 2;
    }
    int spray(uint64_t j) const { return t_->spray(j); }

   private:
    const HostRouter& r_;
    const HotTable* t_;
    int slot_, phase_;
  };

  // The replicated hot set (n digests, hottest first), each object's designated GET rank
  // (`rank`: n values, -1 = sprayed; null = all sprayed) and the spray weights (`w`:
  // nshards non-negative weights, normalised here). n = 0: no spreading. Returns once no
  // reader can still be using the previous table (it is freed here). Writers serialise.
  void set_hot(const Digest* hot, int64_t n, const int32_t* rank, const double* w);
  int64_t nhot() const;
  int hot_rank(const Digest& d) const { return Read(*this).hot_rank(d); }
  bool is_hot(const Digest& d) const { return hot_rank(d) != kNotHot; }
  // dest[i] for a GET stream whose first request has stream position seq0; counts[r] +=
  // requests sent to r. `threads` <= 0: one.
  void route_gets(const Digest* keys, int64_t n, uint64_t seq0, int32_t* dest, int64_t* counts,
                  int threads) const;
  // dest[i] = owner, or -1 (a hot object: every rank); counts[r] += rows rank r stores.
  void route_sets(const Digest* keys, int64_t n, int32_t* dest, int64_t* counts,
                  int threads) const;
  // The 8-lane AVX-512 GET path (on where the CPU has AVX-512F/DQ; off: the scalar rule).
  // Both make the same decisions; the switch is for tests and comparisons.
  bool lanes() const { return lanes_; }
  void set_lanes(bool on);
  // Cumulative spray weights of the current table (nshards doubles, the last exactly 1).
  std::vector<double> cumulative() const;
  // Tables published so far and grace periods waited (tests, stats).
  uint64_t publications() const { return pubs_.load(std::memory_order_relaxed); }

 private:
  int search(uint32_t p) const;
  template <bool kSets>
  int route_one(const HotTable& t, const Digest& d, uint64_t j) const;  // the scalar rule
  template <bool kSets>
  void route_x8(const HotTable& t, const Digest* keys, int64_t a, int64_t b, uint64_t seq0,
                int32_t* dest, int64_t* counts) const;
  template <bool kSets>
  void route_range(const HotTable& t, const Digest* keys, int64_t a, int64_t b, uint64_t seq0,
                   int32_t* dest, int64_t* counts) const;
  // f(a, b, counts) over `threads` slices of [0, n) on the worker pool; counts summed
  void parallel(int64_t n, int threads, int64_t* counts,
                const std::function<void(int64_t, int64_t, int64_t*)>& f) const;
  void worker(int id);
  void set_thresholds(HotTable* t) const;
  int n_;
  std::vector<uint32_t> pts_;
  std::vector<int32_t> own_;
  // per 2^16-wide span: c1 | c2 << 16 | o1 << 32 | o2 << 42 | o3 << 52, bit 63 = more than
  // two points (owner() searches)
  std::vector<uint64_t> span_;
  bool lanes_;
  // published table + grace-period state
  std::atomic<const HotTable*> hot_{nullptr};
  static constexpr int kReadSlots = 64;
  struct alignas(64) ReadSlot {
    std::atomic<int64_t> c[2];
  };
  std::unique_ptr<ReadSlot[]> readers_;
  std::atomic<uint64_t> phase_{0};
  std::atomic<uint64_t> pubs_{0};
  std::mutex set_mu_;
  void grace_period();
  // the worker pool (grown on demand; one job at a time: callers serialise on call_mu_)
  mutable std::mutex call_mu_, mu_;
  mutable std::condition_variable cv_, done_cv_;
  mutable std::vector<std::thread> pool_;
  mutable const std::function<void(int)>* job_ = nullptr;
  mutable uint64_t gen_ = 0;
  mutable int want_ = 0, left_ = 0;
  mutable bool stop_ = false;
};

// Hot-set planning from sampled GET counts (HotSpread.design's "designate" policy, native):
// the top `k` digests by count (count >= min_count; ties by digest), hottest first; each
// designated greedily — hottest first, to the eligible rank with the least load so far,
// starting from the ranks' loads of the sampled non-hot GETs at their owners plus an even
// share of the sprayed objects — and objects above `spray_above` of all sampled GETs
// sprayed over the eligible ranks. `owner(d)` gives a digest's rank; `eligible` is a rank
// mask (bit r). Returns the hot digests, their ranks (-1 = sprayed), the spray weights (1
// for eligible ranks, 0 otherwise), the hot share and the planned per-rank load shares.
struct HotPlan {
  std::vector<Digest> hot;
  std::vector<int32_t> rank;
  std::vector<double> weights;
  double hot_share = 0;
  std::vector<double> planned;
};
// `sticky` (optional): objects that are hot already rank with their count x sticky_factor
// (hysteresis: a refresh does not churn the tail of the set on sampling noise; their loads
// use the true counts).
HotPlan plan_hot(const std::vector<std::pair<Digest, uint64_t>>& counts, int k, int nshards,
                 uint64_t eligible, const std::function<int(const Digest&)>& owner,
                 double spray_above, uint64_t min_count = 2,
                 const std::function<bool(const Digest&)>* sticky = nullptr,
                 double sticky_factor = 1.0);

}  // namespace shellac
