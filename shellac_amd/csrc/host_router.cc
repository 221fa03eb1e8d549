// HostRouter (host_router.h): ketama ownership + hot-object spreading for the host-routed
// multi-GPU topology.
#include "host_router.h"

#include <algorithm>
#include <string>
#include <thread>

namespace shellac {

namespace {
constexpr uint64_t kWeyl = 0x9E3779B97F4A7C15ull;  // 2^64 / golden ratio
}  // namespace

HostRouter::HostRouter(int nshards, int pps)
    : n_(nshards), span_(65536, 0), hot_tab_(1), hot_bits_(1, 0) {
  SH_CHECK(nshards >= 1 && nshards <= 1023 && pps >= 1, "bad router geometry");
  std::vector<std::pair<uint32_t, int>> pts;
  for (int i = 0; i < nshards; ++i)
    for (int j = 0; j < pps; ++j) {  // DigestRing's (and ShardRing's) points
      const std::string s = "shellac-shard-" + std::to_string(i) + "-" + std::to_string(j);
      const Digest d = digest_bytes(reinterpret_cast<const uint8_t*>(s.data()), s.size());
      pts.emplace_back((uint32_t)(d.hi >> 32), i);
    }
  std::stable_sort(pts.begin(), pts.end(),
                   [](const std::pair<uint32_t, int>& a, const std::pair<uint32_t, int>& b) {
                     return a.first < b.first;
                   });
  for (const auto& p : pts) {
    pts_.push_back(p.first);
    own_.push_back(p.second);
  }
  // span s = [a, a + 65535]: its points q1 < q2 (if any); owner(p), t = p - a:
  // t <= q1 - a -> own(q1), t <= q2 - a -> own(q2), else the owner after the last of them
  auto after = [&](uint64_t q) { return q >= 0xFFFFFFFFull ? own_[0] : search((uint32_t)q + 1); };
  for (uint32_t s = 0; s < 65536; ++s) {
    const uint32_t a = s << 16;
    const uint64_t b = (uint64_t)a + 65535u;
    const size_t i0 = (size_t)(std::lower_bound(pts_.begin(), pts_.end(), a) - pts_.begin());
    size_t i1 = i0;
    while (i1 < pts_.size() && pts_[i1] <= b) ++i1;
    const size_t k = i1 - i0;
    uint64_t c1, c2, o1, o2, o3;
    if (k == 0) {
      c1 = c2 = 0xFFFF;
      o1 = o2 = o3 = (uint64_t)after(b);
    } else if (k == 1) {
      c1 = c2 = pts_[i0] - a;
      o1 = (uint64_t)own_[i0];
      o2 = o3 = (uint64_t)after(pts_[i0]);
    } else {
      c1 = pts_[i0] - a;
      c2 = pts_[i0 + 1] - a;
      o1 = (uint64_t)own_[i0];
      o2 = (uint64_t)own_[i0 + 1];
      o3 = (uint64_t)after(pts_[i0 + 1]);
    }
    span_[s] = c1 | c2 << 16 | o1 << 32 | o2 << 42 | o3 << 52 | (k > 2 ? 1ull << 63 : 0ull);
  }
  cw_.assign((size_t)n_, 0.0);
  for (int r = 0; r < n_; ++r) cw_[(size_t)r] = (double)(r + 1) / n_;
  cw_.back() = 1.0;
}

HostRouter::~HostRouter() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : pool_) t.join();
}

int HostRouter::search(uint32_t p) const {
  const auto it = std::lower_bound(pts_.begin(), pts_.end(), p);
  return own_[it == pts_.end() ? 0 : (size_t)(it - pts_.begin())];
}

void HostRouter::set_hot(const Digest* hot, int64_t n, const int32_t* rank, const double* w) {
  nhot_ = 0;
  hot_tab_.assign(1, HotSlot{});
  hot_mask_ = 0;
  hot_bits_.assign(1, 0);
  bits_mask_ = 0;
  if (n > 0) {
    uint64_t slots = 1024;
    while (slots < 2 * (uint64_t)n) slots <<= 1;
    hot_tab_.assign(slots, HotSlot{});
    hot_mask_ = slots - 1;
    uint64_t bits = 1 << 12;
    while (bits < 16 * (uint64_t)n) bits <<= 1;
    hot_bits_.assign(bits / 64, 0);
    bits_mask_ = bits - 1;
    // in the given order (hottest first, HotSpread.plan): the hottest keep their home slot
    for (int64_t i = 0; i < n; ++i) {
      const Digest d = hot[i];
      if (!d.lo && !d.hi) continue;
      const int32_t r = rank ? rank[i] : kSpray;
      SH_CHECK(r >= kSpray && r < n_, "designated rank out of range");
      const uint64_t fb = (d.lo >> 20) & bits_mask_;
      hot_bits_[fb >> 6] |= 1ull << (fb & 63);
      const uint64_t tag = (d.hi & ~0xFFFFull) | (uint64_t)(r + 2);
      for (uint64_t s = d.lo & hot_mask_;; s = (s + 1) & hot_mask_) {
        HotSlot& e = hot_tab_[s];
        if (e.lo == d.lo && ((e.tag ^ d.hi) >> 16) == 0 && (e.tag & 0xFFFF)) {
          e.tag = tag;  // a repeated digest: the last rank
          break;
        }
        if (!(e.tag & 0xFFFF)) {
          e.lo = d.lo;
          e.tag = tag;
          ++nhot_;
          break;
        }
      }
    }
  }
  double tot = 0;
  for (int r = 0; r < n_; ++r) {
    SH_CHECK(w[r] >= 0, "spray weights must be non-negative");
    tot += w[r];
  }
  SH_CHECK(tot > 0, "spray weights sum to zero");
  double acc = 0;
  for (int r = 0; r < n_; ++r) {
    acc += w[r];
    cw_[(size_t)r] = acc / tot;
  }
  cw_.back() = 1.0;
}

uint32_t HostRouter::hot_code_slow(const Digest& d) const {
  for (uint64_t s = d.lo & hot_mask_;; s = (s + 1) & hot_mask_) {
    const HotSlot& e = hot_tab_[s];
    if (hot_match(e, d)) return (uint32_t)(e.tag & 0xFFFFu);
    if (!(e.tag & 0xFFFFu)) return 0;
  }
}

int HostRouter::spray(uint64_t j) const {
  const double u = (double)((j * kWeyl) >> 11) * (1.0 / 9007199254740992.0);  // 2^-53
  int r = 0;  // #{cw <= u} over the first n - 1 weights, branch-free (the rank is random)
  for (int k = 0; k < n_ - 1; ++k) r += cw_[(size_t)k] <= u;
  return r;
}

template <bool kSets>
void HostRouter::route_range(const Digest* keys, int64_t a, int64_t b, uint64_t seq0,
                             int32_t* dest, int64_t* counts) const {
  if (!nhot_) {
    for (int64_t i = a; i < b; ++i) {
      const int o = owner(keys[i]);
      dest[i] = o;
      ++counts[o];
    }
    return;
  }
  // locals: the stores through dest / counts cannot make the compiler reload any of these
  const uint64_t* const span = span_.data();
  const uint64_t* const bits = hot_bits_.data();
  const HotSlot* const tab = hot_tab_.data();
  const uint64_t bmask = bits_mask_, hmask = hot_mask_;
  for (int64_t i = a; i < b; ++i) {
    const Digest d = keys[i];
    // owner (owner()'s span rule)
    const uint32_t p = ring_position(d);
    const uint64_t se = span[p >> 16];
    int o;
    if (__builtin_expect(se >> 63, 0)) {
      o = search(p);
    } else {
      // t <= c1 ? o1 : t <= c2 ? o2 : o3, by masks (g++ turned the ternaries into branches
      // that mispredict on a random stream)
      const uint32_t t = p & 0xFFFFu;
      const uint32_t s1 = 0u - (uint32_t)(t <= (se & 0xFFFFu));
      const uint32_t s2 = 0u - (uint32_t)(t <= ((se >> 16) & 0xFFFFu));
      const uint32_t o1 = (se >> 32) & 1023, o2 = (se >> 42) & 1023, o3 = (se >> 52) & 1023;
      const uint32_t x = o3 ^ ((o2 ^ o3) & s2);
      o = (int)(x ^ ((o1 ^ x) & s1));
    }
    // hot code (hot_code()'s rule)
    const uint64_t fb = (d.lo >> 20) & bmask;
    const uint64_t pass = (bits[fb >> 6] >> (fb & 63)) & 1;
    const HotSlot& e = tab[d.lo & hmask];
    const uint64_t hit = pass & (uint64_t)hot_match(e, d);
    const uint32_t c = __builtin_expect(pass & (hit ^ 1), 0)
                           ? hot_code_slow(d)
                           : (uint32_t)(e.tag & 0xFFFFu & ((uint64_t)0 - hit));
    if (kSets) {
      if (c) {  // (SETs: a hot object's share of a SET stream is small and predictable)
        dest[i] = -1;
        for (int r = 0; r < n_; ++r) ++counts[r];
      } else {
        dest[i] = o;
        ++counts[o];
      }
    } else {
      const uint32_t sel = 0u - (uint32_t)(c >= 2);  // a select by mask, not a branch
      int r = (int)((uint32_t)o ^ (((c - 2) ^ (uint32_t)o) & sel));
      if (c == 1) r = spray(seq0 + (uint64_t)i);  // the few sprayed objects
      dest[i] = r;
      ++counts[r];
    }
  }
}

void HostRouter::worker(int id) {
  uint64_t seen = 0;
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
    if (stop_) return;
    seen = gen_;
    if (id >= want_) continue;
    const std::function<void(int)>* job = job_;
    lk.unlock();
    (*job)(id);
    lk.lock();
    if (--left_ == 0) done_cv_.notify_one();
  }
}

void HostRouter::parallel(int64_t n, int threads, int64_t* counts,
                          const std::function<void(int64_t, int64_t, int64_t*)>& f) const {
  if (threads <= 1 || n < (1 << 16)) {
    f(0, n, counts);
    return;
  }
  threads = (int)std::min<int64_t>(threads, n >> 14);
  std::lock_guard<std::mutex> call(call_mu_);
  std::vector<std::vector<int64_t>> part((size_t)threads, std::vector<int64_t>((size_t)n_, 0));
  const int64_t per = (n + threads - 1) / threads;
  const std::function<void(int)> job = [&](int t) {
    const int64_t lo = std::min(n, t * per), hi = std::min(n, lo + per);
    f(lo, hi, part[(size_t)t].data());
  };
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto* self = const_cast<HostRouter*>(this);
    while ((int)pool_.size() < threads - 1) {
      const int id = (int)pool_.size();
      pool_.emplace_back([self, id] { self->worker(id); });
    }
    job_ = &job;
    want_ = left_ = threads - 1;
    ++gen_;
  }
  cv_.notify_all();
  job(threads - 1);  // the caller's own slice
  {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return left_ == 0; });
    job_ = nullptr;
  }
  for (const auto& p : part)
    for (int r = 0; r < n_; ++r) counts[r] += p[(size_t)r];
}

void HostRouter::route_gets(const Digest* keys, int64_t n, uint64_t seq0, int32_t* dest,
                            int64_t* counts, int threads) const {
  parallel(n, threads, counts, [&](int64_t a, int64_t b, int64_t* c) {
    route_range<false>(keys, a, b, seq0, dest, c);
  });
}

void HostRouter::route_sets(const Digest* keys, int64_t n, int32_t* dest, int64_t* counts,
                            int threads) const {
  parallel(n, threads, counts, [&](int64_t a, int64_t b, int64_t* c) {
    route_range<true>(keys, a, b, 0, dest, c);
  });
}

}  // namespace shellac
