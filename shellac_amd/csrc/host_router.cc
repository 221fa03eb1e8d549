// HostRouter (host_router.h): ketama ownership + hot-object spreading for the host-routed
// multi-GPU topology.
#include "host_router.h"

#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <thread>

namespace shellac {

namespace {
constexpr uint64_t kWeyl = 0x9E3779B97F4A7C15ull;  // 2^64 / golden ratio
const bool kHaveAvx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq");
}  // namespace

HostRouter::HostRouter(int nshards, int pps)
    : n_(nshards), span_(65536, 0), lanes_(kHaveAvx512), readers_(new ReadSlot[kReadSlots]) {
  for (int i = 0; i < kReadSlots; ++i) {
    readers_[i].c[0].store(0, std::memory_order_relaxed);
    readers_[i].c[1].store(0, std::memory_order_relaxed);
  }
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
  auto* t = new HotTable;
  t->cw.assign((size_t)n_, 0.0);
  for (int r = 0; r < n_; ++r) t->cw[(size_t)r] = (double)(r + 1) / n_;
  t->cw.back() = 1.0;
  set_thresholds(t);
  hot_.store(t, std::memory_order_release);
}

void HostRouter::set_lanes(bool on) { lanes_ = on && kHaveAvx512; }

void HostRouter::set_thresholds(HotTable* t) const {
  // cw <= x * 2^-53 <=> x >= ceil(cw * 2^53) for an integer x < 2^53 (exact in doubles)
  t->spray_t.assign(t->cw.size(), 0);
  for (size_t k = 0; k < t->cw.size(); ++k)
    t->spray_t[k] = (uint64_t)std::ceil(t->cw[k] * 9007199254740992.0);
}

HostRouter::~HostRouter() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : pool_) t.join();
  delete hot_.load(std::memory_order_acquire);
}

int HostRouter::search(uint32_t p) const {
  const auto it = std::lower_bound(pts_.begin(), pts_.end(), p);
  return own_[it == pts_.end() ? 0 : (size_t)(it - pts_.begin())];
}

// ---- readers and the grace period -------------------------------------------------
namespace {
std::atomic<unsigned> g_next_slot{0};
int my_read_slot(int slots) {
  thread_local int s = (int)(g_next_slot.fetch_add(1, std::memory_order_relaxed) % (unsigned)slots);
  return s;
}
}  // namespace

HostRouter::Read::Read(const HostRouter& r) : r_(r), slot_(my_read_slot(kReadSlots)) {
  // count in first, then read the table: a writer that published after our count sees it
  // (seq_cst on both sides), one that published before is the table we read
  phase_ = (int)(r.phase_.load(std::memory_order_seq_cst) & 1);
  r.readers_[slot_].c[phase_].fetch_add(1, std::memory_order_seq_cst);
  t_ = r.hot_.load(std::memory_order_seq_cst);
}

HostRouter::Read::~Read() {
  r_.readers_[slot_].c[phase_].fetch_sub(1, std::memory_order_release);
}

void HostRouter::grace_period() {
  // Two phase flips, each followed by a wait for the old phase's readers (the classic
  // sleepable-RCU argument: one flip is not enough for a reader that read the phase, then
  // stalled before counting itself in, across a whole earlier grace period).
  for (int round = 0; round < 2; ++round) {
    const uint64_t p = phase_.fetch_add(1, std::memory_order_seq_cst) & 1;
    for (int spins = 0;; ++spins) {
      int64_t s = 0;
      for (int i = 0; i < kReadSlots; ++i) s += readers_[i].c[p].load(std::memory_order_seq_cst);
      if (s == 0) break;
      if (spins < 64) __builtin_ia32_pause();
      else std::this_thread::yield();
    }
  }
}

int64_t HostRouter::nhot() const { return Read(*this).table().nhot; }

std::vector<double> HostRouter::cumulative() const { return Read(*this).table().cw; }

void HostRouter::set_hot(const Digest* hot, int64_t n, const int32_t* rank, const double* w) {
  std::unique_ptr<HotTable> t(new HotTable);
  if (n > 0) {
    uint64_t slots = 1024;
    while (slots < 4 * (uint64_t)n) slots <<= 1;
    t->tab.assign(slots, HotSlot{});
    t->mask = slots - 1;
    uint64_t bits = 1 << 12;
    while (bits < 16 * (uint64_t)n) bits <<= 1;
    t->bits.assign(bits / 64, 0);
    t->bits_mask = bits - 1;
    // in the given order (hottest first, HotSpread.plan): the hottest keep their home slot
    for (int64_t i = 0; i < n; ++i) {
      const Digest d = hot[i];
      if (!d.lo && !d.hi) continue;
      const int32_t r = rank ? rank[i] : kSpray;
      SH_CHECK(r >= kSpray && r < n_, "designated rank out of range");
      const uint64_t fb = (d.lo >> 20) & t->bits_mask;
      t->bits[fb >> 6] |= 1ull << (fb & 63);
      const uint64_t tag = (d.hi & ~0xFFFFull) | (uint64_t)(r + 2);
      for (uint64_t s = d.lo & t->mask;; s = (s + 1) & t->mask) {
        HotSlot& e = t->tab[s];
        if (e.lo == d.lo && ((e.tag ^ d.hi) >> 16) == 0 && (e.tag & 0xFFFF)) {
          e.tag = tag;  // a repeated digest: the last rank
          break;
        }
        if (!(e.tag & 0xFFFF)) {
          e.lo = d.lo;
          e.tag = tag;
          ++t->nhot;
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
  t->cw.assign((size_t)n_, 0.0);
  double acc = 0;
  for (int r = 0; r < n_; ++r) {
    acc += w[r];
    t->cw[(size_t)r] = acc / tot;
  }
  t->cw.back() = 1.0;
  set_thresholds(t.get());
  std::lock_guard<std::mutex> lk(set_mu_);
  const HotTable* old = hot_.exchange(t.release(), std::memory_order_seq_cst);
  grace_period();  // nobody reads `old` any more
  delete old;
  pubs_.fetch_add(1, std::memory_order_relaxed);
}

uint32_t HostRouter::HotTable::code_slow(const Digest& d) const {
  for (uint64_t s = d.lo & mask;; s = (s + 1) & mask) {
    const HotSlot& e = tab[s];
    if (match(e, d)) return (uint32_t)(e.tag & 0xFFFFu);
    if (!(e.tag & 0xFFFFu)) return 0;
  }
}

int HostRouter::HotTable::spray(uint64_t j) const {
  const double u = (double)((j * kWeyl) >> 11) * (1.0 / 9007199254740992.0);  // 2^-53
  int r = 0;  // #{cw <= u} over the first n - 1 weights, branch-free (the rank is random)
  for (size_t k = 0; k + 1 < cw.size(); ++k) r += cw[k] <= u;
  return r;
}

template <bool kSets>
int HostRouter::route_one(const HotTable& t, const Digest& d, uint64_t j) const {
  const uint32_t c = t.nhot ? t.code(d) : 0;
  if (kSets) return c ? -1 : owner(d);
  return c >= 2 ? (int)c - 2 : c == 1 ? t.spray(j) : owner(d);
}

template <bool kSets>
void HostRouter::route_range(const HotTable& t, const Digest* keys, int64_t a, int64_t b,
                             uint64_t seq0, int32_t* dest, int64_t* counts) const {
  if (lanes_) {
    route_x8<kSets>(t, keys, a, b, seq0, dest, counts);
    return;
  }
  if (!t.nhot) {
    for (int64_t i = a; i < b; ++i) {
      const int o = owner(keys[i]);
      dest[i] = o;
      ++counts[o];
    }
    return;
  }
  // locals: the stores through dest / counts cannot make the compiler reload any of these
  const uint64_t* const span = span_.data();
  const uint64_t* const bits = t.bits.data();
  const HotSlot* const tab = t.tab.data();
  const uint64_t bmask = t.bits_mask, hmask = t.mask;
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
      const uint32_t tt = p & 0xFFFFu;
      const uint32_t s1 = 0u - (uint32_t)(tt <= (se & 0xFFFFu));
      const uint32_t s2 = 0u - (uint32_t)(tt <= ((se >> 16) & 0xFFFFu));
      const uint32_t o1 = (se >> 32) & 1023, o2 = (se >> 42) & 1023, o3 = (se >> 52) & 1023;
      const uint32_t x = o3 ^ ((o2 ^ o3) & s2);
      o = (int)(x ^ ((o1 ^ x) & s1));
    }
    // hot code (HotTable::code()'s rule)
    const uint64_t fb = (d.lo >> 20) & bmask;
    const uint64_t pass = (bits[fb >> 6] >> (fb & 63)) & 1;
    const HotSlot& e = tab[d.lo & hmask];
    const uint64_t hit = pass & (uint64_t)HotTable::match(e, d);
    const uint32_t c = __builtin_expect(pass & (hit ^ 1), 0)
                           ? t.code_slow(d)
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
      if (c == 1) r = t.spray(seq0 + (uint64_t)i);  // the few sprayed objects
      dest[i] = r;
      ++counts[r];
    }
  }
}

// Eight requests per iteration in 512-bit lanes: the span entry, the filter word and the
// home slot are gathered, owner and hot code computed and selected under lane masks, and
// the eight ranks stored as one 32-byte write. Lanes that need more (a span with more than
// two points, a filter pass that missed both probe slots, a GET of a sprayed object over
// more than 64 ranks) are redone by the scalar rule. The per-rank counts are taken from the
// written block afterwards (the increments inside the lane loop would serialise on
// store-to-load forwarding). SETs (kSets): a hot object's lane is -1 (every rank).
template <bool kSets>
__attribute__((target("avx512f,avx512dq"))) void HostRouter::route_x8(
    const HotTable& ht, const Digest* keys, int64_t a, int64_t b, uint64_t seq0, int32_t* dest,
    int64_t* counts) const {
  const long long* const span = reinterpret_cast<const long long*>(span_.data());
  const long long* const bits = reinterpret_cast<const long long*>(ht.bits.data());
  const long long* const tab = reinterpret_cast<const long long*>(ht.tab.data());
  const __m512i ilo = _mm512_setr_epi64(0, 2, 4, 6, 8, 10, 12, 14);
  const __m512i ihi = _mm512_setr_epi64(1, 3, 5, 7, 9, 11, 13, 15);
  const __m512i m16 = _mm512_set1_epi64(0xFFFF), m1023 = _mm512_set1_epi64(1023);
  const __m512i one = _mm512_set1_epi64(1), two = _mm512_set1_epi64(2);
  const __m512i zero = _mm512_setzero_si512(), m63 = _mm512_set1_epi64(63);
  const __m512i lane = _mm512_setr_epi64(0, 1, 2, 3, 4, 5, 6, 7);
  const __m512i weyl = _mm512_set1_epi64((long long)kWeyl);
  const __m512i bmask = _mm512_set1_epi64((long long)ht.bits_mask);
  const __m512i hmask = _mm512_set1_epi64((long long)ht.mask);
  const bool hot = ht.nhot != 0;
  constexpr int64_t kBlock = 2048;  // counted while the block's ranks are in L1
  uint32_t cnt[4][1024];
  for (auto& c : cnt) std::fill(c, c + n_, 0u);
  int64_t fan = 0;
  for (int64_t c0 = a; c0 < b; c0 += kBlock) {
    const int64_t c1 = std::min(b, c0 + kBlock);
    int64_t i = c0;
    for (; i + 8 <= c1; i += 8) {
      const __m512i k0 = _mm512_loadu_si512(keys + i), k1 = _mm512_loadu_si512(keys + i + 4);
      const __m512i lo = _mm512_permutex2var_epi64(k0, ilo, k1);
      const __m512i hi = _mm512_permutex2var_epi64(k0, ihi, k1);
      // owner: t <= c1 ? o1 : t <= c2 ? o2 : o3 from the span entry
      const __m512i se = _mm512_i64gather_epi64(_mm512_srli_epi64(hi, 48), span, 8);
      const __m512i t = _mm512_and_si512(_mm512_srli_epi64(hi, 32), m16);
      const __mmask8 s1 = _mm512_cmple_epu64_mask(t, _mm512_and_si512(se, m16));
      const __mmask8 s2 =
          _mm512_cmple_epu64_mask(t, _mm512_and_si512(_mm512_srli_epi64(se, 16), m16));
      __m512i o = _mm512_mask_blend_epi64(s2, _mm512_and_si512(_mm512_srli_epi64(se, 52), m1023),
                                          _mm512_and_si512(_mm512_srli_epi64(se, 42), m1023));
      o = _mm512_mask_blend_epi64(s1, o, _mm512_and_si512(_mm512_srli_epi64(se, 32), m1023));
      __mmask8 redo = _mm512_cmplt_epi64_mask(se, zero);  // bit 63: search the points
      if (hot) {
        const __m512i fb = _mm512_and_si512(_mm512_srli_epi64(lo, 20), bmask);
        const __m512i w = _mm512_i64gather_epi64(_mm512_srli_epi64(fb, 6), bits, 8);
        const __mmask8 pass =
            _mm512_test_epi64_mask(_mm512_srlv_epi64(w, _mm512_and_si512(fb, m63)), one);
        if (pass) {
          // the home slot, then (where another object holds it) the next one: with the
          // table at most a quarter full a digest that matches neither, and whose second
          // slot is taken too, is rare (it is redone)
          __m512i at = _mm512_slli_epi64(_mm512_and_si512(lo, hmask), 1);
          __m512i elo = _mm512_mask_i64gather_epi64(zero, pass, at, tab, 8);
          __m512i etag = _mm512_mask_i64gather_epi64(zero, pass, _mm512_add_epi64(at, one), tab, 8);
          __m512i code = _mm512_and_si512(etag, m16);
          __mmask8 hit = pass & _mm512_cmpeq_epi64_mask(elo, lo) &
                         _mm512_cmpeq_epi64_mask(
                             _mm512_srli_epi64(_mm512_xor_si512(etag, hi), 16), zero) &
                         _mm512_test_epi64_mask(code, m16);
          const __mmask8 other = pass & ~hit & _mm512_test_epi64_mask(code, m16);
          if (other) {
            at = _mm512_slli_epi64(_mm512_and_si512(_mm512_add_epi64(lo, one), hmask), 1);
            elo = _mm512_mask_i64gather_epi64(zero, other, at, tab, 8);
            etag = _mm512_mask_i64gather_epi64(zero, other, _mm512_add_epi64(at, one), tab, 8);
            const __m512i code1 = _mm512_and_si512(etag, m16);
            const __mmask8 hit1 = other & _mm512_cmpeq_epi64_mask(elo, lo) &
                                  _mm512_cmpeq_epi64_mask(
                                      _mm512_srli_epi64(_mm512_xor_si512(etag, hi), 16), zero) &
                                  _mm512_test_epi64_mask(code1, m16);
            code = _mm512_mask_mov_epi64(code, hit1, code1);
            hit |= hit1;
            redo |= other & ~hit1 & _mm512_test_epi64_mask(code1, m16);
          }
          if (kSets) {
            o = _mm512_mask_mov_epi64(o, hit, _mm512_set1_epi64(-1));
          } else {
          const __mmask8 des = hit & _mm512_cmpge_epu64_mask(code, two);
          o = _mm512_mask_sub_epi64(o, des, code, two);
          const __mmask8 spr = hit & _mm512_cmpeq_epi64_mask(code, one);
          // (a few ranks: computed for every group, as the sprayed lanes come and go at
          // random; more: only when a lane needs it)
          if (n_ <= 16 || spr) {
            if (n_ <= 64) {  // r = #{thresholds <= the lane's 53-bit Weyl draw}
              const __m512i j = _mm512_add_epi64(
                  _mm512_set1_epi64((long long)(seq0 + (uint64_t)i)), lane);
              const __m512i x = _mm512_srli_epi64(_mm512_mullo_epi64(j, weyl), 11);
              __m512i r = zero;
              for (int k = 0; k < n_ - 1; ++k)
                r = _mm512_mask_add_epi64(
                    r, _mm512_cmpge_epu64_mask(x, _mm512_set1_epi64((long long)ht.spray_t[(size_t)k])),
                    r, one);
              o = _mm512_mask_mov_epi64(o, spr, r);
            } else {
              redo |= spr;
            }
          }
          }
        }
      }
      _mm256_storeu_si256(reinterpret_cast<__m256i*>(dest + i), _mm512_cvtepi64_epi32(o));
      if (__builtin_expect(redo != 0, 0))
        for (unsigned m = redo; m; m &= m - 1) {
          const int l = __builtin_ctz(m);
          dest[i + l] = route_one<kSets>(ht, keys[i + l], seq0 + (uint64_t)(i + l));
        }
    }
    for (; i < c1; ++i) dest[i] = route_one<kSets>(ht, keys[i], seq0 + (uint64_t)i);
    if (kSets) {  // -1 (a hot object's SET) counts once for every rank
      for (i = c0; i < c1; ++i) {
        const int32_t r = dest[i];
        if (r < 0) ++fan; else ++cnt[i & 3][r];
      }
      continue;
    }
    for (i = c0; i + 4 <= c1; i += 4) {
      ++cnt[0][dest[i]];
      ++cnt[1][dest[i + 1]];
      ++cnt[2][dest[i + 2]];
      ++cnt[3][dest[i + 3]];
    }
    for (; i < c1; ++i) ++cnt[0][dest[i]];
  }
  for (int r = 0; r < n_; ++r)
    counts[r] += (int64_t)cnt[0][r] + cnt[1][r] + cnt[2][r] + cnt[3][r] + fan;
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
  const Read rd(*this);  // one table for the whole call
  parallel(n, threads, counts, [&](int64_t a, int64_t b, int64_t* c) {
    route_range<false>(rd.table(), keys, a, b, seq0, dest, c);
  });
}

void HostRouter::route_sets(const Digest* keys, int64_t n, int32_t* dest, int64_t* counts,
                            int threads) const {
  const Read rd(*this);
  parallel(n, threads, counts, [&](int64_t a, int64_t b, int64_t* c) {
    route_range<true>(rd.table(), keys, a, b, 0, dest, c);
  });
}

HotPlan plan_hot(const std::vector<std::pair<Digest, uint64_t>>& counts, int k, int nshards,
                 uint64_t eligible, const std::function<int(const Digest&)>& owner,
                 double spray_above, uint64_t min_count,
                 const std::function<bool(const Digest&)>* sticky, double sticky_factor) {
  HotPlan p;
  p.weights.assign((size_t)nshards, 0.0);
  p.planned.assign((size_t)nshards, 0.0);
  std::vector<int> el;
  for (int r = 0; r < nshards; ++r)
    if ((eligible >> r) & 1) {
      el.push_back(r);
      p.weights[(size_t)r] = 1.0;
    }
  uint64_t total = 0;
  for (const auto& c : counts) total += c.second;
  if (k <= 0 || el.empty() || total == 0) {
    if (el.empty()) p.weights.assign((size_t)nshards, 1.0);
    return p;
  }
  // the top k by count (ties by digest, so every caller with the same counts agrees; the
  // low word compared as a signed int64, the order HotSpread.design's tensors sort in)
  std::vector<size_t> idx;
  std::vector<double> rank_w(counts.size());
  for (size_t i = 0; i < counts.size(); ++i) {
    rank_w[i] = (double)counts[i].second;
    if (sticky && sticky_factor != 1.0 && (*sticky)(counts[i].first)) rank_w[i] *= sticky_factor;
    if (counts[i].second >= min_count) idx.push_back(i);
  }
  auto hotter = [&](size_t a, size_t b) {
    const auto &x = counts[a], &y = counts[b];
    if (rank_w[a] != rank_w[b]) return rank_w[a] > rank_w[b];
    if (x.first.lo != y.first.lo) return (int64_t)x.first.lo < (int64_t)y.first.lo;
    return (int64_t)x.first.hi < (int64_t)y.first.hi;
  };
  if ((int64_t)idx.size() > k) {
    std::partial_sort(idx.begin(), idx.begin() + k, idx.end(), hotter);
    idx.resize((size_t)k);
  } else {
    std::sort(idx.begin(), idx.end(), hotter);
  }
  std::vector<uint8_t> is_hot(counts.size(), 0);
  uint64_t hot_total = 0;
  for (size_t i : idx) {
    is_hot[i] = 1;
    hot_total += counts[i].second;
  }
  p.hot_share = (double)hot_total / (double)total;
  // loads: the non-hot sampled GETs at their owners (an ineligible owner's requests stay
  // there: that rank is not a target for hot GETs)
  std::vector<double> load((size_t)nshards, 0.0);
  for (size_t i = 0; i < counts.size(); ++i)
    if (!is_hot[i]) load[(size_t)owner(counts[i].first)] += (double)counts[i].second;
  const double thr = spray_above * (double)total;
  double sprayed = 0;
  for (size_t i : idx)
    if ((double)counts[i].second > thr) sprayed += (double)counts[i].second;
  for (int r : el) load[(size_t)r] += sprayed / (double)el.size();
  for (size_t i : idx) {
    p.hot.push_back(counts[i].first);
    if ((double)counts[i].second > thr) {
      p.rank.push_back(-1);
      continue;
    }
    int best = el[0];  // the least loaded eligible rank (lowest index on ties)
    for (int r : el)
      if (load[(size_t)r] < load[(size_t)best]) best = r;
    load[(size_t)best] += (double)counts[i].second;
    p.rank.push_back(best);
  }
  for (int r = 0; r < nshards; ++r) p.planned[(size_t)r] = load[(size_t)r] / (double)total;
  return p;
}

}  // namespace shellac
