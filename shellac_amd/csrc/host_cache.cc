// Host-DRAM cache shard: same layout and policies as the HBM kernels.
#include "host_cache.h"

#include <sys/mman.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <unordered_map>

namespace shellac {

namespace {

void* map_zeroed(size_t bytes) {
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  SH_CHECK(p != MAP_FAILED, "mmap failed");
  return p;
}

}  // namespace

HostCache::HostCache(uint64_t log_bytes, uint64_t nbuckets, uint32_t max_item, int evict,
                     uint64_t reinsert_max)
    : log_bytes_(log_bytes), nbuckets_(nbuckets), mask_(nbuckets - 1), max_item_(max_item),
      evict_(evict) {
  SH_CHECK(nbuckets >= 2 && (nbuckets & (nbuckets - 1)) == 0, "nbuckets must be a power of two");
  SH_CHECK(log_bytes >= 4096 && log_bytes % 16 == 0, "log_bytes must be >=4096 and %16");
  SH_CHECK(max_item > 0 && item_bytes(max_item) * 2 <= log_bytes, "max_item too large");
  SH_CHECK(max_item <= kVlenMask, "max_item must be < 2 GiB (CLOCK bit in vlen)");
  SH_CHECK(evict == 0 || evict == 1, "unknown eviction policy");
  if (evict_) {
    rmax_ = reinsert_budget(log_bytes, reinsert_max);
    ring_.assign(ring_entries(nbuckets), kRingSkip);
  }
  log_alloc_ = log_bytes + item_bytes(max_item) + 64;
  log_ = static_cast<uint8_t*>(map_zeroed(log_alloc_));
  index_alloc_ = nbuckets * kBucketBytes;
  index_ = static_cast<Entry*>(map_zeroed(index_alloc_));
}

HostCache::~HostCache() {
  munmap(log_, log_alloc_);
  munmap(index_, index_alloc_);
}

uint64_t HostCache::probe_locked(const Digest& d, uint32_t now, uint32_t* vlen,
                                 uint64_t reserve, bool mark) {
  uint64_t best = 0;
  uint32_t bv = 0;
  Entry* be = nullptr;
  const uint64_t bs[2] = {bucket1(d, mask_), bucket2(d, mask_)};
  for (uint64_t b : bs) {
    Entry* e = index_ + b * kEntriesPerBucket;
    for (uint32_t k = 0; k < kEntriesPerBucket; ++k) {
      if (e[k].d0 == d.lo && e[k].d1 == d.hi &&
          entry_live(e[k].loc, e[k].expire, head_ + reserve, log_bytes_, now) && e[k].loc > best) {
        best = e[k].loc;
        bv = entry_vlen(e[k].vlen);
        be = &e[k];
      }
    }
  }
  if (mark && be) be->vlen |= kRefBit;
  if (vlen) *vlen = bv;
  return best;  // 0 = miss, else logical+1
}

void HostCache::lookup(const Digest* keys, int64_t n, uint64_t* loc, uint64_t* size,
                       uint64_t* off, uint32_t now, uint64_t reserve) {
  std::lock_guard<std::mutex> lk(mu_);
  uint64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t vl = 0;
    const uint64_t l = probe_locked(keys[i], now, &vl, reserve, true);
    ctr_.get_ops++;
    if (l) {
      loc[i] = (l - 1) % log_bytes_;
      size[i] = item_bytes(vl);
      ctr_.get_hits++;
      ctr_.get_bytes += vl;
    } else {
      loc[i] = kMissLoc;
      size[i] = 0;
    }
    off[i] = acc;
    acc += size[i];
  }
  off[n] = acc;
}

void HostCache::gather(const uint64_t* loc, const uint64_t* off, int64_t n, uint8_t* out) const {
  std::lock_guard<std::mutex> lk(mu_);
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t sz = off[i + 1] - off[i];
    if (sz) std::memcpy(out + off[i], log_ + loc[i], sz);
  }
}

bool HostCache::insert_locked(const Digest& d, uint64_t loc1, uint32_t vlen, uint32_t expire,
                              uint32_t now) {
  // loc1 = logical + 1. Policy identical to k_set_index.
  const uint64_t b1 = bucket1(d, mask_), b2 = bucket2(d, mask_);
  Entry* slots[8];
  for (int e = 0; e < 8; ++e)
    slots[e] = index_ + (e < 4 ? b1 : b2) * kEntriesPerBucket + (e & 3);
  int target = -1;
  bool evict = false;
  uint32_t lmask = 0;
  for (int e = 0; e < 8; ++e) {
    if (entry_live(slots[e]->loc, slots[e]->expire, head_, log_bytes_, now)) lmask |= 1u << e;
  }
  for (int e = 0; e < 8 && target < 0; ++e)
    if (slots[e]->d0 == d.lo && slots[e]->d1 == d.hi) target = e;
  if (target < 0) {
    const uint32_t dead = ~lmask & 0xffu;
    if (dead) {
      // first bucket while it keeps >= 2 free slots (lookups read it first), else the
      // emptier bucket
      const int live1 = __builtin_popcount(lmask & 0xfu), live2 = __builtin_popcount(lmask & 0xf0u);
      const uint32_t pref = __builtin_popcount(dead & 0x0fu) >= 2
                                ? (dead & 0x0fu)
                                : (live2 < live1 ? (dead & 0xf0u) : (dead & 0x0fu));
      target = __builtin_ctz(pref ? pref : dead);
    } else {
      // all 8 live: move one entry to a dead slot of its own other bucket (one cuckoo
      // step, as k_set_index's relocate_one), else evict the oldest
      for (int e = 0; e < 8 && target < 0; ++e) {
        const Digest de{slots[e]->d0, slots[e]->d1};
        const uint64_t own = e < 4 ? b1 : b2;
        const uint64_t x1 = bucket1(de, mask_), x2 = bucket2(de, mask_);
        const uint64_t ob = x1 == own ? x2 : (x2 == own ? x1 : own);
        if (ob == own) continue;
        for (int k = 0; k < 4; ++k) {
          Entry* a = index_ + ob * kEntriesPerBucket + k;
          if (!entry_live(a->loc, a->expire, head_, log_bytes_, now)) {
            *a = *slots[e];
            target = e;
            break;
          }
        }
      }
      if (target < 0) {
        uint64_t oldest = ~0ull;
        for (int e = 0; e < 8; ++e)
          if (slots[e]->loc < oldest) { oldest = slots[e]->loc; target = e; }
        evict = true;
      }
    }
  }
  Entry* s = slots[target];
  s->d0 = d.lo;
  s->d1 = d.hi;
  s->loc = loc1;
  s->vlen = vlen;
  s->expire = expire;
  if (evict) ctr_.set_evicted++;
  return true;
}

void HostCache::store(const Digest* keys, const uint8_t* values, const uint64_t* val_off,
                      const uint32_t* vlen, const uint32_t* flags, const uint32_t* expire,
                      int64_t n, uint32_t now, uint64_t bytes_bound) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<Row> rows;
  std::vector<uint8_t> stage;
  if (evict_ && rmax_) {
    uint64_t bytes = 0;  // the batch's bytes (dedupe losers included), as the device
    for (int64_t i = 0; i < n; ++i)
      if (vlen[i] != kSkipVlen && vlen[i] <= max_item_) bytes += item_bytes(vlen[i]);
    // the reinsertions share the half-log bound with the batch, capped exactly as
    // HbmCache::store caps them (same bound in, same decisions out)
    uint64_t bound = bytes_bound ? std::max(bytes_bound, bytes) : bytes;
    if (bound > log_bytes_ / 2) bound = bytes;  // (the device refuses such a bound)
    SH_CHECK(bound <= log_bytes_ / 2, "SET batch larger than half the log; split the batch");
    const uint64_t rmax = std::min<uint64_t>(rmax_, log_bytes_ / 2 - bound) / 16 * 16;
    // the device's combined batch: reinsertions (in log order) ahead of the batch
    lead_ = hand_lead(log_bytes_, bound, rmax, lead_);  // every batch (sticky), as HbmCache
    if (rmax) reclaim_locked(n, bytes, rmax, now, &rows, &stage, lead_);
  }
  rows.reserve(rows.size() + (size_t)n);
  for (int64_t i = 0; i < n; ++i)
    rows.push_back(Row{keys[i], values + (vlen[i] == kSkipVlen ? 0 : val_off[i]), vlen[i],
                       flags ? flags[i] : 0u, expire ? expire[i] : 0u});
  store_rows_locked(rows, now);
}

void HostCache::reclaim_locked(int64_t n, uint64_t bytes, uint64_t rmax, uint32_t now,
                               std::vector<Row>* out,
                               std::vector<uint8_t>* stage, bool lead_mode) {
  const int64_t w = hand_window(n);
  const uint64_t rcap = ring_.size(), rmask = rcap - 1;
  const uint64_t avail = ring_tail_ - hand_;
  // the adaptive window (layout.h hand_window_eff) and the reinsertion count cap
  const uint64_t weff = std::min<uint64_t>((uint64_t)hand_window_eff(n, hand_consumed_), avail);
  const uint64_t cmax = (uint64_t)(w - n);
  struct Hot { int64_t j; uint64_t loc, h, hx, c; };  // c: hot entries before it
  std::vector<Hot> hot;
  uint64_t hx = 0, consumed = weff;
  // lead mode: the hand's lead and a pick's safety bound (HbmCache k_rc_emit's rules)
  const uint64_t lead = lead_mode ? rmax + bytes + (bytes >> 2) : 0;
  for (uint64_t j = 0; j < weff; ++j) {
    const uint64_t idx = hand_ + j;
    const uint64_t l = ring_tail_ - idx <= rcap ? ring_[idx & rmask] : kRingSkip;
    if (l == kRingSkip || head_ > l + log_bytes_) continue;  // hole or overwritten
    ItemHeader h;
    std::memcpy(&h, log_ + l % log_bytes_, sizeof h);
    if (h.magic != kItemMagic) continue;
    // stop at the first item `lead` past the overwrite (batch + reinsertions so far)
    if (l + log_bytes_ >= head_ + bytes + std::min(hx, rmax) + lead) {
      consumed = j;
      break;
    }
    const Digest d{h.d0, h.d1};
    const uint64_t bs[2] = {bucket1(d, mask_), bucket2(d, mask_)};
    uint64_t hb = 0;
    for (uint64_t b : bs)
      for (uint32_t k = 0; k < kEntriesPerBucket; ++k) {
        const Entry& e = index_[b * kEntriesPerBucket + k];
        if (e.loc == l + 1 && (e.vlen & kRefBit) && (e.expire == 0 || e.expire > now))
          hb = item_bytes(h.vlen);
      }
    if (hb) hot.push_back(Hot{(int64_t)j, l, hb, hx, (uint64_t)hot.size()});
    hx += hb;
  }
  out->clear();
  uint64_t staged = 0;
  auto picked = [&](const Hot& t) {
    return (uint64_t)t.j < consumed && t.hx + t.h <= rmax && t.c < cmax &&
           (!lead_mode || t.loc + log_bytes_ >= head_ + bytes + rmax);
  };
  for (const Hot& t : hot)
    if (picked(t)) staged = t.hx + t.h;
  stage->assign(staged + 16, 0);
  for (const Hot& t : hot) {
    if (!picked(t)) continue;
    const uint8_t* rec = log_ + t.loc % log_bytes_;
    std::memcpy(stage->data() + t.hx, rec, t.h);
    ItemHeader h;
    std::memcpy(&h, rec, sizeof h);
    out->push_back(Row{Digest{h.d0, h.d1}, stage->data() + t.hx + kItemHeaderBytes, h.vlen,
                       h.flags, h.expire, t.loc + 1});
    ctr_.reinserted++;
    ctr_.reinsert_bytes += h.vlen;
  }
  hand_ += consumed;
  hand_consumed_ = consumed;
  if (ring_tail_ - hand_ > rcap) hand_ = ring_tail_ - rcap;
  // behind the overwrite: jump to the first entry it has not reached (rc_advance's rule)
  auto over = [&](uint64_t idx) {
    const uint64_t l = ring_[idx & rmask];
    return l != kRingSkip && head_ > l + log_bytes_;
  };
  if (catch_up_ && hand_ < ring_tail_ && over(hand_)) {
    uint64_t lo = hand_ + 1, hi = ring_tail_;
    while (lo < hi) {
      const uint64_t mid = lo + (hi - lo) / 2;
      if (over(mid)) lo = mid + 1; else hi = mid;
    }
    hand_ = lo;
  }
}

void HostCache::store_rows_locked(const std::vector<Row>& rows, uint32_t now) {
  const int64_t n = (int64_t)rows.size();
  // last write of a key in the batch wins (dedupe on digest.lo, as on the device)
  std::unordered_map<uint64_t, int64_t> last;
  last.reserve((size_t)n * 2);
  for (int64_t i = 0; i < n; ++i)
    if (rows[i].vlen != kSkipVlen) last[rows[i].key.lo ? rows[i].key.lo : 1] = i;
  std::vector<uint64_t> sz((size_t)n);
  uint64_t total = 0;
  for (int64_t i = 0; i < n; ++i) {
    const Row& r = rows[i];
    if (r.vlen == kSkipVlen) { sz[i] = 0; continue; }
    ctr_.set_ops++;
    const bool win = last[r.key.lo ? r.key.lo : 1] == i && r.vlen <= max_item_;
    sz[i] = win ? item_bytes(r.vlen) : 0;
    if (!win) ctr_.set_dropped++;
    total += sz[i];
  }
  SH_CHECK(total <= log_bytes_ / 2, "SET batch larger than half the log; split the batch");
  const uint64_t base = head_;
  uint64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (!sz[i]) continue;
    const Row& r = rows[i];
    const uint64_t L = base + acc;
    uint8_t* p = log_ + L % log_bytes_;
    ItemHeader h{r.key.lo, r.key.hi, r.vlen, r.flags, r.expire, kItemMagic};
    std::memcpy(p, &h, sizeof h);
    std::memcpy(p + kItemHeaderBytes, r.val, r.vlen);
    const uint64_t pad = sz[i] - kItemHeaderBytes - r.vlen;
    if (pad) std::memset(p + kItemHeaderBytes + r.vlen, 0, pad);
    acc += sz[i];
  }
  head_ = base + total;
  if (evict_) {  // item starts in log order, one ring entry per stored row
    const uint64_t rmask = ring_.size() - 1;
    uint64_t o = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (!sz[i]) continue;
      ring_[ring_tail_++ & rmask] = base + o;
      o += sz[i];
    }
  }
  acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (!sz[i]) continue;
    const Row& r = rows[i];
    if (r.from) {
      // a reinsertion is a move of the entry that still points at the old item (the
      // device's detached hand may run before a SET / DELETE of the key lands; here the
      // hand ran after every earlier batch, so the entry is always still there)
      Entry* src = nullptr;
      for (uint64_t b : {bucket1(r.key, mask_), bucket2(r.key, mask_)})
        for (uint32_t k = 0; k < kEntriesPerBucket && !src; ++k)
          if (index_[b * kEntriesPerBucket + k].loc == r.from) src = &index_[b * kEntriesPerBucket + k];
      if (src) {
        src->loc = base + acc + 1;
        src->vlen = r.vlen;
        src->expire = r.expire;
        ctr_.set_bytes += r.vlen;
      } else {
        ctr_.reinsert_lost++;
      }
      acc += sz[i];
      continue;
    }
    insert_locked(r.key, base + acc + 1, r.vlen, r.expire, now);
    ctr_.set_bytes += r.vlen;
    acc += sz[i];
  }
}

void HostCache::remove(const Digest* keys, int64_t n, uint8_t* found, uint32_t now) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int64_t i = 0; i < n; ++i) {
    const Digest& d = keys[i];
    bool f = false;
    const uint64_t bs[2] = {bucket1(d, mask_), bucket2(d, mask_)};
    for (uint64_t b : bs) {
      Entry* e = index_ + b * kEntriesPerBucket;
      for (uint32_t k = 0; k < kEntriesPerBucket; ++k) {
        if (e[k].loc && e[k].d0 == d.lo && e[k].d1 == d.hi) {
          if (entry_live(e[k].loc, e[k].expire, head_, log_bytes_, now)) f = true;
          e[k].loc = 0;
        }
      }
    }
    ctr_.del_ops++;
    if (f) ctr_.del_hits++;
    if (found) found[i] = f ? 1 : 0;
  }
}

void HostCache::sweep(uint32_t now, uint64_t* live_entries, uint64_t* live_bytes) {
  std::lock_guard<std::mutex> lk(mu_);
  uint64_t live = 0, bytes = 0;
  const uint64_t nslots = nbuckets_ * kEntriesPerBucket;
  for (uint64_t k = 0; k < nslots; ++k) {
    Entry& e = index_[k];
    if (!e.loc) continue;
    if (entry_live(e.loc, e.expire, head_, log_bytes_, now)) {
      ++live;
      bytes += item_bytes(entry_vlen(e.vlen));
    } else {
      e.loc = 0;
      ctr_.swept++;
    }
  }
  if (live_entries) *live_entries = live;
  if (live_bytes) *live_bytes = bytes;
}

uint64_t HostCache::export_keys(Digest* out, uint64_t out_cap, uint32_t now) {
  std::lock_guard<std::mutex> lk(mu_);
  uint64_t m = 0;
  const uint64_t nslots = nbuckets_ * kEntriesPerBucket;
  for (uint64_t k = 0; k < nslots; ++k) {
    const Entry& e = index_[k];
    if (!entry_live(e.loc, e.expire, head_, log_bytes_, now)) continue;
    if (m < out_cap) out[m] = Digest{e.d0, e.d1};
    ++m;
  }
  return m;
}

namespace {
struct SnapHeader {
  char magic[8];
  uint64_t version, log_bytes, nbuckets, max_item, head, index_bytes, log_saved, user[4];
};
constexpr char kSnapMagic[8] = {'S', 'H', 'L', 'C', 'S', 'N', 'P', '1'};
}  // namespace

void HostCache::save(const std::string& path, const uint64_t user[4]) {
  std::lock_guard<std::mutex> lk(mu_);
  const uint64_t slack = item_bytes(max_item_) + 64;
  SnapHeader h{};
  std::memcpy(h.magic, kSnapMagic, 8);
  h.version = 1;
  h.log_bytes = log_bytes_;
  h.nbuckets = nbuckets_;
  h.max_item = max_item_;
  h.head = head_;
  h.index_bytes = nbuckets_ * kBucketBytes;
  h.log_saved = head_ >= log_bytes_ ? log_bytes_ + slack : std::min(head_ + slack, log_bytes_ + slack);
  for (int i = 0; i < 4; ++i) h.user[i] = user ? user[i] : 0;
  FILE* f = std::fopen(path.c_str(), "wb");
  SH_CHECK(f, "cannot open snapshot for writing: " + path);
  bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 &&
            std::fwrite(index_, 1, h.index_bytes, f) == h.index_bytes &&
            std::fwrite(log_, 1, h.log_saved, f) == h.log_saved;
  ok = (std::fclose(f) == 0) && ok;
  SH_CHECK(ok, "snapshot write failed: " + path);
}

void HostCache::load(const std::string& path, uint64_t user[4]) {
  std::lock_guard<std::mutex> lk(mu_);
  FILE* f = std::fopen(path.c_str(), "rb");
  SH_CHECK(f, "cannot open snapshot: " + path);
  SnapHeader h{};
  bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, kSnapMagic, 8) == 0;
  if (!ok || h.log_bytes != log_bytes_ || h.nbuckets != nbuckets_ || h.max_item != max_item_) {
    std::fclose(f);
    throw Error("snapshot " + path + " does not match this shard's geometry");
  }
  ok = std::fread(index_, 1, h.index_bytes, f) == h.index_bytes &&
       std::fread(log_, 1, h.log_saved, f) == h.log_saved;
  std::fclose(f);
  SH_CHECK(ok, "snapshot truncated: " + path);
  head_ = h.head;
  ring_tail_ = hand_ = hand_consumed_ = 0;  // the CLOCK ring is not part of a snapshot (first lap FIFO)
  if (user)
    for (int i = 0; i < 4; ++i) user[i] = h.user[i];
}

std::vector<uint64_t> HostCache::debug_hand() {
  std::lock_guard<std::mutex> lk(mu_);
  const uint64_t rcap = ring_.size();
  const uint64_t loc = rcap && ring_tail_ > hand_ && ring_tail_ - hand_ <= rcap
                           ? ring_[hand_ & (rcap - 1)] : ~0ull;
  return {hand_, ring_tail_, head_, loc};
}

std::vector<uint64_t> HostCache::debug_bucket(uint64_t b) {
  std::lock_guard<std::mutex> lk(mu_);
  SH_CHECK(b < nbuckets_, "bucket out of range");
  std::vector<uint64_t> out;
  for (uint32_t k = 0; k < kEntriesPerBucket; ++k) {
    const Entry& x = index_[b * kEntriesPerBucket + k];
    for (uint64_t w : {x.d0, x.d1, x.loc, (uint64_t)x.vlen | ((uint64_t)x.expire << 32)})
      out.push_back(w);
  }
  return out;
}

void HostCache::debug_set_hand(uint64_t hand, bool catch_up) {
  std::lock_guard<std::mutex> lk(mu_);
  hand_ = hand;
  catch_up_ = catch_up;
}

void HostCache::debug_set_entry(uint64_t b, int slot, uint64_t d0, uint64_t d1, uint64_t loc,
                                uint32_t vlen, uint32_t expire) {
  std::lock_guard<std::mutex> lk(mu_);
  SH_CHECK(b < nbuckets_ && slot >= 0 && slot < (int)kEntriesPerBucket, "entry out of range");
  index_[b * kEntriesPerBucket + slot] = Entry{d0, d1, loc, vlen, expire};
}

void HostCache::flush() {
  std::lock_guard<std::mutex> lk(mu_);
  std::memset(index_, 0, nbuckets_ * kBucketBytes);
}

CacheCounters HostCache::counters() {
  std::lock_guard<std::mutex> lk(mu_);
  return ctr_;
}

uint64_t HostCache::head() {
  std::lock_guard<std::mutex> lk(mu_);
  return head_;
}

bool HostCache::get_one(const Digest& key, std::vector<uint8_t>* out, uint32_t* flags,
                        uint32_t now, uint32_t* expire) {
  std::lock_guard<std::mutex> lk(mu_);
  uint32_t vl = 0;
  const uint64_t l = probe_locked(key, now, &vl, 0, true);
  ctr_.get_ops++;
  if (!l) return false;
  ctr_.get_hits++;
  ctr_.get_bytes += vl;
  const uint8_t* p = log_ + (l - 1) % log_bytes_;
  ItemHeader h;
  std::memcpy(&h, p, sizeof h);
  if (flags) *flags = h.flags;
  if (expire) *expire = h.expire;
  out->assign(p + kItemHeaderBytes, p + kItemHeaderBytes + vl);
  return true;
}

bool HostCache::get_one(const Digest& key, std::string* out, uint32_t* flags, uint32_t now,
                        uint32_t* expire) {
  std::lock_guard<std::mutex> lk(mu_);
  uint32_t vl = 0;
  const uint64_t l = probe_locked(key, now, &vl, 0, true);
  ctr_.get_ops++;
  if (!l) return false;
  ctr_.get_hits++;
  ctr_.get_bytes += vl;
  const uint8_t* p = log_ + (l - 1) % log_bytes_;
  ItemHeader h;
  std::memcpy(&h, p, sizeof h);
  if (flags) *flags = h.flags;
  if (expire) *expire = h.expire;
  out->assign(reinterpret_cast<const char*>(p + kItemHeaderBytes), vl);
  return true;
}

void HostCache::set_one(const Digest& key, const uint8_t* value, uint32_t vlen, uint32_t flags,
                        uint32_t expire, uint32_t now) {
  // value may be unaligned / unpadded: stage through the batch path with val_off 0.
  const uint64_t zero = 0;
  store(&key, value, &zero, &vlen, &flags, &expire, 1, now);
}

// ---------------------------------------------------------------------------------
void host_exclusive_scan(const uint64_t* in, uint64_t* out, int64_t n) {
  uint64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t v = in[i];
    out[i] = acc;
    acc += v;
  }
  out[n] = acc;
}

void host_segcopy(const uint8_t* src, const uint64_t* src_off, const uint64_t* dst_off, int64_t n,
                  uint8_t* dst) {
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t sz = dst_off[i + 1] - dst_off[i];
    // integer address math: src may be null with absolute addresses in src_off
    if (sz) std::memcpy(dst + dst_off[i], reinterpret_cast<const uint8_t*>((uintptr_t)src + src_off[i]), sz);
  }
}

void host_digest_keys(const uint8_t* bytes, const int64_t* offs, int64_t n, Digest* out) {
  for (int64_t i = 0; i < n; ++i)
    out[i] = digest_bytes(bytes + offs[i], (uint64_t)(offs[i + 1] - offs[i]));
}

void host_route_keys(const Digest* keys, int64_t n, const uint32_t* pts, const int32_t* owner,
                     int32_t npts, int32_t* dest, int64_t* counts, int32_t nranks) {
  (void)nranks;
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t p = ring_position(keys[i]);
    const uint32_t* it = std::lower_bound(pts, pts + npts, p);
    const int32_t r = owner[it == pts + npts ? 0 : it - pts];
    dest[i] = r;
    counts[r]++;
  }
}

void host_scatter_by_dest(const int32_t* dest, const int64_t* base, int64_t n, int32_t nranks,
                          int64_t* cursor, int64_t* perm) {
  (void)nranks;
  for (int64_t i = 0; i < n; ++i) perm[i] = base[dest[i]] + cursor[dest[i]]++;
}

void host_permute_records(const void* in, const int64_t* perm, int64_t n, int32_t rec_bytes,
                          void* out) {
  const uint8_t* s = static_cast<const uint8_t*>(in);
  uint8_t* d = static_cast<uint8_t*>(out);
  for (int64_t i = 0; i < n; ++i) std::memcpy(d + perm[i] * rec_bytes, s + i * rec_bytes, rec_bytes);
}

}  // namespace shellac
