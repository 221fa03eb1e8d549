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

HostCache::HostCache(uint64_t log_bytes, uint64_t nbuckets, uint32_t max_item)
    : log_bytes_(log_bytes), nbuckets_(nbuckets), mask_(nbuckets - 1), max_item_(max_item) {
  SH_CHECK(nbuckets >= 2 && (nbuckets & (nbuckets - 1)) == 0, "nbuckets must be a power of two");
  SH_CHECK(log_bytes >= 4096 && log_bytes % 16 == 0, "log_bytes must be >=4096 and %16");
  SH_CHECK(max_item > 0 && item_bytes(max_item) * 2 <= log_bytes, "max_item too large");
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
                                 uint64_t reserve) const {
  uint64_t best = 0;
  uint32_t bv = 0;
  const uint64_t bs[2] = {bucket1(d, mask_), bucket2(d, mask_)};
  for (uint64_t b : bs) {
    const Entry* e = index_ + b * kEntriesPerBucket;
    for (uint32_t k = 0; k < kEntriesPerBucket; ++k) {
      if (e[k].d0 == d.lo && e[k].d1 == d.hi &&
          entry_live(e[k].loc, e[k].expire, head_ + reserve, log_bytes_, now) && e[k].loc > best) {
        best = e[k].loc;
        bv = e[k].vlen;
      }
    }
  }
  if (vlen) *vlen = bv;
  return best;  // 0 = miss, else logical+1
}

void HostCache::lookup(const Digest* keys, int64_t n, uint64_t* loc, uint64_t* size,
                       uint64_t* off, uint32_t now, uint64_t reserve) {
  std::lock_guard<std::mutex> lk(mu_);
  uint64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t vl = 0;
    const uint64_t l = probe_locked(keys[i], now, &vl, reserve);
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
      uint64_t oldest = ~0ull;
      for (int e = 0; e < 8; ++e)
        if (slots[e]->loc < oldest) { oldest = slots[e]->loc; target = e; }
      evict = true;
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
                      int64_t n, uint32_t now) {
  std::lock_guard<std::mutex> lk(mu_);
  // last write of a key in the batch wins (dedupe on digest.lo, as on the device)
  std::unordered_map<uint64_t, int64_t> last;
  last.reserve((size_t)n * 2);
  for (int64_t i = 0; i < n; ++i)
    if (vlen[i] != kSkipVlen) last[keys[i].lo ? keys[i].lo : 1] = i;
  std::vector<uint64_t> sz((size_t)n);
  uint64_t total = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (vlen[i] == kSkipVlen) { sz[i] = 0; continue; }
    ctr_.set_ops++;
    const bool win = last[keys[i].lo ? keys[i].lo : 1] == i && vlen[i] <= max_item_;
    sz[i] = win ? item_bytes(vlen[i]) : 0;
    if (!win) ctr_.set_dropped++;
    total += sz[i];
  }
  SH_CHECK(total <= log_bytes_ / 2, "SET batch larger than half the log; split the batch");
  const uint64_t base = head_;
  uint64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (!sz[i]) continue;
    const uint64_t L = base + acc;
    uint8_t* p = log_ + L % log_bytes_;
    ItemHeader h{keys[i].lo, keys[i].hi, vlen[i], flags ? flags[i] : 0u, expire ? expire[i] : 0u,
                 kItemMagic};
    std::memcpy(p, &h, sizeof h);
    std::memcpy(p + kItemHeaderBytes, values + val_off[i], vlen[i]);
    const uint64_t pad = sz[i] - kItemHeaderBytes - vlen[i];
    if (pad) std::memset(p + kItemHeaderBytes + vlen[i], 0, pad);
    acc += sz[i];
  }
  head_ = base + total;
  acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (!sz[i]) continue;
    insert_locked(keys[i], base + acc + 1, vlen[i], expire ? expire[i] : 0u, now);
    ctr_.set_bytes += vlen[i];
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
      bytes += item_bytes(e.vlen);
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
  if (user)
    for (int i = 0; i < 4; ++i) user[i] = h.user[i];
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
  const uint64_t l = probe_locked(key, now, &vl);
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
