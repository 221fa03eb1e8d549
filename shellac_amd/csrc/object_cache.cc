// ObjectCache: see object_cache.h.
#include "object_cache.h"

#include "keyed.h"

namespace shellac {

namespace {
constexpr int32_t kEmpty = -1, kTomb = -2;
constexpr uint32_t kObjOverhead = 64;  // bookkeeping bytes charged per object
inline size_t hash_of(const Digest& d) { return (size_t)(d.lo ^ (d.lo >> 29)); }
}  // namespace

ObjectCache::ObjectCache(uint64_t capacity_bytes, uint32_t max_item, int stripes)
    : max_item_(max_item) {
  SH_CHECK(stripes > 0 && capacity_bytes > 0, "object cache needs capacity and stripes");
  cap_per_stripe_ = std::max<uint64_t>(capacity_bytes / (uint64_t)stripes, 4096);
  for (int i = 0; i < stripes; ++i) {
    auto s = std::make_unique<Stripe>();
    s->table.assign(1024, kEmpty);
    stripes_.push_back(std::move(s));
  }
}

int32_t* ObjectCache::find(Stripe& s, const Digest& d) {
  const size_t mask = s.table.size() - 1;
  for (size_t h = hash_of(d) & mask, k = 0; k <= mask; h = (h + 1) & mask, ++k) {
    const int32_t v = s.table[h];
    if (v == kEmpty) return nullptr;
    if (v >= 0) {
      const Obj& o = s.slots[(size_t)v];
      if (o.d.lo == d.lo && o.d.hi == d.hi) return &s.table[h];
    }
  }
  return nullptr;
}

void ObjectCache::table_insert(Stripe& s, const Digest& d, int32_t slot) {
  if ((s.used + 1) * 2 > s.table.size()) rehash(s, std::max<size_t>(1024, s.live * 4 + 4));
  const size_t mask = s.table.size() - 1;
  for (size_t h = hash_of(d) & mask;; h = (h + 1) & mask) {
    if (s.table[h] < 0) {
      if (s.table[h] == kEmpty) ++s.used;
      s.table[h] = slot;
      return;
    }
  }
}

void ObjectCache::rehash(Stripe& s, size_t want) {
  size_t cap = 1024;
  while (cap < want) cap <<= 1;
  std::vector<int32_t> t(cap, kEmpty);
  const size_t mask = cap - 1;
  for (int32_t v : s.table) {
    if (v < 0) continue;
    for (size_t h = hash_of(s.slots[(size_t)v].d) & mask;; h = (h + 1) & mask)
      if (t[h] == kEmpty) {
        t[h] = v;
        break;
      }
  }
  s.table.swap(t);
  s.used = s.live;
}

void ObjectCache::erase_slot(Stripe& s, int32_t* pos,
                             std::vector<std::shared_ptr<const std::string>>* dead) {
  const int32_t id = *pos;
  Obj& o = s.slots[(size_t)id];
  s.bytes -= o.bytes;
  dead->push_back(std::move(o.data));  // freed outside the stripe lock
  o = Obj{};
  *pos = kTomb;
  s.free.push_back((uint32_t)id);
  --s.live;
}

// CLOCK: the hand clears a referenced object's bit and passes it once; an unreferenced
// object is evicted. Two laps at most (every bit is clear after one).
void ObjectCache::evict(Stripe& s, std::vector<std::shared_ptr<const std::string>>* dead) {
  const size_t n = s.slots.size();
  for (size_t step = 0; step < 2 * n + 1 && s.bytes > cap_per_stripe_ && s.live > 0; ++step) {
    if (s.hand >= n) s.hand = 0;
    Obj& o = s.slots[s.hand];
    if (o.data) {
      if (o.ref) {
        o.ref = false;
      } else {
        int32_t* pos = find(s, o.d);
        if (pos) {
          erase_slot(s, pos, dead);
          s.st.evictions++;
        }
      }
    }
    ++s.hand;
  }
}

bool ObjectCache::get(const std::string& key, const Digest& d, uint32_t now, Bytes* payload,
                      uint32_t* flags, uint32_t* expire) {
  Stripe& s = stripe(d);
  std::shared_ptr<const std::string> data;
  std::vector<std::shared_ptr<const std::string>> dead;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    s.st.gets++;
    int32_t* pos = find(s, d);
    if (!pos) return false;
    Obj& o = s.slots[(size_t)*pos];
    if (o.expire && o.expire <= now) {
      erase_slot(s, pos, &dead);
      s.st.expired++;
      return false;
    }
    o.ref = true;
    data = o.data;
    if (flags) *flags = o.flags;
    if (expire) *expire = o.expire;
  }
  size_t po = 0;
  if (!keyed_match(data->data(), data->size(), key, &po)) {
    std::lock_guard<std::mutex> lk(s.mu);
    s.st.key_mismatch++;
    return false;
  }
  {
    std::lock_guard<std::mutex> lk(s.mu);
    s.st.hits++;
  }
  *payload = Bytes(data).sub(po, data->size() - po);
  return true;
}

void ObjectCache::set(const std::string& key, const Digest& d, const char* payload, size_t n,
                      uint32_t flags, uint32_t expire, uint32_t now) {
  (void)now;
  if (n > max_item_ || key.size() > kMaxKeyedKey) return;
  auto buf = std::make_shared<std::string>(keyed_size(key.size(), n), '\0');
  write_keyed(reinterpret_cast<uint8_t*>(&(*buf)[0]), key, payload, n);
  std::shared_ptr<const std::string> data = std::move(buf);
  const uint32_t bytes = (uint32_t)data->size() + kObjOverhead;
  Stripe& s = stripe(d);
  std::vector<std::shared_ptr<const std::string>> dead;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    s.st.sets++;
    if (int32_t* pos = find(s, d)) {  // replace in place (the old bytes die outside the lock)
      Obj& o = s.slots[(size_t)*pos];
      s.bytes = s.bytes - o.bytes + bytes;
      dead.push_back(std::move(o.data));
      o.data = std::move(data);
      o.flags = flags;
      o.expire = expire;
      o.bytes = bytes;
    } else {
      uint32_t id;
      if (!s.free.empty()) {
        id = s.free.back();
        s.free.pop_back();
      } else {
        id = (uint32_t)s.slots.size();
        s.slots.emplace_back();
      }
      Obj& o = s.slots[id];
      o.d = d;
      o.data = std::move(data);
      o.flags = flags;
      o.expire = expire;
      o.bytes = bytes;
      o.ref = false;
      s.bytes += bytes;
      ++s.live;
      table_insert(s, d, (int32_t)id);
    }
    if (s.bytes > cap_per_stripe_) evict(s, &dead);
  }
}

bool ObjectCache::del(const std::string& key, const Digest& d, uint32_t now) {
  Stripe& s = stripe(d);
  std::vector<std::shared_ptr<const std::string>> dead;
  std::lock_guard<std::mutex> lk(s.mu);
  int32_t* pos = find(s, d);
  if (!pos) return false;
  const Obj& o = s.slots[(size_t)*pos];
  size_t po = 0;
  const bool live = (!o.expire || o.expire > now) && keyed_match(o.data->data(), o.data->size(), key, &po);
  if (!live && (o.expire && o.expire <= now)) {
    erase_slot(s, pos, &dead);
    return false;
  }
  if (!live) return false;  // another key's object under a colliding digest: keep it
  erase_slot(s, pos, &dead);
  return true;
}

void ObjectCache::clear() {
  for (auto& sp : stripes_) {
    Stripe& s = *sp;
    std::vector<Obj> old;
    {
      std::lock_guard<std::mutex> lk(s.mu);
      old.swap(s.slots);
      s.free.clear();
      s.table.assign(1024, kEmpty);
      s.bytes = s.live = s.used = 0;
      s.hand = 0;
    }
  }
}

ObjectCacheStats ObjectCache::stats() const {
  ObjectCacheStats t;
  for (auto& sp : stripes_) {
    Stripe& s = *sp;
    std::lock_guard<std::mutex> lk(s.mu);
    t.gets += s.st.gets;
    t.hits += s.st.hits;
    t.sets += s.st.sets;
    t.evictions += s.st.evictions;
    t.expired += s.st.expired;
    t.key_mismatch += s.st.key_mismatch;
    t.objects += s.live;
    t.bytes += s.bytes;
  }
  return t;
}

}  // namespace shellac
