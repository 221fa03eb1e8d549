// StreamBuf: an append-only byte stream with an acknowledged read cursor.
//
// Parity with src/python/shellac/server/StreamBuf.py:35-78 (write / ack / seek /
// read / close / buffer / clear / complete / closed / ready). The reference
// builds it on `str +=` (O(n^2) for large bodies, StreamBuf.py:48); here data
// is a list of immutable, reference-counted segments, so a cached response is
// appended by reference (no copy per client) and the reactor drains the unsent
// tail with one writev() over iovecs.
#pragma once

#include <sys/uio.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace shellac {

// An immutable, reference-counted byte range. It either owns a std::string (responses
// built on the host) or views a slice of a larger buffer whose owner it keeps alive —
// the HBM tier hands out hits this way as slices of the pinned buffer the GPU gathered
// them into, so a cached object reaches writev() without a host copy. Pointer-like
// (`if (b)`, `b->data()`, `b->size()`) so it stands in for shared_ptr<const string>.
class ByteRef {
 public:
  ByteRef() = default;
  ByteRef(std::nullptr_t) {}  // NOLINT: implicit, like a null shared_ptr
  ByteRef(std::shared_ptr<const std::string> s)  // NOLINT: implicit on purpose
      : p_(s ? s->data() : nullptr), n_(s ? s->size() : 0), hold_(std::move(s)) {}
  ByteRef(std::shared_ptr<std::string> s)  // NOLINT
      : ByteRef(std::shared_ptr<const std::string>(std::move(s))) {}
  ByteRef(std::shared_ptr<const void> owner, const char* p, size_t n)
      : p_(p), n_(n), hold_(std::move(owner)) {}

  explicit operator bool() const { return hold_ != nullptr; }
  const ByteRef* operator->() const { return this; }
  const char* data() const { return p_; }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  std::string_view view() const { return std::string_view(p_, n_); }
  std::string str() const { return std::string(p_, n_); }
  // [off, off + n) of this range, sharing its owner
  ByteRef sub(size_t off, size_t n) const { return ByteRef(hold_, p_ + off, n); }
  const std::shared_ptr<const void>& owner() const { return hold_; }

 private:
  const char* p_ = nullptr;
  size_t n_ = 0;
  std::shared_ptr<const void> hold_;
};

using Bytes = ByteRef;

class StreamBuf {
 public:
  StreamBuf() = default;
  explicit StreamBuf(std::string data) { if (!data.empty()) write(std::move(data)); }

  void write(std::string data) {
    ready_ = true;
    if (data.empty()) return;
    size_ += data.size();
    segs_.push_back(std::make_shared<const std::string>(std::move(data)));
  }
  // Append a shared segment without copying (cache hits).
  void write_shared(Bytes seg) {
    ready_ = true;
    if (!seg || seg->empty()) return;
    size_ += seg->size();
    segs_.push_back(std::move(seg));
  }
  void ack(uint64_t n) { pos_ += n; }
  void seek(uint64_t pos) { pos_ = pos; }
  void close() { eof_ = true; }
  void clear() {
    segs_.clear();
    size_ = pos_ = dropped_ = 0;
    eof_ = ready_ = false;
  }
  bool complete() const { return eof_ && pos_ >= size_; }
  bool closed() const { return eof_; }
  bool ready() const { return ready_; }
  uint64_t size() const { return size_; }
  uint64_t pos() const { return pos_; }
  uint64_t pending() const { return pos_ >= size_ ? 0 : size_ - pos_; }

  // Unsent tail as one string (Python read()).
  std::string read() const { return slice(pos_); }
  // Everything written (Python buffer()).
  std::string buffer() const { return slice(0); }

  // Fill up to `max` iovecs with the unsent tail; returns count.
  int iov(struct iovec* v, int max) const {
    int k = 0;
    uint64_t off = dropped_;
    for (const auto& s : segs_) {
      const uint64_t end = off + s->size();
      if (end > pos_ && k < max) {
        const uint64_t skip = pos_ > off ? pos_ - off : 0;
        v[k].iov_base = const_cast<char*>(s->data() + skip);
        v[k].iov_len = s->size() - skip;
        ++k;
      }
      off = end;
    }
    return k;
  }
  // Drop fully acknowledged leading segments (reactor use; buffer() then no
  // longer contains them).
  void release_acked() {
    size_t i = 0;
    while (i < segs_.size() && dropped_ + segs_[i]->size() <= pos_) {
      dropped_ += segs_[i]->size();
      ++i;
    }
    if (i) segs_.erase(segs_.begin(), segs_.begin() + (long)i);
  }

 private:
  std::string slice(uint64_t from) const {
    std::string out;
    if (from >= size_) return out;
    out.reserve(size_ - from);
    uint64_t off = dropped_;
    for (const auto& s : segs_) {
      const uint64_t end = off + s->size();
      if (end > from) {
        const uint64_t skip = from > off ? from - off : 0;
        out.append(s->data() + skip, s->size() - skip);
      }
      off = end;
    }
    return out;
  }

  std::vector<Bytes> segs_;
  uint64_t size_ = 0, pos_ = 0, dropped_ = 0;
  bool eof_ = false, ready_ = false;
};

}  // namespace shellac
