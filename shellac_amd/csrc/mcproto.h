// memcached binary protocol: frame layout, opcodes, builders and an incremental
// frame splitter. The reference talks this protocol through pylibmc
// (binary=True, src/python/shellac/server/Server.py:81-83); shellac_amd speaks it
// both as a client (proxy -> remote cache nodes, or a real memcached) and as a
// server (exporting a node's HBM shards to the other nodes of the ring).
#pragma once

#include <arpa/inet.h>

#include <cstdint>
#include <cstring>
#include <string>

namespace shellac {
namespace mc {

constexpr uint8_t kReqMagic = 0x80, kResMagic = 0x81;
constexpr size_t kHeader = 24;

enum Op : uint8_t {
  GET = 0x00, SET = 0x01, ADD = 0x02, REPLACE = 0x03, DELETE = 0x04, INCREMENT = 0x05,
  DECREMENT = 0x06, QUIT = 0x07, FLUSH = 0x08, GETQ = 0x09, NOOP = 0x0a, VERSION = 0x0b,
  GETK = 0x0c, GETKQ = 0x0d, APPEND = 0x0e, PREPEND = 0x0f, STAT = 0x10, SETQ = 0x11,
  ADDQ = 0x12, REPLACEQ = 0x13, DELETEQ = 0x14, QUITQ = 0x17, FLUSHQ = 0x18, TOUCH = 0x1c,
};

enum Status : uint16_t {
  OK = 0x0000, KEY_ENOENT = 0x0001, KEY_EEXISTS = 0x0002, TOO_LARGE = 0x0003, INVALID_ARGS = 0x0004,
  NOT_STORED = 0x0005, DELTA_BADVAL = 0x0006, UNKNOWN_COMMAND = 0x0081, OUT_OF_MEMORY = 0x0082,
};

struct Header {
  uint8_t magic = 0, opcode = 0;
  uint16_t keylen = 0;
  uint8_t extlen = 0, datatype = 0;
  uint16_t status = 0;  // vbucket id in requests
  uint32_t bodylen = 0, opaque = 0;
  uint64_t cas = 0;
};

inline void put16(std::string& s, uint16_t v) { s.push_back((char)(v >> 8)); s.push_back((char)v); }
inline void put32(std::string& s, uint32_t v) {
  for (int i = 3; i >= 0; --i) s.push_back((char)(v >> (8 * i)));
}
inline void put64(std::string& s, uint64_t v) {
  for (int i = 7; i >= 0; --i) s.push_back((char)(v >> (8 * i)));
}
inline uint16_t get16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
inline uint32_t get32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
inline uint64_t get64(const uint8_t* p) { return ((uint64_t)get32(p) << 32) | get32(p + 4); }

inline Header parse_header(const uint8_t* p) {
  Header h;
  h.magic = p[0];
  h.opcode = p[1];
  h.keylen = get16(p + 2);
  h.extlen = p[4];
  h.datatype = p[5];
  h.status = get16(p + 6);
  h.bodylen = get32(p + 8);
  h.opaque = get32(p + 12);
  h.cas = get64(p + 16);
  return h;
}

inline void append_frame(std::string& out, uint8_t magic, uint8_t op, const std::string& key,
                         const std::string& extras, const char* val, size_t vlen,
                         uint16_t status_or_vb, uint32_t opaque, uint64_t cas) {
  out.reserve(out.size() + kHeader + extras.size() + key.size() + vlen);
  out.push_back((char)magic);
  out.push_back((char)op);
  put16(out, (uint16_t)key.size());
  out.push_back((char)extras.size());
  out.push_back(0);
  put16(out, status_or_vb);
  put32(out, (uint32_t)(extras.size() + key.size() + vlen));
  put32(out, opaque);
  put64(out, cas);
  out += extras;
  out += key;
  if (vlen) out.append(val, vlen);
}

inline void request(std::string& out, uint8_t op, const std::string& key, const std::string& extras,
                    const char* val, size_t vlen, uint32_t opaque, uint64_t cas = 0) {
  append_frame(out, kReqMagic, op, key, extras, val, vlen, 0, opaque, cas);
}

inline void response(std::string& out, uint8_t op, uint16_t status, const std::string& key,
                     const std::string& extras, const char* val, size_t vlen, uint32_t opaque,
                     uint64_t cas = 0) {
  append_frame(out, kResMagic, op, key, extras, val, vlen, status, opaque, cas);
}

inline std::string set_extras(uint32_t flags, uint32_t exptime) {
  std::string e;
  put32(e, flags);
  put32(e, exptime);
  return e;
}

// One complete frame view inside a receive buffer.
struct Frame {
  Header h;
  const uint8_t* extras;
  const uint8_t* key;
  const uint8_t* value;
  size_t vlen;
  std::string key_str() const { return std::string((const char*)key, h.keylen); }
};

// Returns bytes of the first complete frame at p (0 if incomplete); fills f.
inline size_t next_frame(const uint8_t* p, size_t n, Frame* f) {
  if (n < kHeader) return 0;
  f->h = parse_header(p);
  const size_t total = kHeader + f->h.bodylen;
  if (n < total) return 0;
  f->extras = p + kHeader;
  f->key = f->extras + f->h.extlen;
  f->value = f->key + f->h.keylen;
  const size_t used = (size_t)f->h.extlen + f->h.keylen;
  f->vlen = f->h.bodylen >= used ? f->h.bodylen - used : 0;
  return total;
}

// memcached exptime: 0 = never, <= 30 days = relative seconds, else unix time.
inline uint32_t exptime_to_relative(uint32_t exptime, uint32_t unix_now) {
  if (exptime == 0) return 0;
  if (exptime <= 60u * 60u * 24u * 30u) return exptime;
  return exptime > unix_now ? exptime - unix_now : 1;
}

}  // namespace mc
}  // namespace shellac
