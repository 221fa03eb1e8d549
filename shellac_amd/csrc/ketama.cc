// MD5 (RFC 1321) and the ketama continuum.
#include "ketama.h"

#include <algorithm>
#include <cstring>

namespace shellac {

namespace {

struct Md5 {
  uint32_t a = 0x67452301, b = 0xefcdab89, c = 0x98badcfe, d = 0x10325476;
  uint64_t len = 0;
  uint8_t buf[64];
  size_t used = 0;

  static uint32_t rol(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
        0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
        0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
        0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
        0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
        0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
        0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
        0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
        0xeb86d391};
    static const int S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t m[16];
    for (int i = 0; i < 16; ++i)
      m[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
             ((uint32_t)p[4 * i + 3] << 24);
    uint32_t A = a, B = b, C = c, D = d;
    for (int i = 0; i < 64; ++i) {
      uint32_t F;
      int g;
      if (i < 16) { F = (B & C) | (~B & D); g = i; }
      else if (i < 32) { F = (D & B) | (~D & C); g = (5 * i + 1) & 15; }
      else if (i < 48) { F = B ^ C ^ D; g = (3 * i + 5) & 15; }
      else { F = C ^ (B | ~D); g = (7 * i) & 15; }
      const uint32_t tmp = D;
      D = C;
      C = B;
      B = B + rol(A + F + K[i] + m[g], S[i]);
      A = tmp;
    }
    a += A; b += B; c += C; d += D;
  }

  void update(const uint8_t* p, size_t n) {
    len += n;
    while (n) {
      const size_t take = std::min(n, 64 - used);
      std::memcpy(buf + used, p, take);
      used += take;
      p += take;
      n -= take;
      if (used == 64) {
        block(buf);
        used = 0;
      }
    }
  }

  void final(uint8_t out[16]) {
    const uint64_t bits = len * 8;
    const uint8_t pad = 0x80;
    update(&pad, 1);
    const uint8_t zero = 0;
    while (used != 56) update(&zero, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (8 * i));
    update(lb, 8);
    const uint32_t w[4] = {a, b, c, d};
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 4; ++k) out[4 * i + k] = (uint8_t)(w[i] >> (8 * k));
  }
};

}  // namespace

void md5(const void* data, size_t len, uint8_t out[16]) {
  Md5 m;
  m.update(static_cast<const uint8_t*>(data), len);
  m.final(out);
}

std::string md5_hex(const std::string& s) {
  uint8_t d[16];
  md5(s.data(), s.size(), d);
  static const char* hx = "0123456789abcdef";
  std::string out(32, '0');
  for (int i = 0; i < 16; ++i) {
    out[2 * i] = hx[d[i] >> 4];
    out[2 * i + 1] = hx[d[i] & 15];
  }
  return out;
}

KetamaRing::KetamaRing(std::vector<Node> nodes, uint32_t ppw) : nodes_(std::move(nodes)), ppw_(ppw) {
  rebuild();
}

void KetamaRing::set_alive(size_t idx, bool alive) {
  if (idx >= nodes_.size() || nodes_[idx].alive == alive) return;
  nodes_[idx].alive = alive;
  rebuild();
}

void KetamaRing::rebuild() {
  pts_.clear();
  for (size_t i = 0; i < nodes_.size(); ++i) {
    if (!nodes_[i].alive) continue;
    const uint32_t digests = (ppw_ * nodes_[i].weight) / 4;
    for (uint32_t k = 0; k < digests; ++k) {
      const std::string s = nodes_[i].name + "-" + std::to_string(k);
      uint8_t d[16];
      md5(s.data(), s.size(), d);
      for (int h = 0; h < 4; ++h) {
        const uint32_t p = ((uint32_t)d[3 + h * 4] << 24) | ((uint32_t)d[2 + h * 4] << 16) |
                           ((uint32_t)d[1 + h * 4] << 8) | (uint32_t)d[h * 4];
        pts_.emplace_back(p, (uint32_t)i);
      }
    }
  }
  std::sort(pts_.begin(), pts_.end());
}

uint32_t KetamaRing::key_hash(const void* key, size_t len) {
  uint8_t d[16];
  md5(key, len, d);
  return ((uint32_t)d[3] << 24) | ((uint32_t)d[2] << 16) | ((uint32_t)d[1] << 8) | (uint32_t)d[0];
}

int KetamaRing::pick_hash(uint32_t h) const {
  if (pts_.empty()) return -1;
  auto it = std::lower_bound(pts_.begin(), pts_.end(), std::make_pair(h, (uint32_t)0));
  if (it == pts_.end()) it = pts_.begin();
  return (int)it->second;
}

int KetamaRing::pick(const void* key, size_t len) const { return pick_hash(key_hash(key, len)); }

}  // namespace shellac
