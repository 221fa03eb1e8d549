// MD5 + ketama consistent-hash continuum.
//
// The reference configures pylibmc with behaviors={'ketama': True}
// (src/python/shellac/server/Server.py:81-83): libmemcached's consistent
// "ketama" distribution with MD5 key hashing. This is the classic libketama
// continuum: every server contributes 40*weight MD5 digests of "host:port-i",
// each digest yields four 32-bit points; a key maps to the first point >= the
// little-endian first word of MD5(key), wrapping around.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace shellac {

void md5(const void* data, size_t len, uint8_t out[16]);
std::string md5_hex(const std::string& s);

class KetamaRing {
 public:
  struct Node {
    std::string name;  // "host:port"
    uint32_t weight = 1;
    bool alive = true;
  };
  explicit KetamaRing(std::vector<Node> nodes = {}, uint32_t points_per_weight = 160);
  void set_alive(size_t idx, bool alive);  // ejection / re-admission rebuilds the continuum
  // Index of the node owning `key`, or -1 if no live node.
  int pick(const void* key, size_t len) const;
  int pick(const std::string& key) const { return pick(key.data(), key.size()); }
  static uint32_t key_hash(const void* key, size_t len);
  int pick_hash(uint32_t h) const;
  size_t size() const { return nodes_.size(); }
  const Node& node(size_t i) const { return nodes_[i]; }
  size_t points() const { return pts_.size(); }

 private:
  void rebuild();
  std::vector<Node> nodes_;
  uint32_t ppw_;
  std::vector<std::pair<uint32_t, uint32_t>> pts_;  // (point, node idx) sorted
};

}  // namespace shellac
