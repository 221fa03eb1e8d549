// Shared helpers for the shellac_amd native core (host C++ and HIP device code).
#pragma once

#include <cstdint>
#include <cstddef>
#include <stdexcept>
#include <string>

#if defined(__HIPCC__)
#define SH_HD __host__ __device__ __forceinline__
#else
#define SH_HD inline
#endif

namespace shellac {

SH_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

SH_HD uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

SH_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

}  // namespace shellac

#define SH_CHECK(cond, msg)                                                         \
  do {                                                                              \
    if (!(cond)) throw ::shellac::Error(std::string("shellac: ") + (msg) + " [" +  \
                                        __FILE__ + ":" + std::to_string(__LINE__) + "]"); \
  } while (0)
