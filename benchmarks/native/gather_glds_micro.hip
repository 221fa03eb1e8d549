// The GET gather's access pattern (records scattered over a log, copied back to back into a
// response buffer) with the two staging primitives of gfx950: loads into VGPRs (what
// k_segcopy does) vs LDS-DMA (`global_load_lds_dwordx4`: the load lands in LDS with no VGPR
// destination, then ds_read + store). The question the round-5 verdict asked: does staging
// through LDS put more bytes in flight and move the gather closer to the HBM roofline?
//
// Workload (the headline step's coalesced gather): 317K records, sizes log-uniform
// 64 B - 4 KiB + a 32-B header (16-B aligned), at random 16-B aligned offsets of a 4 GiB log,
// copied to consecutive offsets of a response buffer. Every kernel: one wave per record at a
// time (grid-stride over records), each lane 16 B per load, U loads in flight per lane.
// Reference: hipMemcpyAsync D2D of the same byte count (contiguous).
//
// build: hipcc --offload-arch=gfx950 -O3 -o bin/gather_glds_micro gather_glds_micro.hip
// run:   bin/gather_glds_micro [records=317000] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define OK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256, kWaves = kBlock / 64;

__global__ void k_fill(uint32_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 32);
}

// register staging: U independent 16-B loads per lane, then their stores
template <int U, bool NT = true>
__global__ __launch_bounds__(kBlock) void k_reg(const uint8_t* __restrict__ src,
                                                const uint64_t* __restrict__ soff,
                                                const uint64_t* __restrict__ doff, int n,
                                                uint8_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int w0 = blockIdx.x * kWaves + (threadIdx.x >> 6), nw = gridDim.x * kWaves;
  for (int j = w0; j < n; j += nw) {
    const uint64_t s = soff[j], d = doff[j], len = (doff[j + 1] - d) >> 4;
    for (uint64_t c0 = 0; c0 < len; c0 += 64 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t c = c0 + u * 64 + lane;
        if (c < len) {
          const u32x4* p = reinterpret_cast<const u32x4*>(src + s) + c;
          v[u] = NT ? __builtin_nontemporal_load(p) : *p;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t c = c0 + u * 64 + lane;
        if (c < len) __builtin_nontemporal_store(v[u], reinterpret_cast<u32x4*>(dst + d) + c);
      }
    }
  }
}

// LDS-DMA staging: U global_load_lds_dwordx4 per lane into the wave's own U KiB of LDS
// (lane-linear: lane l's 16 B land at slot + u KiB + 16 l), wait, then each lane reads back
// its own 16 B and stores them
// AUX: the load's cache policy bits (2 = nontemporal); PAD: extra LDS per workgroup (the
// production gather's 16.4 KB of segment tables), which lowers the co-resident workgroups
template <int U, int AUX = 0, int PAD = 0>
__global__ __launch_bounds__(kBlock) void k_glds(const uint8_t* __restrict__ src,
                                                 const uint64_t* __restrict__ soff,
                                                 const uint64_t* __restrict__ doff, int n,
                                                 uint8_t* __restrict__ dst) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[kWaves][U][1024];
  __shared__ uint32_t s_pad[PAD / 4 + 1];
  if (PAD && n < 0) s_pad[threadIdx.x] = 0;  // (keeps the padding allocated)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int w0 = blockIdx.x * kWaves + wv, nw = gridDim.x * kWaves;
  for (int j = w0; j < n; j += nw) {
    const uint64_t s = soff[j], d = doff[j], len = (doff[j + 1] - d) >> 4;
    for (uint64_t c0 = 0; c0 < len; c0 += 64 * U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t c = c0 + u * 64 + lane;
        if (c < len)
          __builtin_amdgcn_global_load_lds(
              (__attribute__((address_space(1))) void*)(src + s + c * 16),
              (__attribute__((address_space(3))) void*)(&s_buf[wv][u][0]), 16, 0, AUX);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t c = c0 + u * 64 + lane;
        if (c < len) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(&s_buf[wv][u][lane * 16]);
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + d) + c);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next DMA
    }
  }
}

template <typename K>
int resident(K k) {
  int per = 0, cus = 0;
  OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, kBlock, 0));
  OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  return per * cus;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 317000;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const uint64_t log_bytes = 4ull << 30;
  std::mt19937_64 rng(42);
  std::vector<uint64_t> soff(n), doff(n + 1);
  uint64_t tot = 0;
  for (int j = 0; j < n; ++j) {
    const double v = std::exp(std::log(64.0) + (std::log(4096.0) - std::log(64.0)) *
                                                   std::uniform_real_distribution<>(0, 1)(rng));
    const uint64_t bytes = ((uint64_t)v + 32 + 15) / 16 * 16;  // header + value, 16-B units
    soff[j] = (rng() % ((log_bytes - 8192) / 16)) * 16;
    doff[j] = tot;
    tot += bytes;
  }
  doff[n] = tot;
  uint8_t *src, *dst, *ref;
  uint64_t *dso, *ddo;
  OK(hipMalloc(&src, log_bytes));
  OK(hipMalloc(&dst, tot));
  OK(hipMalloc(&ref, tot));
  OK(hipMalloc(&dso, n * 8));
  OK(hipMalloc(&ddo, (n + 1) * 8));
  OK(hipMemcpy(dso, soff.data(), n * 8, hipMemcpyHostToDevice));
  OK(hipMemcpy(ddo, doff.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, nullptr, (uint32_t*)src, log_bytes / 4);
  OK(hipDeviceSynchronize());
  hipEvent_t a, b;
  OK(hipEventCreate(&a));
  OK(hipEventCreate(&b));
  printf("records %d, %.1f MiB gathered (x2 with the writes), %d reps, median us\n", n,
         tot / 1048576.0, reps);
  auto time = [&](const char* name, auto launch) {
    std::vector<float> t;
    for (int r = 0; r < reps + 2; ++r) {
      OK(hipEventRecord(a, nullptr));
      launch();
      OK(hipEventRecord(b, nullptr));
      OK(hipEventSynchronize(b));
      float ms = 0;
      OK(hipEventElapsedTime(&ms, a, b));
      if (r >= 2) t.push_back(ms * 1000.f);
    }
    std::sort(t.begin(), t.end());
    const float med = t[t.size() / 2];
    printf("  %-34s %8.1f us  %6.2f TB/s (read + write)\n", name, med, 2.0 * tot / (med * 1e6));
  };
  // reference result: register staging, U = 4
  hipLaunchKernelGGL(k_reg<4>, dim3(resident(k_reg<4>)), dim3(kBlock), 0, nullptr, src, dso, ddo,
                     n, ref);
  OK(hipDeviceSynchronize());
  std::vector<uint8_t> h_ref(tot), h_out(tot);
  OK(hipMemcpy(h_ref.data(), ref, tot, hipMemcpyDeviceToHost));
  {  // the reference against the host: a sample of records
    std::vector<uint8_t> rec(8192);
    for (int j = 0; j < n; j += 997) {
      const uint64_t len = doff[j + 1] - doff[j];
      OK(hipMemcpy(rec.data(), src + soff[j], len, hipMemcpyDeviceToHost));
      if (memcmp(rec.data(), h_ref.data() + doff[j], len)) {
        fprintf(stderr, "reference gather wrong at record %d\n", j);
        return 1;
      }
    }
  }
  auto check = [&](const char* name) {
    OK(hipMemcpy(h_out.data(), dst, tot, hipMemcpyDeviceToHost));
    if (h_out != h_ref) {
      fprintf(stderr, "%s: output differs from the reference gather\n", name);
      exit(1);
    }
    OK(hipMemset(dst, 0, tot));
  };
#define RUN(K, NAME)                                                                           \
  do {                                                                                         \
    const int g = resident(K);                                                                 \
    time(NAME, [&] { hipLaunchKernelGGL(K, dim3(g), dim3(kBlock), 0, nullptr, src, dso, ddo, n, \
                                        dst); });                                              \
    check(NAME);                                                                               \
  } while (0)
  RUN(k_reg<2>, "registers, U=2");
  RUN(k_reg<4>, "registers, U=4");
  RUN(k_reg<8>, "registers, U=8");
  RUN(k_reg<16>, "registers, U=16");
  RUN(k_glds<2>, "LDS-DMA, U=2");
  RUN(k_glds<4>, "LDS-DMA, U=4");
  RUN(k_glds<8>, "LDS-DMA, U=8");
  RUN(k_glds<16>, "LDS-DMA, U=16");
  RUN((k_reg<4, false>), "registers, U=4, plain loads");
  RUN((k_glds<4, 2>), "LDS-DMA, U=4, nontemporal");
  RUN((k_glds<2, 0, 16448>), "LDS-DMA, U=2, +16.4 KB LDS");
  RUN((k_glds<4, 0, 16448>), "LDS-DMA, U=4, +16.4 KB LDS");
  RUN((k_reg<4, true>), "registers, U=4 (again)");
  RUN((k_glds<4>), "LDS-DMA, U=4 (again)");
  time("hipMemcpyAsync D2D, same bytes",
       [&] { OK(hipMemcpyAsync(dst, ref, tot, hipMemcpyDeviceToDevice, nullptr)); });
  return 0;
}
