// Doorbell round trip host -> resident kernel -> host, two placements of the doorbell word:
// pinned coherent host memory (the kernel polls over PCIe) and fine-grained device memory
// written by the host through the BAR (the kernel polls its own HBM). Prints p50/p99 us.
// Decides where the edge server's job ring lives (HbmCache::serve_get).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#define OK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s\n", hipGetErrorString(e_), #x);              \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

__global__ void pingpong(uint64_t* in, uint64_t* out, int iters) {
  for (int i = 1; i <= iters; ++i) {
    while (__hip_atomic_load(in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != (uint64_t)i)
      __builtin_amdgcn_s_sleep(1);
    __hip_atomic_store(out, (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static int run(const char* name, uint64_t* in_host_view, uint64_t* in_dev_view, uint64_t* out_h,
               uint64_t* out_d, int iters) {
  *in_host_view = 0;
  *out_h = 0;
  hipStream_t s;
  OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(pingpong, dim3(1), dim3(1), 0, s, in_dev_view, out_d, iters);
  OK(hipGetLastError());
  std::vector<double> rt;
  for (int i = 1; i <= iters; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(in_host_view, (uint64_t)i, __ATOMIC_RELEASE);
    const auto lim = t0 + std::chrono::seconds(2);
    while (__atomic_load_n(out_h, __ATOMIC_ACQUIRE) != (uint64_t)i) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() > lim) {
        std::printf("%s: no answer at iteration %d\n", name, i);
        __atomic_store_n(in_host_view, (uint64_t)iters, __ATOMIC_RELEASE);  // let it finish
        break;
      }
    }
    rt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                     .count());
  }
  OK(hipStreamSynchronize(s));
  OK(hipStreamDestroy(s));
  std::sort(rt.begin(), rt.end());
  std::printf("%s: round trip p50 %.2f us  p99 %.2f us\n", name, rt[rt.size() / 2],
              rt[rt.size() * 99 / 100]);
  std::fflush(stdout);
  return 0;
}

int main() {
  const int iters = 5000;
  uint64_t *out_h = nullptr, *out_d = nullptr;
  OK(hipHostMalloc(&out_h, 64, hipHostMallocMapped | hipHostMallocCoherent));
  OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&out_d), out_h, 0));
  uint64_t *hin_h = nullptr, *hin_d = nullptr;
  OK(hipHostMalloc(&hin_h, 64, hipHostMallocMapped | hipHostMallocCoherent));
  OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hin_d), hin_h, 0));
  if (run("host-memory doorbell", hin_h, hin_d, out_h, out_d, iters)) return 1;
  // fine-grained device memory: the host writes it through its BAR mapping (may not be
  // host-accessible on every system: this step runs last)
  uint64_t* vin = nullptr;
  OK(hipExtMallocWithFlags(reinterpret_cast<void**>(&vin), 4096, hipDeviceMallocFinegrained));
  hipPointerAttribute_t at{};
  OK(hipPointerGetAttributes(&at, vin));
  std::printf("fine-grained VRAM: type %d host view %p device view %p\n", (int)at.type,
              at.hostPointer, at.devicePointer);
  std::fflush(stdout);
  uint64_t* hv = at.hostPointer ? static_cast<uint64_t*>(at.hostPointer) : vin;
  if (run("device-memory doorbell", hv, vin, out_h, out_d, iters)) return 1;
  return 0;
}
