// Does hipStreamWaitValue64 work on this box, and on which memory? A stream waits on a
// word that a kernel on another stream raises after ~2 ms; every wait is bounded (the host
// releases the word itself after 3 s), so nothing can hang.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void k_raise(unsigned long long* w, unsigned long long v, long long spin) {
  const long long t0 = clock64();
  while (clock64() - t0 < spin) {}
  __hip_atomic_store(w, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_mark(int* m) { *m = 1; }

static const char* E(hipError_t e) { return hipGetErrorString(e); }

int main() {
  int attr = -1;
  hipError_t e = hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, 0);
  printf("attr CanUseStreamWaitValue = %d (%s)\n", attr, E(e));
  hipStream_t a, b, c;
  hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&c, hipStreamNonBlocking);
  int* mark;
  hipMalloc(&mark, 4);
  for (int kind = 0; kind < 4; ++kind) {
    unsigned long long* w = nullptr;
    const char* name[] = {"signal", "device", "host-coherent", "device-finegrained"};
    if (kind == 0) e = hipExtMallocWithFlags((void**)&w, 64, hipMallocSignalMemory);
    if (kind == 1) e = hipMalloc((void**)&w, 64);
    if (kind == 2) e = hipHostMalloc((void**)&w, 64, hipHostMallocCoherent | hipHostMallocMapped);
    if (kind == 3) e = hipExtMallocWithFlags((void**)&w, 64, hipDeviceMallocFinegrained);
    printf("[%s] alloc: %s\n", name[kind], E(e));
    if (e != hipSuccess) { (void)hipGetLastError(); continue; }
    hipMemset(w, 0, 64);
    hipMemset(mark, 0, 4);
    hipDeviceSynchronize();
    e = hipStreamWaitValue64(a, w, 5, hipStreamWaitValueGte, ~0ull);
    printf("[%s] wait enqueue: %s\n", name[kind], E(e));
    if (e != hipSuccess) { (void)hipGetLastError(); hipFree(w); continue; }
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(1), 0, a, mark);
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_raise, dim3(1), dim3(1), 0, b, w, 7ull, 4000000ll);
    bool early = hipStreamQuery(a) == hipSuccess;
    bool done = false, released = false;
    for (;;) {
      if (hipStreamQuery(a) == hipSuccess) { done = true; break; }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > 3.0 && !released) {  // release it ourselves
        released = true;
        unsigned long long v = 9;
        hipMemcpyAsync(w, &v, 8, hipMemcpyHostToDevice, c);
      }
      if (el > 6.0) break;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    hipStreamSynchronize(b);
    int m = 0;
    hipMemcpy(&m, mark, 4, hipMemcpyDeviceToHost);
    printf("[%s] done=%d early=%d released_by_host=%d mark=%d after %.4f s\n", name[kind], done,
           early, released, m, el);
    if (!done) { printf("ABORT: wait never resolved\n"); return 1; }
    if (kind == 2) hipHostFree(w); else hipFree(w);
  }
  return 0;
}
