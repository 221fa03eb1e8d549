// Cross-queue dependency latency on one MI355X: how long after kernel A's last wave ends
// does kernel B's first wave start, for each way of ordering B after A?
//
// The serving step (models/sharded_cache.py ShardedCache.serve) has two ordering hops on
// its critical path: the SET chain's fix-up (side queue) -> the next lookup (main queue),
// and the lookup -> the gather with the `probe` event recorded between them. A GPU-clock
// trace of the headline step (profiles/r6_trace) shows 15 us and 5 us there. This
// program measures each ordering mechanism in isolation with the kernels' own
// wall_clock64() stamps (100 MHz), so no profiler sits in the way.
//
// build: hipcc --offload-arch=gfx950 -O2 -o bin/hop_micro hop_micro.hip
// run:   bin/hop_micro [reps=40] [busy_us=60]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define OK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int kGrid = 1024, kBlock = 256;

// Every workgroup stamps its start (min) and end (max) into ts[2 slot], ts[2 slot + 1],
// spinning `ticks` of the 100-MHz wall clock in between. flag (optional): the last
// workgroup to finish stores `flag_val` there (a device-side release for wait-value).
__global__ __launch_bounds__(kBlock) void k_busy(unsigned long long* ts, int slot,
                                                 uint64_t ticks, unsigned int* done,
                                                 uint64_t* flag, uint64_t flag_val) {
  __shared__ uint64_t s_t0;
  if (threadIdx.x == 0) {
    s_t0 = wall_clock64();
    atomicMin(&ts[2 * slot], (unsigned long long)s_t0);
  }
  __syncthreads();
  const uint64_t t0 = s_t0;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicMax(&ts[2 * slot + 1], (unsigned long long)wall_clock64());
    if (flag) {
      __threadfence();
      const unsigned int k = atomicAdd(done, 1u);
      if (k == gridDim.x - 1) {
        __threadfence_system();
        __hip_atomic_store(flag, flag_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

__global__ void k_reset(unsigned long long* ts, int n, unsigned int* done) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) ts[i] = (i & 1) ? 0ull : ~0ull;
  if (threadIdx.x == 0) *done = 0;
}

enum Mode {
  kSame,          // s1: A, B
  kSameRecord,    // s1: A, record(e), B
  kCross,         // s1: A, record(e); s2: wait(e), B
  kCrossNoFence,  // as kCross, e created with hipEventDisableSystemFence
  kCrossExt,      // s1: hipExtLaunchKernelGGL(A, stop = e); s2: wait(e), B
  kCrossExtNoFence,
  kWriteValue,    // s1: A, writeValue64(flag); s2: waitValue64(flag >= v), B
  kKernelFlag,    // A's last workgroup stores the flag; s2: waitValue64(flag >= v), B
  kSameWaitDone,  // s1: A, wait(e already complete), B (a satisfied barrier packet)
  kModes
};
static const char* kNames[kModes] = {
    "same queue: A, B",
    "same queue: A, record, B",
    "cross: record / wait (default event)",
    "cross: record / wait (no system fence)",
    "cross: A's own stop event (hipExtLaunch)",
    "cross: A's own stop event, no system fence",
    "cross: writeValue64 / waitValue64",
    "cross: A's last wave stores, waitValue64",
    "same queue: A, wait(satisfied event), B",
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 40;
  const int busy_us = argc > 2 ? atoi(argv[2]) : 60;
  const uint64_t ticks = (uint64_t)busy_us * 100;  // 100 MHz
  hipStream_t s1, s2;
  OK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  OK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e, enf, edone;
  OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  OK(hipEventCreateWithFlags(&enf, hipEventDisableTiming | hipEventDisableSystemFence));
  OK(hipEventCreateWithFlags(&edone, hipEventDisableTiming));
  unsigned long long* ts;
  unsigned int* done;
  uint64_t* flag;
  OK(hipMalloc(&ts, 4 * sizeof(unsigned long long)));
  OK(hipMalloc(&done, sizeof(unsigned int)));
  OK(hipExtMallocWithFlags((void**)&flag, sizeof(uint64_t), hipMallocSignalMemory));
  OK(hipMemset(flag, 0, sizeof(uint64_t)));
  OK(hipEventRecord(edone, s1));
  OK(hipDeviceSynchronize());
  uint64_t fv = 0;
  printf("%-46s %9s %9s %9s   (us, %d reps, A = %d us x %d workgroups)\n", "ordering",
         "median", "p10", "p90", reps, busy_us, kGrid);
  for (int m = 0; m < kModes; ++m) {
    std::vector<double> gap;
    for (int r = 0; r < reps + 3; ++r) {
      hipLaunchKernelGGL(k_reset, dim3(1), dim3(64), 0, s1, ts, 4, done);
      OK(hipStreamSynchronize(s1));
      ++fv;
      const dim3 g(kGrid), b(kBlock);
      switch (m) {
        case kSame:
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 0, ticks, done, nullptr, 0);
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 1, ticks, done, nullptr, 0);
          break;
        case kSameRecord:
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 0, ticks, done, nullptr, 0);
          OK(hipEventRecord(e, s1));
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 1, ticks, done, nullptr, 0);
          break;
        case kCross:
        case kCrossNoFence: {
          hipEvent_t x = m == kCross ? e : enf;
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 0, ticks, done, nullptr, 0);
          OK(hipEventRecord(x, s1));
          OK(hipStreamWaitEvent(s2, x, 0));
          hipLaunchKernelGGL(k_busy, g, b, 0, s2, ts, 1, ticks, done, nullptr, 0);
          break;
        }
        case kCrossExt:
        case kCrossExtNoFence: {
          hipEvent_t x = m == kCrossExt ? e : enf;
          hipExtLaunchKernelGGL(k_busy, g, b, 0, s1, nullptr, x, 0, ts, 0, ticks, done,
                                (uint64_t*)nullptr, (uint64_t)0);
          OK(hipStreamWaitEvent(s2, x, 0));
          hipLaunchKernelGGL(k_busy, g, b, 0, s2, ts, 1, ticks, done, nullptr, 0);
          break;
        }
        case kWriteValue:
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 0, ticks, done, nullptr, 0);
          OK(hipStreamWriteValue64(s1, flag, fv, 0));
          OK(hipStreamWaitValue64(s2, flag, fv, hipStreamWaitValueGte, ~0ull));
          hipLaunchKernelGGL(k_busy, g, b, 0, s2, ts, 1, ticks, done, nullptr, 0);
          break;
        case kKernelFlag:
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 0, ticks, done, flag, fv);
          OK(hipStreamWaitValue64(s2, flag, fv, hipStreamWaitValueGte, ~0ull));
          hipLaunchKernelGGL(k_busy, g, b, 0, s2, ts, 1, ticks, done, nullptr, 0);
          break;
        case kSameWaitDone:
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 0, ticks, done, nullptr, 0);
          OK(hipStreamWaitEvent(s1, edone, 0));
          hipLaunchKernelGGL(k_busy, g, b, 0, s1, ts, 1, ticks, done, nullptr, 0);
          break;
      }
      OK(hipGetLastError());
      OK(hipDeviceSynchronize());
      unsigned long long h[4];
      OK(hipMemcpy(h, ts, sizeof h, hipMemcpyDeviceToHost));
      if (r >= 3) gap.push_back(((double)h[2] - (double)h[1]) / 100.0);
    }
    std::sort(gap.begin(), gap.end());
    const size_t n = gap.size();
    printf("%-46s %9.2f %9.2f %9.2f\n", kNames[m], gap[n / 2], gap[n / 10], gap[n * 9 / 10]);
  }
  return 0;
}
