// Collectives of the routed step (see step_comm.h).
#include "step_comm.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "common.h"

#define SC_OK(expr)                                                                      \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw Error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + #expr);  \
  } while (0)

namespace shellac {

namespace {

// ---- RCCL, resolved at run time ------------------------------------------------------
// torch links its own librccl (soname librccl.so.1); dlopen by soname returns that copy
// when torch is loaded, so one RCCL instance serves both.
struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    SH_CHECK(h != nullptr, std::string("cannot load librccl.so.1: ") + dlerror());
    auto sym = [&](const char* name) {
      void* p = dlsym(h, name);
      SH_CHECK(p != nullptr, std::string("librccl lacks ") + name);
      return p;
    };
    api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(sym("ncclGetUniqueId"));
    api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(sym("ncclCommInitRank"));
    api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(sym("ncclCommDestroy"));
    api.all_gather = reinterpret_cast<decltype(api.all_gather)>(sym("ncclAllGather"));
    api.send = reinterpret_cast<decltype(api.send)>(sym("ncclSend"));
    api.recv = reinterpret_cast<decltype(api.recv)>(sym("ncclRecv"));
    api.group_start = reinterpret_cast<decltype(api.group_start)>(sym("ncclGroupStart"));
    api.group_end = reinterpret_cast<decltype(api.group_end)>(sym("ncclGroupEnd"));
    api.error_string = reinterpret_cast<decltype(api.error_string)>(sym("ncclGetErrorString"));
  });
  return api;
}

void nccl_ok(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw Error(std::string("RCCL error in ") + what + ": " + rccl().error_string(r));
}

class RcclComm final : public StepComm {
 public:
  RcclComm(int world, int rank, int device, const std::vector<std::string>& ids)
      : w_(world), r_(rank) {
    SH_CHECK((int)ids.size() == kChannels, "RCCL comm: one unique id per channel");
    SC_OK(hipSetDevice(device));
    const RcclApi& a = rccl();
    // grouped, so the three initialisations (each collective over the job) overlap
    nccl_ok(a.group_start(), "ncclGroupStart");
    for (int c = 0; c < kChannels; ++c) {
      SH_CHECK(ids[c].size() == sizeof(ncclUniqueId), "RCCL comm: bad unique id");
      ncclUniqueId id;
      std::memcpy(&id, ids[c].data(), sizeof(id));
      nccl_ok(a.comm_init_rank(&comm_[c], world, id, rank), "ncclCommInitRank");
    }
    nccl_ok(a.group_end(), "ncclGroupEnd");
  }
  ~RcclComm() override {
    for (ncclComm_t c : comm_)
      if (c) (void)rccl().comm_destroy(c);
  }
  int world() const override { return w_; }
  int rank() const override { return r_; }

  void all_gather(int64_t* out, const int64_t* in, int64_t words, int, hipStream_t s,
                  int ch) override {
    nccl_ok(rccl().all_gather(in, out, (size_t)words, ncclInt64, comm_[ch], s), "ncclAllGather");
  }

  void all_to_all(uint8_t* rbuf, const std::vector<int64_t>& roff,
                  const std::vector<int64_t>& rbytes, const uint8_t* sbuf,
                  const std::vector<int64_t>& soff, const std::vector<int64_t>& sbytes,
                  hipStream_t s, int ch) override {
    const RcclApi& a = rccl();
    nccl_ok(a.group_start(), "ncclGroupStart");
    // a pair with nothing to move is skipped on both sides: sender and receiver read the
    // same byte count from the all-gathered matrix (or the agreed slot size)
    for (int p = 0; p < w_; ++p) {
      if (p == r_) continue;
      if (sbytes[p] > 0)
        nccl_ok(a.send(sbuf + soff[p], (size_t)sbytes[p], ncclUint8, p, comm_[ch], s), "ncclSend");
      if (rbytes[p] > 0)
        nccl_ok(a.recv(rbuf + roff[p], (size_t)rbytes[p], ncclUint8, p, comm_[ch], s), "ncclRecv");
    }
    nccl_ok(a.group_end(), "ncclGroupEnd");
  }

 private:
  int w_, r_;
  ncclComm_t comm_[kChannels] = {nullptr, nullptr, nullptr};
};

// ---- mirror ----------------------------------------------------------------------------
// out[q K + j] = in[j'] where j' swaps (b W + me) and (b W + q) for b < peer_blocks, q != me:
// what rank q sends to x is what this rank sends to x with the roles of me and q exchanged.
__global__ void k_mirror_gather(int64_t* __restrict__ out, const int64_t* __restrict__ in,
                                int64_t K, int W, int me, int peer_blocks) {
  const int64_t total = K * W;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(t / K);
    int64_t j = t - (int64_t)q * K;
    if (q != me && j < (int64_t)peer_blocks * W) {
      const int64_t b = j / W, e = j - b * W;
      if (e == me) j = b * W + q;
      else if (e == q) j = b * W + me;
    }
    out[t] = in[j];
  }
}

class MirrorComm final : public StepComm {
 public:
  MirrorComm(int world, int rank) : w_(world), r_(rank) {}
  int world() const override { return w_; }
  int rank() const override { return r_; }
  void all_gather(int64_t* out, const int64_t* in, int64_t words, int peer_blocks, hipStream_t s,
                  int) override {
    const int64_t total = words * w_;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 1024);
    hipLaunchKernelGGL(k_mirror_gather, dim3(std::max(grid, 1)), dim3(256), 0, s, out, in, words,
                       w_, r_, peer_blocks);
    SC_OK(hipGetLastError());
  }
  void all_to_all(uint8_t* rbuf, const std::vector<int64_t>& roff,
                  const std::vector<int64_t>& rbytes, const uint8_t* sbuf,
                  const std::vector<int64_t>& soff, const std::vector<int64_t>& sbytes,
                  hipStream_t s, int) override {
    // symmetric traffic: what comes back from p is what went to p. One copy when both
    // sides lay the peers out contiguously in the same order (the routed step always does)
    int64_t lo_s = -1, lo_r = -1, n = 0;
    bool contiguous = true;
    for (int p = 0; p < w_; ++p) {
      if (p == r_ || sbytes[p] == 0) continue;
      SH_CHECK(sbytes[p] == rbytes[p], "mirror all_to_all needs symmetric sizes");
      if (lo_s < 0) {
        lo_s = soff[p];
        lo_r = roff[p];
      }
      if (soff[p] != lo_s + n || roff[p] != lo_r + n) contiguous = false;
      n += sbytes[p];
    }
    if (n == 0) return;
    if (contiguous) {
      SC_OK(hipMemcpyAsync(rbuf + lo_r, sbuf + lo_s, (size_t)n, hipMemcpyDeviceToDevice, s));
      return;
    }
    for (int p = 0; p < w_; ++p)
      if (p != r_ && sbytes[p] > 0)
        SC_OK(hipMemcpyAsync(rbuf + roff[p], sbuf + soff[p], (size_t)sbytes[p],
                             hipMemcpyDeviceToDevice, s));
  }

 private:
  int w_, r_;
};

}  // namespace

std::string rccl_unique_id() {
  ncclUniqueId id;
  nccl_ok(rccl().get_unique_id(&id), "ncclGetUniqueId");
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

std::unique_ptr<StepComm> make_rccl_comm(int world, int rank, int device,
                                         const std::vector<std::string>& ids) {
  return std::make_unique<RcclComm>(world, rank, device, ids);
}

std::unique_ptr<StepComm> make_mirror_comm(int world, int rank) {
  return std::make_unique<MirrorComm>(world, rank);
}

}  // namespace shellac
