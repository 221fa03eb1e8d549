// Collectives of the routed serving step, issued by the native executor
// (RoutedStep::step) without a round trip through Python per call.
//
// The reference has no collectives (one blocking memcached round trip per request,
// src/python/shellac/server/Server.py:335, :432); here every rank exchanges whole
// batches with the others once per step. Three implementations:
//   * RCCL (one process per GPU, the production path): communicators of our own, one
//     per channel, built from unique ids the ranks share through the torch.distributed
//     store; ncclAllGather and grouped ncclSend/ncclRecv enqueued on the caller's HIP
//     stream, so a collective is just another stream-ordered op. librccl is found at run
//     time (dlopen) so the process uses the one copy torch already loaded.
//   * Mirror (bench.py --simulate-world N): rank 0 of a symmetric N-rank job on one GPU;
//     an all-to-all is a local copy, an all-gather a permutation of the own row.
//   * Python callbacks (tests: several ranks on one GPU over gloo), see bind_router.cc.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace shellac {

class StepComm {
 public:
  // Channels map to separate communicators so that collectives issued on different
  // streams never serialise behind each other: the request exchange and the row
  // all-gather (main stream), the reply transfer (its own stream, overlapping the next
  // step), the SET exchange (the SET stream).
  enum Channel { kCtrl = 0, kData = 1, kSet = 2, kChannels = 3 };
  virtual ~StepComm() = default;
  virtual int world() const = 0;
  virtual int rank() const = 0;
  // out[q * words, (q + 1) * words) = rank q's `in` (int64 words). `peer_blocks`: the row
  // starts with that many blocks of one entry per peer (the mirror permutes them).
  virtual void all_gather(int64_t* out, const int64_t* in, int64_t words, int peer_blocks,
                          hipStream_t s, int ch) = 0;
  // Byte all-to-all: sbytes[p] bytes from sbuf + soff[p] go to rank p; rbytes[q] bytes
  // from rank q land at rbuf + roff[q]. Entries for this rank are ignored (self traffic
  // never enters a collective). Stream-ordered on `s`.
  virtual void all_to_all(uint8_t* rbuf, const std::vector<int64_t>& roff,
                          const std::vector<int64_t>& rbytes, const uint8_t* sbuf,
                          const std::vector<int64_t>& soff, const std::vector<int64_t>& sbytes,
                          hipStream_t s, int ch) = 0;
};

// 128-byte RCCL unique id (rank 0 makes one per channel and shares them).
std::string rccl_unique_id();
// Collective: every rank of the job calls it with the same ids (one per channel).
std::unique_ptr<StepComm> make_rccl_comm(int world, int rank, int device,
                                         const std::vector<std::string>& ids);
std::unique_ptr<StepComm> make_mirror_comm(int world, int rank);

}  // namespace shellac
