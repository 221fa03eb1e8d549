// Batch gzip (RFC 1952 members around RFC 1951 DEFLATE data) on one MI355X.
//
// The reference gunzips every origin response and gzips it again at level 6 before
// caching it (src/python/shellac/server/HttpParser.py:124-127, :343-351); the proxy here
// passes gzip bodies through and compresses only identity text bodies (--compress), on
// the CPU. This engine moves that compression to the GPU for whole batches of bodies
// ("batch gzip on GPU for the miss path").
//
// Design (deflate.hip, two passes around a host planning step): every input is cut into
// 32 KiB blocks and every block is one workgroup of ONE wave.
//  1. k_lz77: the wave keeps the block and a 4096-entry hash head table in LDS and parses
//     greedily: at each position the 64 lanes compare the candidate match 64 bytes at a
//     time (one ballot finds the first mismatch) and hash the positions a match covers
//     in parallel. It writes the block's tokens, its literal/length + distance symbol
//     histogram and its CRC-32 register (lane slices combined by GF(2) multiplies).
//  2. host (huffman.cc, a few threads): per block, the cheapest of stored / fixed
//     Huffman / dynamic Huffman by exact bit count, length-limited canonical codes and
//     the dynamic header.
//  3. k_emit: the codes in LDS; each chunk of 64 tokens is placed by a wave prefix sum of
//     their bit lengths and OR-ed into an LDS bit buffer, written out whole.
// Blocks are independent (the window never crosses a block), so a non-final block ends
// with an empty stored block (the zlib sync-flush marker 00 00 FF FF) and the blocks of
// one input concatenate byte-wise. The host folds the blocks' CRC registers per input.
#pragma once

#include <hip/hip_runtime_api.h>

#include "backend.h"

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

namespace shellac {

constexpr int kDeflateBlock = 32768;                 // input bytes per block (= max window)
constexpr int kDeflateStride = kDeflateBlock + 64;   // output bytes reserved per block

struct GzipStats {
  uint64_t inputs = 0, blocks = 0, in_bytes = 0, out_bytes = 0, stored_blocks = 0, inflated = 0;
  // last call, milliseconds: host packing, GPU (copies in + kernel + copies out), assembly
  double last_pack_ms = 0, last_gpu_ms = 0, last_assemble_ms = 0;
};

class GpuGzip {
 public:
  explicit GpuGzip(int device);
  ~GpuGzip();
  GpuGzip(const GpuGzip&) = delete;
  GpuGzip& operator=(const GpuGzip&) = delete;

  // One gzip member per input, in input order (decompressible by zlib / gzip).
  std::vector<std::string> compress(const std::vector<std::string_view>& in);
  // Raw DEFLATE streams only (no gzip header / trailer), for tests and benchmarks.
  std::vector<std::string> deflate(const std::vector<std::string_view>& in);
  // Batch gunzip: one member per input. ok[i] = 1 when member i decoded on the GPU to
  // exactly its ISIZE bytes with a matching CRC-32 (else out[i] is empty: a corrupt
  // member, framing the GPU path does not take, or ISIZE > max_out — the caller may fall
  // back to zlib, which also reports the error).
  std::vector<std::string> inflate(const std::vector<std::string_view>& in,
                                   std::vector<uint8_t>* ok, uint64_t max_out);
  GzipStats stats() const { return stats_; }
  int device() const { return device_; }

 private:
  void run(const std::vector<std::string_view>& in, std::vector<std::string>* out, bool gzip);
  template <typename T>
  T* grow(T** p, size_t* cap, size_t count, bool host);

  int device_;
  hipStream_t stream_ = nullptr;
  std::mutex mu_;
  GzipStats stats_;
  // grow-only staging: pinned host and device copies of the packed input, the block
  // table (src offset, length | final << 31) and the per-block outputs
  uint8_t *h_in_ = nullptr, *d_in_ = nullptr, *h_out_ = nullptr, *d_out_ = nullptr;
  uint64_t *h_tab_ = nullptr, *d_tab_ = nullptr;
  uint32_t *h_len_ = nullptr, *d_len_ = nullptr;
  // two-pass encoding: tokens (device), pass-1 results, per-block plans
  uint32_t *d_tok_ = nullptr, *d_res_ = nullptr, *d_plan_ = nullptr, *d_slot_ = nullptr;
  size_t d_tok_cap_ = 0, d_res_cap_ = 0, d_plan_cap_ = 0, d_slot_cap_ = 0;
  size_t h_in_cap_ = 0, d_in_cap_ = 0, h_out_cap_ = 0, d_out_cap_ = 0, h_tab_cap_ = 0,
         d_tab_cap_ = 0, h_len_cap_ = 0, d_len_cap_ = 0;
};

// Asynchronous front end of GpuGzip for the proxy's miss path: reactor threads submit
// bodies and get a completion; one service thread per GPU collects the submissions of a
// short window (`batch_us`, or `max_batch` bodies) into ONE GpuGzip::compress call, then
// runs each completion (which posts back to its reactor). On a GPU error the completion
// gets ok = false and the original body back, so the caller can fall back to the CPU.
// Inflate jobs (identity variants of gzip objects for clients without gzip) batch the
// same way into GpuGzip::inflate; a member the GPU path does not decode is inflated with
// zlib on the service thread, never on a reactor.
class GzipService : public Compressor {
 public:
  // `workers` threads, each with its own engine and stream, take batches in turn, so one
  // batch's host packing and assembly overlap another's GPU work
  GzipService(int device, int batch_us = 200, size_t max_batch = 4096, int workers = 2);
  ~GzipService() override;
  void submit(std::string body, Done done) override;
  bool can_inflate() const override { return true; }
  void submit_inflate(std::string member, uint64_t max_out, Done done) override;
  void stats(StatList* out) override;
  struct Stats {
    uint64_t batches = 0, bodies = 0, in_bytes = 0, out_bytes = 0, errors = 0;
    uint64_t inflate_batches = 0, inflated_gpu = 0, inflated_cpu = 0, inflate_errors = 0;
  };
  Stats totals();

 private:
  void loop(GpuGzip* gz);
  struct Job {
    std::string body;
    Done done;
    bool inflate = false;
    uint64_t max_out = 0;
  };
  void run_inflate(GpuGzip* gz, std::vector<Job>& batch);
  std::vector<std::unique_ptr<GpuGzip>> gz_;
  int batch_us_;
  size_t max_batch_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  bool stop_ = false;
  Stats st_;
  std::vector<std::thread> th_;
};

}  // namespace shellac
