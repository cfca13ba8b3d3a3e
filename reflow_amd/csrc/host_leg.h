// host_leg.h -- the K1 planner's host leg: a persistent pool of host threads
// (the reference's DigestLimiter pool, local/executor.go:41,522-538) that
// hashes the longest chains of a batch with SHA-NI while the GPU kernels run
// the rest.  Messages resident in HBM stream to each thread through its own
// HIP stream and a pinned double buffer (D2H of chunk c+1 overlaps the hash of
// chunk c); messages in host memory are hashed in place.  Internal header.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace rf {

// D2H chunk of one host thread (a multiple of 64: whole SHA-256 blocks);
// RF_HOST_CHUNK_MB overrides it (tuning experiments).
uint64_t host_chunk_bytes();

// Default host-leg width: min(60, the process's CPU share).  60 is the
// reference's DigestLimiter (local/executor.go:41); the share is the smaller
// of the affinity mask and the cgroup cpu.max quota, divided among the
// node's ranks (LOCAL_WORLD_SIZE, one process per GPU).  RF_HOST_THREADS
// overrides it.
unsigned host_default_threads();

class HostPool {
   public:
    // Per-thread D2H staging, created on first use: one stream per buffer,
    // waited on with hipStreamSynchronize.  Not events: hipEventRecord (and
    // hipStreamWaitEvent) put marker/barrier packets into a hardware queue,
    // and with 4 HW queues per process (GPU_MAX_HW_QUEUES) a worker stream
    // shares one with the GPU legs' streams, so the marker completes only
    // after the duo kernel queued before it -- measured: every host thread
    // stalled for the whole 1.9 s duo run (tools/d2h_probe3.hip: event waits
    // 1000 ms behind a 1 s kernel, stream syncs 29 ms for 1 GiB).
    // One per interleaved message ("lane") of a thread: a stream and two
    // buffers (chunk c+1's D2H lands in one while chunk c is hashed from the
    // other; one stream suffices because c+1 is queued only after c is
    // waited on).
    struct LaneStage {
        hipStream_t s = nullptr;
        uint8_t* buf[2] = {nullptr, nullptr};
    };
    struct Stage {
        LaneStage lane[4];
    };
    HostPool(int device, unsigned n);
    ~HostPool();
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    unsigned size() const { return n_; }
    // fn(w) once on every worker w in [0, size()); returns when all returned.
    void run(const std::function<void(unsigned)>& fn);
    // worker w's staging for `ways` lanes (call from worker w)
    hipError_t stage(unsigned w, int ways, Stage** out);

   private:
    void loop(unsigned w);
    int device_;
    unsigned n_;
    std::vector<std::thread> th_;
    std::vector<Stage> stages_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(unsigned)>* job_ = nullptr;
    uint64_t gen_ = 0;
    unsigned pending_ = 0;
    bool stop_ = false;
};

struct HostTask {
    uint32_t id;    // message id (row of the plan's out32)
    uint64_t off;   // byte offset in the arena
    uint64_t len;
};

// Messages one host thread hashes at once, interleaved (host_sha_blocks_multi):
// RF_HOST_WAYS, default 2 -- on the MI355X box two SHA-NI chains per core
// already out-run the PCIe D2H share of a thread, and fewer lanes keep the
// longest message's own chain fast (DESIGN.md §5 "K1 host leg").
int host_ways();

// out32[i] = SHA256(task i), tasks claimed in array order (callers sort them
// largest first: list scheduling in LPT order).  Exactly one of d_arena (HBM:
// chunked D2H; the caller has waited until its bytes are written) and h_arena
// (host memory) is non-null.  Returns false with *err set on a HIP failure.
bool host_leg_run(HostPool& pool, const HostTask* tasks, uint64_t n, const uint8_t* d_arena,
                  const uint8_t* h_arena, uint8_t* out32, std::string* err);

// Streaming absorb with a carry block: feeds len bytes at p into midstate st
// whose pending partial block is carry[0 .. *carry_len).
void host_sha_absorb(uint32_t st[8], uint8_t carry[64], uint32_t* carry_len, const uint8_t* p, uint64_t len);

}  // namespace rf
