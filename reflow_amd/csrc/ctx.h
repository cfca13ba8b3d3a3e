// ctx.h -- internal: the context object behind rf_ctx* and the helpers the
// C-ABI translation units share (error reporting, device/pinned buffers).
// Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>

#include "host_leg.h"
#include "host_sha.h"
#include "reflow_hip.h"

#include "errors.h"

#define HIPC(x)                                                                                  \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) return rf::fail(RF_EDEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)


// ---------------------------------------------------------------------------
// device buffers
using rf::HostPool;
using rf::host_sha_available;
using rf::host_default_threads;

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct HostBuf {  // pinned staging
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 1 << 16);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    uint8_t* bytes() const { return static_cast<uint8_t*>(p); }
};

// Scratch of the device-form calls (rf_dedup_digests_device,
// rf_bloom_collect_device), which run on the caller's stream, not under the
// context mutex's stream: one buffer per kind of call, handed between
// streams in stream order -- a call waits on its stream for the previous
// user's event and records its own after its last kernel.  (Per-call
// hipMallocAsync/hipFreeAsync blocks from the default pool were tried: on
// ROCm 7.2 a second call's table came back holding the first call's other
// array, tools/dedup_probe.py)
struct StreamScratch {
    std::mutex mu;
    DevBuf buf;
    hipEvent_t last = nullptr;  // never recorded = complete
    // with mu held: a buffer of >= bytes that stream s may use
    hipError_t acquire(size_t bytes, hipStream_t s) {
        hipError_t e = hipSuccess;
        if (!last && (e = hipEventCreateWithFlags(&last, hipEventDisableTiming)) != hipSuccess) return e;
        if (bytes > buf.cap) {
            if ((e = hipEventSynchronize(last)) != hipSuccess) return e;
            return buf.ensure(bytes);
        }
        return hipStreamWaitEvent(s, last, 0);
    }
    hipError_t release(hipStream_t s) { return hipEventRecord(last, s); }
    void destroy() {
        if (last) {
            (void)hipEventSynchronize(last);
            (void)hipEventDestroy(last);
        }
        last = nullptr;
        buf.release();
    }
};

struct rf_ctx {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    std::mutex mu;
    DevBuf d_arena, d_out, d_tmp, d_tab, d_tab2, d_tab3, d_place;
    HostBuf h_stage;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    rf_sha_plan* tplan = nullptr;  // one-shot batches (transient_plan)
    int host_threads = -1;         // K1 host leg: -1 default width, 0 none
    // created on first use; shared so a plan's host leg that runs with the
    // context mutex released keeps its pool alive across rf_set_host_threads
    std::shared_ptr<HostPool> pool;
    StreamScratch sc_dedup, sc_collect;
    // the host leg's measured feed rate (bytes/s) from HBM-resident messages:
    // the last run of a plan whose host leg took >= 1 GiB (0: none yet; the
    // planner then assumes kD2HLink), and the width it ran at
    double host_link_bps = 0.0;
    unsigned host_link_threads = 0;
};

// Host-leg width of a context (0 when the CPU has no SHA extensions).
inline unsigned ctx_host_threads(rf_ctx* ctx) {
    if (!host_sha_available()) return 0;
    return ctx->host_threads < 0 ? host_default_threads() : (unsigned)ctx->host_threads;
}

// (caller holds ctx->mu)
inline std::shared_ptr<HostPool> ctx_pool_ref(rf_ctx* ctx) {
    const unsigned n = ctx_host_threads(ctx);
    if (!n) return nullptr;
    if (ctx->pool && ctx->pool->size() != n) ctx->pool.reset();
    if (!ctx->pool) ctx->pool = std::make_shared<HostPool>(ctx->device, n);
    return ctx->pool;
}
inline HostPool* ctx_pool(rf_ctx* ctx) { return ctx_pool_ref(ctx).get(); }


// Blocking copy / memset on the context's own (non-blocking) stream, never
// the legacy null stream: a legacy-stream operation is ordered after every
// stream of the device, and HIP refuses it (hipErrorStreamCaptureImplicit)
// while another thread captures a hipGraph -- several contexts in one
// process (ranks as threads, a server's concurrent callers) must not.
inline hipError_t sync_copy(rf_ctx* c, void* dst, const void* src, size_t n, hipMemcpyKind k) {
    if (!n) return hipSuccess;
    hipError_t e = hipMemcpyAsync(dst, src, n, k, c->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(c->stream);
}
inline hipError_t sync_memset(rf_ctx* c, void* dst, int v, size_t n) {
    if (!n) return hipSuccess;
    hipError_t e = hipMemsetAsync(dst, v, n, c->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(c->stream);
}

struct DevGuard {
    explicit DevGuard(int d) { (void)hipSetDevice(d); }
};

inline hipStream_t pick(rf_ctx* ctx, void* stream) {
    return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}
