// capi.cpp -- implementation of include/reflow_hip.h (the drop-in C-ABI).
//
// Host-side runtime around the gfx950 kernels: contexts and streams, the K1
// planner (largest-first order, lane- vs wave-per-message split), the
// Fileset material builder (executor.go:214-233), the digest-DAG loader
// (levels, reverse edges, padded templates) and the bloom wire formats
// (bloom.go:264-325, bitset.go:628-721).  No CPU fallback: every digest is
// computed by a HIP kernel; a missing device or code object is RF_EDEVICE.
#include <hip/hip_runtime.h>

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "engine.h"
#include "host_leg.h"
#include "ctx.h"
#include "graph_internal.h"
#include "host_sha.h"
#include "reflow_hip.h"
#include "walk.h"
#include "wire.h"

using namespace rf;

extern "C" int rf_device_count(int* n) {
    ARG(n, "null out");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        return fail(RF_EDEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *n = c;
    return RF_OK;
}

extern "C" int rf_init(int device, rf_ctx** out) {
    ARG(out, "null out");
    *out = nullptr;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess || c == 0)
        return fail(RF_EDEVICE, "no HIP device (%s)", hipGetErrorString(e));
    if (device < 0 || device >= c) return fail(RF_EINVAL, "device %d out of range [0,%d)", device, c);
    HIPC(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPC(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RF_EDEVICE, "device %d is %s; this library is built for gfx950 only", device,
                    prop.gcnArchName);
    e = probe_kernels();
    if (e != hipSuccess)
        return fail(RF_EDEVICE, "gfx950 code object not loadable: %s", hipGetErrorString(e));
    rf_ctx* ctx = new rf_ctx();
    ctx->device = device;
    ctx->n_cu = prop.multiProcessorCount;
    e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return fail(RF_EDEVICE, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    *out = ctx;
    return RF_OK;
}

extern "C" void rf_destroy(rf_ctx* ctx) {
    if (!ctx) return;
    DevGuard g(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    ctx->d_arena.release();
    ctx->d_out.release();
    ctx->d_tmp.release();
    ctx->d_tab.release();
    ctx->d_tab2.release();
    ctx->d_tab3.release();
    ctx->d_place.release();
    ctx->h_stage.release();
    ctx->sc_dedup.destroy();
    ctx->sc_collect.destroy();
    rf_sha_plan_destroy(ctx->tplan);
    ctx->pool.reset();
    if (ctx->t0) (void)hipEventDestroy(ctx->t0);
    if (ctx->t1) (void)hipEventDestroy(ctx->t1);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

extern "C" int rf_sync(rf_ctx* ctx) {
    ARG(ctx, "null ctx");
    DevGuard g(ctx->device);
    HIPC(hipStreamSynchronize(ctx->stream));
    return RF_OK;
}

extern "C" int rf_set_host_threads(rf_ctx* ctx, int n) {
    ARG(ctx, "null ctx");
    ARG(n >= -1 && n <= 1024, "host threads must be -1 (default), 0 (none) or 1..1024");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->host_threads = n;
    ctx->pool.reset();  // a host leg running unlocked keeps its own reference
    return RF_OK;
}

extern "C" int rf_host_rate(rf_ctx* ctx, int* ways, double* thread_bytes_per_s) {
    ARG(ctx, "null ctx");
    const int w = host_ways();
    if (ways) *ways = w;
    if (thread_bytes_per_s) *thread_bytes_per_s = host_sha_rate(w);
    return RF_OK;
}

extern "C" int rf_host_info(rf_ctx* ctx, int* threads, double* core_bytes_per_s, int* sha_ext) {
    ARG(ctx, "null ctx");
    if (threads) *threads = (int)ctx_host_threads(ctx);
    if (core_bytes_per_s) *core_bytes_per_s = host_sha_rate();
    if (sha_ext) *sha_ext = host_sha_available() ? 1 : 0;
    return RF_OK;
}


// ---------------------------------------------------------------------------
// device memory / timing
extern "C" int rf_malloc(rf_ctx* ctx, uint64_t bytes, void** out) {
    ARG(ctx && out, "null argument");
    DevGuard g(ctx->device);
    *out = nullptr;
    hipError_t e = hipMalloc(out, std::max<uint64_t>(bytes, 16));
    if (e != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? RF_ENOMEM : RF_EDEVICE, "hipMalloc(%llu): %s",
                    (unsigned long long)bytes, hipGetErrorString(e));
    return RF_OK;
}

extern "C" int rf_free(rf_ctx* ctx, void* p) {
    ARG(ctx, "null ctx");
    DevGuard g(ctx->device);
    if (p) HIPC(hipFree(p));
    return RF_OK;
}

extern "C" int rf_memcpy_h2d(rf_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
    ARG(ctx && (bytes == 0 || (dst && src)), "null argument");
    DevGuard g(ctx->device);
    if (bytes) HIPC(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    return RF_OK;
}

extern "C" int rf_memcpy_d2h(rf_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
    ARG(ctx && (bytes == 0 || (dst && src)), "null argument");
    DevGuard g(ctx->device);
    if (bytes) HIPC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    return RF_OK;
}

extern "C" int rf_memset_d(rf_ctx* ctx, void* dst, int value, uint64_t bytes) {
    ARG(ctx && (bytes == 0 || dst), "null argument");
    DevGuard g(ctx->device);
    if (bytes) HIPC(hipMemsetAsync(dst, value, bytes, ctx->stream));
    return RF_OK;
}

extern "C" int rf_memcpy_d2d(rf_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
    ARG(ctx && (bytes == 0 || (dst && src)), "null argument");
    DevGuard g(ctx->device);
    if (bytes) HIPC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return RF_OK;
}

extern "C" void* rf_stream(rf_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

extern "C" int rf_timer_start(rf_ctx* ctx) {
    ARG(ctx, "null ctx");
    DevGuard g(ctx->device);
    if (!ctx->t0) HIPC(hipEventCreate(&ctx->t0));
    if (!ctx->t1) HIPC(hipEventCreate(&ctx->t1));
    HIPC(hipEventRecord(ctx->t0, ctx->stream));
    return RF_OK;
}

extern "C" int rf_timer_stop(rf_ctx* ctx, float* ms) {
    ARG(ctx && ms && ctx->t0, "timer not started");
    DevGuard g(ctx->device);
    HIPC(hipEventRecord(ctx->t1, ctx->stream));
    HIPC(hipEventSynchronize(ctx->t1));
    HIPC(hipEventElapsedTime(ms, ctx->t0, ctx->t1));
    return RF_OK;
}

// ---------------------------------------------------------------------------
// RCCL
struct rf_comm {
    rf_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    DevBuf scratch;
};

#define NCCLC(x)                                                                          \
    do {                                                                                  \
        ncclResult_t r_ = (x);                                                            \
        if (r_ != ncclSuccess) return fail(RF_EDEVICE, "%s: %s", #x, ncclGetErrorString(r_)); \
    } while (0)

extern "C" int rf_comm_unique_id(uint8_t id[128]) {
    ARG(id, "null id");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    NCCLC(ncclGetUniqueId(&u));
    memcpy(id, &u, 128);
    return RF_OK;
}

extern "C" int rf_comm_init(rf_ctx* ctx, int nranks, int rank, const uint8_t id[128], rf_comm** out) {
    ARG(ctx && id && out && nranks >= 1 && rank >= 0 && rank < nranks, "bad comm arguments");
    DevGuard g(ctx->device);
    ncclUniqueId u;
    memcpy(&u, id, 128);
    auto* c = new rf_comm();
    c->ctx = ctx;
    c->nranks = nranks;
    c->rank = rank;
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(RF_EDEVICE, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    *out = c;
    return RF_OK;
}

extern "C" void rf_comm_destroy(rf_comm* c) {
    if (!c) return;
    DevGuard g(c->ctx->device);
    c->scratch.release();
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
}

extern "C" int rf_comm_allgather(rf_comm* c, const void* d_send, void* d_recv, uint64_t bytes,
                                 void* stream) {
    ARG(c && (bytes == 0 || (d_send && d_recv)), "null argument");
    DevGuard g(c->ctx->device);
    NCCLC(ncclAllGather(d_send, d_recv, bytes, ncclUint8, c->comm, pick(c->ctx, stream)));
    return RF_OK;
}

extern "C" int rf_comm_allreduce_or(rf_comm* c, void* d_words, uint64_t nwords, void* stream) {
    ARG(c && (nwords == 0 || d_words), "null argument");
    DevGuard g(c->ctx->device);
    if (!nwords) return RF_OK;
    hipStream_t s = pick(c->ctx, stream);
    HIPC(c->scratch.ensure(8ull * nwords * c->nranks));
    NCCLC(ncclAllGather(d_words, c->scratch.p, nwords, ncclUint64, c->comm, s));
    HIPC(launch_or_reduce(c->scratch.as<uint64_t>(), nwords, c->nranks,
                          static_cast<uint64_t*>(d_words), s));
    return RF_OK;
}

// ---------------------------------------------------------------------------
// K1 planner
struct rf_sha_plan {
    rf_ctx* ctx = nullptr;
    std::mutex mu;  // one run of a plan at a time (its host leg runs without ctx->mu)
    uint64_t n = 0;
    uint32_t n_lanes = 0, n_solo = 0, n_host = 0, grid = 0, n_shards = 1;
    bool duo = true;  // wave-per-message kernel: two-lane chain (default) or one-lane
    bool pair = false;  // lane messages on k1_sha256_pair (latency-bound small sets)
    bool octo = false;  // ... or on k1_sha256_octo (eight per wave, two-lane chain)
    DevBuf d_offs, d_lens, d_order, d_heads;  // d_order = [lanes order | solo order]
    // host leg: messages hashed by the context's HostPool, largest first;
    // their digests go to HBM through h_dig -> d_dig -> scatter into out32
    std::vector<HostTask> host;
    DevBuf d_host_ids, d_host_dig;
    HostBuf h_host_dig;
    hipEvent_t e_hcopy = nullptr;
    bool hcopy_pending = false;
    float last_ms_host = 0.f;
    hipStream_t side = nullptr;
    hipEvent_t e0 = nullptr, e_solo = nullptr, e_lanes = nullptr, e1 = nullptr;
    bool ran = false;
    rf_sha_stats st{};
};

// Measured per-block chain latencies of the GPU legs:
//   duo chain            1.13 us/block (one wave per message, one per SIMD)
//   pair chain           1.9 us/block on configs[0] (lane messages <= 16 per
//                        SIMD: one pair workgroup per CU) but 31-42 s on the
//                        same 19M-block message run to run beside the duo
//                        chains of configs[1]: modelled at the lanes rate,
//                        so a lane message never sets the makespan
//   octo chain           1.3 us/block (eight messages per wave; sets of <= 4
//                        messages per SIMD, so the chain waves do not share)
//   lanes, latency-bound 3.2 us/block; throughput 64 B x 35 T lane-ops/s / 1464
// For the size-sorted messages nbs[h..n) (blocks, descending; suf = suffix
// sums) the GPU makespan of putting the k largest on duo waves is
//   M(k) = max(duo: nbs[h] x 1.13 us if k > 0,
//              lane set: max(nbs[h+k] x t_lane(n-h-k), suf[h+k] x 1464 / 35e12))
// minimised over k <= #SIMDs; ties keep the smaller k.
static double gpu_model(const std::vector<uint64_t>& nbs, const std::vector<double>& suf, uint64_t h,
                        uint32_t n_cu, uint32_t flags, uint64_t* k_out) {
    const double t_duo = 1.13e-6, t_octo = 1.3e-6, t_pair = 3.2e-6, t_lanes = 3.2e-6, blk_rate = 35e12 / 1464.0;
    const uint64_t n = nbs.size();
    *k_out = 0;
    if (h >= n) return 0.0;
    const uint64_t cnt = n - h;
    if (flags & RF_SHA_ALL_SOLO) {
        *k_out = cnt;
        return (double)nbs[h] * t_duo;
    }
    const uint64_t n_simd = 4ull * n_cu;
    const uint64_t cap = (flags & RF_SHA_NO_SOLO) ? 0 : std::min<uint64_t>(cnt, n_simd);
    const bool pair_ok = !(flags & RF_SHA_NO_PAIR), octo_ok = !(flags & RF_SHA_NO_OCTO);
    double best = 1e300;
    for (uint64_t k = 0; k <= cap; ++k) {
        const uint64_t lanes = cnt - k;
        double m = k ? (double)nbs[h] * t_duo : 0.0;
        if (lanes) {
            const double tl = (octo_ok && lanes <= 4 * n_simd)   ? t_octo
                              : (pair_ok && lanes <= 16 * n_simd) ? t_pair
                                                                  : t_lanes;
            m = std::max(m, std::max((double)nbs[h + k] * tl, suf[h + k] / blk_rate));
        }
        if (m < best * 0.98) {
            best = m;
            *k_out = k;
        }
    }
    return best;
}

// The host leg's inputs to the split: its slots (threads x interleaved
// lanes), one slot's SHA-NI rate (bytes/s: a core's measured rate with
// `ways` messages interleaved, divided among them) and, for messages resident
// in HBM, the D2H link rate every host-leg byte crosses.
struct HostModel {
    unsigned slots = 0;
    double rate = 0.0;
    double link = 0.0;  // 0: messages already in host memory
};

// Sustained D2H rate the host leg's copies reach on the MI355X box (PCIe
// Gen5 x16; tools/host_leg_probe.py all-host runs) -- the
// planner's assumption until a run measures the leg (rf_ctx::host_link_bps):
// round 5's model kept three duo chains (1,314 ms) beside a host leg that
// finished in 1,266 ms at 53.3 GB/s, because this figure and the 2 % margin
// priced moving them to the host above the chains.
static constexpr double kD2HLink = 52e9;
static constexpr uint64_t kLinkCalibBytes = 1ull << 30;  // a host leg this large calibrates the link

// The feed rate the planner prices the host leg's HBM-resident bytes at:
// the context's last measurement at the current width (a whole leg's bytes
// over its wall time: the D2H copies and the SHA-NI threads together), else
// kD2HLink.  (caller holds ctx->mu)
static double host_link_rate(const rf_ctx* ctx, unsigned threads) {
    if (ctx->host_link_bps > 0 && ctx->host_link_threads == threads)
        return std::min(std::max(ctx->host_link_bps, 0.25 * kD2HLink), 4.0 * kD2HLink);
    return kD2HLink;
}

extern "C" int rf_host_link(rf_ctx* ctx, double* bytes_per_s, int* measured) {
    ARG(ctx, "null ctx");
    std::lock_guard<std::mutex> lk(ctx->mu);
    const unsigned threads = ctx_host_threads(ctx);
    const bool m = ctx->host_link_bps > 0 && ctx->host_link_threads == threads;
    if (bytes_per_s) *bytes_per_s = host_link_rate(ctx, threads);
    if (measured) *measured = m ? 1 : 0;
    return RF_OK;
}

// Which messages go to the host leg (the h largest) and how the rest split
// over the GPU kernels.  The host leg's makespan for the h largest messages
// is list scheduling in LPT order over its slots (what the pool's shared
// largest-first queue does), each message costing len/rate plus a fixed
// 20 us (its first D2H chunk / queue hop), bounded below by the link; plus
// 100 us to wake the pool.  host(h) grows with h, gpu(h) shrinks, so
// the best h sits at their crossing; the smallest h reaching the best
// makespan (2% margin) wins, so the GPU keeps every message the host leg
// would not finish sooner.
static void plan_split(const std::vector<uint64_t>& nb, const uint64_t* lens, std::vector<uint32_t>& order,
                       uint32_t n_cu, uint32_t flags, const HostModel& hm, uint32_t* n_host_out,
                       uint32_t* n_solo_out) {
    const uint64_t n = nb.size();
    order.resize(n);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return nb[a] > nb[b]; });
    std::vector<uint64_t> nbs(n);
    std::vector<double> suf(n + 1, 0.0);
    for (uint64_t i = 0; i < n; ++i) nbs[i] = nb[order[i]];
    for (uint64_t i = n; i-- > 0;) suf[i] = suf[i + 1] + (double)nbs[i];
    uint64_t h = 0;
    const bool host_ok = hm.slots > 0 && hm.rate > 0 && !(flags & RF_SHA_NO_HOST);
    if (host_ok && (flags & RF_SHA_ALL_HOST)) {
        h = n;
    } else if (host_ok && n) {
        std::vector<double> host_t(n + 1, 0.0);
        std::vector<double> load(hm.slots, 0.0);  // min-heap of slot loads (s)
        double maxload = 0, bytes = 0;
        for (uint64_t i = 0; i < n; ++i) {
            std::pop_heap(load.begin(), load.end(), std::greater<double>());
            load.back() += (double)lens[order[i]] / hm.rate + 20e-6;
            maxload = std::max(maxload, load.back());
            std::push_heap(load.begin(), load.end(), std::greater<double>());
            bytes += (double)lens[order[i]];
            host_t[i + 1] = std::max(maxload, hm.link > 0 ? bytes / hm.link : 0.0) + 100e-6;
        }
        std::vector<double> gmemo(n + 1, -1.0);
        auto gpu_t = [&](uint64_t x) {
            if (gmemo[x] < 0) {
                uint64_t k;
                gmemo[x] = gpu_model(nbs, suf, x, n_cu, flags, &k);
            }
            return gmemo[x];
        };
        // smallest x with host_t[x] >= gpu_t(x) (true at x = n, gpu_t(n) = 0)
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (host_t[mid] >= gpu_t(mid)) hi = mid; else lo = mid + 1;
        }
        const uint64_t x0 = lo;
        double best = gpu_t(0);
        uint64_t best_h = 0;
        for (uint64_t c : {x0 > 0 ? x0 - 1 : 0, x0}) {
            const double m = std::max(host_t[c], gpu_t(c));
            if (m < best * 0.98) {
                best = m;
                best_h = c;
            }
        }
        // the smallest h with the same makespan (gpu_t is a step function
        // of h: below the crossing the host leg only adds threads' work)
        if (best_h > 0 && host_t[best_h] < gpu_t(best_h)) {
            const double target = gpu_t(best_h);
            uint64_t a = 0, b = best_h;
            while (a < b) {
                const uint64_t mid = (a + b) / 2;
                if (gpu_t(mid) <= target) b = mid; else a = mid + 1;
            }
            best_h = a;
        }
        h = best_h;
    }
    uint64_t k = 0;
    gpu_model(nbs, suf, h, n_cu, flags, &k);
    // order = [host (largest first)..., lanes..., solo...]
    std::vector<uint32_t> o2;
    o2.reserve(n);
    for (uint64_t i = 0; i < h; ++i) o2.push_back(order[i]);
    for (uint64_t i = h + k; i < n; ++i) o2.push_back(order[i]);
    for (uint64_t i = h; i < h + k; ++i) o2.push_back(order[i]);
    order.swap(o2);
    *n_host_out = (uint32_t)h;
    *n_solo_out = (uint32_t)k;
}

extern "C" void rf_sha_plan_destroy(rf_sha_plan* p);

// Fills plan p for (offs, lens): host-side split, device copies of the
// offsets/lengths/order (buffers only grow), stream and events created once.
// host_resident: the messages will be in host memory at run time (no D2H in
// the host leg's cost).
static int plan_setup(rf_ctx* ctx, rf_sha_plan* p, const uint64_t* offs, const uint64_t* lens, uint64_t n,
                      uint32_t flags, bool host_resident) {
    ARG(n == 0 || (offs && lens), "null offs/lens");
    ARG(n < 0xffffffffull, "too many messages");
    ARG(!((flags & RF_SHA_ALL_HOST) && (flags & RF_SHA_NO_HOST)), "RF_SHA_ALL_HOST with RF_SHA_NO_HOST");
    std::vector<uint64_t> nb(n);
    uint64_t total_blocks = 0, max_blocks = 0, total_bytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (offs[i] % 16) return fail(RF_EINVAL, "offs[%llu] not 16-byte aligned", (unsigned long long)i);
        nb[i] = (lens[i] + 9 + 63) / 64;
        total_blocks += nb[i];
        max_blocks = std::max(max_blocks, nb[i]);
        total_bytes += lens[i];
    }
    HostModel hm;
    const unsigned threads = (flags & RF_SHA_NO_HOST) ? 0u : ctx_host_threads(ctx);
    if ((flags & RF_SHA_ALL_HOST) && threads == 0)
        return fail(RF_EINVAL, "RF_SHA_ALL_HOST: the host leg is off (no SHA extensions, or 0 host threads)");
    const int ways = host_ways();
    hm.slots = threads * (unsigned)ways;
    hm.rate = threads ? host_sha_rate(ways) / ways : 0.0;
    hm.link = host_resident ? 0.0 : host_link_rate(ctx, threads);
    p->ctx = ctx;
    p->n = n;
    p->ran = false;
    p->st = rf_sha_stats{};
    std::vector<uint32_t> order;
    uint32_t n_solo = 0, n_host = 0;
    plan_split(nb, lens, order, (uint32_t)ctx->n_cu, flags, hm, &n_host, &n_solo);
    p->n_host = n_host;
    p->n_solo = n_solo;
    p->duo = !(flags & RF_SHA_ONE_LANE_CHAIN);
    p->n_lanes = (uint32_t)(n - n_solo - n_host);
    p->host.resize(n_host);
    for (uint32_t i = 0; i < n_host; ++i) p->host[i] = HostTask{order[i], offs[order[i]], lens[order[i]]};
    // The lanes kernel is persistent: enough 256-thread blocks for every lane
    // message, capped at 5 blocks per CU (its VGPR-limited residency).
    const uint64_t want = (p->n_lanes + sha_lanes_block() - 1) / sha_lanes_block();
    p->grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)ctx->n_cu * 5));
    p->n_shards = std::max<uint32_t>(1, std::min<uint32_t>(64, p->grid * 4));
    // Few lane messages (<= 16 per SIMD: one 64-message pair workgroup per CU)
    // are latency-bound on their wave's issue rate: split schedule and rounds
    // over two waves (k1_sha256_pair).
    p->pair = !(flags & RF_SHA_NO_PAIR) && p->n_lanes > 0 && p->n_lanes <= 16ull * 4 * ctx->n_cu;
    // Up to 4 lane messages per SIMD: eight per wave on the two-lane chain
    // (k1_sha256_octo), 8 instead of 14 chain instructions per round.
    p->octo = !(flags & RF_SHA_NO_OCTO) && p->n_lanes > 0 && p->n_lanes <= 4ull * 4 * ctx->n_cu;
    const uint64_t n_gpu = n - n_host;
    hipError_t e = hipSuccess;
    if ((e = p->d_offs.ensure(8 * std::max<uint64_t>(n, 1))) != hipSuccess ||
        (e = p->d_lens.ensure(8 * std::max<uint64_t>(n, 1))) != hipSuccess ||
        (e = p->d_order.ensure(4 * std::max<uint64_t>(n_gpu, 1))) != hipSuccess ||
        (e = p->d_heads.ensure(4 * 64)) != hipSuccess ||
        (e = p->d_host_ids.ensure(4 * std::max<uint64_t>(n_host, 1))) != hipSuccess ||
        (e = p->d_host_dig.ensure(32 * std::max<uint64_t>(n_host, 1))) != hipSuccess)
        return fail(RF_ENOMEM, "plan alloc: %s", hipGetErrorString(e));
    if (p->hcopy_pending) {  // a previous run's digest upload still reads h_host_dig
        HIPC(hipEventSynchronize(p->e_hcopy));
        p->hcopy_pending = false;
    }
    HIPC(p->h_host_dig.ensure(32 * std::max<uint64_t>(n_host, 1)));
    if (n) {
        HIPC(sync_copy(ctx, p->d_offs.p, offs, 8 * n, hipMemcpyHostToDevice));
        HIPC(sync_copy(ctx, p->d_lens.p, lens, 8 * n, hipMemcpyHostToDevice));
        if (n_gpu) HIPC(sync_copy(ctx, p->d_order.p, order.data() + n_host, 4 * n_gpu, hipMemcpyHostToDevice));
        if (n_host) HIPC(sync_copy(ctx, p->d_host_ids.p, order.data(), 4 * n_host, hipMemcpyHostToDevice));
    }
    if (!p->side) HIPC(hipStreamCreateWithFlags(&p->side, hipStreamNonBlocking));
    for (hipEvent_t* ev : {&p->e0, &p->e_solo, &p->e_lanes, &p->e1})
        if (!*ev) HIPC(hipEventCreate(ev));
    if (!p->e_hcopy) HIPC(hipEventCreateWithFlags(&p->e_hcopy, hipEventDisableTiming));
    uint64_t host_bytes = 0;
    for (const HostTask& t : p->host) host_bytes += t.len;
    p->st.n_msgs = n;
    p->st.n_solo = n_solo;
    p->st.n_host = n_host;
    p->st.host_bytes = host_bytes;
    p->st.host_threads = n_host ? threads : 0;
    p->st.total_blocks = total_blocks;
    p->st.max_blocks = max_blocks;
    p->st.total_bytes = total_bytes;
    return RF_OK;
}

static int plan_create_nolock(rf_ctx* ctx, const uint64_t* offs, const uint64_t* lens, uint64_t n,
                              uint32_t flags, rf_sha_plan** out) {
    ARG(ctx && out, "null argument");
    *out = nullptr;
    DevGuard g(ctx->device);
    auto* p = new rf_sha_plan();
    const int rc = plan_setup(ctx, p, offs, lens, n, flags, false);
    if (rc) {
        rf_sha_plan_destroy(p);
        return rc;
    }
    *out = p;
    return RF_OK;
}

// The context's own plan for one-shot batches (rf_sha256_batch/arena, the
// Fileset digests): its stream, events and device buffers are created once
// (a fresh plan costs ~4 ms of stream/event/allocation setup per call).
// The messages of these batches sit in host memory (the pinned stage).
static int transient_plan(rf_ctx* ctx, const uint64_t* offs, const uint64_t* lens, uint64_t n,
                          rf_sha_plan** out) {
    if (!ctx->tplan) ctx->tplan = new rf_sha_plan();
    *out = ctx->tplan;
    return plan_setup(ctx, ctx->tplan, offs, lens, n, 0, true);
}

extern "C" int rf_sha_plan_create(rf_ctx* ctx, const uint64_t* offs, const uint64_t* lens,
                                  uint64_t n, uint32_t flags, rf_sha_plan** out) {
    ARG(ctx, "null ctx");
    std::lock_guard<std::mutex> lk(ctx->mu);
    return plan_create_nolock(ctx, offs, lens, n, flags, out);
}

// GPU legs are queued asynchronously on s (and the plan's side stream); the
// host leg runs on the context's pool meanwhile and this call returns when
// it is done, with the upload + scatter of its digests queued on s.  The
// host leg reads h_arena (host memory) when given, else d_arena via D2H.
// ctx_lock (rf_sha_plan_run): the context mutex, released while the host leg
// hashes -- ~1.3 s on configs[1], during which other calls on the context
// (graph steps, probes, assoc) proceed; the plan's own mutex is held.
static int plan_run_locked(rf_sha_plan* p, const void* d_arena, void* d_out, hipStream_t s,
                           const uint8_t* h_arena = nullptr, std::unique_lock<std::mutex>* ctx_lock = nullptr) {
    HIPC(hipEventRecord(p->e0, s));
    const uint32_t* order = p->d_order.as<uint32_t>();
    if (p->n_lanes) HIPC(hipMemsetAsync(p->d_heads.p, 0, 4 * 64, s));
    if (p->n_solo) {
        HIPC(hipStreamWaitEvent(p->side, p->e0, 0));
        SoloArgs sa{static_cast<const uint8_t*>(d_arena), p->d_offs.as<uint64_t>(),
                    p->d_lens.as<uint64_t>(), order + p->n_lanes, p->n_solo,
                    static_cast<uint8_t*>(d_out)};
        HIPC(launch_sha_solo(sa, p->duo, p->side));
        HIPC(hipEventRecord(p->e_solo, p->side));
    }
    if (p->n_lanes && p->octo) {
        SoloArgs oa{static_cast<const uint8_t*>(d_arena), p->d_offs.as<uint64_t>(), p->d_lens.as<uint64_t>(),
                    order, p->n_lanes, static_cast<uint8_t*>(d_out)};
        HIPC(launch_sha_octo(oa, s));
    } else if (p->n_lanes && p->pair) {
        SoloArgs pa{static_cast<const uint8_t*>(d_arena), p->d_offs.as<uint64_t>(), p->d_lens.as<uint64_t>(),
                    order, p->n_lanes, static_cast<uint8_t*>(d_out)};
        HIPC(launch_sha_pair(pa, s));
    } else if (p->n_lanes) {
        LanesArgs la{static_cast<const uint8_t*>(d_arena), p->d_offs.as<uint64_t>(),
                     p->d_lens.as<uint64_t>(), order, p->n_lanes, p->n_shards,
                     p->d_heads.as<uint32_t>(), static_cast<uint8_t*>(d_out)};
        HIPC(launch_sha_lanes(la, p->grid, s));
    }
    HIPC(hipEventRecord(p->e_lanes, s));
    p->last_ms_host = 0.f;
    if (p->n_host) {
        std::shared_ptr<HostPool> pool = ctx_pool_ref(p->ctx);
        if (!pool) return fail(RF_EINVAL, "plan has a host leg but the context's host leg is off");
        if (p->hcopy_pending) {
            HIPC(hipEventSynchronize(p->e_hcopy));
            p->hcopy_pending = false;
        }
        // the arena's bytes are written once the work queued on s before e0
        // is done (a host-side wait: see HostPool::Stage on stream-side waits)
        if (!h_arena) HIPC(hipEventSynchronize(p->e0));
        const auto t0 = std::chrono::steady_clock::now();
        std::string err;
        if (ctx_lock) ctx_lock->unlock();
        const bool ok = host_leg_run(*pool, p->host.data(), p->n_host,
                                     h_arena ? nullptr : static_cast<const uint8_t*>(d_arena), h_arena,
                                     p->h_host_dig.bytes(), &err);
        if (ctx_lock) ctx_lock->lock();
        if (!ok) return fail(RF_EDEVICE, "%s", err.c_str());
        p->last_ms_host = (float)std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (!h_arena && p->st.host_bytes >= kLinkCalibBytes && p->last_ms_host > 0) {  // calibrate the link
            p->ctx->host_link_bps = (double)p->st.host_bytes / (p->last_ms_host * 1e-3);
            p->ctx->host_link_threads = (unsigned)pool->size();
        }
        HIPC(hipMemcpyAsync(p->d_host_dig.p, p->h_host_dig.p, 32ull * p->n_host, hipMemcpyHostToDevice, s));
        HIPC(hipEventRecord(p->e_hcopy, s));
        p->hcopy_pending = true;
        HIPC(launch_scatter_digests(static_cast<uint8_t*>(d_out), p->d_host_ids.as<uint32_t>(),
                                    p->d_host_dig.as<uint8_t>(), p->n_host, s));
    }
    if (p->n_solo) HIPC(hipStreamWaitEvent(s, p->e_solo, 0));
    HIPC(hipEventRecord(p->e1, s));
    p->ran = true;
    return RF_OK;
}

extern "C" int rf_sha_plan_run(rf_sha_plan* p, const void* d_arena, void* d_out32, void* stream) {
    ARG(p, "null plan");
    ARG(p->n == 0 || (d_arena && d_out32), "null device buffer");
    std::lock_guard<std::mutex> plk(p->mu);
    std::unique_lock<std::mutex> lk(p->ctx->mu);
    DevGuard g(p->ctx->device);
    return plan_run_locked(p, d_arena, d_out32, pick(p->ctx, stream), nullptr, &lk);
}

extern "C" int rf_sha_plan_stats(rf_sha_plan* p, rf_sha_stats* out) {
    ARG(p && out, "null argument");
    DevGuard g(p->ctx->device);
    if (p->ran) {
        HIPC(hipEventSynchronize(p->e1));
        float ms = 0;
        HIPC(hipEventElapsedTime(&ms, p->e0, p->e1));
        p->st.last_ms_total = ms;
        HIPC(hipEventElapsedTime(&ms, p->e0, p->e_lanes));
        p->st.last_ms_lanes = p->n_lanes ? ms : 0.f;
        if (p->n_solo) {
            HIPC(hipEventElapsedTime(&ms, p->e0, p->e_solo));
            p->st.last_ms_solo = ms;
        } else {
            p->st.last_ms_solo = 0.f;
        }
        p->st.last_ms_host = p->last_ms_host;
    }
    *out = p->st;
    return RF_OK;
}

extern "C" void rf_sha_plan_destroy(rf_sha_plan* p) {
    if (!p) return;
    if (p->ctx) {
        DevGuard g(p->ctx->device);
        if (p->side) {
            (void)hipStreamSynchronize(p->side);
            (void)hipStreamDestroy(p->side);
        }
        if (p->hcopy_pending) (void)hipEventSynchronize(p->e_hcopy);
        for (hipEvent_t ev : {p->e0, p->e_solo, p->e_lanes, p->e1, p->e_hcopy})
            if (ev) (void)hipEventDestroy(ev);
    }
    p->d_offs.release();
    p->d_lens.release();
    p->d_order.release();
    p->d_heads.release();
    p->d_host_ids.release();
    p->d_host_dig.release();
    p->h_host_dig.release();
    delete p;
}

// The packed messages already in ctx->d_arena (queued on ctx->stream): plan,
// run, download.  h_arena: the same bytes in host memory, for the host leg.
static int sha_device_packed(rf_ctx* ctx, const std::vector<uint64_t>& offs, const std::vector<uint64_t>& lens,
                             uint8_t* out32, const uint8_t* h_arena, rf_sha_plan* planned = nullptr) {
    const uint64_t n = lens.size();
    HIPC(ctx->d_out.ensure(32 * n));
    rf_sha_plan* p = planned;
    if (!p) {
        int rc = transient_plan(ctx, offs.data(), lens.data(), n, &p);
        if (rc) return rc;
    }
    int rc = plan_run_locked(p, ctx->d_arena.p, ctx->d_out.p, ctx->stream, h_arena);
    if (rc == RF_OK) {
        hipError_t e = hipMemcpyAsync(out32, ctx->d_out.p, 32 * n, hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) rc = fail(RF_EDEVICE, "sha256 batch: %s", hipGetErrorString(e));
    }
    return rc;
}

// Host-buffer batch packed in the pinned stage: plan first, upload only the
// bytes of the messages the GPU legs hash (runs of consecutive GPU messages),
// run, download.
static int sha_host_packed(rf_ctx* ctx, const std::vector<uint64_t>& offs,
                           const std::vector<uint64_t>& lens, uint64_t arena_bytes,
                           uint8_t* out32) {
    const uint64_t n = lens.size();
    HIPC(ctx->d_arena.ensure(arena_bytes + 64));
    rf_sha_plan* p = nullptr;
    int rc = transient_plan(ctx, offs.data(), lens.data(), n, &p);
    if (rc) return rc;
    if (p->n_host == 0) {
        HIPC(hipMemcpyAsync(ctx->d_arena.p, ctx->h_stage.p, arena_bytes, hipMemcpyHostToDevice, ctx->stream));
    } else if (p->n_host < n) {
        std::vector<uint8_t> on_host(n, 0);
        for (const HostTask& t : p->host) on_host[t.id] = 1;
        for (uint64_t i = 0; i < n;) {
            if (on_host[i]) {
                ++i;
                continue;
            }
            uint64_t j = i;
            while (j + 1 < n && !on_host[j + 1]) ++j;
            const uint64_t b0 = offs[i], b1 = offs[j] + lens[j];
            if (b1 > b0)
                HIPC(hipMemcpyAsync(ctx->d_arena.as<uint8_t>() + b0, ctx->h_stage.bytes() + b0, b1 - b0,
                                    hipMemcpyHostToDevice, ctx->stream));
            i = j + 1;
        }
    }
    return sha_device_packed(ctx, offs, lens, out32, ctx->h_stage.bytes(), p);
}

extern "C" int rf_sha256_batch(rf_ctx* ctx, const uint8_t* const* msgs, const uint64_t* lens,
                               uint64_t n, uint8_t* out32) {
    ARG(ctx && (n == 0 || (msgs && lens && out32)), "null argument");
    if (n == 0) return RF_OK;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard g(ctx->device);
    std::vector<uint64_t> offs(n), ls(lens, lens + n);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) {
        ARG(msgs[i] || lens[i] == 0, "null message with nonzero length");
        offs[i] = pos;
        pos += (lens[i] + 63) & ~63ull;
    }
    HIPC(ctx->h_stage.ensure(pos + 64));
    for (uint64_t i = 0; i < n; ++i)
        if (lens[i]) memcpy(ctx->h_stage.bytes() + offs[i], msgs[i], lens[i]);
    return sha_host_packed(ctx, offs, ls, pos, out32);
}

extern "C" int rf_sha256_arena(rf_ctx* ctx, const uint8_t* arena, const uint64_t* offs,
                               const uint64_t* lens, uint64_t n, uint8_t* out32) {
    ARG(ctx && (n == 0 || (arena && offs && lens && out32)), "null argument");
    if (n == 0) return RF_OK;
    std::vector<const uint8_t*> ptrs(n);
    for (uint64_t i = 0; i < n; ++i) ptrs[i] = arena + offs[i];
    return rf_sha256_batch(ctx, ptrs.data(), lens, n, out32);
}

extern "C" int rf_gen_fill(rf_ctx* ctx, void* d_arena, const uint64_t* d_offs,
                           const uint64_t* d_lens, uint64_t n, uint64_t seed, uint64_t arena_bytes,
                           void* stream) {
    ARG(ctx && d_arena && (n == 0 || (d_offs && d_lens)), "null argument");
    ARG(arena_bytes % 16 == 0, "arena_bytes must be a multiple of 16");
    DevGuard g(ctx->device);
    HIPC(launch_gen_fill(static_cast<uint8_t*>(d_arena), d_offs, d_lens, n, seed, arena_bytes,
                         pick(ctx, stream)));
    return RF_OK;
}

// ---------------------------------------------------------------------------
// Fileset digest (executor.go:205-233)
//
// Material of set s = Σ over its groups, entries sorted bytewise (sort.Strings):
// path ‖ 0x00 0x05 ‖ id, written straight into the packed host stage (sets at
// 64-B aligned offsets).  With ids32 == nullptr the ID bytes are left for the
// device (k_place_ids): *place gets (material byte, entry) per entry.
static int fileset_material(rf_ctx* ctx, uint64_t n_sets, const uint64_t* set_group, const uint64_t* group_entry,
                            const char* const* paths, const uint32_t* path_lens, const uint8_t* ids32,
                            std::vector<uint64_t>& offs, std::vector<uint64_t>& lens, uint64_t& arena_bytes,
                            std::vector<uint64_t>* place_off, std::vector<uint32_t>* place_entry) {
    const uint64_t n_groups = set_group[n_sets];
    ARG(n_groups == 0 || group_entry, "null group_entry");
    const uint64_t n_entries = n_groups ? group_entry[n_groups] : 0;
    ARG(n_entries == 0 || (paths && path_lens), "null entries");
    offs.assign(n_sets, 0);
    lens.assign(n_sets, 0);
    uint64_t pos = 0;
    for (uint64_t s = 0; s < n_sets; ++s) {
        ARG(set_group[s] <= set_group[s + 1], "set_group not monotone");
        uint64_t len = 0;
        for (uint64_t gi = set_group[s]; gi < set_group[s + 1]; ++gi) {
            ARG(group_entry[gi] <= group_entry[gi + 1], "group_entry not monotone");
            for (uint64_t e = group_entry[gi]; e < group_entry[gi + 1]; ++e) {
                ARG(paths[e] || path_lens[e] == 0, "null path");
                len += path_lens[e] + 34ull;
            }
        }
        offs[s] = pos;
        lens[s] = len;
        pos += (len + 63) & ~63ull;
    }
    arena_bytes = pos;
    HIPC(ctx->h_stage.ensure(pos + 64));
    uint8_t* out = ctx->h_stage.bytes();
    std::vector<uint32_t> idx;
    for (uint64_t s = 0; s < n_sets; ++s) {
        uint64_t w = offs[s];
        for (uint64_t gi = set_group[s]; gi < set_group[s + 1]; ++gi) {
            idx.resize(group_entry[gi + 1] - group_entry[gi]);
            std::iota(idx.begin(), idx.end(), (uint32_t)group_entry[gi]);
            std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
                const size_t la = path_lens[a], lb = path_lens[b];
                const int c = memcmp(paths[a], paths[b], std::min(la, lb));
                return c < 0 || (c == 0 && la < lb);
            });
            for (uint32_t e : idx) {
                if (path_lens[e]) memcpy(out + w, paths[e], path_lens[e]);
                w += path_lens[e];
                out[w++] = 0x00;
                out[w++] = 0x05;
                if (ids32) {
                    memcpy(out + w, ids32 + 32ull * e, 32);
                } else {
                    place_off->push_back(w);
                    place_entry->push_back(e);
                }
                w += 32;
            }
        }
    }
    return RF_OK;
}

extern "C" int rf_fileset_digest_batch(rf_ctx* ctx, uint64_t n_sets, const uint64_t* set_group,
                                       const uint64_t* group_entry, const char* const* paths,
                                       const uint32_t* path_lens, const uint8_t* ids32,
                                       uint8_t* out32) {
    ARG(ctx && set_group && out32, "null argument");
    if (n_sets == 0) return RF_OK;
    ARG(set_group[n_sets] == 0 || group_entry, "null group_entry");
    ARG(set_group[n_sets] == 0 || group_entry[set_group[n_sets]] == 0 || ids32, "null ids32");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard g(ctx->device);
    std::vector<uint64_t> offs, lens;
    uint64_t arena_bytes = 0;
    int rc = fileset_material(ctx, n_sets, set_group, group_entry, paths, path_lens, ids32, offs, lens,
                              arena_bytes, nullptr, nullptr);
    if (rc) return rc;
    return sha_host_packed(ctx, offs, lens, arena_bytes, out32);
}

extern "C" int rf_fileset_digest_device(rf_ctx* ctx, uint64_t n_sets, const uint64_t* set_group,
                                        const uint64_t* group_entry, const char* const* paths,
                                        const uint32_t* path_lens, const void* d_ids32, uint8_t* out32) {
    ARG(ctx && set_group && out32, "null argument");
    if (n_sets == 0) return RF_OK;
    ARG(set_group[n_sets] == 0 || group_entry, "null group_entry");
    ARG(set_group[n_sets] == 0 || group_entry[set_group[n_sets]] == 0 || d_ids32, "null d_ids32");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard g(ctx->device);
    std::vector<uint64_t> offs, lens, place_off;
    std::vector<uint32_t> place_entry;
    uint64_t arena_bytes = 0;
    int rc = fileset_material(ctx, n_sets, set_group, group_entry, paths, path_lens, nullptr, offs, lens,
                              arena_bytes, &place_off, &place_entry);
    if (rc) return rc;
    const uint64_t n = n_sets, np = place_off.size();
    HIPC(ctx->d_arena.ensure(arena_bytes + 64));
    HIPC(ctx->d_out.ensure(32 * n));
    HIPC(ctx->d_place.ensure(12 * np + 16));
    HIPC(hipMemcpyAsync(ctx->d_arena.p, ctx->h_stage.p, arena_bytes, hipMemcpyHostToDevice, ctx->stream));
    uint64_t* d_off = ctx->d_place.as<uint64_t>();
    uint32_t* d_ent = reinterpret_cast<uint32_t*>(d_off + np);
    HIPC(hipMemcpyAsync(d_off, place_off.data(), 8 * np, hipMemcpyHostToDevice, ctx->stream));
    HIPC(hipMemcpyAsync(d_ent, place_entry.data(), 4 * np, hipMemcpyHostToDevice, ctx->stream));
    HIPC(launch_place_ids(ctx->d_arena.as<uint8_t>(), d_off, d_ent, np, static_cast<const uint8_t*>(d_ids32),
                          ctx->stream));
    rf_sha_plan* p = nullptr;
    rc = transient_plan(ctx, offs.data(), lens.data(), n, &p);
    if (rc) return rc;
    rc = plan_run_locked(p, ctx->d_arena.p, ctx->d_out.p, ctx->stream);
    if (rc == RF_OK) {
        hipError_t e = hipMemcpyAsync(out32, ctx->d_out.p, 32 * n, hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) rc = fail(RF_EDEVICE, "fileset digest: %s", hipGetErrorString(e));
    }
    return rc;
}

// ---------------------------------------------------------------------------
// Executor.install (local/executor.go:514-557): walk a tree the way
// internal/walker/walker.go:33-99 does, digest every non-directory entry
// (repository/file/repository.go:50-63: ID = SHA256(contents)) and build
// Fileset{Map: relpath -> File{ID, Size}}.
//   * os.Stat semantics: symlinks are followed; ENOENT (e.g. a dangling link)
//     skips the entry (walker.go:40-43); any other stat/readdir error fails.
//   * directory entries sorted bytewise (readDirNames, walker.go:88-99),
//     depth-first pre-order (children prepended to the todo list, :52-55).
//   * relpath = filepath.Rel(root, path): "." for a root that is a file.
//   * Size = the Stat size (executor.go:525 takes w.Info().Size()).
// Files are read by a pool of host threads (<= 60, the DigestLimiter of
// local/executor.go:41) straight into the pinned stage, in chunks of at most
// kInstallChunk bytes, and each chunk is one K1 batch.
struct rf_install {
    std::vector<std::string> rel;
    std::vector<std::string> full;
    std::vector<int64_t> sizes;
    std::vector<uint8_t> ids;
    uint8_t fileset[32];
};

static constexpr uint64_t kInstallChunk = 8ull << 30;
static constexpr uint64_t kInstallSeg = 32ull << 20;

// Read file f (expected `want` bytes) into dst; the content must not have
// changed size since the walk's stat.
static bool install_read(const std::string& f, uint8_t* dst, uint64_t want, std::string& err) {
    const int fd = ::open(f.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
        err = "open " + f + ": " + strerror(errno);
        return false;
    }
    uint64_t got = 0;
    for (;;) {
        uint8_t probe;
        uint8_t* p = got < want ? dst + got : &probe;
        const size_t ask = got < want ? (size_t)std::min<uint64_t>(want - got, 1ull << 30) : 1;
        const ssize_t r = ::read(fd, p, ask);
        if (r < 0) {
            if (errno == EINTR) continue;
            err = "read " + f + ": " + strerror(errno);
            ::close(fd);
            return false;
        }
        if (r == 0) break;
        got += (uint64_t)r;
        if (got > want) break;
    }
    ::close(fd);
    if (got != want) {
        err = "file " + f + " changed size while it was digested";
        return false;
    }
    return true;
}

extern "C" int rf_install_dir(rf_ctx* ctx, const char* root, rf_install** out) {
    ARG(ctx && root && out, "null argument");
    *out = nullptr;
    std::unique_ptr<rf_install> in(new rf_install());
    // RF_INSTALL_TIMING=1: phase times on stderr (diagnostic)
    const bool timing = getenv("RF_INSTALL_TIMING") != nullptr;
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_begin = now();
    int rc = walk_tree(root, in->rel, in->full, in->sizes);
    if (rc) return rc;
    const double t_walk = now();
    const uint64_t n = in->rel.size();
    in->ids.assign(32 * n, 0);
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard g(ctx->device);
    for (uint64_t c0 = 0; c0 < n;) {
        // chunk [c0, c1): walk order, at most kInstallChunk bytes (or one file)
        uint64_t c1 = c0, pos = 0;
        std::vector<uint64_t> offs, lens;
        while (c1 < n) {
            const uint64_t len = (uint64_t)in->sizes[c1];
            const uint64_t alen = (len + 63) & ~63ull;
            if (c1 > c0 && pos + alen > kInstallChunk) break;
            offs.push_back(pos);
            lens.push_back(len);
            pos += alen;
            ++c1;
        }
        HIPC(ctx->h_stage.ensure(pos + 64));
        HIPC(ctx->d_arena.ensure(pos + 64));
        uint8_t* stage = ctx->h_stage.bytes();
        // segments of >= kInstallSeg bytes (consecutive files): the H2D copy of
        // a segment is queued as soon as its last file is read, overlapping
        // the reads of the next ones (files are claimed in order)
        std::vector<uint64_t> seg_first{0};
        for (uint64_t i = 0, acc = 0; i < c1 - c0; ++i) {
            acc += (lens[i] + 63) & ~63ull;
            if (acc >= kInstallSeg && i + 1 < c1 - c0) {
                seg_first.push_back(i + 1);
                acc = 0;
            }
        }
        seg_first.push_back(c1 - c0);
        const uint64_t nseg = seg_first.size() - 1;
        std::vector<uint64_t> seg_of(c1 - c0);
        std::unique_ptr<std::atomic<uint64_t>[]> left(new std::atomic<uint64_t>[nseg]);
        for (uint64_t sg = 0; sg < nseg; ++sg) {
            left[sg] = seg_first[sg + 1] - seg_first[sg];
            for (uint64_t i = seg_first[sg]; i < seg_first[sg + 1]; ++i) seg_of[i] = sg;
        }
        std::atomic<uint64_t> next{0};
        std::mutex emu;
        std::condition_variable cv;
        std::string first_err;
        auto worker = [&]() {
            for (uint64_t i; (i = next.fetch_add(1)) < c1 - c0;) {
                std::string err;
                if (!install_read(in->full[c0 + i], stage + offs[i], lens[i], err)) {
                    std::lock_guard<std::mutex> el(emu);
                    if (first_err.empty()) first_err = err;
                }
                if (left[seg_of[i]].fetch_sub(1) == 1) {
                    std::lock_guard<std::mutex> el(emu);
                    cv.notify_all();
                }
            }
        };
        const uint64_t hw = std::max(1u, std::thread::hardware_concurrency());
        const uint64_t nt = std::min<uint64_t>({60, hw, c1 - c0});
        std::vector<std::thread> pool;
        for (uint64_t t = 0; t < nt; ++t) pool.emplace_back(worker);
        hipError_t he = hipSuccess;
        for (uint64_t sg = 0; sg < nseg; ++sg) {  // this thread queues the copies, in order
            {
                std::unique_lock<std::mutex> el(emu);
                cv.wait(el, [&] { return left[sg].load() == 0; });
            }
            const uint64_t b0 = offs[seg_first[sg]];
            const uint64_t b1 = seg_first[sg + 1] < c1 - c0 ? offs[seg_first[sg + 1]] : pos;
            if (he == hipSuccess)
                he = hipMemcpyAsync(ctx->d_arena.as<uint8_t>() + b0, stage + b0, b1 - b0, hipMemcpyHostToDevice,
                                    ctx->stream);
        }
        for (auto& t : pool) t.join();
        if (timing) {
            const double tr = now();
            (void)hipStreamSynchronize(ctx->stream);
            fprintf(stderr, "[install] walk %.2f ms, reads done %.2f ms, copies done %.2f ms (%llu files, %llu threads)\n",
                    t_walk - t_begin, tr - t_begin, now() - t_begin, (unsigned long long)(c1 - c0),
                    (unsigned long long)nt);
        }
        if (!first_err.empty()) {
            (void)hipStreamSynchronize(ctx->stream);
            return fail(RF_EIO, "%s", first_err.c_str());
        }
        HIPC(he);
        rc = sha_device_packed(ctx, offs, lens, in->ids.data() + 32 * c0, ctx->h_stage.bytes());
        if (rc) return rc;
        c0 = c1;
    }
    // Fileset{Map}.Digest: one set, one group, all entries
    std::vector<const char*> paths(n);
    std::vector<uint32_t> plen(n);
    for (uint64_t i = 0; i < n; ++i) {
        paths[i] = in->rel[i].data();
        plen[i] = (uint32_t)in->rel[i].size();
    }
    const uint64_t set_group[2] = {0, 1}, group_entry[2] = {0, n};
    std::vector<uint64_t> offs, lens;
    uint64_t arena_bytes = 0;
    rc = fileset_material(ctx, 1, set_group, group_entry, paths.data(), plen.data(), in->ids.data(), offs, lens,
                          arena_bytes, nullptr, nullptr);
    if (rc) return rc;
    const double t_ids = now();
    rc = sha_host_packed(ctx, offs, lens, arena_bytes, in->fileset);
    if (rc) return rc;
    if (timing) fprintf(stderr, "[install] ids %.2f ms, fileset digest %.2f ms\n", t_ids - t_begin, now() - t_begin);
    *out = in.release();
    return RF_OK;
}

extern "C" int rf_install_info(const rf_install* in, uint64_t* n_entries, uint64_t* path_bytes,
                               uint8_t fileset_digest32[32]) {
    ARG(in, "null install");
    uint64_t pb = 0;
    for (const std::string& r : in->rel) pb += r.size();
    if (n_entries) *n_entries = in->rel.size();
    if (path_bytes) *path_bytes = pb;
    if (fileset_digest32) memcpy(fileset_digest32, in->fileset, 32);
    return RF_OK;
}

extern "C" int rf_install_entries(const rf_install* in, char* paths, uint64_t* path_offs, uint8_t* ids32,
                                  int64_t* sizes) {
    ARG(in, "null install");
    const uint64_t n = in->rel.size();
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (path_offs) path_offs[i] = w;
        if (paths && !in->rel[i].empty()) memcpy(paths + w, in->rel[i].data(), in->rel[i].size());
        w += in->rel[i].size();
    }
    if (path_offs) path_offs[n] = w;
    if (ids32 && n) memcpy(ids32, in->ids.data(), 32 * n);
    if (sizes && n) memcpy(sizes, in->sizes.data(), 8 * n);
    return RF_OK;
}

extern "C" void rf_install_destroy(rf_install* in) { delete in; }

// ---------------------------------------------------------------------------
// Fileset JSON marshal: wire.cpp (host-only)
extern "C" int rf_fileset_value_digest_batch(rf_ctx* ctx, const rf_fileset_tree* t, const uint32_t* roots,
                                             uint64_t n, uint8_t* out32) {
    ARG(ctx && (n == 0 || (roots && out32)), "null argument");
    if (n == 0) return RF_OK;
    int rc = fileset_check_tree(t);
    if (rc) return rc;
    std::string arena;
    std::vector<uint64_t> offs(n), lens(n);
    for (uint64_t i = 0; i < n; ++i) {
        offs[i] = arena.size();
        if ((rc = fileset_marshal_append(t, roots[i], arena))) return rc;
        lens[i] = arena.size() - offs[i];
    }
    return rf_sha256_arena(ctx, reinterpret_cast<const uint8_t*>(arena.data()), offs.data(), lens.data(),
                           n, out32);
}

// ---------------------------------------------------------------------------
// Digest DAG
// Device buffers of a graph of J jobs, S slots, L levels, H holes and
// tmpl_bytes of padded templates (contents not uploaded: rf_graph_load and
// rf_graph_restore fill them), the per-step state zeroed and gr->g pointed at
// them.  Caller holds ctx->mu.
int graph_device_alloc(rf_graph* gr, uint32_t J, uint32_t S, uint32_t L, uint64_t H, uint64_t tmpl_bytes) {
    rf_ctx* ctx = gr->ctx;
    GraphDev& G = gr->g;
    G.n_jobs = J;
    G.n_slots = S;
    G.n_levels = L;
    hipError_t e;
    if ((e = gr->b_meta.ensure(std::max<size_t>(32ull * J, 64))) != hipSuccess ||
        (e = gr->b_holes.ensure(std::max<size_t>(8ull * H, 64))) != hipSuccess ||  // k2 reads element 0 always
        (e = gr->b_cons_ptr.ensure(std::max<size_t>(4ull * (S + 1), 64))) != hipSuccess ||
        (e = gr->b_cons_job.ensure(std::max<size_t>(8ull * H, 64))) != hipSuccess ||
        (e = gr->b_tmpl.ensure(std::max<size_t>(tmpl_bytes, 64))) != hipSuccess ||
        (e = gr->b_slots.ensure(32ull * std::max<uint32_t>(S, 1))) != hipSuccess ||
        (e = gr->b_dirty.ensure(4ull * (J + 1))) != hipSuccess ||
        (e = gr->b_list.ensure(4ull * std::max<uint32_t>(J, 1))) != hipSuccess ||
        (e = gr->b_lmeta.ensure(32ull * std::max<uint32_t>(J, 1))) != hipSuccess ||
        (e = gr->b_counts.ensure(8ull * counts_half_words(L))) != hipSuccess ||  // two halves (plain-step parity)
        (e = gr->b_counts_last.ensure(4ull * (L + 1))) != hipSuccess ||
        (e = gr->b_lvl_start.ensure(std::max<size_t>(4ull * (L + 1), 64))) != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? RF_ENOMEM : RF_EDEVICE, "graph alloc: %s", hipGetErrorString(e));
    HIPC(sync_memset(ctx, gr->b_slots.p, 0, 32ull * std::max<uint32_t>(S, 1)));
    HIPC(sync_memset(ctx, gr->b_dirty.p, 0, 4ull * (J + 1)));
    HIPC(sync_memset(ctx, gr->b_counts.p, 0, 8ull * counts_half_words(L)));
    HIPC(sync_memset(ctx, gr->b_counts_last.p, 0, 4ull * (L + 1)));
    G.meta = gr->b_meta.as<uint4>();
    G.holes = gr->b_holes.as<uint2>();
    G.cons_ptr = gr->b_cons_ptr.as<uint32_t>();
    G.cons = gr->b_cons_job.as<uint2>();
    G.tmpl = gr->b_tmpl.as<uint8_t>();
    G.slots = gr->b_slots.as<uint8_t>();
    G.dirty = gr->b_dirty.as<uint32_t>();
    G.list = gr->b_list.as<uint32_t>();
    G.lmeta = gr->b_lmeta.as<uint4>();
    G.counts = gr->b_counts.as<uint32_t>();
    G.counts_other = G.counts + counts_half_words(L);
    G.counts_last = gr->b_counts_last.as<uint32_t>();
    gr->last_counts = G.counts_last;
    G.lvl_start_dev = gr->b_lvl_start.as<uint32_t>();
    if (!gr->e0) HIPC(hipEventCreate(&gr->e0));
    if (!gr->e1) HIPC(hipEventCreate(&gr->e1));
    return RF_OK;
}

// fn(lo, hi) over [0, n) in ranges of `grain`, on the context's host threads
// (the load's copy loops; fn must not throw)
template <class F>
static void load_parallel(rf_ctx* ctx, uint64_t n, uint64_t grain, F fn) {
    const uint64_t nr = (n + grain - 1) / grain;
    const uint64_t nt = std::min<uint64_t>(std::max(1u, ctx_host_threads(ctx)), nr);
    if (nt <= 1) {
        if (n) fn(0, n);
        return;
    }
    std::atomic<uint64_t> next{0};
    auto work = [&] {
        for (uint64_t r; (r = next.fetch_add(1)) < nr;) fn(r * grain, std::min(n, (r + 1) * grain));
    };
    std::vector<std::thread> pool;
    for (uint64_t t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
}

// Stable counting sort of idx by key[idx] in [0, nkey) -> out
static void counting_pass(const std::vector<uint32_t>& idx, const uint32_t* key, uint32_t nkey,
                          std::vector<uint32_t>& out) {
    std::vector<uint32_t> at(nkey + 1, 0);
    for (uint32_t i : idx) at[key[i] + 1]++;
    for (uint32_t k = 0; k < nkey; ++k) at[k + 1] += at[k];
    out.resize(idx.size());
    for (uint32_t i : idx) out[at[key[i]]++] = i;
}

int graph_build_plan(rf_graph* gr) {
    GraphDev& G = gr->g;
    if (!RF_SLOT_PLAN) return RF_OK;
    hipError_t e = gr->b_plan.ensure(48ull * std::max<uint32_t>(G.n_slots, 1));
    if (e != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? RF_ENOMEM : RF_EDEVICE, "graph plan: %s", hipGetErrorString(e));
    G.plan = gr->b_plan.as<uint4>();
    HIPC(launch_slot_plan(G, gr->ctx->stream));
    HIPC(hipStreamSynchronize(gr->ctx->stream));
    return RF_OK;
}

extern "C" int rf_graph_load(rf_ctx* ctx, const rf_graph_desc* d, rf_graph** out) {
    ARG(ctx && d && out, "null argument");
    *out = nullptr;
    const uint32_t J = d->n_jobs, S = d->n_slots;
    ARG(J == 0 || (d->out_slot && d->tmpl_off && d->tmpl_len && d->hole_ptr), "null job arrays");
    ARG(d->hole_ptr == nullptr || d->hole_ptr[0] == 0 || J == 0, "hole_ptr[0] must be 0");
    const uint64_t H = J ? d->hole_ptr[J] : 0;
    ARG(H == 0 || (d->hole_pos && d->hole_slot), "null hole arrays");
    ARG(H < 0xffffffffull, "too many holes");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    auto* gr = new rf_graph();
    std::unique_ptr<rf_graph, void (*)(rf_graph*)> guard(gr, [](rf_graph* x) { rf_graph_destroy(x); });
    gr->ctx = ctx;
    // RF_LOWER_TIMING=1: this load's phases on stderr (diagnostic, read per load)
    const bool timing = getenv("RF_LOWER_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!timing) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[load] %s %.3f s\n", what, std::chrono::duration<double>(now - t_last).count());
        t_last = now;
    };
    gr->producer.assign(S, -1);
    std::vector<uint32_t> nblk(J);
    for (uint32_t j = 0; j < J; ++j) {
        const uint32_t s = d->out_slot[j];
        if (s >= S) return fail(RF_EINVAL, "job %u: out_slot %u >= n_slots %u", j, s, S);
        if (gr->producer[s] >= 0) return fail(RF_EINVAL, "slot %u written by jobs %lld and %u", s,
                                              (long long)gr->producer[s], j);
        gr->producer[s] = j;
        if (d->tmpl_off[j] + d->tmpl_len[j] > d->blob_len)
            return fail(RF_EINVAL, "job %u: template outside blob", j);
        if (d->hole_ptr[j + 1] < d->hole_ptr[j]) return fail(RF_EINVAL, "hole_ptr not monotone");
        uint64_t last_end = 0;
        for (uint64_t h = d->hole_ptr[j]; h < d->hole_ptr[j + 1]; ++h) {
            if (d->hole_slot[h] >= S) return fail(RF_EINVAL, "job %u: hole slot out of range", j);
            if ((uint64_t)d->hole_pos[h] + 32 > d->tmpl_len[j])
                return fail(RF_EINVAL, "job %u: hole past template end", j);
            if (h > d->hole_ptr[j] && d->hole_pos[h] < last_end)
                return fail(RF_EINVAL, "job %u: holes unsorted or overlapping", j);
            last_end = (uint64_t)d->hole_pos[h] + 32;
        }
        nblk[j] = (uint32_t)((d->tmpl_len[j] + 9 + 63) / 64);
    }
    lap("validate");
    // topological levels (Kahn)
    std::vector<uint32_t> indeg(J, 0), level(J, 0);
    std::vector<uint64_t> cptr(S + 1, 0);  // slot -> consumer jobs (external ids)
    for (uint64_t h = 0; h < H; ++h) cptr[d->hole_slot[h] + 1]++;
    for (uint32_t s = 0; s < S; ++s) cptr[s + 1] += cptr[s];
    std::vector<uint32_t> cjob(H);
    {
        std::vector<uint64_t> fillp(cptr.begin(), cptr.end() - 1);
        for (uint32_t j = 0; j < J; ++j)
            for (uint64_t h = d->hole_ptr[j]; h < d->hole_ptr[j + 1]; ++h) {
                const uint32_t s = d->hole_slot[h];
                cjob[fillp[s]++] = j;
                if (gr->producer[s] >= 0) indeg[j]++;
            }
    }
    std::vector<uint32_t> q;
    q.reserve(J);
    // jobs given producers first (the C++ lowering's post-order, the bench
    // layouts): the levels in one forward pass, q = the given order
    bool ordered = true;
    for (uint32_t j = 0; j < J && ordered; ++j) {
        uint32_t lv = 0;
        for (uint64_t h = d->hole_ptr[j]; h < d->hole_ptr[j + 1]; ++h) {
            const int64_t p = gr->producer[d->hole_slot[h]];
            if (p < 0) continue;
            if ((uint64_t)p >= j) {
                ordered = false;
                break;
            }
            lv = std::max(lv, level[(uint32_t)p] + 1);
        }
        level[j] = lv;
    }
    if (ordered) {
        for (uint32_t j = 0; j < J; ++j) q.push_back(j);
    } else {  // Kahn
        std::fill(level.begin(), level.end(), 0u);
        for (uint32_t j = 0; j < J; ++j)
            if (!indeg[j]) q.push_back(j);
        for (size_t qi = 0; qi < q.size(); ++qi) {
            const uint32_t j = q[qi], s = d->out_slot[j];
            for (uint64_t c = cptr[s]; c < cptr[s + 1]; ++c) {
                const uint32_t k = cjob[c];
                level[k] = std::max(level[k], level[j] + 1);
                if (--indeg[k] == 0) q.push_back(k);
            }
        }
        if (q.size() != J) return fail(RF_EINVAL, "job graph has a cycle (%zu of %u jobs ordered)", q.size(), J);
    }
    uint32_t L = 0;
    for (uint32_t j = 0; j < J; ++j) L = std::max(L, level[j] + 1);
    lap("levels");
    // Fused chains (k2_level_pc): job j's fusion target is a consumer k whose
    // material has exactly one hole -- j's digest -- so k depends on nothing
    // else and can be hashed right after j, in the same lane, without being
    // queued.  Its reverse edge is moved to the end of j's consumer range.
    std::vector<int64_t> fuse(J, -1);
    std::vector<uint8_t> fused_target(J, 0);
    for (uint32_t j = 0; j < J; ++j) {
        const uint32_t s = d->out_slot[j];
        for (uint64_t c = cptr[s]; c < cptr[s + 1]; ++c) {
            const uint32_t k = cjob[c];
            if (d->hole_ptr[k + 1] - d->hole_ptr[k] == 1 && !fused_target[k]) {
                fuse[j] = k;
                fused_target[k] = 1;
                std::swap(cjob[c], cjob[cptr[s + 1] - 1]);
                break;
            }
        }
    }
    // Slot fusion: an input slot's consumer whose only hole is that slot
    // depends on nothing else, so the lane that writes the slot (k3_mark_slots,
    // k_part_apply) hashes it -- and its fusion chain -- at once instead of
    // queueing it.  At most one per slot, moved to the front of the slot's
    // range and flagged there (kSlotFused).  Jobs without holes can never be
    // queued either.  RF_K2_SLOT_FUSE=0: off (A/B).
    std::vector<uint8_t> slot_fused(J, 0);
    {
        static const bool on = RF_DIAG_KNOB("RF_K2_SLOT_FUSE", 1) != 0;
        if (on)
            for (uint32_t s = 0; s < S; ++s) {
                if (gr->producer[s] >= 0) continue;
                for (uint64_t c = cptr[s]; c < cptr[s + 1]; ++c) {
                    const uint32_t k = cjob[c];
                    if (d->hole_ptr[k + 1] - d->hole_ptr[k] == 1 && !slot_fused[k]) {
                        slot_fused[k] = 1;
                        std::swap(cjob[c], cjob[cptr[s]]);
                        break;
                    }
                }
            }
    }
    auto queueable = [&](uint32_t j) {
        return !fused_target[j] && !slot_fused[j] && d->hole_ptr[j + 1] > d->hole_ptr[j];
    };
    // Sinks (jobs nothing reads: physical cache keys, roots) may run at any
    // level after their inputs: move them to the last level that launches
    // anyway (one holding queueable non-sink jobs), where they fill their own
    // workgroups beside that level's longer chains instead of lengthening an
    // earlier level's (configs[2]: the pE1 keys, 4 blocks, left level 0's
    // 1+2-block Val -> Coerce chains waiting).
    // RF_K2_SINK_ALAP=3: the last such level whose non-sink queueable jobs
    // number at least 1/64 of the sinks (the fill level) -- a level wide
    // enough that the sinks do not wait behind a few long merge jobs (the 100M
    // layout's part roots, 15 blocks each, held its 140k pE1 keys in the
    // throughput form's lanes: 0.820 -> 0.781 ms/step; configs[2] and the
    // 8-rank piece unchanged, profiles/r03/s3/sink_fill_ab.log).  Default (2):
    // those sinks in a level of their own whose list a plain step attaches to
    // the last throughput-form launch from their inputs' level up to the fill
    // level, else to the fill level's launch (4-rank piece 0.408 -> 0.380
    // ms/step, sink_attach_ab.log).  1: the last level (A/B); 0: off.
    uint32_t sink_fill = ~0u, sink_min = 0;
    {
        static const int alap = (int)RF_DIAG_KNOB("RF_K2_SINK_ALAP", 2);
        auto sink = [&](uint32_t j) { return cptr[d->out_slot[j]] == cptr[d->out_slot[j] + 1]; };
        int64_t lq = -1;
        std::vector<uint64_t> nsq(L, 0);
        uint64_t n_sink = 0;
        for (uint32_t j = 0; j < J; ++j)
            if (queueable(j)) {
                if (!sink(j)) {
                    lq = std::max<int64_t>(lq, level[j]);
                    nsq[level[j]]++;
                } else {
                    n_sink++;
                }
            }
        if (alap >= 2)
            for (int64_t l = lq; l > 0; --l)
                if (nsq[l] * 64 >= n_sink) {
                    lq = l;
                    break;
                }
        if (alap == 2 && lq > 0) {
            // the sinks whose inputs are final by the fill level get a level of
            // their own, the last; its list runs attached to a level launch
            // (GraphDev kLvlSink, graph_enqueue)
            uint32_t smin = 0, nm = 0;
            for (uint32_t j = 0; j < J; ++j)
                if (queueable(j) && sink(j) && level[j] <= (uint32_t)lq) {
                    smin = std::max(smin, level[j]);
                    level[j] = L;
                    ++nm;
                }
            if (nm) {
                sink_fill = (uint32_t)lq;
                sink_min = smin;
                ++L;
            }
        } else if (alap && lq > 0) {
            for (uint32_t j = 0; j < J; ++j)
                if (queueable(j) && sink(j) && level[j] < (uint32_t)lq) level[j] = (uint32_t)lq;
        }
    }
    lap("fusion + sinks");
    // internal order: level ascending, blocks descending (similar lanes per wave)
    std::vector<uint32_t> perm(J);
    std::iota(perm.begin(), perm.end(), 0u);
    {
        const uint32_t maxb = J ? *std::max_element(nblk.begin(), nblk.end()) : 0;
        if (maxb < (1u << 22)) {  // two stable counting passes: blocks descending, then level
            std::vector<uint32_t> key(J), tmp;
            for (uint32_t j = 0; j < J; ++j) key[j] = maxb - nblk[j];
            counting_pass(perm, key.data(), maxb + 1, tmp);
            counting_pass(tmp, level.data(), L, perm);
        } else {
            std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) {
                return level[a] != level[b] ? level[a] < level[b] : nblk[a] > nblk[b];
            });
        }
    }
    gr->ext2int.assign(J, 0);
    for (uint32_t i = 0; i < J; ++i) gr->ext2int[perm[i]] = i;
    gr->g.lvl_start.assign(L + 1, 0);
    for (uint32_t j = 0; j < J; ++j) gr->g.lvl_start[level[j] + 1]++;
    for (uint32_t l = 0; l < L; ++l) {
        gr->max_level_jobs = std::max(gr->max_level_jobs, gr->g.lvl_start[l + 1]);
        gr->g.lvl_start[l + 1] += gr->g.lvl_start[l];
    }
    lap("order");
    // host arrays in internal order: 32-B job records, {pos, slot} holes,
    // padded templates (64-B blocks, FIPS padding pre-applied)
    std::vector<uint32_t> meta(8ull * J, 0), holes(2ull * H);
    std::vector<uint64_t> job_off(J);
    // Constant leading blocks: a job whose first hole starts in block L > 0
    // begins every hash with the same L blocks -- hashed once at load into a
    // midstate (k2_midstates); the record's template offset and block count
    // skip them and its hole positions move back by 64 L (jobs without holes
    // are hashed only by a full recompute and keep their blocks).
    std::vector<uint32_t> lead(J, 0), lead_start(J, 0);
    uint64_t n_lead = 0;
    uint64_t tb = 0;
    {
        // offsets first (a prefix pass), then the records on host threads
        std::vector<uint32_t> hoff(J);
        uint64_t hcur = 0;
        for (uint32_t i = 0; i < J; ++i) {
            const uint32_t j = perm[i];
            job_off[i] = tb;
            hoff[i] = (uint32_t)hcur;
            tb += 64ull * nblk[j];
            hcur += d->hole_ptr[j + 1] - d->hole_ptr[j];
        }
        std::atomic<uint64_t> a_lead{0}, a_blocks{0};
        std::atomic<bool> pos2{true};
        // slot-fused jobs (the mark kernels' first): all without constant
        // leading blocks and with their hole at one position -> GraphDev::sf_pos
        std::mutex sf_mu;
        bool sf_ok = true;
        uint32_t sf_at = ~0u;
        load_parallel(ctx, J, 16384, [&](uint64_t i0, uint64_t i1) {
            uint64_t nl = 0, nb = 0;
            bool p2 = true, sok = true;
            uint32_t sat = ~0u;
            for (uint64_t i = i0; i < i1; ++i) {
                const uint32_t j = perm[i];
                const uint32_t s = d->out_slot[j];
                const uint32_t ld = d->hole_ptr[j + 1] > d->hole_ptr[j]
                                        ? std::min<uint32_t>(d->hole_pos[d->hole_ptr[j]] / 64, nblk[j] - 1) : 0;
                lead[i] = ld;
                lead_start[i] = (uint32_t)(job_off[i] / 64);
                nl += ld != 0;
                uint32_t* m = &meta[8ull * i];
                uint64_t hc = hoff[i];
                m[0] = (uint32_t)(job_off[i] / 64) + ld;
                m[1] = nblk[j] - ld;
                m[2] = (uint32_t)hc;
                for (uint64_t h = d->hole_ptr[j]; h < d->hole_ptr[j + 1]; ++h, ++hc) {
                    holes[2 * hc] = d->hole_pos[h] - 64 * ld;
                    holes[2 * hc + 1] = d->hole_slot[h];
                }
                m[3] = (uint32_t)hc;
                m[4] = s;
                m[5] = (uint32_t)cptr[s];
                m[6] = (uint32_t)cptr[s + 1];
                m[7] = fuse[j] >= 0 ? gr->ext2int[(uint32_t)fuse[j]] : 0xffffffffu;
                // (cb0 = 2 and fused_hole need every one at material byte 2:
                // relative byte 2 after constant leading blocks is not enough,
                // such a target starts from a midstate)
                if (fused_target[j] && (holes[2 * m[2]] != 2 || ld != 0)) p2 = false;
                if (slot_fused[j]) {
                    if (ld != 0 || (sat != ~0u && sat != holes[2 * m[2]])) sok = false;
                    sat = holes[2 * m[2]];
                }
                nb += nblk[j] - ld;
            }
            a_lead += nl;
            a_blocks += nb;
            if (!p2) pos2 = false;
            if (!sok || sat != ~0u) {
                std::lock_guard<std::mutex> lk(sf_mu);
                if (!sok || (sf_at != ~0u && sf_at != sat)) sf_ok = false;
                sf_at = sat;
            }
        });
        gr->g.sf_pos = sf_ok ? sf_at : ~0u;
        n_lead = a_lead;
        gr->total_blocks += a_blocks;
        if (!pos2) gr->g.fuse_pos2 = false;
    }
    // levels none of whose jobs has constant leading blocks: their listed
    // jobs start from the IV without a midstate load (k2_level_lf)
    gr->g.lvl_lead0.assign(L, 1);
    for (uint32_t l = 0; l < L; ++l)
        for (uint32_t i = gr->g.lvl_start[l]; i < gr->g.lvl_start[l + 1] && gr->g.lvl_lead0[l]; ++i)
            if (lead[i]) gr->g.lvl_lead0[l] = 0;
    lap("records");
    if (tb / 64 >= 0xffffffffull) return fail(RF_EINVAL, "templates exceed 256 GiB");
    // every byte is written below (template, zero tail, padding): no zero fill
    const uint64_t tmpl_size = std::max<uint64_t>(tb, 64);
    std::unique_ptr<uint8_t[]> tmpl(new (std::nothrow) uint8_t[tmpl_size]);
    if (!tmpl) return fail(RF_ENOMEM, "graph templates: %llu bytes", (unsigned long long)tmpl_size);
    if (tb < 64) memset(tmpl.get(), 0, 64);
    load_parallel(ctx, J, 4096, [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; ++i) {
            const uint32_t j = perm[i];
            uint8_t* t = tmpl.get() + job_off[i];
            const uint64_t len = d->tmpl_len[j];
            if (len) memcpy(t, d->blob + d->tmpl_off[j], len);
            // the kernels OR digests into the holes: keep them zero
            for (uint64_t h = d->hole_ptr[j]; h < d->hole_ptr[j + 1]; ++h) memset(t + d->hole_pos[h], 0, 32);
            t[len] = 0x80;
            uint8_t* e = t + 64ull * nblk[j];
            memset(t + len + 1, 0, (size_t)(e - 8 - (t + len + 1)));
            const uint64_t bits = len * 8;
            for (int b = 0; b < 8; ++b) e[-1 - b] = (uint8_t)(bits >> (8 * b));
        }
    });
    lap("templates");
    std::vector<uint32_t> cons_ptr(S + 1), cons_job(2 * H);  // {internal job, level}
    for (uint32_t s = 0; s <= S; ++s) cons_ptr[s] = (uint32_t)cptr[s];
    for (uint64_t c = 0; c < H; ++c) {
        cons_job[2 * c] = gr->ext2int[cjob[c]];
        cons_job[2 * c + 1] = level[cjob[c]] | (slot_fused[cjob[c]] ? 0x80000000u : 0u);  // kSlotFused
    }
    gr->hole_count = H;
    // 1: the level has queueable jobs (k2_level_pc<2>); 2: they average at
    // least RF_K2_WIDE blocks (default 8; 0 = never), so the producer's
    // assembly + expansion outlasts the chain's rounds (k2_level_pc<3>)
    gr->g.inc_level.assign(L, 0);
    {
        const uint64_t wide = [] {  // read per load: tests force a mode
            const char* v = getenv("RF_K2_WIDE");
            return v ? (uint64_t)strtoull(v, nullptr, 10) : 8ull;
        }();
        // the average over the level's non-sink queueable jobs: sinks moved
        // here run in their own short workgroups, the chains set the shape
        std::vector<uint64_t> qj(L, 0), qb(L, 0), qall(L, 0);
        for (uint32_t j = 0; j < J; ++j)
            if (queueable(j)) {
                qall[level[j]] += 1;
                if (cptr[d->out_slot[j]] == cptr[d->out_slot[j] + 1]) continue;  // a sink
                qj[level[j]] += 1;
                qb[level[j]] += nblk[j];
            }
        for (uint32_t l = 0; l < L; ++l)
            if (qall[l]) gr->g.inc_level[l] = (wide && qj[l] && qb[l] >= wide * qj[l]) ? 2 : 1;
        // the octo form (k2_level_oct) for levels of few long jobs -- a merge
        // tree above the fill level: at most kOctMaxLevel queueable jobs, each
        // without a fusion target, with <= kOctMaxBlocks blocks and <=
        // kOctMaxHoles holes (its whole material staged in LDS).  RF_K2_OCT=0:
        // off (A/B)
        const bool oct_on = [] {  // (read per load, like the form thresholds)
            const char* v = getenv("RF_K2_OCT");
            return !(v && atoi(v) == 0);
        }();
        if (oct_on) {
            std::vector<uint8_t> ok(L, 1);
            for (uint32_t j = 0; j < J; ++j)  // (every job of the level: rf_graph_restore checks the same)
                if (fuse[j] >= 0 || nblk[j] > kOctMaxBlocks || d->hole_ptr[j + 1] - d->hole_ptr[j] > kOctMaxHoles)
                    ok[level[j]] = 0;
            for (uint32_t l = 0; l < L; ++l)
                if ((gr->g.inc_level[l] & kLvlForm) == 2 && ok[l] && qall[l] <= kOctMaxLevel)
                    gr->g.inc_level[l] |= kLvlOct;
        }
        if (sink_fill != ~0u) {
            gr->g.inc_level[L - 1] |= kLvlSink;
            gr->g.inc_level[sink_fill] |= kLvlFill;
            gr->g.inc_level[sink_min] |= kLvlSinkMin;
        }
    }
    gr->g.sink_attach_ok = true;
    gr->tmpl_bytes = tb;
    lap("reverse edges + forms");
    // upload
    GraphDev& G = gr->g;
    if (int rc = graph_device_alloc(gr, J, S, L, H, tmpl_size)) return rc;
    hipError_t e;
    if ((e = sync_copy(ctx, gr->b_meta.p, meta.data(), 32ull * J, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = sync_copy(ctx, gr->b_holes.p, holes.data(), 8ull * H, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = sync_copy(ctx, gr->b_cons_ptr.p, cons_ptr.data(), 4ull * (S + 1), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = sync_copy(ctx, gr->b_cons_job.p, cons_job.data(), 8ull * H, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = sync_copy(ctx, gr->b_tmpl.p, tmpl.get(), tmpl_size, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = sync_copy(ctx, gr->b_lvl_start.p, G.lvl_start.data(), 4ull * (L + 1), hipMemcpyHostToDevice)) != hipSuccess)
        return fail(RF_EDEVICE, "graph upload: %s", hipGetErrorString(e));
    tmpl.reset();
    lap("upload");
    auto up = [&](DevBuf& b, const void* src, size_t bytes) -> hipError_t {
        hipError_t e = b.ensure(std::max<size_t>(bytes, 64));
        if (e != hipSuccess) return e;
        return bytes ? sync_copy(ctx, b.p, src, bytes, hipMemcpyHostToDevice) : hipSuccess;
    };
    G.stream_handover = RF_DIAG_KNOB("RF_K2_STREAM", 0) == 1;  // (the streamed hand-over: diagnostic builds)
    graph_forms_from_env(G);
    G.n_cu = graph_ovf_cus(ctx, &G.ovf_mode);
    if (n_lead && !getenv("RF_K2_NO_MIDSTATE")) {  // (RF_K2_NO_MIDSTATE: A/B)
        struct Tmp {
            DevBuf b;
            ~Tmp() { b.release(); }
        } d_start, d_lead;
        if ((e = up(d_start.b, lead_start.data(), 4ull * J)) != hipSuccess ||
            (e = up(d_lead.b, lead.data(), 4ull * J)) != hipSuccess || (e = gr->b_mid.ensure(32ull * J)) != hipSuccess)
            return fail(e == hipErrorOutOfMemory ? RF_ENOMEM : RF_EDEVICE, "graph midstates: %s", hipGetErrorString(e));
        HIPC(launch_graph_midstates(G.tmpl, d_start.b.as<uint32_t>(), d_lead.b.as<uint32_t>(), J,
                                    gr->b_mid.as<uint4>(), ctx->stream));
        HIPC(hipStreamSynchronize(ctx->stream));
        G.mid = gr->b_mid.as<uint4>();
    } else if (n_lead) {  // A/B: keep every block, the records as if no job had a constant prefix
        G.hole_in_b0 = false;
        G.fuse_pos2 = false;  // (a target's hole may move past byte 2: fused_hole loads the records)
        G.sf_pos = ~0u;
        for (uint32_t i = 0; i < J; ++i) {
            if (!lead[i]) continue;
            meta[8ull * i] -= lead[i];
            meta[8ull * i + 1] += lead[i];
            gr->total_blocks += lead[i];
            for (uint32_t h = meta[8ull * i + 2]; h < meta[8ull * i + 3]; ++h) holes[2ull * h] += 64 * lead[i];
        }
        HIPC(sync_copy(ctx, gr->b_meta.p, meta.data(), 32ull * J, hipMemcpyHostToDevice));
        HIPC(sync_copy(ctx, gr->b_holes.p, holes.data(), 8ull * H, hipMemcpyHostToDevice));
    }
    // split block 0: every fusion target's one hole at byte 2 (fuse_pos2),
    // so its block 1 is template only
    G.split_b0 = G.hole_in_b0 && G.fuse_pos2 ? graph_split_on() : 0u;
    lap("midstates");
    if (int rc = graph_build_plan(gr)) return rc;
    if (RF_DIAG_KNOB("RF_K2_STAMPS", 0)) {  // diagnostic build: per-phase times of workgroup 0 of each level
        HIPC(gr->b_stamps.ensure(8ull * 128 * (L + 1)));  // (row L: the mark kernel's)
        HIPC(sync_memset(ctx, gr->b_stamps.p, 0, 8ull * 128 * (L + 1)));
        G.stamps = static_cast<unsigned long long*>(gr->b_stamps.p);
    }
    if (RF_DIAG_KNOB("RF_K2_WGSTAMPS", 0)) {  // diagnostic build: every incremental level kernel's workgroups
        const uint64_t bytes = 8ull * 4 * 2048 * std::max<uint32_t>(L, 1);
        HIPC(gr->b_wgst.ensure(bytes));
        HIPC(sync_memset(ctx, gr->b_wgst.p, 0, bytes));
        G.wgst = static_cast<unsigned long long*>(gr->b_wgst.p);
    }
    guard.release();
    *out = gr;
    return RF_OK;
}

extern "C" void rf_graph_destroy(rf_graph* gr) {
    if (!gr) return;
    if (gr->ctx) {
        DevGuard dg(gr->ctx->device);
        for (DevBuf* b : {&gr->b_meta, &gr->b_holes, &gr->b_cons_ptr, &gr->b_cons_job, &gr->b_tmpl,
                          &gr->b_slots, &gr->b_dirty, &gr->b_list, &gr->b_lmeta, &gr->b_counts, &gr->b_counts_last,
                          &gr->b_lvl_start, &gr->b_tmp_idx, &gr->b_tmp_dig, &gr->b_stamps, &gr->b_mid, &gr->b_wgst, &gr->b_plan})
            b->release();
        if (gr->e0) (void)hipEventDestroy(gr->e0);
        if (gr->e1) (void)hipEventDestroy(gr->e1);
        if (gr->exec_inc) (void)hipGraphExecDestroy(gr->exec_inc);
        if (gr->exec_upd) (void)hipGraphExecDestroy(gr->exec_upd);
        if (gr->graph_upd) (void)hipGraphDestroy(gr->graph_upd);
        if (gr->exec_full) (void)hipGraphExecDestroy(gr->exec_full);
        graph_part_release(gr);
    }
    delete gr;
}

static int graph_check_inputs(rf_graph* gr, const uint32_t* slots, uint32_t n) {
    // the first offending entry in index order (ranges checked on host threads
    // for large batches: an Eval's every File ID at once)
    std::atomic<uint64_t> bad{~0ull};
    load_parallel(gr->ctx, n, 1u << 20, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i)
            if (slots[i] >= gr->g.n_slots || gr->producer[slots[i]] >= 0) {
                uint64_t b = bad.load();
                while (i < b && !bad.compare_exchange_weak(b, i)) {
                }
                return;
            }
    });
    const uint64_t i = bad.load();
    if (i == ~0ull) return RF_OK;
    if (slots[i] >= gr->g.n_slots) return fail(RF_EINVAL, "slot %u out of range", slots[i]);
    return fail(RF_EINVAL, "slot %u is the output of job %lld", slots[i], (long long)gr->producer[slots[i]]);
}


extern "C" int rf_graph_set_slots(rf_graph* gr, const uint32_t* slots, const uint8_t* digests32,
                                  uint32_t n) {
    ARG(gr && (n == 0 || (slots && digests32)), "null argument");
    if (!n) return RF_OK;
    // RF_LOWER_TIMING=1: a large batch's phases on stderr (as rf_graph_load's)
    static const bool timing = getenv("RF_LOWER_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!timing || n < (1u << 20)) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[set_slots] %s %.3f s\n", what, std::chrono::duration<double>(now - t_last).count());
        t_last = now;
    };
    if (int rc = graph_check_inputs(gr, slots, n)) return rc;
    lap("validate");
    rf_ctx* ctx = gr->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    HIPC(gr->b_tmp_idx.ensure(4ull * n));
    HIPC(gr->b_tmp_dig.ensure(32ull * n));
    lap("buffers");
    HIPC(hipMemcpyAsync(gr->b_tmp_idx.p, slots, 4ull * n, hipMemcpyHostToDevice, ctx->stream));
    HIPC(hipMemcpyAsync(gr->b_tmp_dig.p, digests32, 32ull * n, hipMemcpyHostToDevice, ctx->stream));
    if (timing && n >= (1u << 20)) HIPC(hipStreamSynchronize(ctx->stream));
    lap("upload");
    if (!gr->initialized) {
        // never recomputed: the next recompute is a full one, which hashes
        // every job from the slots as they stand -- the inputs are only
        // written (an Eval's first File IDs: 20M slot-fused chains hashed and
        // their consumers queued, all of it discarded by the full pass, 0.4 s)
        HIPC(launch_scatter_digests(gr->g.slots, gr->b_tmp_idx.as<uint32_t>(), gr->b_tmp_dig.as<uint8_t>(), n,
                                    ctx->stream));
    } else {
        HIPC(launch_graph_mark_slots(gr->g, gr->b_tmp_idx.as<uint32_t>(), gr->b_tmp_dig.as<uint8_t>(), n,
                                     ctx->stream));
    }
    HIPC(hipStreamSynchronize(ctx->stream));
    lap("mark");
    gr->marked += n;
    return RF_OK;
}

extern "C" int rf_graph_set_slots_device(rf_graph* gr, const void* d_slots, const void* d_digests32,
                                         uint32_t n, void* stream) {
    ARG(gr && (n == 0 || (d_slots && d_digests32)), "null argument");
    std::lock_guard<std::mutex> lk(gr->ctx->mu);
    DevGuard dg(gr->ctx->device);
    if (!gr->initialized) {  // (as rf_graph_set_slots: the next recompute is a full one)
        HIPC(launch_scatter_digests(gr->g.slots, static_cast<const uint32_t*>(d_slots),
                                    static_cast<const uint8_t*>(d_digests32), n, pick(gr->ctx, stream)));
    } else {
        HIPC(launch_graph_mark_slots(gr->g, static_cast<const uint32_t*>(d_slots),
                                     static_cast<const uint8_t*>(d_digests32), n, pick(gr->ctx, stream)));
    }
    gr->marked += n;
    return RF_OK;
}

// A level that can receive this many chains (min(level jobs, input slots
// marked since the last step)) runs in the lane-per-job throughput form
// (k2_level_lf): from 24k for levels of short jobs (the latency form holds
// 16k chains at full speed, one 64-job workgroup per CU), from 64k for levels
// of long jobs (inc_level 2: a lane alone hashes an 18-block job at ~5 us a
// block, memory-latency-bound, against the three-wave latency form's ~1.5).
static constexpr uint64_t kThruSlots = RF_K2_THRU_DEFAULT, kThruSlotsWide = RF_K2_THRU_WIDE_DEFAULT;

// The CU count the latency form's overflow lanes size for (k2_level_pl
// ovf): the device's, or RF_K2_OVF_CU (tests: a small graph's levels
// overflow a pretended 4-CU chip); and their mode, RF_K2_OVF (0 off, 1 on,
// 2 at the chains' wave priority).  Read at load / restore.
uint32_t graph_ovf_cus(const rf_ctx* ctx, uint32_t* mode) {
    // the overflow lanes (measured slower): diagnostic builds only
    *mode = (uint32_t)std::min<long>(std::max<long>(RF_DIAG_KNOB("RF_K2_OVF", 0), 0), 2);
    const char* v = getenv("RF_K2_OVF_CU");
    return v && atoi(v) > 0 ? (uint32_t)atoi(v) : (uint32_t)ctx->n_cu;
}

// Split block 0 of the fused links (k2_level_pl cb0 = 2): RF_K2_SPLIT = 0
// off, 1 the producer expands K+W[32..63], 2 (default) K+W[16..63] (A/B;
// read at load and restore, never per step).
uint32_t graph_split_on() {
    const char* v = getenv("RF_K2_SPLIT");
    const int m = v ? atoi(v) : 2;
    return m < 0 ? 0u : m > 2 ? 2u : (uint32_t)m;
}

// The form thresholds of a graph being loaded or restored: the defaults, or
// RF_K2_THRU / RF_K2_THRU_WIDE (tests and A/B runs force either form); read
// here once, never per step (a libc call per step, and racy against setenv
// in threaded callers).  rf_graph_set_forms changes them later.
void graph_forms_from_env(GraphDev& G) {
    {
        const char* v = getenv("RF_K2_SINK_AT");
        G.sink_at = v ? (uint32_t)std::min(std::max(atoi(v), 0), 4) : 2u;
    }
    {
        const char* v = getenv("RF_K2_SPLIT_HALF");
        G.split_half = v && atoi(v) == 1 ? 1u : 0u;
        G.dbg_mark = (uint32_t)RF_DIAG_KNOB("RF_K2_DBG_MARK", 0);  // (diagnostic builds: stats wrong, digests right)
    }
    const char* tv = getenv("RF_K2_THRU");
    const char* tw = getenv("RF_K2_THRU_WIDE");
    G.cfg_thru = tv ? (uint64_t)strtoull(tv, nullptr, 10) : kThruSlots;
    G.cfg_thru_wide = tw ? (uint64_t)strtoull(tw, nullptr, 10) : tv ? G.cfg_thru : kThruSlotsWide;
    G.cfg_thru_mark = tv ? G.cfg_thru : RF_K2_THRU_MARK_DEFAULT;
}

extern "C" int rf_graph_set_forms(rf_graph* gr, uint64_t thru, uint64_t thru_wide, uint64_t thru_mark) {
    ARG(gr, "null argument");
    std::lock_guard<std::mutex> lk(gr->ctx->mu);
    gr->g.cfg_thru = thru;
    gr->g.cfg_thru_wide = thru_wide;
    gr->g.cfg_thru_mark = thru_mark;
    return RF_OK;
}

extern "C" int rf_graph_adopt_slots(rf_graph* gr, rf_graph* src) {
    ARG(gr && src && gr != src, "null argument");
    ARG(gr->ctx == src->ctx, "graphs of different contexts");
    rf_ctx* ctx = gr->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    if (gr->g.n_slots != src->g.n_slots)
        return fail(RF_EINVAL, "adopt_slots: slot tables differ: %u vs %u slots", gr->g.n_slots, src->g.n_slots);
    if (gr->marked || src->marked) return fail(RF_EPRECONDITION, "adopt_slots: a change set is pending");
    if (!src->initialized) return fail(RF_EPRECONDITION, "adopt_slots: the source graph was never recomputed");
    if (gr->g.n_slots) {
        HIPC(hipMemcpyAsync(gr->g.slots, src->g.slots, 32ull * gr->g.n_slots, hipMemcpyDeviceToDevice, ctx->stream));
        HIPC(hipStreamSynchronize(ctx->stream));
    }
    gr->initialized = true;
    return RF_OK;
}

// The launch sequence (one kernel per level + a step-end kernel) only reads
// device-side list lengths, so it is fixed for a loaded graph: capture it once
// per mode into a hipGraph and replay (kernel boundaries ~1.5 us instead of a
// host launch each; MI355X_MICROARCH "boundary" / "graph-replay-floor").  An
// incremental step leaves the dirty set empty (each hashed job clears its
// bit); a full one discards whatever set_slots queued.
// lvl_lo / lvl_hi / swap (plain incremental steps only): launch the levels in
// [lvl_lo, lvl_hi), and whether this call ends the step (swaps the cursor
// halves) -- a partitioned step may split its levels around the boundary
// exchange (recompute_rounds, GraphPart::defer_lvl)
static int graph_enqueue(rf_graph* gr, int full, hipStream_t s, bool plain = false, uint32_t lvl_lo = 0,
                         uint32_t lvl_hi = ~0u, bool swap = true) {
    GraphDev& G = gr->g;
    struct MarkedReset {  // every step consumes the change set marked before it
        rf_graph* gr;
        bool on;
        ~MarkedReset() {
            if (on) gr->marked = 0;
        }
    } marked_reset{gr, swap || full || !plain};
    bool any = false;
    for (uint32_t l = 0; l < G.n_levels; ++l) any |= (G.inc_level[l] & kLvlForm) != 0;
    if (plain && !full && any) {
        // the level-kernel forms for this step: a level that can receive at
        // least cfg_thru chains (default kThruSlots; cfg_thru_wide, default
        // kThruSlotsWide, for levels of long jobs) fills the chip, and the
        // lane-per-job form (k2_level_lf) outruns the two-lane latency form
        // (k2_level_pl) there -- DESIGN.md §5
        G.step_marked = gr->marked;
        G.thru_slots = G.cfg_thru;
        G.thru_slots_wide = G.cfg_thru_wide;
        // the sink level's list rides on the launch of the last level from
        // kLvlSinkMin to kLvlFill that runs in the throughput form (the short
        // sink jobs fill SIMDs its waves leave idle; the latency form is a
        // poor fit for them), else on the fill level's (GraphDev kLvlSink).  The choice depends only on the
        // step's forms, so the calls of a deferred partitioned step agree.
        uint32_t sink = ~0u, attach = ~0u;
        {
            uint32_t fill = ~0u, smin = 0;
            for (uint32_t l = 0; l < G.n_levels; ++l) {
                if (G.inc_level[l] & kLvlSink) sink = l;
                if (G.inc_level[l] & kLvlFill) fill = l;
                if (G.inc_level[l] & kLvlSinkMin) smin = l;
            }
            if (sink != ~0u && fill != ~0u && G.sink_attach_ok) {
                // (sink_at 4: the level above the fill level first, A/B)
                if (G.sink_at == 4) {
                    uint32_t most = 0;
                    for (uint32_t l = fill + 1; l < sink; ++l)
                        if ((G.inc_level[l] & kLvlForm) && G.lvl_start[l + 1] - G.lvl_start[l] > most) {
                            most = G.lvl_start[l + 1] - G.lvl_start[l];
                            attach = l;
                        }
                }
                for (uint32_t l = fill + 1; l-- > smin && attach == ~0u;)
                    if ((G.inc_level[l] & kLvlForm) && graph_level_lf(G, l)) attach = l;
                // no throughput-form level to fill: a level above the fill
                // level (a merge tree: few long jobs on a nearly idle chip)
                // rather than the fill level itself, whose latency-form chains
                // the sinks' workgroups would share CUs with (the 8-rank
                // piece's OpK level: 67 us, its chains alone ~50) -- the one
                // with the most jobs, so the sinks run beside its longest
                // stretch of work (octo-form levels take the list in
                // workgroups of their own).  GraphDev::sink_at (RF_K2_SINK_AT,
                // read at load): 0 = the fill level, 1 = the last latency-form
                // level above it, 3 = above the fill level without the
                // spare-CU rule below (A/B and tests), 2 = all of these
                const uint32_t sink_at = G.sink_at;
                // else an earlier latency-form level (from smin) whose chains
                // leave CUs free -- its workgroups estimated from the step's
                // marked slots (a bound on the chains reaching it): the sinks
                // run there one per lane at the lowest priority (k2_level_pl
                // sink lanes) and the fill level's chains keep their CUs
                // (configs[2]: the Exec level, 220 workgroups on 256 CUs)
                if (attach == ~0u && sink_at == 2)
                    for (uint32_t l = smin; l <= fill && attach == ~0u; ++l)
                        if ((G.inc_level[l] & kLvlForm) && !(G.inc_level[l] & kLvlOct) && !graph_level_lf(G, l)) {
                            const uint64_t jobs = std::min<uint64_t>(G.lvl_start[l + 1] - G.lvl_start[l], G.step_marked);
                            if ((jobs + 63) / 64 + 16 <= gr->ctx->n_cu) attach = l;
                        }
                if (attach == ~0u && sink_at == 1)
                    for (uint32_t l = sink; l-- > fill + 1 && attach == ~0u;)
                        if ((G.inc_level[l] & kLvlForm) && !(G.inc_level[l] & kLvlOct)) attach = l;
                if (attach == ~0u && (sink_at == 2 || sink_at == 3)) {
                    uint32_t most = 0;
                    for (uint32_t l = fill + 1; l < sink; ++l)
                        if ((G.inc_level[l] & kLvlForm) && G.lvl_start[l + 1] - G.lvl_start[l] > most) {
                            most = G.lvl_start[l + 1] - G.lvl_start[l];
                            attach = l;
                        }
                }
                if (attach == ~0u) attach = fill;
            }
        }
        // the first launched level zeroes the previous step's half; the next
        // step (and set_slots / imports before it) uses that half
        bool first = true;
        if (lvl_lo == 0) G.last_levels_lf = G.last_levels_oct = G.last_levels_half = 0;
        G.last_sink_attach = attach;
        for (uint32_t l = lvl_lo; l < std::min(lvl_hi, G.n_levels); ++l) {
            if (!(G.inc_level[l] & kLvlForm) || (l == sink && attach != ~0u)) continue;
            HIPC(launch_graph_level(G, l, 0, s, first ? G.counts_other : nullptr, l == attach ? sink : ~0u));
            G.last_levels_lf += graph_level_lf(G, l) ? 1u : 0u;
            G.last_levels_oct += (G.inc_level[l] & kLvlOct) ? 1u : 0u;  // (RF_K2_CHAIN=14 aside)
            G.last_levels_half += graph_level_half(G, l) ? 1u : 0u;
            first = false;
        }
        gr->last_counts = G.counts;
        if (swap) std::swap(G.counts, G.counts_other);
        return RF_OK;
    }
    // captured sequences: the latency form, 64-job workgroups (no per-step
    // choice may be frozen into a graph from the last plain step's change set)
    G.thru_slots = G.thru_slots_wide = ~0ull;
    G.step_marked = 0;
    for (uint32_t l = 0; l < G.n_levels; ++l) HIPC(launch_graph_level(G, l, full, s));
    HIPC(launch_graph_step_end(G, full, s));
    gr->last_counts = G.counts_last;
    if (full) {
        HIPC(hipMemsetAsync(G.dirty, 0, 4ull * (G.n_jobs + 1), s));
        HIPC(hipMemsetAsync(G.counts_other, 0, 4ull * counts_half_words(G.n_levels), s));  // both halves clear
    }
    return RF_OK;
}

static int graph_capture(rf_graph* gr, int full, hipGraphExec_t* out) {
    hipStream_t cs = nullptr;
    HIPC(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t graph = nullptr;
    int rc = RF_OK;
    hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
        rc = graph_enqueue(gr, full, cs);
        e = hipStreamEndCapture(cs, &graph);
    }
    if (e == hipSuccess && rc == RF_OK) e = hipGraphInstantiate(out, graph, nullptr, nullptr, 0);
    if (graph) (void)hipGraphDestroy(graph);
    (void)hipStreamDestroy(cs);
    if (rc != RF_OK) return rc;
    if (e != hipSuccess) return fail(RF_EDEVICE, "graph capture: %s", hipGetErrorString(e));
    return RF_OK;
}

// An incremental step launches only its few queueable levels (configs[2]:
// two level kernels): queued back to back as plain launches they start
// sooner than as a replayed hipGraph (same-box A/B: 0.1827 -> 0.1752 ms per
// step), and with the cursor halves alternating (GraphDev::counts_other) no
// step-end kernel is needed.  The full recompute (every level) keeps its
// graph.  RF_K2_GRAPH=1: the incremental graph (A/B).
// RF_K2_EVENTS=1: record the timing events on asynchronous recomputes too
static bool events_always() {
    static const bool on = RF_DIAG_KNOB("RF_K2_EVENTS", 0) == 1;
    return on;
}

static bool inc_plain() {
    static const bool on = RF_DIAG_KNOB("RF_K2_GRAPH", 0) != 1;
    return on;
}

bool graph_plain_steps() { return inc_plain(); }

int graph_recompute_locked(rf_graph* gr, int full, hipStream_t s, uint32_t lvl_lo, uint32_t lvl_hi, bool swap) {
    if (!gr->initialized) full = 1;
    const bool no_graph = inc_plain();
    static const bool full_plain = RF_DIAG_KNOB("RF_K2_FULL_GRAPH", 1) == 0;  // (A/B: the full recompute as plain launches)
    if ((no_graph && !full) || (full_plain && full)) {
        // the timing events (rf_graph_stats.last_ms) only where a caller waits
        // anyway: each event record put a ~6 us bubble on either side of the
        // step's level launches (rocprofv3 trace)
        const bool ev = gr->time_next || events_always();
        if (ev) HIPC(hipEventRecord(gr->e0, s));
        if (int rc = graph_enqueue(gr, full, s, true, lvl_lo, lvl_hi, swap)) return rc;
        if (ev) HIPC(hipEventRecord(gr->e1, s));
        gr->timed = ev;
        gr->initialized = true;
        return RF_OK;
    }
    hipGraphExec_t& ex = full ? gr->exec_full : gr->exec_inc;
    if (!ex && gr->g.n_levels)
        if (int rc = graph_capture(gr, full, &ex)) return rc;
    gr->marked = 0;
    HIPC(hipEventRecord(gr->e0, s));
    if (ex) HIPC(hipGraphLaunch(ex, s));
    gr->last_counts = gr->g.counts_last;
    HIPC(hipEventRecord(gr->e1, s));
    gr->timed = true;
    gr->initialized = true;
    return RF_OK;
}

// Mark + incremental levels as ONE graph launch: the mark kernel is the
// graph's first node and only its parameters change between calls
// (hipGraphExecKernelNodeSetParams, host side), so a step is one launch --
// no separate mark launch and no gap before the first level.
static int graph_capture_upd(rf_graph* gr, const MarkArgs& ma, const hipKernelNodeParams& mp) {
    hipStream_t cs = nullptr;
    HIPC(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t graph = nullptr;
    int rc = RF_OK;
    hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
        e = hipLaunchKernel(mp.func, mp.gridDim, mp.blockDim, mp.kernelParams, 0, cs);
        if (e == hipSuccess) rc = graph_enqueue(gr, 0, cs);
        const hipError_t e2 = hipStreamEndCapture(cs, &graph);
        if (e == hipSuccess) e = e2;
    }
    (void)ma;
    if (e == hipSuccess && rc == RF_OK) {  // the mark node: the kernel node running k3_mark_slots
        size_t nn = 0;
        e = hipGraphGetNodes(graph, nullptr, &nn);
        std::vector<hipGraphNode_t> nodes(nn);
        if (e == hipSuccess && nn) e = hipGraphGetNodes(graph, nodes.data(), &nn);
        for (size_t i = 0; e == hipSuccess && i < nn && !gr->upd_mark; ++i) {
            hipGraphNodeType t;
            if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
            hipKernelNodeParams kp{};
            if (hipGraphKernelNodeGetParams(nodes[i], &kp) == hipSuccess && kp.func == graph_mark_kernel())
                gr->upd_mark = nodes[i];
        }
        if (e == hipSuccess && !gr->upd_mark) e = hipErrorNotFound;
        if (e == hipSuccess) e = hipGraphInstantiate(&gr->exec_upd, graph, nullptr, nullptr, 0);
    }
    (void)hipStreamDestroy(cs);
    if (rc != RF_OK || e != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        gr->upd_mark = nullptr;
        gr->exec_upd = nullptr;
        return rc != RF_OK ? rc : fail(RF_EDEVICE, "update graph capture: %s", hipGetErrorString(e));
    }
    gr->graph_upd = graph;
    return RF_OK;
}

extern "C" int rf_graph_update_recompute_async(rf_graph* gr, const void* d_slots, const void* d_digests32,
                                               uint32_t n, void* stream) {
    ARG(gr && (n == 0 || (d_slots && d_digests32)), "null argument");
    std::lock_guard<std::mutex> lk(gr->ctx->mu);
    DevGuard dg(gr->ctx->device);
    hipStream_t s = pick(gr->ctx, stream);
    if (!gr->initialized || inc_plain()) {  // mark, then the level launches (first call: the full sequence)
        HIPC(launch_graph_mark_slots(gr->g, static_cast<const uint32_t*>(d_slots),
                                     static_cast<const uint8_t*>(d_digests32), n, s));
        gr->marked += n;
        return graph_recompute_locked(gr, gr->initialized ? 0 : 1, s);
    }
    MarkArgs ma;
    hipKernelNodeParams mp{};
    graph_mark_params(gr->g, static_cast<const uint32_t*>(d_slots), static_cast<const uint8_t*>(d_digests32), n,
                      &ma, &mp);
    if (!gr->exec_upd) {
        if (int rc = graph_capture_upd(gr, ma, mp)) return rc;
    } else {
        HIPC(hipGraphExecKernelNodeSetParams(gr->exec_upd, gr->upd_mark, &mp));
    }
    HIPC(hipEventRecord(gr->e0, s));
    HIPC(hipGraphLaunch(gr->exec_upd, s));
    HIPC(hipEventRecord(gr->e1, s));
    gr->timed = true;
    return RF_OK;
}

// The last step's jobs per level, [L] the jobs hashed inside fused chains
// (a plain step's cursor half: its fused parts folded in; k3_step_end has
// already folded them into counts_last).  Synchronizes s.
int graph_read_counts(rf_graph* gr, hipStream_t s, std::vector<uint32_t>& counts) {
    const uint32_t L = gr->g.n_levels;
    const bool half = gr->last_counts != gr->g.counts_last;
    std::vector<uint32_t> raw(half ? counts_half_words(L) : L + 1, 0);
    if (L) HIPC(hipMemcpyAsync(raw.data(), gr->last_counts, 4ull * raw.size(), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (L && half) {
        for (uint32_t k = 0; k < kFusedParts; ++k) raw[L] += raw[L + 1 + kPartStride * k];
        for (uint32_t l = 0; l < L; ++l)  // the levels' list runs (engine.h kListShards)
            for (uint32_t k = 0; k < kListShards; ++k) raw[l] += raw[list_shard_off(L) + k * cursor_lp(L) + l];
    }
    raw.resize(L + 1);
    counts.swap(raw);
    return RF_OK;
}

extern "C" int rf_graph_recompute_async(rf_graph* gr, int full, void* stream) {
    ARG(gr, "null graph");
    std::lock_guard<std::mutex> lk(gr->ctx->mu);
    DevGuard dg(gr->ctx->device);
    return graph_recompute_locked(gr, full, pick(gr->ctx, stream));
}

// RF_K2_WGSTAMPS=1 diagnostic: per launched level, the workgroups that took
// jobs -- how many, their durations (min / median / max), how late the last
// one started, and how many shared a CU with another working workgroup (and
// their mean duration against the ones alone) -- then the records are cleared.
static void wgst_report(rf_graph* gr) {
    const GraphDev& G = gr->g;
    std::vector<unsigned long long> w(4ull * 2048 * G.n_levels);
    if (sync_copy(gr->ctx, w.data(), G.wgst, 8 * w.size(), hipMemcpyDeviceToHost) != hipSuccess) return;
    unsigned long long step0 = ~0ull;  // the step's first workgroup start, any level
    for (size_t i = 0; i < w.size(); i += 4)
        if (w[i + 1]) step0 = std::min(step0, w[i]);
    for (uint32_t l = 0; l < G.n_levels; ++l) {
        const unsigned long long* r = &w[4ull * 2048 * l];
        // every workgroup of the launch (working or not): its first start and
        // last end on the step's clock
        unsigned long long a0 = ~0ull, a1 = 0;
        uint32_t nall = 0;
        for (uint32_t i = 0; i < 2048; ++i)
            if (r[4 * i + 1]) {
                a0 = std::min(a0, r[4 * i]);
                a1 = std::max(a1, r[4 * i + 1]);
                ++nall;
            }
        std::vector<uint32_t> act;
        unsigned long long t0 = ~0ull;
        for (uint32_t i = 0; i < 2048; ++i)
            if (r[4 * i + 1] && r[4 * i + 3]) {
                act.push_back(i);
                t0 = std::min(t0, r[4 * i]);
            }
        if (act.empty()) continue;
        std::map<unsigned long long, std::vector<uint32_t>> cu;  // xcc | se/sh/cu -> workgroups
        std::vector<double> dur;
        double late = 0;
        for (uint32_t i : act) {
            const unsigned long long hw = r[4 * i + 2];
            cu[((hw >> 32) << 8) | ((hw >> 8) & 0xff)].push_back(i);
            dur.push_back((r[4 * i + 1] - r[4 * i]) * 0.01);
            late = std::max(late, (r[4 * i] - t0) * 0.01);
        }
        std::vector<double> ds = dur;
        std::sort(ds.begin(), ds.end());
        // start-time spread: workgroups starting more than 5 / 20 / 50 us
        // after the first (a launch wider than the resident set waits)
        uint32_t l5 = 0, l20 = 0, l50 = 0, maxcu = 0;
        for (uint32_t i : act) {
            const double st = (r[4 * i] - t0) * 0.01;
            l5 += st > 5, l20 += st > 20, l50 += st > 50;
        }
        for (auto& kv : cu) maxcu = std::max<uint32_t>(maxcu, (uint32_t)kv.second.size());
        fprintf(stderr, "[wgstamps] level %u: started >5us late %u, >20us %u, >50us %u; most workgroups on one CU %u\n",
                l, l5, l20, l50, maxcu);
        double sh = 0, al = 0;
        uint32_t nsh = 0, nal = 0, cus_shared = 0;
        for (auto& kv : cu) {
            if (kv.second.size() > 1) ++cus_shared;
            for (uint32_t i : kv.second) {
                const double d = (r[4 * i + 1] - r[4 * i]) * 0.01;
                if (kv.second.size() > 1) sh += d, ++nsh;
                else al += d, ++nal;
            }
        }
        fprintf(stderr,
                "[wgstamps] level %u: launch %u workgroups, first start %.1f, last end %.1f us into the step; "
                "%zu working on %zu CUs (%u CUs shared); us min %.1f median %.1f max %.1f; last start +%.1f; "
                "mean alone %.1f (%u), shared %.1f (%u)\n",
                l, nall, (a0 - step0) * 0.01, (a1 - step0) * 0.01, act.size(), cu.size(), cus_shared, ds.front(),
                ds[ds.size() / 2], ds.back(), late, nal ? al / nal : 0.0, nal, nsh ? sh / nsh : 0.0, nsh);
    }
    (void)sync_memset(gr->ctx, G.wgst, 0, 8 * w.size());
}

extern "C" int rf_graph_recompute(rf_graph* gr, int full, uint64_t* out_recomputed) {
    ARG(gr, "null graph");
    rf_ctx* ctx = gr->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    gr->time_next = true;
    const int rc0 = graph_recompute_locked(gr, full, ctx->stream);
    gr->time_next = false;
    if (rc0) return rc0;
    std::vector<uint32_t> counts;
    if (int rc = graph_read_counts(gr, ctx->stream, counts)) return rc;
    uint64_t tot = 0;
    for (uint32_t l = 0; l <= gr->g.n_levels; ++l) tot += counts[l];
    if (gr->g.wgst && !full) wgst_report(gr);
    if (gr->g.stamps && !full) {  // diagnostic print: per level, chain wave then producer wave
        std::vector<unsigned long long> st(128ull * gr->g.n_levels);
        HIPC(sync_copy(ctx, st.data(), gr->g.stamps, 8 * st.size(), hipMemcpyDeviceToHost));
        fprintf(stderr, "[counts] jobs per level:");
        for (uint32_t l = 0; l <= gr->g.n_levels; ++l) fprintf(stderr, " %u", counts[l]);
        fprintf(stderr, " (last: fused)\n");
        for (uint32_t l = 0; l < gr->g.n_levels; ++l)
            for (int w = 0; w < 2; ++w) {
                const unsigned long long* x = &st[128ull * l + 64 * w];
                if (!x[0]) continue;
                fprintf(stderr, "[stamps] level %u wave %d:", l, w);
                for (int k = 1; k < 64 && x[k]; ++k) fprintf(stderr, " %.2f", (x[k] - x[k - 1]) * 0.01);
                fprintf(stderr, " (us)\n");
            }
        // the mark kernel's workgroups 0..31: start (from the first), then the
        // lanes' latest time at each phase end (MarkStamp)
        std::vector<unsigned long long> mk(128);
        HIPC(sync_copy(ctx, mk.data(), gr->g.stamps + 128ull * gr->g.n_levels, 8 * mk.size(), hipMemcpyDeviceToHost));
        unsigned long long m0 = ~0ull;
        for (int b = 0; b < 32; ++b)
            if (mk[4 * b + 3]) m0 = std::min(m0, mk[4 * b]);
        for (int b = 0; b < 32; ++b) {
            const unsigned long long* x = &mk[4 * b];
            if (!x[3]) continue;
            fprintf(stderr, "[mark stamps] wg %d: start +%.2f, slot loaded %.2f, chain %.2f, appends %.2f, drained %.2f us\n",
                    b, (x[0] - m0) * 0.01, (uint32_t)x[1] * 0.01, (uint32_t)(x[1] >> 32) * 0.01,
                    (uint32_t)x[2] * 0.01, (uint32_t)(x[2] >> 32) * 0.01);
        }
        (void)sync_memset(ctx, gr->g.stamps + 128ull * gr->g.n_levels, 0, 8 * mk.size());
    }
    gr->last_recomputed = tot;
    if (out_recomputed) *out_recomputed = tot;
    return RF_OK;
}

extern "C" int rf_graph_get_slots(rf_graph* gr, const uint32_t* slots, uint32_t n, uint8_t* out32) {
    ARG(gr && (n == 0 || (slots && out32)), "null argument");
    if (!n) return RF_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (slots[i] >= gr->g.n_slots) return fail(RF_EINVAL, "slot %u out of range", slots[i]);
    rf_ctx* ctx = gr->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    HIPC(gr->b_tmp_idx.ensure(4ull * n));
    HIPC(gr->b_tmp_dig.ensure(32ull * n));
    HIPC(hipMemcpyAsync(gr->b_tmp_idx.p, slots, 4ull * n, hipMemcpyHostToDevice, ctx->stream));
    HIPC(launch_gather_slots(gr->g.slots, gr->b_tmp_idx.as<uint32_t>(), n, gr->b_tmp_dig.as<uint8_t>(),
                             ctx->stream));
    HIPC(hipMemcpyAsync(out32, gr->b_tmp_dig.p, 32ull * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    return RF_OK;
}

extern "C" int rf_graph_gather_device(rf_graph* gr, const void* d_slots, uint32_t n, void* d_out32,
                                      void* stream) {
    ARG(gr && (n == 0 || (d_slots && d_out32)), "null argument");
    DevGuard dg(gr->ctx->device);
    HIPC(launch_gather_slots(gr->g.slots, static_cast<const uint32_t*>(d_slots), n,
                             static_cast<uint8_t*>(d_out32), pick(gr->ctx, stream)));
    return RF_OK;
}

extern "C" int rf_graph_stats_get(rf_graph* gr, rf_graph_stats* out) {
    ARG(gr && out, "null argument");
    std::lock_guard<std::mutex> lk(gr->ctx->mu);
    DevGuard dg(gr->ctx->device);
    *out = rf_graph_stats{};
    out->n_jobs = gr->g.n_jobs;
    out->n_slots = gr->g.n_slots;
    out->n_levels = gr->g.n_levels;
    out->max_level_jobs = gr->max_level_jobs;
    out->total_blocks = gr->total_blocks;
    out->hole_count = gr->hole_count;
    out->template_bytes = gr->tmpl_bytes;
    out->last_recomputed = gr->last_recomputed;
    out->last_levels_lf = gr->g.last_levels_lf;
    out->last_mark_lf = gr->g.last_mark_lf;
    out->last_levels_oct = gr->g.last_levels_oct;
    out->split_block0 = gr->g.split_b0;
    out->last_sink_attach = gr->g.last_sink_attach;
    out->last_levels_half = gr->g.last_levels_half;
    if (gr->timed) {
        HIPC(hipEventSynchronize(gr->e1));
        HIPC(hipEventElapsedTime(&out->last_ms, gr->e0, gr->e1));
    }
    return RF_OK;
}

// ---------------------------------------------------------------------------
// Bloom filter
struct rf_bloom {
    rf_ctx* ctx = nullptr;
    BloomDev b;
    DevBuf words, len_dev, keys, out, sizes, dead, tiles, idx, nb;
};

static int bloom_make(rf_ctx* ctx, uint64_t m, uint64_t k, const uint64_t* words, uint64_t nwords,
                      uint64_t length, rf_bloom** out) {
    ARG(ctx && out, "null argument");
    ARG(m >= 1, "bloom m must be >= 1 (location() divides by m)");
    ARG(k < (1ull << 31), "bloom k too large");
    // bitset words needed for `length` bits (bitset.go:89-94), without wrapping
    const uint64_t need = length / 64 + (length % 64 != 0);
    ARG(!words || nwords >= need, "fewer words than the bitset length needs");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    auto* bl = new rf_bloom();
    bl->ctx = ctx;
    // capacity: enough words for any location < m (Add may grow length to m)
    const uint64_t cap = std::max<uint64_t>(std::max(std::max(nwords, need), (m + 63) / 64), 1);
    hipError_t e;
    if ((e = bl->words.ensure(8 * cap)) != hipSuccess || (e = bl->len_dev.ensure(8)) != hipSuccess) {
        delete bl;
        return fail(RF_ENOMEM, "bloom alloc: %s", hipGetErrorString(e));
    }
    HIPC(sync_memset(ctx, bl->words.p, 0, 8 * cap));
    // the bitset holds exactly wordsNeeded(length) words (bitset.go:89-94,
    // ReadFrom); words past them stay zero, as extendSetMaybe exposes them
    if (need && words) HIPC(sync_copy(ctx, bl->words.p, words, 8 * need, hipMemcpyHostToDevice));
    HIPC(sync_copy(ctx, bl->len_dev.p, &length, 8, hipMemcpyHostToDevice));
    bl->b.m = m;
    bl->b.k = k;
    bl->b.length = length;
    bl->b.nwords = cap;
    bl->b.words = bl->words.as<uint64_t>();
    bl->b.len_dev = bl->len_dev.as<uint64_t>();
    *out = bl;
    return RF_OK;
}

extern "C" int rf_bloom_load(rf_ctx* ctx, uint64_t m, uint64_t k, const uint64_t* words,
                             uint64_t nwords, uint64_t length, rf_bloom** out) {
    return bloom_make(ctx, m, k, words, nwords, length, out);
}

extern "C" int rf_bloom_new(rf_ctx* ctx, uint64_t m, uint64_t k, rf_bloom** out) {
    // bloom.New: max(1,m), max(1,k), bitset.New(m) (length = m as given)
    return bloom_make(ctx, std::max<uint64_t>(1, m), std::max<uint64_t>(1, k), nullptr, 0, m, out);
}

extern "C" int rf_bloom_load_binary(rf_ctx* ctx, const uint8_t* buf, size_t len, rf_bloom** out) {
    uint64_t m = 0, k = 0, length = 0;
    std::vector<uint64_t> w;
    int rc = bloom_parse_binary(buf, len, &m, &k, &length, w);
    return rc ? rc : bloom_make(ctx, m, k, w.data(), w.size(), length, out);
}

extern "C" int rf_bloom_load_json(rf_ctx* ctx, const char* json, size_t len, rf_bloom** out) {
    uint64_t m = 0, k = 0, length = 0;
    std::vector<uint64_t> w;
    int rc = bloom_parse_json(json, len, &m, &k, &length, w);
    return rc ? rc : bloom_make(ctx, m, k, w.data(), w.size(), length, out);
}

extern "C" void rf_bloom_destroy(rf_bloom* bl) {
    if (!bl) return;
    DevGuard dg(bl->ctx->device);
    bl->words.release();
    bl->len_dev.release();
    for (DevBuf* d : {&bl->keys, &bl->out, &bl->sizes, &bl->dead, &bl->tiles, &bl->idx, &bl->nb}) d->release();
    delete bl;
}

extern "C" int rf_bloom_probe_device(rf_bloom* bl, const void* d_digests32, uint64_t n, void* d_out,
                                     void* stream) {
    ARG(bl && (n == 0 || (d_digests32 && d_out)), "null argument");
    DevGuard dg(bl->ctx->device);
    HIPC(launch_bloom_probe(bl->b, static_cast<const uint8_t*>(d_digests32), n,
                            static_cast<uint8_t*>(d_out), pick(bl->ctx, stream)));
    return RF_OK;
}

extern "C" int rf_bloom_probe(rf_bloom* bl, const uint8_t* digests32, uint64_t n, uint8_t* out) {
    ARG(bl && (n == 0 || (digests32 && out)), "null argument");
    if (!n) return RF_OK;
    rf_ctx* ctx = bl->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    HIPC(bl->keys.ensure(32 * n));
    HIPC(bl->out.ensure(n));
    HIPC(hipMemcpyAsync(bl->keys.p, digests32, 32 * n, hipMemcpyHostToDevice, ctx->stream));
    HIPC(launch_bloom_probe(bl->b, bl->keys.as<uint8_t>(), n, bl->out.as<uint8_t>(), ctx->stream));
    HIPC(hipMemcpyAsync(out, bl->out.p, n, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    return RF_OK;
}

extern "C" int rf_bloom_add_device(rf_bloom* bl, const void* d_digests32, uint64_t n, void* stream) {
    ARG(bl && (n == 0 || d_digests32), "null argument");
    DevGuard dg(bl->ctx->device);
    HIPC(launch_bloom_add(bl->b, static_cast<const uint8_t*>(d_digests32), n, pick(bl->ctx, stream)));
    return RF_OK;
}

extern "C" int rf_bloom_add(rf_bloom* bl, const uint8_t* digests32, uint64_t n) {
    ARG(bl && (n == 0 || digests32), "null argument");
    if (!n) return RF_OK;
    rf_ctx* ctx = bl->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    HIPC(bl->keys.ensure(32 * n));
    HIPC(hipMemcpyAsync(bl->keys.p, digests32, 32 * n, hipMemcpyHostToDevice, ctx->stream));
    HIPC(launch_bloom_add(bl->b, bl->keys.as<uint8_t>(), n, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    return RF_OK;
}

extern "C" int rf_bloom_params(rf_bloom* bl, uint64_t* m, uint64_t* k, uint64_t* length,
                               uint64_t* nwords) {
    ARG(bl, "null bloom");
    DevGuard dg(bl->ctx->device);
    uint64_t len = 0;
    HIPC(sync_copy(bl->ctx, &len, bl->b.len_dev, 8, hipMemcpyDeviceToHost));
    if (m) *m = bl->b.m;
    if (k) *k = bl->b.k;
    if (length) *length = len;
    if (nwords) *nwords = (len + 63) / 64;
    return RF_OK;
}

extern "C" int rf_bloom_words(rf_bloom* bl, uint64_t* words, uint64_t nwords) {
    ARG(bl && (nwords == 0 || words), "null argument");
    ARG(nwords <= bl->b.nwords, "nwords exceeds filter capacity");
    DevGuard dg(bl->ctx->device);
    if (nwords) HIPC(sync_copy(bl->ctx, words, bl->b.words, 8 * nwords, hipMemcpyDeviceToHost));
    return RF_OK;
}

// ---- Liveset wire formats out (bloom.go:264-301, bitset.go:623-702) ----------
// The bitset as the device holds it: its length and wordsNeeded(length)
// words (bitset.go:628-640); the byte layout is wire.cpp's.
static int bloom_host_words(rf_bloom* bl, uint64_t* length, std::vector<uint64_t>& w) {
    HIPC(sync_copy(bl->ctx, length, bl->b.len_dev, 8, hipMemcpyDeviceToHost));
    const uint64_t nw = (*length + 63) / 64;
    if (nw > bl->b.nwords) return fail(RF_EINVAL, "bitset length exceeds filter capacity");
    w.resize(nw);
    if (nw) HIPC(sync_copy(bl->ctx, w.data(), bl->b.words, 8 * nw, hipMemcpyDeviceToHost));
    return RF_OK;
}

extern "C" int rf_bloom_marshal_binary(rf_bloom* bl, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    ARG(bl, "null bloom");
    DevGuard dg(bl->ctx->device);
    uint64_t length = 0;
    std::vector<uint64_t> w;
    int rc = bloom_host_words(bl, &length, w);
    return rc ? rc : rf_bloom_format_binary(bl->b.m, bl->b.k, length, w.data(), w.size(), out, cap, out_len);
}

extern "C" int rf_bloom_marshal_json(rf_bloom* bl, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    ARG(bl, "null bloom");
    DevGuard dg(bl->ctx->device);
    uint64_t length = 0;
    std::vector<uint64_t> w;
    int rc = bloom_host_words(bl, &length, w);
    return rc ? rc : rf_bloom_format_json(bl->b.m, bl->b.k, length, w.data(), w.size(), out, cap, out_len);
}

// ---- Repository.Collect over a batch of objects (repository/file/repository.go:304-327)
extern "C" int rf_bloom_collect_device(rf_bloom* bl, const void* d_digests32, const void* d_sizes, uint64_t n,
                                       void* d_dead_idx, void* d_counts2, void* stream) {
    ARG(bl && (n == 0 || (d_digests32 && d_dead_idx)) && d_counts2, "null argument");
    ARG(n < (1ull << 32), "collect batch too large (n < 2^32)");
    DevGuard dg(bl->ctx->device);
    hipStream_t s = pick(bl->ctx, stream);
    HIPC(hipMemsetAsync(d_counts2, 0, 16, s));
    if (!n) return RF_OK;
    // scratch handed between streams in stream order (StreamScratch, ctx.h)
    StreamScratch& sc = bl->ctx->sc_collect;
    std::lock_guard<std::mutex> lk(sc.mu);
    const size_t dead_bytes = (n + 255) / 256 * 256;
    HIPC(sc.acquire(dead_bytes + 4 * bloom_collect_tiles(n), s));
    uint8_t* dead = sc.buf.as<uint8_t>();
    hipError_t e = launch_bloom_collect(bl->b, static_cast<const uint8_t*>(d_digests32),
                                        static_cast<const int64_t*>(d_sizes), n, dead,
                                        reinterpret_cast<uint32_t*>(dead + dead_bytes),
                                        static_cast<uint64_t*>(d_dead_idx), static_cast<uint64_t*>(d_counts2), s);
    HIPC(sc.release(s));
    if (e != hipSuccess) return fail(RF_EDEVICE, "collect: %s", hipGetErrorString(e));
    return RF_OK;
}

extern "C" int rf_bloom_collect(rf_bloom* bl, const uint8_t* digests32, const int64_t* sizes, uint64_t n,
                                uint64_t* dead_idx, uint64_t* n_dead, int64_t* dead_bytes) {
    ARG(bl && (n == 0 || (digests32 && dead_idx)) && n_dead, "null argument");
    rf_ctx* ctx = bl->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    HIPC(bl->keys.ensure(32 * std::max<uint64_t>(n, 1)));
    HIPC(bl->idx.ensure(8 * std::max<uint64_t>(n, 1)));
    HIPC(bl->nb.ensure(16));
    if (n) HIPC(hipMemcpyAsync(bl->keys.p, digests32, 32 * n, hipMemcpyHostToDevice, ctx->stream));
    if (n && sizes) {
        HIPC(bl->sizes.ensure(8 * n));
        HIPC(hipMemcpyAsync(bl->sizes.p, sizes, 8 * n, hipMemcpyHostToDevice, ctx->stream));
    }
    int rc = rf_bloom_collect_device(bl, bl->keys.p, sizes ? bl->sizes.p : nullptr, n, bl->idx.p, bl->nb.p,
                                     ctx->stream);
    if (rc) return rc;
    uint64_t nb[2] = {0, 0};
    HIPC(hipMemcpyAsync(nb, bl->nb.p, 16, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    if (nb[0]) HIPC(sync_copy(bl->ctx, dead_idx, bl->idx.p, 8 * nb[0], hipMemcpyDeviceToHost));
    *n_dead = nb[0];
    if (dead_bytes) *dead_bytes = (int64_t)nb[1];
    return RF_OK;
}

// ---------------------------------------------------------------------------
// K5: Canonicalize's flowMap (flow.go:814-843, flowMap.Get/Put :881-907)
// Scratch of a device-form call: the context's StreamScratch, handed
// between the callers' streams in stream order (ctx.h).
static int dedup_on_stream(rf_ctx* ctx, const void* d_digests32, uint32_t n, void* d_canon, void* d_n_unique,
                           hipStream_t s) {
    StreamScratch& sc = ctx->sc_dedup;
    std::lock_guard<std::mutex> lk(sc.mu);
    const size_t tab_bytes = 4ull * dedup_table_slots(n);
    HIPC(sc.acquire(tab_bytes + 4ull * std::max<uint32_t>(n, 1), s));
    uint32_t* tab = sc.buf.as<uint32_t>();
    hipError_t e = launch_dedup(static_cast<const uint8_t*>(d_digests32), n, tab, tab + tab_bytes / 4,
                                static_cast<uint32_t*>(d_canon), static_cast<uint32_t*>(d_n_unique), s);
    HIPC(sc.release(s));
    if (e != hipSuccess) return fail(RF_EDEVICE, "dedup: %s", hipGetErrorString(e));
    return RF_OK;
}

extern "C" int rf_dedup_digests_device(rf_ctx* ctx, const void* d_digests32, uint32_t n, void* d_canon,
                                       void* d_n_unique, void* stream) {
    ARG(ctx && d_n_unique && (n == 0 || (d_digests32 && d_canon)), "null argument");
    ARG(n <= (1u << 30), "dedup batch too large (n <= 2^30)");
    DevGuard dg(ctx->device);
    return dedup_on_stream(ctx, d_digests32, n, d_canon, d_n_unique, pick(ctx, stream));
}

extern "C" int rf_dedup_digests(rf_ctx* ctx, const uint8_t* digests32, uint32_t n, uint32_t* canon,
                                uint32_t* n_unique) {
    ARG(ctx && n_unique && (n == 0 || (digests32 && canon)), "null argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    HIPC(ctx->d_arena.ensure(32ull * std::max<uint32_t>(n, 1)));
    HIPC(ctx->d_tab3.ensure(4ull * std::max<uint32_t>(n, 1) + 64));
    uint32_t* d_canon = ctx->d_tab3.as<uint32_t>();
    uint32_t* d_nu = d_canon + std::max<uint32_t>(n, 1);
    if (n) HIPC(hipMemcpyAsync(ctx->d_arena.p, digests32, 32ull * n, hipMemcpyHostToDevice, ctx->stream));
    HIPC(ctx->d_tab.ensure(4ull * dedup_table_slots(n)));
    HIPC(ctx->d_tab2.ensure(4ull * std::max<uint32_t>(n, 1)));
    HIPC(launch_dedup(ctx->d_arena.as<uint8_t>(), n, ctx->d_tab.as<uint32_t>(), ctx->d_tab2.as<uint32_t>(), d_canon,
                      d_nu, ctx->stream));
    if (n) HIPC(hipMemcpyAsync(canon, d_canon, 4ull * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipMemcpyAsync(n_unique, d_nu, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    if (*n_unique & 0x80000000u) return fail(RF_EDEVICE, "dedup: probe bound exceeded (table not usable)");
    return RF_OK;
}

// ---------------------------------------------------------------------------
// HBM assoc (assoc.Assoc, assoc/assoc.go:26-38; test/testutil/assoc.go:34-56)
struct rf_assoc {
    rf_ctx* ctx = nullptr;
    uint32_t cap = 0;
    // the last Get launched on a caller's stream (rf_assoc_get_device): a
    // rehash frees the old table only after it
    hipEvent_t e_reader = nullptr;
    bool reader_pending = false;
    DevBuf tag, keys, vals, count;                                   // the table
    DevBuf b_keys, b_vals, b_exp, b_canon, b_aslot, b_cls, b_rem, b_next, b_cnt, b_status, b_found;  // batch scratch
    AssocView view() {
        return AssocView{tag.as<uint32_t>(), keys.as<uint4>(), vals.as<uint4>(), cap - 1, count.as<uint32_t>()};
    }
};

static hipError_t assoc_alloc_table(rf_assoc* a, uint32_t cap, hipStream_t s) {
    hipError_t e;
    if ((e = a->tag.ensure(4ull * cap)) != hipSuccess || (e = a->keys.ensure(32ull * cap)) != hipSuccess ||
        (e = a->vals.ensure(32ull * cap)) != hipSuccess || (e = a->count.ensure(64)) != hipSuccess)
        return e;
    a->cap = cap;
    if ((e = hipMemsetAsync(a->tag.p, 0, 4ull * cap, s)) != hipSuccess) return e;
    return hipMemsetAsync(a->count.p, 0, 4, s);
}

extern "C" int rf_assoc_new(rf_ctx* ctx, uint64_t capacity, rf_assoc** out) {
    ARG(ctx && out, "null argument");
    ARG(capacity < (1ull << 30), "assoc capacity too large");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    auto* a = new rf_assoc();
    a->ctx = ctx;
    uint32_t cap = 1024;
    while (cap < 2 * capacity) cap <<= 1;
    hipError_t e = assoc_alloc_table(a, cap, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        delete a;
        return fail(e == hipErrorOutOfMemory ? RF_ENOMEM : RF_EDEVICE, "assoc alloc: %s", hipGetErrorString(e));
    }
    *out = a;
    return RF_OK;
}

extern "C" void rf_assoc_destroy(rf_assoc* a) {
    if (!a) return;
    DevGuard dg(a->ctx->device);
    if (a->e_reader) {
        if (a->reader_pending) (void)hipEventSynchronize(a->e_reader);
        (void)hipEventDestroy(a->e_reader);
    }
    for (DevBuf* d : {&a->tag, &a->keys, &a->vals, &a->count, &a->b_keys, &a->b_vals, &a->b_exp, &a->b_canon,
                      &a->b_aslot, &a->b_cls, &a->b_rem, &a->b_next, &a->b_cnt, &a->b_status, &a->b_found})
        d->release();
    delete a;
}

// keep the table at most half full after inserting up to `incoming` new keys
static int assoc_reserve(rf_assoc* a, uint64_t incoming) {
    rf_ctx* ctx = a->ctx;
    uint32_t used = 0;
    HIPC(hipMemcpyAsync(&used, a->count.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    const uint64_t need = (uint64_t)used + incoming;
    if (2 * need <= a->cap) return RF_OK;
    uint64_t cap = a->cap;
    while (cap < 2 * need) cap <<= 1;
    ARG(cap <= (1ull << 31), "assoc table would exceed 2^31 slots");
    rf_assoc old;  // move the old table out
    std::swap(old.tag, a->tag);
    std::swap(old.keys, a->keys);
    std::swap(old.vals, a->vals);
    std::swap(old.count, a->count);
    old.cap = a->cap;
    HIPC(assoc_alloc_table(a, (uint32_t)cap, ctx->stream));
    HIPC(launch_assoc_rehash(old.view(), old.cap, a->view(), ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    if (a->reader_pending) {  // a device-form Get on another stream may still read the old table
        HIPC(hipEventSynchronize(a->e_reader));
        a->reader_pending = false;
    }
    old.tag.release();
    old.keys.release();
    old.vals.release();
    old.count.release();
    return RF_OK;
}

// Put over device-resident keys / values / expects (d_status: int32 per op).
static int assoc_put_locked(rf_assoc* a, int kind, const uint8_t* d_exp, const uint8_t* d_keys, const uint8_t* d_vals,
                            uint64_t n, int32_t* d_status) {
    rf_ctx* ctx = a->ctx;
    hipStream_t s = ctx->stream;
    int rc = assoc_reserve(a, n);
    if (rc) return rc;
    HIPC(a->b_canon.ensure(4 * n + 64));
    HIPC(a->b_aslot.ensure(4 * n));
    HIPC(a->b_cls.ensure(8 * n));
    HIPC(a->b_rem.ensure(4 * n));
    HIPC(a->b_next.ensure(4 * n));
    HIPC(a->b_cnt.ensure(64));
    // distinct keys of the batch (K5 dedup), then find-or-insert them
    uint32_t* canon = a->b_canon.as<uint32_t>();
    uint32_t* d_nu = canon + n;
    HIPC(ctx->d_tab.ensure(4ull * dedup_table_slots((uint32_t)n)));
    HIPC(ctx->d_tab2.ensure(4ull * n));
    HIPC(launch_dedup(d_keys, (uint32_t)n, ctx->d_tab.as<uint32_t>(), ctx->d_tab2.as<uint32_t>(), canon, d_nu, s));
    // a batch that hit the dedup probe bound has canon[i] = ~0 for some ops:
    // the insert / claim / apply kernels index by canon, so stop here
    uint32_t nu = 0;
    HIPC(hipMemcpyAsync(&nu, d_nu, 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (nu & 0x80000000u) return fail(RF_EDEVICE, "assoc put: dedup probe bound exceeded (batch not applied)");
    HIPC(launch_assoc_insert(a->view(), (uint32_t)kind, d_keys, canon, (uint32_t)n, a->b_aslot.as<uint32_t>(), s));
    // ops in batch order per key: round r applies each key's r-th op
    HIPC(launch_iota(a->b_rem.as<uint32_t>(), (uint32_t)n, s));
    HIPC(hipMemsetAsync(a->b_cls.p, 0, 8 * n, s));
    uint32_t* cnt = a->b_cnt.as<uint32_t>();  // cnt[0] = remaining, cnt[1] = next
    uint32_t n_rem = (uint32_t)n;
    HIPC(hipMemcpyAsync(cnt, &n_rem, 4, hipMemcpyHostToDevice, s));
    uint32_t* rem = a->b_rem.as<uint32_t>();
    uint32_t* next = a->b_next.as<uint32_t>();
    for (uint32_t round = 1; n_rem; ++round) {
        HIPC(hipMemsetAsync(cnt + 1, 0, 4, s));
        HIPC(launch_assoc_round(a->view(), rem, cnt, n_rem, canon, (unsigned long long*)a->b_cls.p, round,
                                a->b_aslot.as<uint32_t>(), d_exp, d_vals, d_status, next, cnt + 1, s));
        HIPC(hipMemcpyAsync(&n_rem, cnt + 1, 4, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        HIPC(hipMemcpyAsync(cnt, cnt + 1, 4, hipMemcpyDeviceToDevice, s));
        std::swap(rem, next);
    }
    return RF_OK;
}

extern "C" int rf_assoc_put_device(rf_assoc* a, int kind, const void* d_expect32, const void* d_keys32,
                                   const void* d_vals32, uint64_t n, void* d_status) {
    ARG(a && (n == 0 || (d_keys32 && d_vals32 && d_status)), "null argument");
    ARG(kind >= 0 && kind < (1 << 30), "bad assoc kind");
    ARG(n <= (1u << 30), "assoc batch too large");
    if (!n) return RF_OK;
    std::lock_guard<std::mutex> lk(a->ctx->mu);
    DevGuard dg(a->ctx->device);
    int rc = assoc_put_locked(a, kind, static_cast<const uint8_t*>(d_expect32), static_cast<const uint8_t*>(d_keys32),
                              static_cast<const uint8_t*>(d_vals32), n, static_cast<int32_t*>(d_status));
    if (rc) return rc;
    HIPC(hipStreamSynchronize(a->ctx->stream));
    return RF_OK;
}

extern "C" int rf_assoc_put(rf_assoc* a, int kind, const uint8_t* expect32, const uint8_t* keys32,
                            const uint8_t* vals32, uint64_t n, int32_t* status) {
    ARG(a && (n == 0 || (keys32 && vals32 && status)), "null argument");
    ARG(kind >= 0 && kind < (1 << 30), "bad assoc kind");
    ARG(n <= (1u << 30), "assoc batch too large");
    if (!n) return RF_OK;
    rf_ctx* ctx = a->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    hipStream_t s = ctx->stream;
    HIPC(a->b_keys.ensure(32 * n));
    HIPC(a->b_vals.ensure(32 * n));
    HIPC(a->b_status.ensure(4 * n));
    HIPC(hipMemcpyAsync(a->b_keys.p, keys32, 32 * n, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(a->b_vals.p, vals32, 32 * n, hipMemcpyHostToDevice, s));
    if (expect32) {
        HIPC(a->b_exp.ensure(32 * n));
        HIPC(hipMemcpyAsync(a->b_exp.p, expect32, 32 * n, hipMemcpyHostToDevice, s));
    }
    int rc = assoc_put_locked(a, kind, expect32 ? a->b_exp.as<uint8_t>() : nullptr, a->b_keys.as<uint8_t>(),
                              a->b_vals.as<uint8_t>(), n, a->b_status.as<int32_t>());
    if (rc) return rc;
    HIPC(hipMemcpyAsync(status, a->b_status.p, 4 * n, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    return RF_OK;
}

extern "C" int rf_assoc_get_device(rf_assoc* a, int kind, const void* d_keys32, uint64_t n, void* d_vals32,
                                   void* d_found, void* stream) {
    ARG(a && (n == 0 || (d_keys32 && d_vals32 && d_found)), "null argument");
    std::lock_guard<std::mutex> lk(a->ctx->mu);  // no Put may swap the table meanwhile
    DevGuard dg(a->ctx->device);
    hipStream_t s = pick(a->ctx, stream);
    HIPC(launch_assoc_get(a->view(), (uint32_t)kind, static_cast<const uint8_t*>(d_keys32), n,
                          static_cast<uint8_t*>(d_vals32), static_cast<uint8_t*>(d_found), s));
    if (s != a->ctx->stream) {  // Puts run on ctx->stream, ordered after it already
        if (!a->e_reader) HIPC(hipEventCreateWithFlags(&a->e_reader, hipEventDisableTiming));
        HIPC(hipEventRecord(a->e_reader, s));
        a->reader_pending = true;
    }
    return RF_OK;
}

extern "C" int rf_assoc_get(rf_assoc* a, int kind, const uint8_t* keys32, uint64_t n, uint8_t* vals32,
                            uint8_t* found) {
    ARG(a && (n == 0 || (keys32 && vals32 && found)), "null argument");
    if (!n) return RF_OK;
    rf_ctx* ctx = a->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    HIPC(a->b_keys.ensure(32 * n));
    HIPC(a->b_vals.ensure(32 * n));
    HIPC(a->b_found.ensure(n));
    HIPC(hipMemcpyAsync(a->b_keys.p, keys32, 32 * n, hipMemcpyHostToDevice, ctx->stream));
    HIPC(launch_assoc_get(a->view(), (uint32_t)kind, a->b_keys.as<uint8_t>(), n, a->b_vals.as<uint8_t>(),
                          a->b_found.as<uint8_t>(), ctx->stream));
    HIPC(hipMemcpyAsync(vals32, a->b_vals.p, 32 * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipMemcpyAsync(found, a->b_found.p, n, hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    return RF_OK;
}

// Eval.lookup over a batch of nodes (eval.go:1172-1220): one Get batch over
// every node's cache keys (the BatchGetItem the TODO at eval.go:1199-1201
// asks for), first hit per node selected on the device.  Read only.
static int check_key_ptr(const uint64_t* key_ptr, uint64_t n_nodes) {
    ARG(key_ptr[0] == 0, "key_ptr[0] must be 0");
    for (uint64_t i = 0; i < n_nodes; ++i) ARG(key_ptr[i] <= key_ptr[i + 1], "key_ptr not monotone");
    ARG(key_ptr[n_nodes] <= (1u << 30), "lookup batch too large");
    return RF_OK;
}

extern "C" int rf_assoc_lookup(rf_assoc* a, int kind, const uint8_t* keys32, const uint64_t* key_ptr, uint64_t n_nodes,
                               int32_t* which, uint8_t* vals32, uint8_t* key_found, uint8_t* key_vals32) {
    ARG(a && key_ptr && (n_nodes == 0 || (which && vals32)), "null argument");
    ARG(kind >= 0 && kind < (1 << 30), "bad assoc kind");
    if (!n_nodes) return RF_OK;
    if (int rc = check_key_ptr(key_ptr, n_nodes)) return rc;
    const uint64_t nk = key_ptr[n_nodes];
    ARG(nk == 0 || keys32, "null keys");
    rf_ctx* ctx = a->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    hipStream_t s = ctx->stream;
    // scratch: keys + per-key values (b_keys, b_vals), found per key, the
    // node CSR and per-node outputs (b_exp region)
    HIPC(a->b_keys.ensure(32 * nk + 32));
    HIPC(a->b_vals.ensure(32 * nk + 32));
    HIPC(a->b_found.ensure(nk + 16));
    const uint64_t off_which = (8 * (n_nodes + 1) + 15) & ~15ull, off_out = (off_which + 4 * n_nodes + 15) & ~15ull;
    HIPC(a->b_exp.ensure(off_out + 32 * n_nodes));
    uint64_t* d_ptr = a->b_exp.as<uint64_t>();
    int32_t* d_which = reinterpret_cast<int32_t*>(a->b_exp.as<uint8_t>() + off_which);
    uint8_t* d_out = a->b_exp.as<uint8_t>() + off_out;
    if (nk) HIPC(hipMemcpyAsync(a->b_keys.p, keys32, 32 * nk, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(d_ptr, key_ptr, 8 * (n_nodes + 1), hipMemcpyHostToDevice, s));
    HIPC(launch_assoc_get(a->view(), (uint32_t)kind, a->b_keys.as<uint8_t>(), nk, a->b_vals.as<uint8_t>(),
                          a->b_found.as<uint8_t>(), s));
    HIPC(launch_assoc_select(a->b_found.as<uint8_t>(), a->b_vals.as<uint8_t>(), d_ptr, n_nodes, d_which, d_out, s));
    HIPC(hipMemcpyAsync(which, d_which, 4 * n_nodes, hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(vals32, d_out, 32 * n_nodes, hipMemcpyDeviceToHost, s));
    if (key_found && nk) HIPC(hipMemcpyAsync(key_found, a->b_found.p, nk, hipMemcpyDeviceToHost, s));
    if (key_vals32 && nk) HIPC(hipMemcpyAsync(key_vals32, a->b_vals.p, 32 * nk, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    return RF_OK;
}

// Read repair of the nodes the caller verified (eval.go:1227-1258): Put(zero
// expect) of the node's value under its other keys (blind) or under the ones
// the Get found missing (precise), as one Put batch in node order, key order.
extern "C" int rf_assoc_repair(rf_assoc* a, int kind, const uint8_t* keys32, const uint64_t* key_ptr, uint64_t n_nodes,
                               const int32_t* which, const uint8_t* vals32, const uint8_t* key_found) {
    ARG(a && key_ptr && (n_nodes == 0 || (which && vals32)), "null argument");
    ARG(kind >= 0 && kind < (1 << 30), "bad assoc kind");
    if (!n_nodes) return RF_OK;
    if (int rc = check_key_ptr(key_ptr, n_nodes)) return rc;
    const uint64_t nk = key_ptr[n_nodes];
    ARG(nk == 0 || keys32, "null keys");
    std::vector<uint8_t> rk, rv;
    for (uint64_t i = 0; i < n_nodes; ++i) {
        if (which[i] < 0) continue;
        ARG((uint64_t)which[i] < key_ptr[i + 1] - key_ptr[i], "which[i] past the node's keys");
        for (uint64_t k = key_ptr[i]; k < key_ptr[i + 1]; ++k) {
            if ((int64_t)(k - key_ptr[i]) == which[i] || (key_found && key_found[k])) continue;
            rk.insert(rk.end(), keys32 + 32 * k, keys32 + 32 * k + 32);
            rv.insert(rv.end(), vals32 + 32 * i, vals32 + 32 * i + 32);
        }
    }
    const uint64_t nr = rk.size() / 32;
    if (!nr) return RF_OK;
    rf_ctx* ctx = a->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    hipStream_t s = ctx->stream;
    HIPC(a->b_keys.ensure(32 * nr));
    HIPC(a->b_vals.ensure(32 * nr));
    HIPC(a->b_status.ensure(4 * nr));
    HIPC(hipMemcpyAsync(a->b_keys.p, rk.data(), 32 * nr, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(a->b_vals.p, rv.data(), 32 * nr, hipMemcpyHostToDevice, s));
    int rc = assoc_put_locked(a, kind, nullptr, a->b_keys.as<uint8_t>(), a->b_vals.as<uint8_t>(), nr,
                              a->b_status.as<int32_t>());
    if (rc) return rc;
    HIPC(hipStreamSynchronize(s));
    return RF_OK;
}

extern "C" int rf_assoc_get_abbrev(rf_assoc* a, int kind, const uint8_t* keys32, const uint8_t* nhex, uint64_t n,
                                   uint8_t* keys_out32, uint8_t* vals32, int32_t* status) {
    ARG(a && (n == 0 || (keys32 && nhex && keys_out32 && vals32 && status)), "null argument");
    for (uint64_t i = 0; i < n; ++i) ARG(nhex[i] >= 8 && nhex[i] <= 64, "abbreviated keys need 8..64 hex digits (ID4)");
    if (!n) return RF_OK;
    rf_ctx* ctx = a->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    hipStream_t s = ctx->stream;
    HIPC(a->b_keys.ensure(32 * 64 + 64));
    HIPC(a->b_cnt.ensure(4 * 64 * 2));
    uint32_t* cnt = a->b_cnt.as<uint32_t>();
    for (uint64_t b = 0; b < n; b += 64) {
        const uint32_t q = (uint32_t)std::min<uint64_t>(64, n - b);
        HIPC(hipMemcpyAsync(a->b_keys.p, keys32 + 32 * b, 32 * q, hipMemcpyHostToDevice, s));
        HIPC(hipMemcpyAsync(a->b_keys.as<uint8_t>() + 32 * 64, nhex + b, q, hipMemcpyHostToDevice, s));
        HIPC(hipMemsetAsync(cnt, 0, 4 * 64, s));
        HIPC(launch_assoc_abbrev(a->view(), (uint32_t)kind, a->cap, a->b_keys.as<uint8_t>(),
                                 a->b_keys.as<uint8_t>() + 32 * 64, q, cnt, cnt + 64, s));
        uint32_t h[128];
        HIPC(hipMemcpyAsync(h, cnt, 4 * 128, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        for (uint32_t j = 0; j < q; ++j) {
            const uint64_t i = b + j;
            if (h[j] == 0) {
                status[i] = RF_ENOTFOUND;
            } else if (h[j] > 1) {
                status[i] = RF_EINVAL;  // "more than one key matched" (dydbassoc.go:145-146)
            } else {
                HIPC(sync_copy(ctx, keys_out32 + 32 * i, a->keys.as<uint8_t>() + 32ull * h[64 + j], 32,
                               hipMemcpyDeviceToHost));
                HIPC(sync_copy(ctx, vals32 + 32 * i, a->vals.as<uint8_t>() + 32ull * h[64 + j], 32,
                               hipMemcpyDeviceToHost));
                status[i] = RF_OK;
            }
        }
    }
    return RF_OK;
}

extern "C" int rf_assoc_stats(rf_assoc* a, uint64_t* occupied, uint64_t* capacity) {
    ARG(a, "null assoc");
    DevGuard dg(a->ctx->device);
    uint32_t used = 0;
    HIPC(sync_copy(a->ctx, &used, a->count.p, 4, hipMemcpyDeviceToHost));
    if (occupied) *occupied = used;
    if (capacity) *capacity = a->cap;
    return RF_OK;
}
