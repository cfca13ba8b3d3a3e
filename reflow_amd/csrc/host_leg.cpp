// host_leg.cpp -- host thread pool and the K1 planner's host leg (host_leg.h).
#include "host_leg.h"

#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>

#include "host_sha.h"

namespace rf {

uint64_t host_chunk_bytes() {
    static const uint64_t c = [] {
        const char* v = getenv("RF_HOST_CHUNK_MB");
        const uint64_t mb = v ? (uint64_t)std::max(1, atoi(v)) : 8ull;
        return mb << 20;
    }();
    return c;
}

// RF_HOST_LEG_TIMING=1: per-run totals of the host threads' time waiting for
// D2H chunks and hashing (stderr; diagnostic).
static bool leg_timing() {
    static const bool on = getenv("RF_HOST_LEG_TIMING") != nullptr;
    return on;
}
static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// CPUs the cgroup (v2 cpu.max, or v1 cfs quota) lets this process use; 0 = no limit.
static unsigned cgroup_cpus() {
    long long q = -1, p = 0;
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char qs[64] = {0};
        if (fscanf(f, "%63s %lld", qs, &p) == 2 && strcmp(qs, "max") != 0) q = atoll(qs);
        fclose(f);
    } else {
        FILE* fq = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r");
        FILE* fp = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r");
        if (fq && fp && fscanf(fq, "%lld", &q) == 1 && fscanf(fp, "%lld", &p) == 1) {
        } else {
            q = -1;
        }
        if (fq) fclose(fq);
        if (fp) fclose(fp);
    }
    if (q <= 0 || p <= 0) return 0;
    return (unsigned)std::max<long long>(1, (q + p - 1) / p);
}

unsigned host_default_threads() {
    if (const char* v = getenv("RF_HOST_THREADS")) return (unsigned)std::max(0, atoi(v));
    cpu_set_t set;
    unsigned share = 1;
    if (sched_getaffinity(0, sizeof set, &set) == 0) share = (unsigned)CPU_COUNT(&set);
    if (const unsigned q = cgroup_cpus()) share = std::min(share, q);
    if (const char* l = getenv("LOCAL_WORLD_SIZE")) {
        const int lws = atoi(l);
        if (lws > 1) share = std::max(1u, share / (unsigned)lws);
    }
    return std::max(1u, std::min(60u, share));
}

HostPool::HostPool(int device, unsigned n) : device_(device), n_(n), stages_(n) {
    th_.reserve(n);
    for (unsigned w = 0; w < n; ++w) th_.emplace_back([this, w] { loop(w); });
}

HostPool::~HostPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
    (void)hipSetDevice(device_);
    for (Stage& s : stages_)
        for (int i = 0; i < 2; ++i) {
            if (s.s[i]) {
                (void)hipStreamSynchronize(s.s[i]);
                (void)hipStreamDestroy(s.s[i]);
            }
            if (s.buf[i]) (void)hipHostFree(s.buf[i]);
        }
}

void HostPool::loop(unsigned w) {
    (void)hipSetDevice(device_);
    uint64_t seen = 0;
    for (;;) {
        const std::function<void(unsigned)>* job;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            job = job_;
        }
        (*job)(w);
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_cv_.notify_all();
        }
    }
}

void HostPool::run(const std::function<void(unsigned)>& fn) {
    std::lock_guard<std::mutex> rl(run_mu_);
    std::unique_lock<std::mutex> lk(mu_);
    job_ = &fn;
    pending_ = n_;
    ++gen_;
    cv_.notify_all();
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
}

hipError_t HostPool::stage(unsigned w, Stage** out) {
    Stage& s = stages_[w];
    *out = &s;
    if (s.buf[1]) return hipSuccess;
    hipError_t e;
    for (int i = 0; i < 2; ++i) {
        if (!s.s[i] && (e = hipStreamCreateWithFlags(&s.s[i], hipStreamNonBlocking)) != hipSuccess) return e;
        if (s.buf[i]) continue;
        void* p = nullptr;
        if ((e = hipHostMalloc(&p, host_chunk_bytes(), hipHostMallocDefault)) != hipSuccess) return e;
        s.buf[i] = static_cast<uint8_t*>(p);
    }
    return hipSuccess;
}

// One message resident in HBM: chunk c+1's D2H is queued before chunk c is
// hashed, so the copy engine and the core overlap.  wait/hash (optional)
// accumulate the seconds spent waiting for chunks and hashing.
static hipError_t hash_device_message(HostPool::Stage* st, const uint8_t* src, uint64_t len, uint8_t* out32,
                                      double* wait, double* hash) {
    const uint64_t C = host_chunk_bytes();
    uint32_t h[8];
    host_sha_init(h);
    const uint64_t nch = len ? (len + C - 1) / C : 0;
    auto issue = [&](uint64_t c) -> hipError_t {
        const uint64_t off = c * C, sz = std::min(C, len - off);
        return hipMemcpyAsync(st->buf[c & 1], src + off, sz, hipMemcpyDeviceToHost, st->s[c & 1]);
    };
    hipError_t e = hipSuccess;
    if (nch) e = issue(0);
    for (uint64_t c = 0; c < nch && e == hipSuccess; ++c) {
        if (c + 1 < nch && (e = issue(c + 1)) != hipSuccess) break;
        const double t0 = wait ? now_s() : 0;
        if ((e = hipStreamSynchronize(st->s[c & 1])) != hipSuccess) break;
        const double t1 = wait ? now_s() : 0;
        const uint64_t sz = std::min(C, len - c * C);
        host_sha_blocks(h, st->buf[c & 1], sz / 64);
        if (c + 1 == nch) host_sha_final(h, st->buf[c & 1] + (sz & ~63ull), sz & 63, len, out32);
        if (wait) {
            *wait += t1 - t0;
            *hash += now_s() - t1;
        }
    }
    if (e == hipSuccess && nch == 0) host_sha_final(h, nullptr, 0, 0, out32);
    return e;
}

bool host_leg_run(HostPool& pool, const HostTask* tasks, uint64_t n, const uint8_t* d_arena,
                  const uint8_t* h_arena, uint8_t* out32, std::string* err) {
    std::atomic<uint64_t> next{0};
    std::atomic<bool> bad{false};
    std::mutex emu;
    const bool timing = leg_timing();
    std::vector<double> tw(pool.size(), 0.0), th(pool.size(), 0.0), tt(pool.size(), 0.0);
    const double t_run = timing ? now_s() : 0;
    pool.run([&](unsigned w) {
        const double t_start = timing ? now_s() : 0;
        HostPool::Stage* st = nullptr;
        if (d_arena) {
            const hipError_t e = pool.stage(w, &st);
            if (e != hipSuccess) {
                std::lock_guard<std::mutex> lk(emu);
                if (!bad.exchange(true)) *err = std::string("host leg stage: ") + hipGetErrorString(e);
                return;
            }
        }
        for (uint64_t i; !bad.load(std::memory_order_relaxed) && (i = next.fetch_add(1)) < n;) {
            const HostTask& t = tasks[i];
            if (h_arena) {
                host_sha256(h_arena + t.off, t.len, out32 + 32 * i);
                continue;
            }
            const hipError_t e = hash_device_message(st, d_arena + t.off, t.len, out32 + 32 * i,
                                                     timing ? &tw[w] : nullptr, timing ? &th[w] : nullptr);
            if (e != hipSuccess) {
                std::lock_guard<std::mutex> lk(emu);
                if (!bad.exchange(true)) *err = std::string("host leg D2H: ") + hipGetErrorString(e);
            }
        }
        if (timing) tt[w] = now_s() - t_start;
    });
    if (timing) {
        double sw = 0, sh = 0, mx = 0;
        for (unsigned w = 0; w < pool.size(); ++w) {
            sw += tw[w];
            sh += th[w];
            mx = std::max(mx, tt[w]);
        }
        uint64_t bytes = 0;
        for (uint64_t i = 0; i < n; ++i) bytes += tasks[i].len;
        fprintf(stderr, "[host leg] %u threads, %llu msgs, %.2f GB: wall %.1f ms, slowest thread %.1f ms; "
                        "sum wait %.1f ms, sum hash %.1f ms (%.2f GB/s per hashing thread)\n",
                pool.size(), (unsigned long long)n, bytes / 1e9, (now_s() - t_run) * 1e3, mx * 1e3, sw * 1e3,
                sh * 1e3, sh > 0 ? bytes / sh / 1e9 : 0.0);
    }
    return !bad.load();
}

void host_sha_absorb(uint32_t st[8], uint8_t carry[64], uint32_t* carry_len, const uint8_t* p, uint64_t len) {
    uint32_t c = *carry_len;
    if (c) {
        const uint64_t take = std::min<uint64_t>(64 - c, len);
        memcpy(carry + c, p, take);
        c += (uint32_t)take;
        p += take;
        len -= take;
        if (c < 64) {
            *carry_len = c;
            return;
        }
        host_sha_blocks(st, carry, 1);
        c = 0;
    }
    const uint64_t nb = len / 64;
    host_sha_blocks(st, p, nb);
    const uint64_t rest = len - 64 * nb;
    if (rest) memcpy(carry, p + 64 * nb, rest);
    *carry_len = (uint32_t)rest;
}

}  // namespace rf
