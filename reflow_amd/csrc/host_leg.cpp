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

#include "diag.h"
#include "host_sha.h"

namespace rf {

uint64_t host_chunk_bytes() {
    static const uint64_t c = (uint64_t)std::max<long>(1, RF_DIAG_KNOB("RF_HOST_CHUNK_MB", 8)) << 20;
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
        for (LaneStage& l : s.lane) {
            if (l.s) {
                (void)hipStreamSynchronize(l.s);
                (void)hipStreamDestroy(l.s);
            }
            for (uint8_t* b : l.buf)
                if (b) (void)hipHostFree(b);
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

hipError_t HostPool::stage(unsigned w, int ways, Stage** out) {
    Stage& s = stages_[w];
    *out = &s;
    hipError_t e;
    for (int k = 0; k < ways; ++k) {
        LaneStage& l = s.lane[k];
        if (!l.s && (e = hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking)) != hipSuccess) return e;
        for (uint8_t*& b : l.buf) {
            if (b) continue;
            void* p = nullptr;
            if ((e = hipHostMalloc(&p, host_chunk_bytes(), hipHostMallocDefault)) != hipSuccess) return e;
            b = static_cast<uint8_t*>(p);
        }
    }
    return hipSuccess;
}

int host_ways() {
    static const int w = (int)std::min<long>(4, std::max<long>(1, RF_DIAG_KNOB("RF_HOST_WAYS", 2)));
    return w;
}

namespace {
// One message in flight on a host thread.  Its bytes come in chunks of C
// (from the message start, so every chunk but the last is whole blocks):
// from HBM through the lane's double buffer, or straight from host memory.
struct Lane {
    bool active = false, ready = false;
    uint64_t task = 0, len = 0, nch = 0, c = 0, pos = 0;
    int buf = 0;
    const uint8_t* src = nullptr;
    uint32_t st[8];
};
}  // namespace

bool host_leg_run(HostPool& pool, const HostTask* tasks, uint64_t n, const uint8_t* d_arena,
                  const uint8_t* h_arena, uint8_t* out32, std::string* err) {
    std::atomic<uint64_t> next{0};
    std::atomic<bool> bad{false};
    std::mutex emu;
    const bool timing = leg_timing();
    const int W = host_ways();
    const uint64_t C = host_chunk_bytes();
    std::vector<double> tw(pool.size(), 0.0), th(pool.size(), 0.0), tt(pool.size(), 0.0);
    const double t_run = timing ? now_s() : 0;
    auto fail_with = [&](const char* what, hipError_t e) {
        std::lock_guard<std::mutex> lk(emu);
        if (!bad.exchange(true)) *err = std::string(what) + hipGetErrorString(e);
    };
    pool.run([&](unsigned w) {
        const double t_start = timing ? now_s() : 0;
        HostPool::Stage* st = nullptr;
        if (d_arena) {
            const hipError_t e = pool.stage(w, W, &st);
            if (e != hipSuccess) return fail_with("host leg stage: ", e);
        }
        Lane L[4];
        auto chunk_len = [&](const Lane& x) { return std::min(C, x.len - x.c * C); };
        auto data = [&](const Lane& x, int k) -> const uint8_t* {
            return h_arena ? x.src + x.c * C : st->lane[k].buf[x.buf];
        };
        auto issue = [&](Lane& x, int k, uint64_t c, int b) -> bool {
            const uint64_t off = c * C;
            const hipError_t e = hipMemcpyAsync(st->lane[k].buf[b], x.src + off, std::min(C, x.len - off),
                                                hipMemcpyDeviceToHost, st->lane[k].s);
            if (e != hipSuccess) fail_with("host leg D2H: ", e);
            return e == hipSuccess;
        };
        // next message into lane slot k (zero-length ones finish on the spot)
        auto claim = [&](int k) {
            Lane& x = L[k];
            x.active = false;
            for (uint64_t i; !bad.load(std::memory_order_relaxed) && (i = next.fetch_add(1)) < n;) {
                x.task = i;
                x.len = tasks[i].len;
                x.src = (h_arena ? h_arena : d_arena) + tasks[i].off;
                host_sha_init(x.st);
                if (!x.len) {
                    host_sha_final(x.st, nullptr, 0, 0, out32 + 32 * i);
                    continue;
                }
                x.nch = (x.len + C - 1) / C;
                x.c = x.pos = 0;
                x.buf = 0;
                x.ready = h_arena != nullptr;
                if (!h_arena && !issue(x, k, 0, 0)) return;
                x.active = true;
                return;
            }
        };
        for (int k = 0; k < W; ++k) claim(k);
        for (;;) {
            int idx[4], na = 0;
            for (int k = 0; k < W; ++k)
                if (L[k].active) idx[na++] = k;
            if (!na || bad.load(std::memory_order_relaxed)) break;
            // chunks not yet waited on: wait, then queue the lane's next chunk
            // into the buffer its previous chunk has left
            for (int a = 0; a < na; ++a) {
                Lane& x = L[idx[a]];
                if (x.ready) continue;
                const double t0 = timing ? now_s() : 0;
                const hipError_t e = hipStreamSynchronize(st->lane[idx[a]].s);
                if (timing) tw[w] += now_s() - t0;
                if (e != hipSuccess) return fail_with("host leg D2H: ", e);
                x.ready = true;
                if (x.c + 1 < x.nch && !issue(x, idx[a], x.c + 1, x.buf ^ 1)) return;
            }
            // whole blocks every active lane has left in its current chunk
            uint64_t m = ~0ull;
            for (int a = 0; a < na; ++a) {
                const Lane& x = L[idx[a]];
                m = std::min(m, (chunk_len(x) - x.pos) / 64);
            }
            const double t1 = timing ? now_s() : 0;
            if (m) {
                uint32_t* sp[4];
                const uint8_t* pp[4];
                for (int a = 0; a < na; ++a) {
                    sp[a] = L[idx[a]].st;
                    pp[a] = data(L[idx[a]], idx[a]) + L[idx[a]].pos;
                }
                host_sha_blocks_multi(na, sp, pp, m);
                for (int a = 0; a < na; ++a) L[idx[a]].pos += 64 * m;
            }
            for (int a = 0; a < na; ++a) {
                Lane& x = L[idx[a]];
                const uint64_t cl = chunk_len(x);
                if (cl - x.pos >= 64) continue;  // blocks left in this chunk
                if (x.c + 1 < x.nch) {           // on to the next chunk (its copy is queued)
                    ++x.c;
                    x.pos = 0;
                    x.buf ^= 1;
                    x.ready = h_arena != nullptr;
                } else {  // the tail: pad, finish, take the next message
                    host_sha_final(x.st, data(x, idx[a]) + x.pos, cl - x.pos, x.len, out32 + 32 * x.task);
                    claim(idx[a]);
                }
            }
            if (timing) th[w] += now_s() - t1;
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
        fprintf(stderr, "[host leg] %u threads x %d ways, %llu msgs, %.2f GB: wall %.1f ms, slowest thread %.1f ms; "
                        "sum wait %.1f ms, sum hash %.1f ms (%.2f GB/s per hashing thread)\n",
                pool.size(), W, (unsigned long long)n, bytes / 1e9, (now_s() - t_run) * 1e3, mx * 1e3, sw * 1e3,
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
