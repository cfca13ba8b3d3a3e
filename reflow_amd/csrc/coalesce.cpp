// coalesce.cpp -- concurrent callers coalesced into device batches
// (SURVEY §8(b) "Threading": the reference digests files in <=60 goroutines,
// local/executor.go:41,522-538, and looks up cache keys in one goroutine per
// node, eval.go:402-411; each would be its own tiny device batch).
//
// Group commit: a request joins the pending list; the first caller that finds
// no flush in progress becomes the flusher -- it waits up to max_wait_us
// (or until max_batch requests are pending), takes the whole list, runs ONE
// batched call (rf_sha256_batch / rf_bloom_probe / rf_assoc_get) without the
// lock held, then publishes every result and wakes the waiters.  Requests
// that arrive during a flush form the next batch; one of their callers flushes
// it.  Blocking calls (Go-friendly: a goroutine blocks in cgo) and async ones
// (submit returns a ticket, poll/wait complete it) share the queue.
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "errors.h"

using rf::fail;

namespace {
struct Req {
    const uint8_t* in = nullptr;  // message (SHA) or 32-B key
    uint64_t len = 0;
    uint8_t* out32 = nullptr;     // digest / value
    uint8_t* out_flag = nullptr;  // probe answer / found
    int rc = RF_OK;
    bool done = false;
    bool async = false;           // owned by the queue until polled
};
}  // namespace

struct rf_coalescer {
    int kind = 0;
    rf_ctx* ctx = nullptr;
    rf_bloom* bloom = nullptr;
    rf_assoc* assoc = nullptr;
    int assoc_kind = 0;
    uint64_t max_batch = 4096;
    uint64_t max_wait_us = 200;
    std::mutex mu;
    std::condition_variable cv_more;  // the flusher waits for a fuller batch
    std::condition_variable cv_done;  // callers wait for their result
    std::vector<Req*> pending;
    bool flushing = false;
    uint64_t batches = 0, requests = 0, largest = 0;
};

static int run_batch(rf_coalescer* c, std::vector<Req*>& b) {
    const uint64_t n = b.size();
    if (c->kind == RF_COALESCE_SHA256) {
        std::vector<const uint8_t*> msgs(n);
        std::vector<uint64_t> lens(n);
        std::vector<uint8_t> out(32 * n);
        for (uint64_t i = 0; i < n; ++i) {
            msgs[i] = b[i]->in;
            lens[i] = b[i]->len;
        }
        int rc = rf_sha256_batch(c->ctx, msgs.data(), lens.data(), n, out.data());
        if (rc == RF_OK)
            for (uint64_t i = 0; i < n; ++i) memcpy(b[i]->out32, &out[32 * i], 32);
        return rc;
    }
    std::vector<uint8_t> keys(32 * n), flag(n), vals(c->kind == RF_COALESCE_ASSOC_GET ? 32 * n : 0);
    for (uint64_t i = 0; i < n; ++i) memcpy(&keys[32 * i], b[i]->in, 32);
    int rc = c->kind == RF_COALESCE_PROBE
                 ? rf_bloom_probe(c->bloom, keys.data(), n, flag.data())
                 : rf_assoc_get(c->assoc, c->assoc_kind, keys.data(), n, vals.data(), flag.data());
    if (rc == RF_OK)
        for (uint64_t i = 0; i < n; ++i) {
            *b[i]->out_flag = flag[i];
            if (b[i]->out32) memcpy(b[i]->out32, &vals[32 * i], 32);
        }
    return rc;
}

// With c->mu held by lk: become the flusher, run batches until the queue is
// empty or `until` is done (its caller's request), then hand over.
static void flush(rf_coalescer* c, std::unique_lock<std::mutex>& lk, const Req* until) {
    c->flushing = true;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(c->max_wait_us);
    c->cv_more.wait_until(lk, deadline, [&] { return c->pending.size() >= c->max_batch; });
    std::vector<Req*> b;
    if (c->pending.size() <= c->max_batch) {
        b.swap(c->pending);
    } else {  // the oldest max_batch; the rest wait for the next flush
        b.assign(c->pending.begin(), c->pending.begin() + c->max_batch);
        c->pending.erase(c->pending.begin(), c->pending.begin() + c->max_batch);
    }
    lk.unlock();
    const int rc = b.empty() ? RF_OK : run_batch(c, b);
    lk.lock();
    ++c->batches;
    c->requests += b.size();
    if (b.size() > c->largest) c->largest = b.size();
    for (Req* r : b) {
        r->rc = rc;
        r->done = true;
    }
    c->flushing = false;
    c->cv_done.notify_all();  // results, and a pending caller may take over the next flush
    (void)until;
}

// Block until r is done, flushing whenever nobody else is.
static int wait_req(rf_coalescer* c, std::unique_lock<std::mutex>& lk, Req* r) {
    while (!r->done) {
        if (!c->flushing) {
            flush(c, lk, r);
        } else {
            c->cv_done.wait(lk);
        }
    }
    return r->rc;
}

static Req* enqueue(rf_coalescer* c, std::unique_lock<std::mutex>& lk, Req* r) {
    (void)lk;
    c->pending.push_back(r);
    if (c->pending.size() >= c->max_batch) c->cv_more.notify_one();
    return r;
}

extern "C" int rf_coalescer_open(rf_ctx* ctx, int kind, void* target, int assoc_kind, uint64_t max_batch,
                                 uint64_t max_wait_us, rf_coalescer** out) {
    ARG(ctx && out, "null argument");
    ARG(kind == RF_COALESCE_SHA256 || kind == RF_COALESCE_PROBE || kind == RF_COALESCE_ASSOC_GET,
        "unknown coalescer kind");
    ARG(kind == RF_COALESCE_SHA256 || target, "probe / assoc coalescers need their filter / table");
    ARG(max_batch >= 1, "max_batch must be >= 1");
    auto* c = new rf_coalescer();
    c->kind = kind;
    c->ctx = ctx;
    if (kind == RF_COALESCE_PROBE) c->bloom = static_cast<rf_bloom*>(target);
    if (kind == RF_COALESCE_ASSOC_GET) c->assoc = static_cast<rf_assoc*>(target);
    c->assoc_kind = assoc_kind;
    c->max_batch = max_batch;
    c->max_wait_us = max_wait_us;
    *out = c;
    return RF_OK;
}

extern "C" void rf_coalescer_close(rf_coalescer* c) {
    if (!c) return;
    {
        // drain: a caller still blocked in the queue finishes first
        std::unique_lock<std::mutex> lk(c->mu);
        while (!c->pending.empty() || c->flushing) {
            if (!c->flushing) flush(c, lk, nullptr);
            else c->cv_done.wait(lk);
        }
    }
    delete c;
}

extern "C" int rf_coalesce_sha256(rf_coalescer* c, const uint8_t* msg, uint64_t len, uint8_t* out32) {
    ARG(c && out32 && (len == 0 || msg), "null argument");
    ARG(c->kind == RF_COALESCE_SHA256, "not a SHA-256 coalescer");
    Req r;
    r.in = msg;
    r.len = len;
    r.out32 = out32;
    std::unique_lock<std::mutex> lk(c->mu);
    enqueue(c, lk, &r);
    return wait_req(c, lk, &r);
}

extern "C" int rf_coalesce_probe(rf_coalescer* c, const uint8_t* digest32, uint8_t* contains) {
    ARG(c && digest32 && contains, "null argument");
    ARG(c->kind == RF_COALESCE_PROBE, "not a probe coalescer");
    Req r;
    r.in = digest32;
    r.out_flag = contains;
    std::unique_lock<std::mutex> lk(c->mu);
    enqueue(c, lk, &r);
    return wait_req(c, lk, &r);
}

extern "C" int rf_coalesce_assoc_get(rf_coalescer* c, const uint8_t* key32, uint8_t* val32, uint8_t* found) {
    ARG(c && key32 && val32 && found, "null argument");
    ARG(c->kind == RF_COALESCE_ASSOC_GET, "not an assoc coalescer");
    Req r;
    r.in = key32;
    r.out32 = val32;
    r.out_flag = found;
    std::unique_lock<std::mutex> lk(c->mu);
    enqueue(c, lk, &r);
    return wait_req(c, lk, &r);
}

// ---- async: a ticket per request ---------------------------------------------
struct rf_coalesce_ticket {
    Req r;
};

extern "C" int rf_coalesce_sha256_async(rf_coalescer* c, const uint8_t* msg, uint64_t len, uint8_t* out32,
                                        rf_coalesce_ticket** out) {
    ARG(c && out32 && out && (len == 0 || msg), "null argument");
    ARG(c->kind == RF_COALESCE_SHA256, "not a SHA-256 coalescer");
    auto* t = new rf_coalesce_ticket();
    t->r.in = msg;
    t->r.len = len;
    t->r.out32 = out32;
    t->r.async = true;
    std::unique_lock<std::mutex> lk(c->mu);
    enqueue(c, lk, &t->r);
    *out = t;
    return RF_OK;
}

extern "C" int rf_coalesce_poll(rf_coalescer* c, rf_coalesce_ticket* t, int* done) {
    ARG(c && t && done, "null argument");
    std::unique_lock<std::mutex> lk(c->mu);
    // nobody flushing and this request still queued: it will not complete on
    // its own, so a poll that finds it so flushes without waiting for more
    if (!t->r.done && !c->flushing && !c->pending.empty()) {
        const uint64_t w = c->max_wait_us;
        c->max_wait_us = 0;
        flush(c, lk, &t->r);
        c->max_wait_us = w;
    }
    *done = t->r.done ? 1 : 0;
    return t->r.done ? t->r.rc : RF_OK;
}

extern "C" int rf_coalesce_wait(rf_coalescer* c, rf_coalesce_ticket* t) {
    ARG(c && t, "null argument");
    std::unique_lock<std::mutex> lk(c->mu);
    return wait_req(c, lk, &t->r);
}

extern "C" void rf_coalesce_ticket_free(rf_coalescer* c, rf_coalesce_ticket* t) {
    if (!t) return;
    if (c) {  // still queued: complete it first (the queue holds its address)
        std::unique_lock<std::mutex> lk(c->mu);
        (void)wait_req(c, lk, &t->r);
    }
    delete t;
}

extern "C" int rf_coalescer_stats(rf_coalescer* c, uint64_t* batches, uint64_t* requests, uint64_t* largest) {
    ARG(c, "null coalescer");
    std::lock_guard<std::mutex> lk(c->mu);
    if (batches) *batches = c->batches;
    if (requests) *requests = c->requests;
    if (largest) *largest = c->largest;
    return RF_OK;
}
