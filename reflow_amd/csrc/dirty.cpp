// dirty.cpp -- Eval.dirty for a whole Flow graph (rf_flow_dirty), on K3's
// reachability kernel (k3_reach.hip).
#include <hip/hip_runtime.h>
#include <string.h>

#include <vector>

#include "ctx.h"
#include "engine.h"

using namespace rf;

extern "C" int rf_flow_dirty(rf_ctx* ctx, uint64_t n, const uint64_t* dep_ptr, const uint32_t* deps,
                             const uint8_t* is_extern, int no_cache_extern, uint8_t* dirty) {
    ARG(ctx && (n == 0 || (dep_ptr && is_extern && dirty)), "null argument");
    ARG(n < (1ull << 32), "too many nodes");
    if (!n) return RF_OK;
    // eval.go:875-877: without NoCacheExtern nothing is dirty
    if (!no_cache_extern) {
        memset(dirty, 0, n);
        return RF_OK;
    }
    ARG(dep_ptr[0] == 0, "dep_ptr[0] must be 0");
    const uint64_t E = dep_ptr[n];
    ARG(E == 0 || deps, "null deps");
    // reverse edges: dep -> the nodes that list it (consumers)
    std::vector<uint64_t> cptr(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) {
        ARG(dep_ptr[i] <= dep_ptr[i + 1], "dep_ptr not monotone");
        for (uint64_t e = dep_ptr[i]; e < dep_ptr[i + 1]; ++e) {
            if (deps[e] >= n) return fail(RF_EINVAL, "node %llu: dep %u out of range", (unsigned long long)i, deps[e]);
            cptr[deps[e] + 1]++;
        }
    }
    for (uint64_t i = 0; i < n; ++i) cptr[i + 1] += cptr[i];
    std::vector<uint32_t> cons(std::max<uint64_t>(E, 1));
    {
        std::vector<uint64_t> fill(cptr.begin(), cptr.end() - 1);
        for (uint64_t i = 0; i < n; ++i)
            for (uint64_t e = dep_ptr[i]; e < dep_ptr[i + 1]; ++e) cons[fill[deps[e]]++] = (uint32_t)i;
    }
    std::vector<uint32_t> seed;
    const uint64_t nw = (n + 31) / 32;
    std::vector<uint32_t> bits(nw, 0);
    for (uint64_t i = 0; i < n; ++i)
        if (is_extern[i]) {  // eval.go:878-880
            seed.push_back((uint32_t)i);
            bits[i >> 5] |= 1u << (i & 31);
        }
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    hipStream_t s = ctx->stream;
    // scratch: cons_ptr, cons, bits, two frontiers, counter
    DevBuf b_ptr, b_cons, b_bits, b_f0, b_f1, b_cnt;
    struct Free {
        DevBuf* b[6];
        ~Free() {
            for (DevBuf* x : b) x->release();
        }
    } free_all{{&b_ptr, &b_cons, &b_bits, &b_f0, &b_f1, &b_cnt}};
    HIPC(b_ptr.ensure(8 * (n + 1)));
    HIPC(b_cons.ensure(4 * cons.size()));
    HIPC(b_bits.ensure(4 * nw));
    HIPC(b_f0.ensure(4 * n));
    HIPC(b_f1.ensure(4 * n));
    HIPC(b_cnt.ensure(64));
    HIPC(hipMemcpyAsync(b_ptr.p, cptr.data(), 8 * (n + 1), hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(b_cons.p, cons.data(), 4 * cons.size(), hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(b_bits.p, bits.data(), 4 * nw, hipMemcpyHostToDevice, s));
    if (!seed.empty()) HIPC(hipMemcpyAsync(b_f0.p, seed.data(), 4 * seed.size(), hipMemcpyHostToDevice, s));
    uint32_t n_front = (uint32_t)seed.size();
    uint32_t* f0 = b_f0.as<uint32_t>();
    uint32_t* f1 = b_f1.as<uint32_t>();
    while (n_front) {  // one level per launch: a dep's consumers are marked
        HIPC(hipMemsetAsync(b_cnt.p, 0, 4, s));
        HIPC(launch_reach_step(f0, n_front, b_ptr.as<uint64_t>(), b_cons.as<uint32_t>(), b_bits.as<uint32_t>(), f1,
                               b_cnt.as<uint32_t>(), s));
        HIPC(hipMemcpyAsync(&n_front, b_cnt.p, 4, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        std::swap(f0, f1);
    }
    HIPC(hipMemcpyAsync(bits.data(), b_bits.p, 4 * nw, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    for (uint64_t i = 0; i < n; ++i) dirty[i] = (bits[i >> 5] >> (i & 31)) & 1;
    return RF_OK;
}
