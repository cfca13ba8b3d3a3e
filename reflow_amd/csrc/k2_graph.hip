// k2_graph.hip -- K2/K3: level-synchronous incremental digest DAG.
//
// Replaces the recursive, sync.Once-memoized Flow.Digest / WriteDigest of
// /root/reference/flow.go:653-750, PhysicalDigest :764-792 and CacheKeys
// :796-802.  The reference recomputes every digest of a fresh Eval
// (eval.go:240-272 -> Canonicalize flow.go:814-843); here only the transitive
// dependents of changed inputs are rehashed.
//
// Data layout in HBM (DESIGN.md "Data layout"):
//   tmpl      per job, its digest material with SHA padding already applied
//             (64-B aligned, nblk*64 bytes); WD holes carry the 0x00 0x05
//             prefix and 32 bytes that are rewritten from the slot table.
//   meta      32-B job record (template offset, blocks, hole range, out slot,
//             consumer range): two 16-B loads per job.
//   holes     {byte position, slot} pairs.
//   slots     [S][32] digest table (node digests, physical keys, File IDs).
//   dirty     bitset over jobs in level order.
//   cons      slot -> consumer jobs (reverse edges for the frontier).
// Per level: k3_compact turns the level's dirty bits into a dense job list,
// then k2_hash gives each listed job one lane: patch holes from the slot
// table, hash the padded template, write the slot and -- only if the digest
// changed -- atomicOr the consumers' dirty bits (early cut-off).  A fused
// per-workgroup compaction was measured 4x slower on the incremental step:
// small, heavy levels (the wide K) got too few workgroups.
#include "engine.h"
#include "sha256_dev.h"

namespace rf {

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v += t;
    }
    return v;
}

// Write the 32 digest bytes D (as 8 little-endian words) at byte `pos` of a
// 4-B aligned buffer, preserving the neighbouring bytes.
__device__ __forceinline__ void patch_digest(uint32_t* wb, uint32_t pos, const uint32_t (&D)[8]) {
    const uint32_t w0 = pos >> 2, s = pos & 3;
    if (s == 0) {
#pragma unroll
        for (int m = 0; m < 8; ++m) wb[w0 + m] = D[m];
    } else {
        const uint32_t sh = 8 * s, keep = (1u << sh) - 1u;
        wb[w0] = (wb[w0] & keep) | (D[0] << sh);
#pragma unroll
        for (int m = 1; m < 8; ++m) wb[w0 + m] = (D[m - 1] >> (32 - sh)) | (D[m] << sh);
        wb[w0 + 8] = (wb[w0 + 8] & ~keep) | (D[7] >> (32 - sh));
    }
}

struct LevelArgs {
    uint32_t s, e, lvl;  // internal job range of the level
    int full;
    const uint4* meta;
    const uint2* holes;
    const uint32_t* cons_job;
    uint8_t* tmpl;
    uint8_t* slots;
    uint32_t* dirty;
    uint32_t* counts;
};

__device__ __forceinline__ void hash_job(const LevelArgs& a, uint32_t p) {
    const uint4 m0 = a.meta[2 * p], m1 = a.meta[2 * p + 1];
    uint8_t* t = a.tmpl + 64ull * m0.x;
    uint32_t* tw = reinterpret_cast<uint32_t*>(t);
    // 1. patch holes from the slot table
    for (uint32_t h = m0.z; h < m0.w; ++h) {
        const uint2 hp = a.holes[h];
        const uint4* src = reinterpret_cast<const uint4*>(a.slots + 32ull * hp.y);
        const uint4 lo = src[0], hi = src[1];
        const uint32_t D[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        patch_digest(tw, hp.x, D);
    }
    // 2. hash the padded template (full blocks only)
    ShaState st;
    st.init();
    const uint4* q = reinterpret_cast<const uint4*>(t);
    for (uint32_t b = 0; b < m0.y; ++b) {
        const uint4 r0 = q[4 * b], r1 = q[4 * b + 1], r2 = q[4 * b + 2], r3 = q[4 * b + 3];
        uint32_t w[16] = {bswap32(r0.x), bswap32(r0.y), bswap32(r0.z), bswap32(r0.w),
                          bswap32(r1.x), bswap32(r1.y), bswap32(r1.z), bswap32(r1.w),
                          bswap32(r2.x), bswap32(r2.y), bswap32(r2.z), bswap32(r2.w),
                          bswap32(r3.x), bswap32(r3.y), bswap32(r3.z), bswap32(r3.w)};
        sha256_compress(st, w);
    }
    uint4 nlo, nhi;
    nlo.x = bswap32(st.h[0]); nlo.y = bswap32(st.h[1]); nlo.z = bswap32(st.h[2]); nlo.w = bswap32(st.h[3]);
    nhi.x = bswap32(st.h[4]); nhi.y = bswap32(st.h[5]); nhi.z = bswap32(st.h[6]); nhi.w = bswap32(st.h[7]);
    // 3. store; propagate only on change (early cut-off)
    uint4* dst = reinterpret_cast<uint4*>(a.slots + 32ull * m1.x);
    bool changed = true;
    if (!a.full) {
        const uint4 olo = dst[0], ohi = dst[1];
        changed = (olo.x != nlo.x) | (olo.y != nlo.y) | (olo.z != nlo.z) | (olo.w != nlo.w) |
                  (ohi.x != nhi.x) | (ohi.y != nhi.y) | (ohi.z != nhi.z) | (ohi.w != nhi.w);
    }
    if (changed) {
        dst[0] = nlo;
        dst[1] = nhi;
        if (!a.full) {
            for (uint32_t c = m1.y; c < m1.z; ++c) {
                const uint32_t j = a.cons_job[c];
                atomicOr(&a.dirty[j >> 5], 1u << (j & 31));
            }
        }
    }
}

// K3: compact the dirty jobs of the level's range [s, e) into a dense global
// list (wave popcount prefix, one atomic per wave) so K2 gets one full lane
// per dirty job whatever the dirty density (2% on an incremental step).
__global__ __launch_bounds__(256) void k3_compact(const uint32_t* __restrict__ dirty, uint32_t s,
                                                  uint32_t e, uint32_t* __restrict__ list,
                                                  uint32_t* __restrict__ counts, uint32_t lvl) {
    const uint32_t w_lo = s >> 5, w_hi = (e + 31) >> 5;
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = blockIdx.x * blockDim.x; base < (w_hi - w_lo); base += gridDim.x * blockDim.x) {
        const uint32_t wi = w_lo + base + threadIdx.x;
        uint32_t bits = 0;
        if (wi < w_hi) {
            bits = dirty[wi];
            const uint32_t first = wi << 5;
            if (first < s) bits &= ~0u << (s - first);
            if (first + 32 > e) bits &= (e - first >= 32) ? ~0u : ((1u << (e - first)) - 1u);
        }
        const uint32_t c = __popc(bits);
        const uint32_t incl = wave_incl_scan(c);
        const uint32_t total = __shfl(incl, 63, 64);
        uint32_t wbase = 0;
        if (lane == 63 && total) wbase = atomicAdd(&counts[lvl], total);
        wbase = __shfl(wbase, 63, 64);
        uint32_t pos = wbase + incl - c;
        while (bits) {
            const uint32_t b = __ffs(bits) - 1;
            bits &= bits - 1;
            list[pos++] = (wi << 5) + b;
        }
    }
}

// K2: one lane per listed job of the level.
__global__ __launch_bounds__(256) void k2_hash(LevelArgs a, const uint32_t* __restrict__ list) {
    const uint32_t n = a.counts[a.lvl];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        hash_job(a, list[i]);
}

// set_slots: write input digests, dirty their consumers when they changed.
__global__ __launch_bounds__(256) void k3_mark_slots(const uint32_t* __restrict__ sl,
                                                     const uint8_t* __restrict__ dig, uint32_t n,
                                                     uint8_t* slots, const uint32_t* cons_ptr,
                                                     const uint32_t* cons_job, uint32_t* dirty) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t s = sl[i];
        const uint4* src = reinterpret_cast<const uint4*>(dig + 32ull * i);
        uint4* dst = reinterpret_cast<uint4*>(slots + 32ull * s);
        const uint4 nlo = src[0], nhi = src[1], olo = dst[0], ohi = dst[1];
        const bool changed = (olo.x != nlo.x) | (olo.y != nlo.y) | (olo.z != nlo.z) |
                             (olo.w != nlo.w) | (ohi.x != nhi.x) | (ohi.y != nhi.y) |
                             (ohi.z != nhi.z) | (ohi.w != nhi.w);
        if (changed) {
            dst[0] = nlo;
            dst[1] = nhi;
            for (uint32_t c = cons_ptr[s]; c < cons_ptr[s + 1]; ++c) {
                const uint32_t j = cons_job[c];
                atomicOr(&dirty[j >> 5], 1u << (j & 31));
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_gather_slots(const uint8_t* __restrict__ slots,
                                                      const uint32_t* __restrict__ idx, uint32_t n,
                                                      uint8_t* __restrict__ out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint4* src = reinterpret_cast<const uint4*>(slots + 32ull * idx[i]);
        uint4* dst = reinterpret_cast<uint4*>(out + 32ull * i);
        dst[0] = src[0];
        dst[1] = src[1];
    }
}

// OR of nranks gathered copies of an nwords bitset (RCCL has no bitwise OR).
__global__ __launch_bounds__(256) void k_or_reduce(const uint64_t* __restrict__ g, uint64_t nwords,
                                                   int nranks, uint64_t* __restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nwords;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t v = 0;
        for (int r = 0; r < nranks; ++r) v |= g[(uint64_t)r * nwords + i];
        out[i] = v;
    }
}

static uint32_t grid_for(uint64_t items, uint32_t cap) {
    uint64_t g = (items + 255) / 256;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (uint32_t)g;
}

hipError_t launch_graph_mark_slots(const GraphDev& g, const uint32_t* slots, const uint8_t* digests,
                                   uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k3_mark_slots, dim3(grid_for(n, 4096)), dim3(256), 0, s, slots, digests, n,
                       g.slots, g.cons_ptr, g.cons_job, g.dirty);
    return hipGetLastError();
}

hipError_t launch_graph_level(const GraphDev& g, uint32_t lvl, int full, hipStream_t s) {
    const uint32_t b = g.lvl_start[lvl], e = g.lvl_start[lvl + 1];
    if (e <= b) return hipSuccess;
    const uint32_t words = ((e + 31) >> 5) - (b >> 5);
    hipLaunchKernelGGL(k3_compact, dim3(grid_for(words, 2048)), dim3(256), 0, s, g.dirty, b, e, g.list,
                       g.counts, lvl);
    LevelArgs a{b, e, lvl, full, g.meta, g.holes, g.cons_job, g.tmpl, g.slots, g.dirty, g.counts};
    hipLaunchKernelGGL(k2_hash, dim3(grid_for(e - b, 16384)), dim3(256), 0, s, a, g.list);
    return hipGetLastError();
}

hipError_t launch_or_reduce(const uint64_t* gathered, uint64_t nwords, int nranks, uint64_t* out,
                            hipStream_t s) {
    if (!nwords) return hipSuccess;
    hipLaunchKernelGGL(k_or_reduce, dim3(grid_for(nwords, 4096)), dim3(256), 0, s, gathered, nwords,
                       nranks, out);
    return hipGetLastError();
}

hipError_t launch_gather_slots(const uint8_t* slots, const uint32_t* idx, uint32_t n, uint8_t* out,
                               hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather_slots, dim3(grid_for(n, 4096)), dim3(256), 0, s, slots, idx, n, out);
    return hipGetLastError();
}

}  // namespace rf
