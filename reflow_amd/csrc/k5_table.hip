// k5_table.hip -- K5: digest-keyed hash table in HBM (Canonicalize's flowMap).
//
// Replaces the mutex-guarded map[digest.Digest]*Flow of flowMap.Get/Put
// (/root/reference/flow.go:881-907) that Flow.Canonicalize (:814-843) fills
// node by node: semantically equal flows (same Flow.Digest) collapse into the
// first one Put.  Batched: every node digest (numbered in canonicalize's
// post-order, which is the order of its Puts) is inserted at once; a node's
// canonical representative is the smallest index with its digest, which is the
// node the reference's first Put registers (DESIGN.md K5 argues why skipped
// subtrees never hold that minimum).
//
// Layout: open addressing, linear probing, a power-of-two table of u32 node
// indices (empty = ~0), at most half full.  The probe start is the digest's
// first 8 bytes (SHA-256 output: uniform), and a slot whose index points at an
// equal 32-B digest is a hit -- slots store indices, the digests stay in their
// input array, so an insert is: one slot read, one CAS (or an atomicMin on a
// hit), one 32-B compare read.  All of it is random access: the bound is the
// random-gather rate, not HBM bandwidth.
#include "engine.h"

namespace rf {

constexpr uint32_t kEmpty = 0xffffffffu;

__device__ __forceinline__ bool dig_eq(const uint4& alo, const uint4& ahi, const uint8_t* b) {
    const uint4* q = reinterpret_cast<const uint4*>(b);
    const uint4 blo = q[0], bhi = q[1];
    return ((alo.x ^ blo.x) | (alo.y ^ blo.y) | (alo.z ^ blo.z) | (alo.w ^ blo.w) | (ahi.x ^ bhi.x) |
            (ahi.y ^ bhi.y) | (ahi.z ^ bhi.z) | (ahi.w ^ bhi.w)) == 0;
}

// Insert node i; slot_of[i] = the slot that holds its digest class.  A slot's
// value only ever moves from empty to an index and then down (atomicMin), and
// every index a slot ever holds has the slot's digest, so a stale read of a
// non-empty slot still names the right class.
__global__ __launch_bounds__(256) void k5_dedup_insert(const uint8_t* __restrict__ dig, uint32_t n,
                                                       uint32_t* __restrict__ table, uint32_t mask,
                                                       uint32_t* __restrict__ slot_of) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint4* d = reinterpret_cast<const uint4*>(dig + 32ull * i);
        const uint4 lo = d[0], hi = d[1];
        uint32_t slot = lo.x & mask;
        for (;;) {
            uint32_t cur = __hip_atomic_load(&table[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == kEmpty) {
                cur = atomicCAS(&table[slot], kEmpty, i);
                if (cur == kEmpty) break;  // claimed: this node opens its class
            }
            if (dig_eq(lo, hi, dig + 32ull * cur)) {
                if (i < cur) atomicMin(&table[slot], i);
                break;
            }
            slot = (slot + 1) & mask;
        }
        slot_of[i] = slot;
    }
}

__global__ __launch_bounds__(256) void k5_dedup_resolve(uint32_t n, const uint32_t* __restrict__ table,
                                                        const uint32_t* __restrict__ slot_of,
                                                        uint32_t* __restrict__ canon,
                                                        uint32_t* __restrict__ n_unique) {
    // one counter word takes ~88 atomics/us (MI355X_MICROARCH "dequeue"): count
    // per thread over the grid-stride loop, one atomicAdd per block
    __shared__ uint32_t s_w[4];
    uint32_t uniq = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t c = table[slot_of[i]];
        canon[i] = c;
        uniq += c == i;
    }
    for (int o = 32; o > 0; o >>= 1) uniq += __shfl_xor(uniq, o, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = uniq;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        if (t) atomicAdd(n_unique, t);
    }
}

uint32_t dedup_table_slots(uint32_t n) {
    uint32_t cap = 64;
    while (cap < 2ull * n && cap < (1u << 31)) cap <<= 1;
    return cap;
}

hipError_t launch_dedup(const uint8_t* dig, uint32_t n, uint32_t* table, uint32_t* slot_of, uint32_t* canon,
                        uint32_t* n_unique, hipStream_t s) {
    const uint32_t cap = dedup_table_slots(n);
    hipError_t e = hipMemsetAsync(table, 0xff, 4ull * cap, s);
    if (e == hipSuccess) e = hipMemsetAsync(n_unique, 0, 4, s);
    if (e != hipSuccess || n == 0) return e;
    uint32_t grid = (n + 255) / 256;
    if (grid > 16384) grid = 16384;
    hipLaunchKernelGGL(k5_dedup_insert, dim3(grid), dim3(256), 0, s, dig, n, table, cap - 1, slot_of);
    hipLaunchKernelGGL(k5_dedup_resolve, dim3(grid < 2048 ? grid : 2048), dim3(256), 0, s, n, table, slot_of,
                       canon, n_unique);
    return hipGetLastError();
}

}  // namespace rf
