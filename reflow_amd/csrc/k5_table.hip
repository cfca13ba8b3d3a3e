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
// indices (empty = ~0), at most half full.  The probe start is key_hash of
// all eight digest words, and a slot whose index points at an
// equal 32-B digest is a hit -- slots store indices, the digests stay in their
// input array, so an insert is: one slot read, one CAS (or an atomicMin on a
// hit), one 32-B compare read.  All of it is random access: the bound is the
// random-gather rate, not HBM bandwidth.
#include "engine.h"

namespace rf {

constexpr uint32_t kEmpty = 0xffffffffu;
constexpr uint32_t kMaxProbe = 1u << 16;

// 32-bit slot hash over all eight words of a 32-B key.  Each word enters
// through an xor with a rotated partner and an odd multiply (bijections), so
// two keys that differ in any single word never share a pre-finaliser value,
// and the finaliser (also a bijection) spreads them over the low bits.  Keys
// are usually SHA-256 output (any word would do), but callers may hand in
// digests that share all but a few bytes.
__device__ __forceinline__ uint32_t key_hash(const uint4& lo, const uint4& hi) {
    uint32_t h = ((lo.x ^ __builtin_rotateleft32(lo.y, 5)) * 0x9E3779B1u) ^
                 ((lo.z ^ __builtin_rotateleft32(lo.w, 11)) * 0x85EBCA77u) ^
                 ((hi.x ^ __builtin_rotateleft32(hi.y, 17)) * 0xC2B2AE3Du) ^
                 ((hi.z ^ __builtin_rotateleft32(hi.w, 23)) * 0x27D4EB2Fu);
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    return h;
}

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
        uint32_t slot = key_hash(lo, hi) & mask;
        // bounded probing: the table is >= 2n slots (load <= 1/2), where
        // linear probing's runs are a few slots long; the bound guarantees
        // that every wave exits, and a batch that hits it is flagged
        uint32_t probes = 0;
        for (;; ++probes) {
            if (probes >= kMaxProbe) {
                slot = kEmpty;
                break;
            }
            uint32_t cur = __hip_atomic_load(&table[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == kEmpty) {
                cur = atomicCAS(&table[slot], kEmpty, i);
                if (cur == kEmpty) break;  // claimed: this node opens its class
            }
            if (cur >= n) {  // not an index of this batch: the table was not cleared
                slot = kEmpty;
                break;
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
        const uint32_t so = slot_of[i];
        if (so == kEmpty) {  // insert gave up (see k5_dedup_insert): flag the batch
            canon[i] = kEmpty;
            atomicOr(n_unique, 0x80000000u);
            continue;
        }
        const uint32_t c = table[so];
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

__global__ __launch_bounds__(256) void k5_fill_u32(uint32_t* __restrict__ p, uint32_t v, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

hipError_t launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    uint64_t g = (n + 255) / 256;
    hipLaunchKernelGGL(k5_fill_u32, dim3((uint32_t)(g > 16384 ? 16384 : g)), dim3(256), 0, s, p, v, n);
    return hipGetLastError();
}

hipError_t launch_dedup(const uint8_t* dig, uint32_t n, uint32_t* table, uint32_t* slot_of, uint32_t* canon,
                        uint32_t* n_unique, hipStream_t s, bool clear_table) {
    const uint32_t cap = dedup_table_slots(n);
    hipError_t e = clear_table ? hipMemsetAsync(table, 0xff, 4ull * cap, s) : hipSuccess;
    if (e == hipSuccess) e = hipMemsetAsync(n_unique, 0, 4, s);
    if (e != hipSuccess || n == 0) return e;
    uint32_t grid = (n + 255) / 256;
    if (grid > 16384) grid = 16384;
    hipLaunchKernelGGL(k5_dedup_insert, dim3(grid), dim3(256), 0, s, dig, n, table, cap - 1, slot_of);
    hipLaunchKernelGGL(k5_dedup_resolve, dim3(grid < 2048 ? grid : 2048), dim3(256), 0, s, n, table, slot_of,
                       canon, n_unique);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// HBM-resident assoc (assoc.Assoc, assoc/assoc.go:26-38) with the in-memory
// implementation's semantics (test/testutil/assoc.go:34-56): (kind, key) ->
// value; Put with a nonzero `expect` is a compare-and-set, a zero value
// deletes.  Table: open addressing on key_hash(key), a tag word per
// slot (0 empty, 1 being written, 2 + kind ready), keys and values 32 B each.
// Deleted entries keep their slot with a zero value (Get: NotExist).
constexpr uint32_t kTagEmpty = 0, kTagBusy = 1, kTagReady = 2;



// Add a per-thread count to a global counter: one atomic per wave.  Called by
// every lane of the wave after its grid-stride loop (converged).
__device__ __forceinline__ void wave_count_add(uint32_t* counter, uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(counter, v);
}

__device__ __forceinline__ bool key_eq(const uint4* k, const uint4& lo, const uint4& hi) {
    const uint4 a = k[0], b = k[1];
    return ((a.x ^ lo.x) | (a.y ^ lo.y) | (a.z ^ lo.z) | (a.w ^ lo.w) | (b.x ^ hi.x) | (b.y ^ hi.y) |
            (b.z ^ hi.z) | (b.w ^ hi.w)) == 0;
}

// Insert (or find) the batch's DISTINCT keys (canon[i] == i).  A slot is
// claimed empty -> busy with one CAS and its key written with plain stores --
// no per-slot fences (an acquire load + release store per insert, a cache
// invalidate and a store drain each, made a 1e8-key Put 234 ms).  A busy slot
// is a key of this launch, never this lane's (the batch's keys are distinct),
// so it is skipped without reading its key, which another XCD's L2 may not
// show yet; k5_assoc_publish turns this launch's claims into ready tags after
// the kernel boundary.  slot_of[i] carries bit 31 for a claim.
__global__ __launch_bounds__(256) void k5_assoc_insert(AssocView t, uint32_t kind, const uint8_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ canon, uint32_t n,
                                                       uint32_t* __restrict__ slot_of) {
    const uint32_t ready = kTagReady + kind;
    uint32_t added = 0;  // one atomicAdd per wave: a single counter word serialises ~88 atomics/us
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (canon[i] != i) continue;
        const uint4* k = reinterpret_cast<const uint4*>(keys + 32ull * i);
        const uint4 lo = k[0], hi = k[1];
        uint32_t slot = key_hash(lo, hi) & t.mask, mark = 0;
        for (;;) {
            uint32_t tg = __hip_atomic_load(&t.tag[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tg == kTagEmpty) {
                tg = atomicCAS(&t.tag[slot], kTagEmpty, kTagBusy);
                if (tg == kTagEmpty) {
                    t.keys[2 * slot] = lo;
                    t.keys[2 * slot + 1] = hi;
                    t.vals[2 * slot] = make_uint4(0, 0, 0, 0);
                    t.vals[2 * slot + 1] = make_uint4(0, 0, 0, 0);
                    ++added;
                    mark = 0x80000000u;
                    break;
                }
            }
            // ready tags were set by earlier launches: their keys are visible
            if (tg == ready && key_eq(&t.keys[2 * slot], lo, hi)) break;
            slot = (slot + 1) & t.mask;
        }
        slot_of[i] = slot | mark;
    }
    wave_count_add(t.count, added);
}

// The insert launch's claims become ready (and slot_of plain slot indices).
__global__ __launch_bounds__(256) void k5_assoc_publish(AssocView t, uint32_t kind, const uint32_t* __restrict__ canon,
                                                        uint32_t n, uint32_t* __restrict__ slot_of) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (canon[i] != i) continue;
        const uint32_t so = slot_of[i];
        if (so & 0x80000000u) {
            t.tag[so & 0x7fffffffu] = kTagReady + kind;
            slot_of[i] = so & 0x7fffffffu;
        }
    }
}

__device__ __forceinline__ uint32_t assoc_find(const AssocView& t, uint32_t kind, const uint4& lo, const uint4& hi) {
    const uint32_t ready = kTagReady + kind;
    uint32_t slot = key_hash(lo, hi) & t.mask;
    for (;;) {
        const uint32_t tg = t.tag[slot];
        if (tg == kTagEmpty) return kEmpty;
        if (tg == ready && key_eq(&t.keys[2 * slot], lo, hi)) return slot;
        slot = (slot + 1) & t.mask;
    }
}

// One round of a Put batch: every remaining op claims its key's class with
// atomicMax((round << 32) | ~i) -- the smallest index of the class wins the
// round -- then winners apply in index order across rounds.
__global__ __launch_bounds__(256) void k5_assoc_claim(const uint32_t* __restrict__ rem, const uint32_t* __restrict__ n_rem,
                                                      const uint32_t* __restrict__ canon,
                                                      unsigned long long* __restrict__ cls, uint32_t round) {
    const uint32_t n = *n_rem;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
        const uint32_t i = rem[q];
        if (canon[i] == kEmpty) continue;  // never reached: the host stops a flagged batch
        atomicMax(&cls[canon[i]],((unsigned long long)round << 32) | (unsigned long long)(~i));
    }
}

__global__ __launch_bounds__(256) void k5_assoc_apply(AssocView t, const uint32_t* __restrict__ rem,
                                                      const uint32_t* __restrict__ n_rem,
                                                      const uint32_t* __restrict__ canon,
                                                      const unsigned long long* __restrict__ cls, uint32_t round,
                                                      const uint32_t* __restrict__ slot_of,
                                                      const uint8_t* __restrict__ expect, const uint8_t* __restrict__ vals,
                                                      int32_t* __restrict__ status, uint32_t* __restrict__ next,
                                                      uint32_t* __restrict__ n_next) {
    const uint32_t n = *n_rem;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
        const uint32_t i = rem[q];
        const uint32_t c = canon[i];
        if (c == kEmpty) continue;
        if (cls[c] !=(((unsigned long long)round << 32) | (unsigned long long)(~i))) {
            next[atomicAdd(n_next, 1u)] = i;  // a later op of the same key: next round
            continue;
        }
        const uint32_t slot = slot_of[c];
        uint4* v = &t.vals[2 * slot];
        if (expect) {
            const uint4* e = reinterpret_cast<const uint4*>(expect + 32ull * i);
            const uint4 elo = e[0], ehi = e[1];
            const bool nz = (elo.x | elo.y | elo.z | elo.w | ehi.x | ehi.y | ehi.z | ehi.w) != 0;
            if (nz && !key_eq(v, elo, ehi)) {  // testutil/assoc.go:38-40
                status[i] = 7;                 // RF_EPRECONDITION
                continue;
            }
        }
        const uint4* nv = reinterpret_cast<const uint4*>(vals + 32ull * i);
        v[0] = nv[0];  // a zero value deletes (Get then reports NotExist)
        v[1] = nv[1];
        status[i] = 0;
    }
}

__global__ __launch_bounds__(256) void k5_assoc_get(AssocView t, uint32_t kind, const uint8_t* __restrict__ keys,
                                                    uint64_t n, uint8_t* __restrict__ vals, uint8_t* __restrict__ found) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4* k = reinterpret_cast<const uint4*>(keys + 32ull * i);
        const uint4 lo = k[0], hi = k[1];
        const uint32_t slot = assoc_find(t, kind, lo, hi);
        uint4 a = make_uint4(0, 0, 0, 0), b = a;
        if (slot != kEmpty) {
            a = t.vals[2 * slot];
            b = t.vals[2 * slot + 1];
        }
        uint4* o = reinterpret_cast<uint4*>(vals + 32ull * i);
        o[0] = a;
        o[1] = b;
        found[i] = (a.x | a.y | a.z | a.w | b.x | b.y | b.z | b.w) != 0;
    }
}

// Eval.lookup for a batch of nodes (eval.go:1202-1221): node i's cache keys
// are [key_ptr[i], key_ptr[i+1]) of a k5_assoc_get batch in CacheKeys order;
// the first key found wins.  One lane per node.
__global__ __launch_bounds__(256) void k5_assoc_select(const uint8_t* __restrict__ found,
                                                       const uint8_t* __restrict__ vals,
                                                       const uint64_t* __restrict__ key_ptr, uint64_t n,
                                                       int32_t* __restrict__ which, uint8_t* __restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = key_ptr[i], e = key_ptr[i + 1];
        int32_t w = -1;
        uint4 lo = make_uint4(0, 0, 0, 0), hi = lo;
        for (uint64_t k = b; k < e; ++k)
            if (found[k]) {
                w = (int32_t)(k - b);
                const uint4* v = reinterpret_cast<const uint4*>(vals + 32ull * k);
                lo = v[0];
                hi = v[1];
                break;
            }
        which[i] = w;
        uint4* o = reinterpret_cast<uint4*>(out + 32ull * i);
        o[0] = lo;
        o[1] = hi;
    }
}

// Abbreviated keys (dydbassoc.go:111-147: the ID4 index narrows, Expands
// decides): every live entry of the kind is compared with each of the q
// queries' first nhex hex digits; per query, the number of matches and one
// matching slot.
__global__ __launch_bounds__(256) void k5_assoc_abbrev(AssocView t, uint32_t kind, uint32_t cap,
                                                       const uint8_t* __restrict__ qkeys, const uint8_t* __restrict__ nhex,
                                                       uint32_t q, uint32_t* __restrict__ matches,
                                                       uint32_t* __restrict__ hit_slot) {
    const uint32_t ready = kTagReady + kind;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += gridDim.x * blockDim.x) {
        if (t.tag[s] != ready) continue;
        const uint4 vlo = t.vals[2 * s], vhi = t.vals[2 * s + 1];
        if ((vlo.x | vlo.y | vlo.z | vlo.w | vhi.x | vhi.y | vhi.z | vhi.w) == 0) continue;  // deleted
        const uint8_t* key = reinterpret_cast<const uint8_t*>(&t.keys[2 * s]);
        for (uint32_t j = 0; j < q; ++j) {
            const uint32_t nh = nhex[j];
            bool eq = true;
            for (uint32_t b = 0; b < nh / 2 && eq; ++b) eq = key[b] == qkeys[32 * j + b];
            if (eq && (nh & 1)) eq = (key[nh / 2] >> 4) == (qkeys[32 * j + nh / 2] >> 4);
            if (eq) {
                atomicAdd(&matches[j], 1u);
                hit_slot[j] = s;
            }
        }
    }
}

// Rehash every occupied slot into a larger (empty) table; keys are distinct.
__global__ __launch_bounds__(256) void k5_assoc_rehash(AssocView from, uint32_t cap_from, AssocView to) {
    uint32_t added = 0;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < cap_from; s += gridDim.x * blockDim.x) {
        const uint32_t tg = from.tag[s];
        if (tg < kTagReady) continue;
        const uint4 lo = from.keys[2 * s], hi = from.keys[2 * s + 1];
        // keys are distinct and nothing compares them in this launch: claim
        // the slot with its final tag, no fences (the kernel boundary publishes)
        uint32_t slot = key_hash(lo, hi) & to.mask;
        while (atomicCAS(&to.tag[slot], kTagEmpty, tg) != kTagEmpty) slot = (slot + 1) & to.mask;
        to.keys[2 * slot] = lo;
        to.keys[2 * slot + 1] = hi;
        to.vals[2 * slot] = from.vals[2 * s];
        to.vals[2 * slot + 1] = from.vals[2 * s + 1];
        ++added;
    }
    wave_count_add(to.count, added);
}

// rem[q] = q: a Put batch's first round holds every op, in index order
__global__ __launch_bounds__(256) void k5_iota(uint32_t* __restrict__ out, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = i;
}

static uint32_t grid256(uint64_t n) {
    uint64_t g = (n + 255) / 256;
    return (uint32_t)(g < 1 ? 1 : g > 16384 ? 16384 : g);
}

hipError_t launch_assoc_insert(const AssocView& t, uint32_t kind, const uint8_t* keys, const uint32_t* canon,
                               uint32_t n, uint32_t* slot_of, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k5_assoc_insert, dim3(grid256(n)), dim3(256), 0, s, t, kind, keys, canon, n, slot_of);
    hipLaunchKernelGGL(k5_assoc_publish, dim3(grid256(n)), dim3(256), 0, s, t, kind, canon, n, slot_of);
    return hipGetLastError();
}

hipError_t launch_assoc_round(const AssocView& t, const uint32_t* rem, const uint32_t* n_rem, uint32_t n_max,
                              const uint32_t* canon, unsigned long long* cls, uint32_t round,
                              const uint32_t* slot_of, const uint8_t* expect, const uint8_t* vals,
                              int32_t* status, uint32_t* next, uint32_t* n_next, hipStream_t s) {
    if (!n_max) return hipSuccess;
    hipLaunchKernelGGL(k5_assoc_claim, dim3(grid256(n_max)), dim3(256), 0, s, rem, n_rem, canon, cls, round);
    hipLaunchKernelGGL(k5_assoc_apply, dim3(grid256(n_max)), dim3(256), 0, s, t, rem, n_rem, canon, cls, round,
                       slot_of, expect, vals, status, next, n_next);
    return hipGetLastError();
}

hipError_t launch_assoc_get(const AssocView& t, uint32_t kind, const uint8_t* keys, uint64_t n, uint8_t* vals,
                            uint8_t* found, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k5_assoc_get, dim3(grid256(n)), dim3(256), 0, s, t, kind, keys, n, vals, found);
    return hipGetLastError();
}

hipError_t launch_assoc_select(const uint8_t* found, const uint8_t* vals, const uint64_t* key_ptr, uint64_t n,
                              int32_t* which, uint8_t* out, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k5_assoc_select, dim3(grid256(n)), dim3(256), 0, s, found, vals, key_ptr, n, which, out);
    return hipGetLastError();
}

hipError_t launch_assoc_abbrev(const AssocView& t, uint32_t kind, uint32_t cap, const uint8_t* qkeys,
                               const uint8_t* nhex, uint32_t q, uint32_t* matches, uint32_t* hit_slot,
                               hipStream_t s) {
    hipLaunchKernelGGL(k5_assoc_abbrev, dim3(grid256(cap)), dim3(256), 0, s, t, kind, cap, qkeys, nhex, q,
                       matches, hit_slot);
    return hipGetLastError();
}

hipError_t launch_iota(uint32_t* out, uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k5_iota, dim3(grid256(n)), dim3(256), 0, s, out, n);
    return hipGetLastError();
}

hipError_t launch_assoc_rehash(const AssocView& from, uint32_t cap_from, const AssocView& to, hipStream_t s) {
    hipLaunchKernelGGL(k5_assoc_rehash, dim3(grid256(cap_from)), dim3(256), 0, s, from, cap_from, to);
    return hipGetLastError();
}

}  // namespace rf
