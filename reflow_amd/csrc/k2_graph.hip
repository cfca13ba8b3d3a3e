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
//             (64-B aligned, nblk*64 bytes) and ZERO bytes at every hole; it is
//             never written after load.
//   meta      32-B job record (template offset, blocks, hole range, out slot,
//             consumer range): two 16-B loads per job.
//   holes     {byte position, slot} pairs, sorted by position per job.
//   slots     [S][32] digest table (node digests, physical keys, File IDs).
//   dirty     one word per job in level order: "already queued this step"
//             (a word each, not a bit: a bitset packed 32 consumers into one
//             word, and a merge node's producers -- 32 of them for each of
//             the word's 32 jobs -- serialised their atomics on it).
//   list      [J] per-level work lists; level l's list lives at lvl_start[l]
//             (a level can never hold more dirty jobs than it has jobs).
//   cons      slot -> consumer jobs (reverse edges for the frontier).
// The frontier needs no compaction pass: whoever changes a slot (set_slots,
// or a job whose digest changed -- early cut-off) sets its consumers' dirty
// bits and appends the newly set ones to their levels' lists, one atomicAdd
// per (wave, level).  One kernel per level then gives each listed job one
// lane, which assembles the job's material block by block in a private LDS
// ring (template block + digests OR-ed into the zero holes), hashes it and
// propagates.  A level's jobs all depend only on lower levels, so a level's
// list is complete when its kernel starts.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "engine.h"
#include "sha256_dev.h"
#include "lag_chain.h"

namespace rf {

constexpr uint32_t kLevelBlock = 256;
constexpr uint32_t kRing = 33;  // words per lane: a 32-word ring + 1 (odd stride: no bank conflicts)
// Diagnostic builds (-DRF_DIAG, diag.h) only: the phase stamps, the
// per-workgroup records, the timing probes (LevelArgs::dbg_twice) and the
// measured-dead kernel forms.  In the release build every such branch folds
// away at compile time and the dead forms are not instantiated.
#ifdef RF_DIAG
constexpr bool kDiag = true;
#else
constexpr bool kDiag = false;
#endif

struct LevelArgs;
__device__ __forceinline__ uint32_t dbg_mode(const LevelArgs& a);
struct LevelArgs {
    uint32_t s, e, lvl;  // internal job range of the level
    int full;
    uint32_t dbg_twice;  // diagnostic: hash every block twice (RF_DBG_HASH2), result unchanged
    const uint4* __restrict__ meta;
    const uint2* __restrict__ holes;
    const uint2* __restrict__ cons;          // {consumer job, its level}
    const uint32_t* __restrict__ lvl_start;  // [L+1] on device
    uint32_t n_levels;
    const uint8_t* __restrict__ tmpl;
    uint8_t* slots;
    uint32_t* dirty;
    uint32_t* list;
    uint32_t* counts;
    unsigned long long* stamps;  // diagnostic (RF_K2_STAMPS): phase times of workgroup 0, else null
    const uint4* __restrict__ mid;  // [2J] initial chaining values, or null (= IV for every job)
    const uint32_t* __restrict__ cons_ptr;  // [S+1] slot -> reverse-edge range (mark / apply kernels)
    uint4* lmeta;                           // [2J] the listed jobs' records, beside list
    uint32_t cb0;  // k2_level_pl<2,false>: chain-built block 0 of fused jobs (1: via the ring, 2: in registers)
    // k2_level_pl: workgroups take the level's list from its END -- the jobs
    // appended last (the chains that reached this level) before the sinks the
    // mark kernel queued early (ALAP-moved physical keys): at 100M nodes the
    // sinks alone fill the first ~2k workgroups of the OpK level
    uint32_t rev;
    uint32_t* zero_counts;  // [L+1] the previous plain step's cursor half, zeroed by workgroup 0 (or null)
    unsigned long long* wgst;  // diagnostic (RF_K2_WGSTAMPS=1): per-workgroup records [L][kWgStamps][4], else null
    // an attached sink list (k2_level_pl / k2_level_lf): the sink level lvl2's
    // list (at s2) is taken after this level's own, in the same launch
    // (graph_enqueue, GraphDev kLvlSink); lvl2 = ~0u: none
    uint32_t s2 = 0, lvl2 = ~0u;
    // split block 0 (k2_level_pl<2> cb0 = 2, GraphDev::split_b0): the
    // producer expands the upper half of a fusion target's block 0 and builds
    // its template-only block 1 during the job before it
    uint32_t split = 0;
    uint32_t oct_wg = 0;  // k2_level_oct: workgroups of the level's own list (the rest run the sink list)
    // k2_level_pl: nonzero = workgroups from sink_wg on run the attached sink
    // list one job per lane at the lowest priority (lf_job), the rest the
    // level's own list; ovf = 1: the own list only up to sink_wg x 64 jobs
    // (one batch per latency-form workgroup, one per CU), its overflow one
    // chain per lane in those lane workgroups too, before the sinks
    uint32_t sink_wg = 0, ovf = 0;
    uint32_t handoff = 1;  // k2_level_pl cb0 = 2: the producer hands the chain its next target's operands
    uint32_t n_cu = 256;   // the device's CUs (k2_level_lf's issue priorities)
    // GraphDev::fuse_pos2: every fusion target's one hole at byte 2 of its
    // first block, reading its producer's slot -- its hole record need not be
    // loaded (fused_hole)
    uint32_t fuse_pos2 = 0;
    uint32_t sf_pos = ~0u;  // GraphDev::sf_pos (slot-fused jobs, the mark kernels)
    // GraphDev::lvl_lead0 of lvl / lvl2: the listed jobs start from the IV
    uint32_t lead0 = 0, lead0_2 = 0;
    const uint4* __restrict__ plan = nullptr;  // [3S] the mark kernels' per-slot plan (GraphDev::plan), or null
};
// The diagnostic mode of a launch (LevelArgs::dbg_twice): always 0 in a release build.
__device__ __forceinline__ uint32_t dbg_mode(const LevelArgs& a) { return kDiag ? a.dbg_twice : 0u; }

// A level's append cursors (engine.h kListShards): run k of level l holds
// the listed jobs whose ids fall in [lvl_start[l] + k * 2^sh, ... + 2^sh),
// its cursor at list_shard_off(L) + k * Lp + l.
__device__ __forceinline__ const uint32_t* shard_cursors(const LevelArgs& a, uint32_t l) {
    return a.counts + list_shard_off(a.n_levels) + l;
}
// Jobs listed at level l this step.
__device__ __forceinline__ uint32_t level_count(const LevelArgs& a, uint32_t l) {
    if constexpr (kLegacyLists) return a.counts[l];
    const uint32_t* c = shard_cursors(a, l);
    const uint32_t lp = cursor_lp(a.n_levels);
    uint32_t n = 0;
#pragma unroll
    for (uint32_t k = 0; k < kListShards; ++k) n += c[k * lp];
    return n;
}
// The list position of level l's i-th listed job: runs in order, each run's
// entries from its start (branch-free over the runs).
__device__ __forceinline__ uint32_t level_pos(const LevelArgs& a, uint32_t l, uint32_t i) {
    if constexpr (kLegacyLists) return a.lvl_start[l] + i;
    const uint32_t* c = shard_cursors(a, l);
    const uint32_t lp = cursor_lp(a.n_levels), b = a.lvl_start[l];
    const uint32_t sh = list_shard_shift(a.lvl_start[l + 1] - b);
    uint32_t k = 0;
#pragma unroll
    for (uint32_t q = 0; q < kListShards; ++q) {
        const uint32_t cq = c[q * lp];
        const bool past = k == q && i >= cq;
        i -= past ? cq : 0u;
        k += past ? 1u : 0u;
    }
    return b + (k << sh) + i;
}

// A level launch's list runs, staged in LDS once per workgroup (stage_runs,
// then a barrier): per list -- the level's own, then the attached sink
// level's -- the runs' prefix counts [0 .. kListShards], the level's first
// list position and its run shift.  (Mapping from the cursors in global
// memory at every lookup put the latency form over its register budget:
// 256 VGPRs + an AGPR, one wave a SIMD.)
constexpr uint32_t kRunWords = kListShards + 3;
static_assert(2 * kListShards <= 64, "one wave stages both lists' runs");
__device__ __forceinline__ void stage_runs(const LevelArgs& a, uint32_t* sr) {
    if constexpr (kLegacyLists) return;
    // wave 0, lane t < 2 kListShards: list t / kListShards, run t % kListShards --
    // every cursor loaded at once, then a prefix scan within each list's lanes
    if (threadIdx.x < 64) {
        const uint32_t t = threadIdx.x, w = t / kListShards, k = t % kListShards;
        const uint32_t l = w ? a.lvl2 : a.lvl;
        const bool on = t < 2 * kListShards && l != ~0u;
        uint32_t v = on ? shard_cursors(a, l)[k * cursor_lp(a.n_levels)] : 0u;
#pragma unroll
        for (uint32_t o = 1; o < kListShards; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)v, o, 64);
            v += k >= o ? u : 0u;
        }
        if (t < 2 * kListShards) {
            uint32_t* p = sr + kRunWords * w;
            p[k + 1] = v;
            if (k == 0) {
                const uint32_t b = on ? a.lvl_start[l] : 0u;
                p[0] = 0;
                p[kListShards + 1] = b;
                p[kListShards + 2] = on ? list_shard_shift(a.lvl_start[l + 1] - b) : 0u;
            }
        }
    }
}
// The list position of a staged list's i-th entry (i < its count): the run
// holding it by binary search over the prefix counts (empty runs skipped).
__device__ __forceinline__ uint32_t run_pos(const uint32_t* p, uint32_t i) {
    uint32_t k = 0;
#pragma unroll
    for (uint32_t st = kListShards / 2; st; st >>= 1) k += p[k + st] <= i ? st : 0u;
    return p[kListShards + 1] + (k << p[kListShards + 2]) + (i - p[k]);
}

// Entries of a level launch: the level's own list (from its end when rev),
// then the attached sink list.  Offsets into a.list / a.lmeta; sr: the
// workgroup's staged runs (stage_runs, after its barrier).
struct LaunchList {
    const uint32_t* sr;
    uint32_t n1, n;
    __device__ __forceinline__ LaunchList(const LevelArgs& a, const uint32_t* staged)
        : sr(staged),
          n1(kLegacyLists ? a.counts[a.lvl] : staged[kListShards]),
          n(n1 + (kLegacyLists ? (a.lvl2 != ~0u ? a.counts[a.lvl2] : 0u) : staged[kRunWords + kListShards])) {}
    __device__ __forceinline__ uint32_t at(const LevelArgs& a, uint32_t i) const {
        if constexpr (kLegacyLists) return i < n1 ? a.s + (a.rev ? n1 - 1 - i : i) : a.s2 + (i - n1);
        return i < n1 ? run_pos(sr, a.rev ? n1 - 1 - i : i) : run_pos(sr + kRunWords, i - n1);
    }
};

// Diagnostic per-workgroup record of an incremental level kernel: start and
// end (s_memrealtime, 100 MHz), the hardware ids of the CU it ran on
// (HW_REG_HW_ID | HW_REG_XCC_ID << 32) and the jobs it took from the list.
constexpr uint32_t kWgStamps = 2048;
struct WgStamp {
    unsigned long long t0 = 0;
    uint32_t jobs = 0;
    __device__ __forceinline__ void begin(const LevelArgs& a) {
        if (kDiag && a.wgst && threadIdx.x == 0) t0 = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ void end(const LevelArgs& a) {
        if (!(kDiag && a.wgst) || threadIdx.x != 0 || blockIdx.x >= kWgStamps) return;
        uint32_t hw, xcc;
        __asm__ volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)"
                         : "=s"(hw), "=s"(xcc));
        unsigned long long* r = a.wgst + 4ull * (a.lvl * kWgStamps + blockIdx.x);
        r[0] = t0;
        r[1] = __builtin_amdgcn_s_memrealtime();
        r[2] = hw | ((unsigned long long)xcc << 32);
        r[3] = jobs;
    }
};

// This wave's fused-job counter (engine.h kFusedParts): one of the parts
// after the half's level counts, picked by workgroup and wave.
__device__ __forceinline__ uint32_t* fused_part(const LevelArgs& a) {
    const uint32_t k = (blockIdx.x * 5u + (threadIdx.x >> 6)) & (kFusedParts - 1);
    return &a.counts[a.n_levels + 1 + kPartStride * k];
}

// (first level kernel of a plain incremental step) the previous step's
// cursor half back to zero -- nobody reads or appends to it during this step
__device__ __forceinline__ void zero_other_counts(const LevelArgs& a) {
    if (a.zero_counts && blockIdx.x == 0)
        for (uint32_t l = threadIdx.x; l < counts_half_words(a.n_levels); l += blockDim.x) a.zero_counts[l] = 0;
}

// Reverse edges of an INPUT slot: bit 31 of the level field flags its
// slot-fused consumer (at most one, first in the slot's range): a job whose
// only hole is that slot, hashed by the lane that writes the slot
// (mark_input_slot) instead of being queued (rf_graph_load).
constexpr uint32_t kSlotFused = 0x80000000u;

// A job's initial chaining value (GraphDev::mid).
__device__ __forceinline__ void init_state(const LevelArgs& a, uint32_t p, ShaState& st) {
    if (a.mid) {
        const uint4 lo = a.mid[2ull * p], hi = a.mid[2ull * p + 1];
        st.h[0] = lo.x; st.h[1] = lo.y; st.h[2] = lo.z; st.h[3] = lo.w;
        st.h[4] = hi.x; st.h[5] = hi.y; st.h[6] = hi.z; st.h[7] = hi.w;
    } else {
        st.init();
    }
}

// Append the lanes' jobs j (need) at level lv to their levels' lists, each
// with its 32-B record (q0, q1) beside it in lmeta, so a level kernel's first
// job starts one HBM round trip earlier (list -> record -> template was three
// dependent loads).  A job joins its level's run (engine.h kListShards, by
// its id): one atomicAdd per
// distinct run in the wave, all issued before any result is used.  Called by
// every lane of the wave.
__device__ __forceinline__ void append_jobs(const LevelArgs& a, bool need, uint32_t j, uint32_t lv, const uint4& q0,
                                            const uint4& q1) {
    const uint32_t lane = __lane_id();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    if constexpr (kLegacyLists) {  // (A/B build: round 4's one cursor a level)
        uint64_t mask = __ballot(need);
        while (mask) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)mask) - 1;
            const uint32_t lvl = __builtin_amdgcn_readfirstlane(__shfl(lv, leader, 64));
            const bool mine = need && lv == lvl;
            const uint64_t same = __ballot(mine);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(&a.counts[lvl], (uint32_t)__popcll(same));
            base = a.lvl_start[lvl] + __shfl(base, leader, 64);
            if (mine) {
                const uint32_t at = base + (uint32_t)__popcll(same & lt);
                a.list[at] = j;
                a.lmeta[2ull * at] = q0;
                a.lmeta[2ull * at + 1] = q1;
                need = false;
            }
            mask = __ballot(need);
        }
        return;
    }
    // per distinct level (its start and run shift in scalar registers), per
    // distinct run among that level's lanes: one atomic, its result kept in
    // the leader lane; every lane's slot taken after the last one is issued
    uint32_t old = 0, ml = 0, rb = 0;
    uint64_t ms = 0;
    bool left = need;
    while (__any(left)) {
        const uint32_t ld = (uint32_t)__ffsll((unsigned long long)__ballot(left)) - 1;
        const uint32_t lvl = __builtin_amdgcn_readfirstlane(__shfl(lv, ld, 64));
        const uint32_t b = a.lvl_start[lvl];
        const uint32_t sh = list_shard_shift(a.lvl_start[lvl + 1] - b);
        const bool here = left && lv == lvl;
        const uint32_t k = here ? (j - b) >> sh : 0u;
        bool run = here;
        while (__any(run)) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)__ballot(run)) - 1;
            const uint32_t kk = __builtin_amdgcn_readfirstlane(__shfl(k, leader, 64));
            const bool mine = run && k == kk;
            const uint64_t same = __ballot(mine);
            if (lane == leader)
                old = atomicAdd(&a.counts[list_shard_off(a.n_levels) + kk * cursor_lp(a.n_levels) + lvl],
                                (uint32_t)__popcll(same));
            if (mine) {
                ml = leader;
                ms = same;
                rb = b + (kk << sh);
                run = false;
            }
        }
        left = left && !here;
    }
    const uint32_t base = (uint32_t)__shfl((int)old, (int)ml, 64);
    if (need) {
        const uint32_t at = rb + base + (uint32_t)__popcll(ms & lt);
        a.list[at] = j;
        a.lmeta[2ull * at] = q0;
        a.lmeta[2ull * at + 1] = q1;
    }
}

// Mark consumers [c, ce) of the lanes whose slot changed (c == ce otherwise)
// dirty, queueing the newly dirty ones (their records are fetched beside the
// dirty-flag atomic).  Wave-uniform loop.
__device__ __forceinline__ void propagate(const LevelArgs& a, uint32_t c, uint32_t ce) {
    while (__any(c < ce)) {
        bool need = false;
        uint2 jl = make_uint2(0, 0);
        uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
        if (c < ce) {
            jl = a.cons[c++];
            q0 = a.meta[2ull * jl.x];
            q1 = a.meta[2ull * jl.x + 1];
            need = atomicOr(&a.dirty[jl.x], 1u) == 0u;
        }
        append_jobs(a, need, jl.x, jl.y, q0, q1);
    }
}

// OR digest D (8 LE words) into the lane's ring at material byte `pos`; the
// template holds zero bytes there, and the 00 05 prefix around it.
__device__ __forceinline__ void or_digest(uint32_t* ring, uint32_t pos, const uint32_t (&D)[8]) {
    const uint32_t x = pos >> 2, sh = 32 - 8 * (pos & 3);
    uint32_t prev = 0;
#pragma unroll
    for (int m = 0; m < 9; ++m) {
        const uint32_t cur = m < 8 ? D[m] : 0u;
        const uint32_t v = (uint32_t)((((uint64_t)cur << 32) | prev) >> sh);
        atomicOr(&ring[(x + m) & 31], v);
        prev = cur;
    }
}

// w[0..15] = the big-endian words of the 16 ring words at r, the eight
// two-word LDS reads issued back to back and waited for once (compiled
// from C++, the throughput form at its register limit issued them one at a
// time, each waited for in full)
__device__ __forceinline__ void ring_read16(const uint32_t* r, uint32_t (&w)[16]) {
    const uint32_t lds = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint32_t*)r);
    uint64_t x0, x1, x2, x3, x4, x5, x6, x7;
    __asm__ volatile(
        "ds_read2_b32 %0, %8 offset1:1\n\t"
        "ds_read2_b32 %1, %8 offset0:2 offset1:3\n\t"
        "ds_read2_b32 %2, %8 offset0:4 offset1:5\n\t"
        "ds_read2_b32 %3, %8 offset0:6 offset1:7\n\t"
        "ds_read2_b32 %4, %8 offset0:8 offset1:9\n\t"
        "ds_read2_b32 %5, %8 offset0:10 offset1:11\n\t"
        "ds_read2_b32 %6, %8 offset0:12 offset1:13\n\t"
        "ds_read2_b32 %7, %8 offset0:14 offset1:15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3), "=&v"(x4), "=&v"(x5), "=&v"(x6), "=&v"(x7)
        : "v"(lds)
        : "memory");
    const uint64_t x[8] = {x0, x1, x2, x3, x4, x5, x6, x7};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        w[2 * k] = bswap32((uint32_t)x[k]);
        w[2 * k + 1] = bswap32((uint32_t)(x[k] >> 32));
    }
}

__device__ __forceinline__ void ring_put(uint32_t* ring, uint32_t half, const uint4 (&t)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        ring[half + 4 * q] = t[q].x;
        ring[half + 4 * q + 1] = t[q].y;
        ring[half + 4 * q + 2] = t[q].z;
        ring[half + 4 * q + 3] = t[q].w;
    }
}

// Assembles a job's material block by block in the lane's LDS ring (a
// template block with the slot digests OR-ed into its zero holes).  Software
// pipeline: while block b is consumed, the template of block b+2 and the (at
// most two: holes are >= 32 B apart) holes that start in block b+1 -- records
// and slot digests -- are in flight.
// A fusion target's hole record: loaded, or -- when every target's one hole
// is at material byte 2 (LevelArgs::fuse_pos2; then it has no constant
// leading blocks either and starts from the IV) -- (2, ~0u) without a load
// (the slot is its producer's, whose digest the caller hands over).  The record load
// was a random access into the 1.2 GB hole array at every chain link, ~5 %
// of the 100M step (timing probe, profiles/r06/probe_loads/).
// jf: the job is fused to another job (a fusion target); a slot-fused job
// (the mark kernels' first, reading an input slot) has its hole elsewhere
// (OpVal: byte 8), its record is always loaded.
__device__ __forceinline__ uint2 fused_hole(const LevelArgs& a, uint32_t h, bool jf = true) {
    if (jf) return a.fuse_pos2 ? make_uint2(2u, ~0u) : a.holes[h];
    return a.sf_pos != ~0u ? make_uint2(a.sf_pos, ~0u) : a.holes[h];  // (slot-fused: GraphDev::sf_pos)
}
// Whether a fused job (jf: to a job; else to an input slot) starts from the IV
// without a midstate load.
__device__ __forceinline__ bool fused_iv(const LevelArgs& a, bool jf) {
    return jf ? a.fuse_pos2 != 0 : a.sf_pos != ~0u;
}

struct PendingHole {
    uint2 r;  // (material byte, slot), or ~0 past the job's last hole
    uint4 lo, hi;
};

__device__ __forceinline__ void vm_drain() { __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct MatCursor {
    // holes hn .. hn+3 in flight with their slot digests, and the records of
    // hn+4 and hn+5: a block applies at most two holes (they are >= 32 B apart),
    // so a record arrives a block before its digest load is issued, and the
    // digest a block before it is applied
    const uint4* __restrict__ T;
    uint32_t nb, he, hn;
    PendingHole q0, q1, q2, q3;
    uint2 r4, r5;
    uint4 t[4];
    uint32_t fslot = ~0u;  // a slot whose new digest is handed over in registers (fused chains)
    uint4 flo, fhi;

    // unconditional load (index 0 past the job's holes; the hole array always
    // has an element), so independent record loads issue back to back with no
    // branch forcing a wait between them
    __device__ __forceinline__ uint2 record(const LevelArgs& a, uint32_t h) const {
        const uint2 v = a.holes[h < he ? h : 0u];
        return h < he ? v : make_uint2(~0u, 0u);
    }
    __device__ __forceinline__ void digest(const LevelArgs& a, PendingHole& q, const uint2& r) const {
        q.r = r;
        const uint8_t* slot = a.slots + 32ull * (q.r.y == ~0u ? 0u : q.r.y);
        const uint4* src = reinterpret_cast<const uint4*>(slot);
        q.lo = src[0];
        q.hi = src[1];
    }
    __device__ __forceinline__ void apply(uint32_t* ring, const PendingHole& q) const {
        const bool f = q.r.y == fslot;
        const uint4 lo = f ? flo : q.lo, hi = f ? fhi : q.hi;
        const uint32_t D[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        or_digest(ring, q.r.x, D);
    }
    __device__ __forceinline__ void begin(const LevelArgs& a, const uint4& m0, uint32_t* ring) {
        T = reinterpret_cast<const uint4*>(a.tmpl) + 4ull * m0.x;
        nb = m0.y;
        he = m0.w;
        hn = m0.z;  // first hole not yet applied
        // all six records first, then the four digest loads: one HBM round
        // trip each way instead of four dependent record -> digest pairs
        const uint2 r0 = record(a, hn), r1 = record(a, hn + 1), r2 = record(a, hn + 2), r3 = record(a, hn + 3);
        r4 = record(a, hn + 4);
        r5 = record(a, hn + 5);
        uint4 t0[4];
        t0[0] = T[0]; t0[1] = T[1]; t0[2] = T[2]; t0[3] = T[3];
        // block 1's template with block 0's, not after block 0's wait (two
        // round trips in a row at every job's start)
        if (nb > 1) {
            t[0] = T[4]; t[1] = T[5]; t[2] = T[6]; t[3] = T[7];
        }
        digest(a, q0, r0);
        digest(a, q1, r1);
        digest(a, q2, r2);
        digest(a, q3, r3);
        ring_put(ring, 0, t0);
    }
    // begin() for a fused job: its one hole reads the slot handed over in
    // registers, and its first two template blocks and hole record were
    // prefetched while its producer was hashed
    __device__ __forceinline__ void begin_pre(const uint4& m0, const uint4* __restrict__ tmpl, const uint4 (&nt)[8],
                                              const uint2& nr, uint32_t* ring) {
        T = tmpl + 4ull * m0.x;
        nb = m0.y;
        he = m0.w;
        hn = m0.z;
        q0.r = nr;
        q1.r = q2.r = q3.r = r4 = r5 = make_uint2(~0u, 0u);
        t[0] = nt[0]; t[1] = nt[1]; t[2] = nt[2]; t[3] = nt[3];
        ring_put(ring, 0, t);
        t[0] = nt[4]; t[1] = nt[5]; t[2] = nt[6]; t[3] = nt[7];
    }
    // begin() for a job with one hole, whose digest is handed over in
    // registers (fslot / flo / fhi): only its hole record and template blocks
    // are loaded (hash_fused_chain_lean; then block(..., one = true))
    __device__ __forceinline__ void begin_fused(const LevelArgs& a, const uint4& m0, uint32_t* ring, bool jf = true) {
        T = reinterpret_cast<const uint4*>(a.tmpl) + 4ull * m0.x;
        nb = m0.y;
        he = m0.w;
        hn = m0.z;
        q0.r = fused_hole(a, m0.z, jf);
        q0.r.y = fslot;  // (its one hole reads the handed-over slot: apply uses flo/fhi)
        q1.r = q2.r = q3.r = r4 = r5 = make_uint2(~0u, 0u);
        uint4 t0[4];
        t0[0] = T[0]; t0[1] = T[1]; t0[2] = T[2]; t0[3] = T[3];
        if (nb > 1) {  // (with block 0's: see begin)
            t[0] = T[4]; t[1] = T[5]; t[2] = T[6]; t[3] = T[7];
        }
        ring_put(ring, 0, t0);
    }
    // begin() for a fused job whose block 0 the chain wave builds (k2_level_pl,
    // cb0): the ring already holds its template blocks 0 and 1 with the
    // producer's digest OR-ed into the one hole, so the cursor starts at block
    // 1 with no hole left; t is block 2's template
    __device__ __forceinline__ void begin_chain(const uint4& m0, const uint4* __restrict__ tmpl) {
        T = tmpl + 4ull * m0.x;
        nb = m0.y;
        he = m0.w;
        hn = m0.z;
        q0.r = q1.r = q2.r = q3.r = r4 = r5 = make_uint2(~0u, 0u);
        if (nb > 2) {
            t[0] = T[8]; t[1] = T[9]; t[2] = T[10]; t[3] = T[11];
        }
    }
    // the 16 big-endian words of block b (blocks taken in order).  one: every
    // active lane of the wave holds a fused job (begin_pre: its single hole is
    // q0) -- wave-uniform, so that path has no queue rotation: no record or
    // digest loads and no register moves of loads in flight (each such move
    // compiled to an s_waitcnt vmcnt(0), an HBM round trip inside the block)
    __device__ __forceinline__ void block(const LevelArgs& a, uint32_t b, uint32_t* ring, uint32_t (&w)[16],
                                          bool one = false) {
        const uint32_t half = (b & 1) * 16;
        if (b + 1 < nb) {
            ring_put(ring, half ^ 16, t);
            if (b + 2 < nb) {
                const uint4* s = T + 4 * (b + 2);
                t[0] = s[0]; t[1] = s[1]; t[2] = s[2]; t[3] = s[3];
            }
        }
        // holes that start in block b (they may run into block b+1)
        const uint32_t lim = 64 * (b + 1);
        if (one) {
            if (q0.r.x < lim) {
                apply(ring, q0);
                q0.r = make_uint2(~0u, 0u);
            }
        } else if (q0.r.x < lim) {
            apply(ring, q0);
            if (q1.r.x < lim) {
                apply(ring, q1);
                q0 = q2;
                q1 = q3;
                hn += 2;
                digest(a, q2, r4);
                digest(a, q3, r5);
                r4 = record(a, hn + 4);
                r5 = record(a, hn + 5);
            } else {
                q0 = q1;
                q1 = q2;
                q2 = q3;
                hn += 1;
                digest(a, q3, r4);
                r4 = r5;
                r5 = record(a, hn + 5);
            }
        }
        ring_read16(ring + half, w);
    }
};

// The producer wave's material cursor in k2_level_pl: MatCursor's template
// stream, with the holes in chunks of kHC per job.  While chunk c is applied
// from the lane's LDS buffer, chunk c+1's digests and chunk c+2's records are
// in flight in fixed registers; at the first hole of chunk c+1 (a transition)
// chunk c+1's records and digests go to LDS buffer (c+1) & 1, chunk c+2's
// records move in, and chunk c+2's digests and chunk c+3's records are
// issued.  Every register move or store reads loads issued a chunk (about two
// blocks) earlier: MatCursor's queue moved digests issued one block earlier
// and waited for them (an 18-block Merge job's producer took 1.1-1.9 us a
// block against the chain's 1.36, RF_K2_STAMPS=3).
// Chunks of two holes (round 3, session 3): a transition every block or so,
// each staging half as much, instead of a heavy one every other block (the
// per-block barrier makes the slowest block set the pace): 8-rank piece
// 0.330 -> 0.325 ms/step, configs[2] unchanged; 3 measured the same as 2
// (profiles/r03/s3/hole_chunk_ab.log).  -DRF_HOLE_CHUNK=4: the previous form.
#ifndef RF_HOLE_CHUNK
#define RF_HOLE_CHUNK 2
#endif
constexpr uint32_t kHC = RF_HOLE_CHUNK;  // holes per chunk
constexpr uint32_t kHq = 2 * kHC * 9 + 1;  // words per lane: [2 chunks][kHC holes][pos + 8 digest words] + 1 (odd stride)
struct ChunkCursor {
    const uint4* __restrict__ T;
    uint32_t nb, he, h0, hn, staged;  // holes [h0, he), hn the next to apply, staged: chunks in LDS
    uint4 t[4];
    uint32_t fslot = ~0u;  // a slot whose new digest is handed over in registers (fused chains)
    uint4 flo, fhi;
    uint2 single;          // one-hole fused jobs (begin_pre): the hole's record
    uint2 rn[kHC], rnn[kHC];   // records of chunks c+1 and c+2
    uint4 dlo[kHC], dhi[kHC];  // digests of chunk c+1
    uint32_t* hq;          // the lane's LDS buffers

    __device__ __forceinline__ uint2 record(const LevelArgs& a, uint32_t h) const {
        const uint2 v = a.holes[h < he ? h : 0u];
        return h < he ? v : make_uint2(~0u, 0u);
    }
    __device__ __forceinline__ void load_records(const LevelArgs& a, uint32_t c, uint2 (&r)[kHC]) const {
#pragma unroll
        for (uint32_t q = 0; q < kHC; ++q) r[q] = record(a, h0 + kHC * c + q);
    }
    __device__ __forceinline__ void load_digests(const LevelArgs& a, const uint2 (&r)[kHC]) {
#pragma unroll
        for (uint32_t q = 0; q < kHC; ++q) {
            const uint4* src = reinterpret_cast<const uint4*>(a.slots + 32ull * (r[q].x == ~0u ? 0u : r[q].y));
            dlo[q] = src[0];
            dhi[q] = src[1];
        }
    }
    // chunk c's records r and digests dlo/dhi into LDS buffer c & 1
    __device__ __forceinline__ void stash(uint32_t c, const uint2 (&r)[kHC]) const {
        uint32_t* q = hq + (c & 1) * 9 * kHC;
#pragma unroll
        for (uint32_t k = 0; k < kHC; ++k) {
            const bool f = r[k].y == fslot && r[k].x != ~0u;
            const uint4 lo = f ? flo : dlo[k], hi = f ? fhi : dhi[k];
            q[9 * k] = r[k].x;
            q[9 * k + 1] = lo.x; q[9 * k + 2] = lo.y; q[9 * k + 3] = lo.z; q[9 * k + 4] = lo.w;
            q[9 * k + 5] = hi.x; q[9 * k + 6] = hi.y; q[9 * k + 7] = hi.z; q[9 * k + 8] = hi.w;
        }
    }
    __device__ __forceinline__ void begin(const LevelArgs& a, const uint4& m0, uint32_t* ring) {
        T = reinterpret_cast<const uint4*>(a.tmpl) + 4ull * m0.x;
        nb = m0.y;
        he = m0.w;
        h0 = hn = m0.z;
        single = make_uint2(~0u, 0u);
        uint2 r0[kHC];
        load_records(a, 0, r0);
        load_records(a, 1, rn);
        load_records(a, 2, rnn);
        t[0] = T[0]; t[1] = T[1]; t[2] = T[2]; t[3] = T[3];
        load_digests(a, r0);
        stash(0, r0);
        load_digests(a, rn);  // chunk 1's, in flight until its transition
        staged = 1;
        ring_put(ring, 0, t);
        if (nb > 1) {
            t[0] = T[4]; t[1] = T[5]; t[2] = T[6]; t[3] = T[7];
        }
    }
    // (as MatCursor's) a fused job: one hole, its digest handed over in registers
    __device__ __forceinline__ void begin_pre(const uint4& m0, const uint4* __restrict__ tmpl, const uint4 (&nt)[8],
                                              const uint2& nr, uint32_t* ring) {
        T = tmpl + 4ull * m0.x;
        nb = m0.y;
        he = m0.w;
        h0 = hn = m0.z;
        single = nr;
        t[0] = nt[0]; t[1] = nt[1]; t[2] = nt[2]; t[3] = nt[3];
        ring_put(ring, 0, t);
        t[0] = nt[4]; t[1] = nt[5]; t[2] = nt[6]; t[3] = nt[7];
    }
    __device__ __forceinline__ void begin_chain(const uint4& m0, const uint4* __restrict__ tmpl) {
        T = tmpl + 4ull * m0.x;
        nb = m0.y;
        he = m0.w;
        h0 = hn = m0.z;
        single = make_uint2(~0u, 0u);
        if (nb > 2) {
            t[0] = T[8]; t[1] = T[9]; t[2] = T[10]; t[3] = T[11];
        }
    }
    // the next hole hn: its chunk staged first (a transition), then applied
    // if it starts below lim
    __device__ __forceinline__ void next_hole(const LevelArgs& a, uint32_t* ring, uint32_t lim) {
        if (hn >= he) return;
        const uint32_t c = (hn - h0) / kHC;
        if (c >= staged) {  // chunk c (= staged) enters: stash it, move the pipeline on
            stash(c, rn);
#pragma unroll
            for (uint32_t q = 0; q < kHC; ++q) rn[q] = rnn[q];
            load_digests(a, rn);
            load_records(a, c + 2, rnn);
            staged = c + 1;
        }
        const uint32_t* q = hq + (c & 1) * 9 * kHC + 9 * ((hn - h0) % kHC);
        const uint32_t pos = q[0];
        if (pos < lim) {
            const uint32_t D[8] = {q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[8]};
            or_digest(ring, pos, D);
            ++hn;
        }
    }
    // block b's template-only bookkeeping without assembling it (its K+W
    // rows came from elsewhere: split block 0's precomputed block 1)
    __device__ __forceinline__ void skip(uint32_t b, uint32_t* ring) {
        if (b + 1 < nb) ring_put(ring, ((b & 1) * 16) ^ 16, t);
        if (b + 2 < nb) {
            const uint4* s = T + 4 * (b + 2);
            t[0] = s[0]; t[1] = s[1]; t[2] = s[2]; t[3] = s[3];
        }
    }
    __device__ __forceinline__ void block(const LevelArgs& a, uint32_t b, uint32_t* ring, uint32_t (&w)[16],
                                          bool one = false) {
        const uint32_t half = (b & 1) * 16;
        // the next block's template into the ring first (a hole may run into
        // it); block b+2's template is issued only after the holes: the
        // compiler's waits in a transition are vmcnt(0), and a load issued
        // just before them would be waited for in full
        if (b + 1 < nb) ring_put(ring, half ^ 16, t);
        const uint32_t lim = 64 * (b + 1);
        if (one) {
            if (single.x < lim) {  // (the hole reads the handed-over slot: begin_pre)
                const uint32_t D[8] = {flo.x, flo.y, flo.z, flo.w, fhi.x, fhi.y, fhi.z, fhi.w};
                or_digest(ring, single.x, D);
                single = make_uint2(~0u, 0u);
            }
        } else {
            // holes that start in block b: at most two (they are >= 32 B apart)
            next_hole(a, ring, lim);
            next_hole(a, ring, lim);
        }
        if (b + 2 < nb) {
            const uint4* s = T + 4 * (b + 2);
            t[0] = s[0]; t[1] = s[1]; t[2] = s[2]; t[3] = s[3];
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = bswap32(ring[half + i]);
    }
};

// Store the digest into its slot if it changed (always in full mode).
__device__ __forceinline__ bool finish_job(const LevelArgs& a, const uint4& m1, const ShaState& st) {
    uint4* dst = reinterpret_cast<uint4*>(a.slots + 32ull * m1.x);
    uint4 nlo, nhi;
    nlo.x = bswap32(st.h[0]); nlo.y = bswap32(st.h[1]); nlo.z = bswap32(st.h[2]); nlo.w = bswap32(st.h[3]);
    nhi.x = bswap32(st.h[4]); nhi.y = bswap32(st.h[5]); nhi.z = bswap32(st.h[6]); nhi.w = bswap32(st.h[7]);
    bool changed = true;
    if (!a.full) {
        const uint4 olo = dst[0], ohi = dst[1];
        changed = (olo.x != nlo.x) | (olo.y != nlo.y) | (olo.z != nlo.z) | (olo.w != nlo.w) |
                  (ohi.x != nhi.x) | (ohi.y != nhi.y) | (ohi.z != nhi.z) | (ohi.w != nhi.w);
    }
    if (changed) {
        dst[0] = nlo;
        dst[1] = nhi;
    }
    return changed;
}

// As finish_job, with the old digest already loaded (incremental mode).
__device__ __forceinline__ bool finish_job_pre(const LevelArgs& a, const uint4& m1, const ShaState& st,
                                               const uint4& olo, const uint4& ohi) {
    uint4 nlo, nhi;
    nlo.x = bswap32(st.h[0]); nlo.y = bswap32(st.h[1]); nlo.z = bswap32(st.h[2]); nlo.w = bswap32(st.h[3]);
    nhi.x = bswap32(st.h[4]); nhi.y = bswap32(st.h[5]); nhi.z = bswap32(st.h[6]); nhi.w = bswap32(st.h[7]);
    const bool changed = (olo.x != nlo.x) | (olo.y != nlo.y) | (olo.z != nlo.z) | (olo.w != nlo.w) |
                         (ohi.x != nhi.x) | (ohi.y != nhi.y) | (ohi.z != nhi.z) | (ohi.w != nhi.w);
    if (changed) {
        uint4* dst = reinterpret_cast<uint4*>(a.slots + 32ull * m1.x);
        dst[0] = nlo;
        dst[1] = nhi;
    }
    return changed;
}

// propagate() with the first two reverse edges already in registers.
__device__ __forceinline__ void propagate_pre(const LevelArgs& a, uint32_t c, uint32_t ce, const uint2 (&pre)[2]) {
    for (int k = 0; k < 2; ++k) {
        bool need = false;
        const uint2 jl = pre[k];
        uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
        if (c < ce) {
            ++c;
            q0 = a.meta[2ull * jl.x];
            q1 = a.meta[2ull * jl.x + 1];
            need = atomicOr(&a.dirty[jl.x], 1u) == 0u;
        }
        append_jobs(a, need, jl.x, jl.y, q0, q1);
    }
    propagate(a, c, ce);
}

// Hash job p in one lane; returns whether its slot changed.
__device__ __forceinline__ bool hash_job(const LevelArgs& a, uint32_t p, uint32_t* ring, uint32_t& cb,
                                         uint32_t& ce) {
    const uint4 m0 = a.meta[2 * p], m1 = a.meta[2 * p + 1];
    ShaState st;
    init_state(a, p, st);  // (before the cursor's loads: see hash_fused_chain_lean)
    MatCursor cur;
    cur.begin(a, m0, ring);
    for (uint32_t b = 0; b < cur.nb; ++b) {
        uint32_t w[16];
        cur.block(a, b, ring, w);
        if (dbg_mode(a) == 1) {  // (2 = RF_K2_STAMPS=2, not a hashing mode)
            ShaState s2 = st;
            uint32_t w2[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) w2[i] = w[i] ^ (dbg_mode(a) - 1);
            sha256_compress(s2, w2);
            st.h[0] ^= s2.h[0] & (dbg_mode(a) - 1);
        }
        sha256_compress(st, w);
    }
    cb = m1.y;
    ce = m1.z;
    return finish_job(a, m1, st);
}

// K2+K3, one level: every listed job (incremental) or every job of the level
// (full).  Incremental: the job leaves the dirty set, and if its digest
// changed its consumers join their levels' lists.
__global__ __launch_bounds__(kLevelBlock) void k2_level(LevelArgs a) {
    __shared__ uint32_t ring_all[kLevelBlock * kRing];
    uint32_t* ring = &ring_all[threadIdx.x * kRing];
    const uint32_t n = a.full ? (a.e - a.s) : level_count(a, a.lvl);
    for (uint32_t base = blockIdx.x * kLevelBlock; base < n; base += gridDim.x * kLevelBlock) {
        const uint32_t i = base + threadIdx.x;
        uint32_t cb = 0, ce = 0;
        if (i < n) {
            const uint32_t p = a.full ? a.s + i : a.list[level_pos(a, a.lvl, i)];
            const bool changed = hash_job(a, p, ring, cb, ce);
            if (!a.full) {
                a.dirty[p] = 0u;
                if (!changed) ce = cb;
            }
        }
        if (!a.full) propagate(a, cb, ce);
    }
}

// Incremental levels are latency-bound (a level's dirty jobs fill a few
// hundred waves, one per SIMD): a lane-per-job hash costs ~1400 issued
// instructions per block on one wave (~3 us).  Here a workgroup of two waves
// splits that work for 64 jobs: the producer wave assembles each job's next
// block and expands its message schedule (K[t]+W[t], 64 words) into a
// double-buffered LDS row per job, while the chain wave runs the 64 rounds of
// the current block from LDS (14 instructions per round: ~910 per block).
// One workgroup barrier per block; the chain then stores, clears the queued
// bit and propagates like k2_level.
// Workgroup barrier for LDS hand-overs only.  __syncthreads() is a release /
// acquire fence as well, which waits for every outstanding global load and
// store of the wave (s_waitcnt vmcnt(0)): each block would then wait out the
// HBM latency of the template and hole loads just issued for later blocks.
// Nothing here is passed between the two waves through global memory.
__device__ __forceinline__ void lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

#ifndef RF_K2_JOIN_WAIT
#define RF_K2_JOIN_WAIT 0  // (A/B build: 1 = the compiler's wait at the join)
#endif
constexpr uint32_t kPcRow = 68;  // words per K+W row: 16-B reads of 64 rows hit distinct banks

// Fused chains: a job whose only input is one job's digest, and which that
// job names as its fusion target (meta[2j+1].w, rf_graph_load), is never
// queued; whoever hashes its producer hashes it next, in the same lane, as
// soon as the producer's digest changed -- no level barrier between them (the
// 1000align pair chain Exec -> Coerce -> K -> ... is ten such jobs deep).  The
// producer's new digest reaches the fused job's material through LDS.
#define RF_STAMP(k)                                                                        \
    do {                                                                                   \
        if (kDiag && a.stamps && blockIdx.x == 0 && lane == 0 && wave < 2 && (k) < 64)             \
            a.stamps[128 * a.lvl + 64 * wave + (k)] = __builtin_amdgcn_s_memrealtime();    \
    } while (0)

// kW = 2: chain + producer.  kW = 3 (levels of long jobs, e.g. the
// per-sample OpK with 18 blocks, where the producer's ~2.4 us per block
// exceeded the chain's ~1.9 us): the producer only assembles each block and
// hands its 16 big-endian words through LDS (wbuf) to an expander wave, which
// writes the K+W row a block later; the chain lags two blocks.
constexpr uint32_t kWRow = 20;  // words per assembled-block row: 16-B accesses of 16 lanes hit distinct banks

#ifdef RF_DIAG  // the one-lane chain form (RF_K2_CHAIN=14, A/B): diagnostic builds only
template <uint32_t kW>
__global__ __launch_bounds__(64 * kW) void k2_level_pc(LevelArgs a) {
    static_assert(kW == 2 || kW == 3, "chain + producer (+ expander)");
    constexpr uint32_t lag = kW - 1;  // iterations between a block's assembly and its rounds
    __shared__ __attribute__((aligned(16))) uint32_t kw[2 * 64 * kPcRow];
    __shared__ __attribute__((aligned(16))) uint32_t wbuf[kW == 3 ? 2 * 64 * kWRow : 4];
    __shared__ uint32_t ring_all[64 * kRing];
    __shared__ uint4 s_dig[64][2];   // the last job's new digest (raw words)
    __shared__ uint32_t s_next[64];  // the lane's next (fused) job, or ~0
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // 0 chain, 1 producer, 2 expander
    const uint32_t lane = threadIdx.x & 63;
    uint32_t* ring = &ring_all[lane * kRing];
    zero_other_counts(a);
    const uint32_t n = level_count(a, a.lvl);
    for (uint32_t base = blockIdx.x * 64; base < n; base += gridDim.x * 64) {
        const uint32_t i = base + lane;
        bool has = i < n;
        uint32_t p = has ? a.list[level_pos(a, a.lvl, i)] : 0u;
        uint32_t fslot = ~0u;  // the previous job's out slot (fused hand-over)
        uint32_t sk = 0;
        // the fusion target's meta, first template blocks, hole record (producer)
        // and old digest + first reverse edges (chain), prefetched while its
        // producer is hashed: a fused job starts without a dependent HBM chain
        // nnm: the target's own fusion target's meta, fetched a job ahead, so a
        // fused job's successor record never costs an HBM round trip on its block 0
        uint4 nm0 = make_uint4(0, 0, 0, 0), nm1 = nm0, nolo = nm0, nohi = nm0, nnm0 = nm0, nnm1 = nm0;
        uint4 nt[8];
        uint2 nr = make_uint2(0, 0);
        uint2 npre[2] = {make_uint2(0, 0), make_uint2(0, 0)};
        // both waves hold the same per-lane job, so this loop is uniform
        while (__any(has)) {
            RF_STAMP(sk); ++sk;
            const bool fused = fslot != ~0u;
            uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
            if (has) {
                if (fused) {
                    m0 = nm0;
                    m1 = nm1;
                    nm0 = nnm0;  // = meta[m1.w], valid when m1.w != ~0
                    nm1 = nnm1;
                } else {
                    m0 = a.meta[2 * p];
                    m1 = a.meta[2 * p + 1];
                }
            }
            const bool nfu = has && m1.w != ~0u;
            if (nfu && !fused) {
                nm0 = a.meta[2ull * m1.w];
                nm1 = a.meta[2ull * m1.w + 1];
            }
            uint32_t maxnb = m0.y;
            for (int o = 32; o > 0; o >>= 1) maxnb = max(maxnb, (uint32_t)__shfl_xor((int)maxnb, o, 64));
            maxnb = __builtin_amdgcn_readfirstlane(maxnb);
            MatCursor cur;
            ShaState st;
            init_state(a, has ? p : 0u, st);
            uint4 olo = make_uint4(0, 0, 0, 0), ohi = olo;
            uint2 pre[2] = {make_uint2(0, 0), make_uint2(0, 0)};
            if (wave == 1 && has) {
                cur.fslot = fslot;
                if (fused) {
                    cur.flo = s_dig[lane][0];
                    cur.fhi = s_dig[lane][1];
                    cur.begin_pre(m0, reinterpret_cast<const uint4*>(a.tmpl), nt, nr, ring);
                } else {
                    cur.begin(a, m0, ring);
                }
            }
            if (wave == 0 && has) {  // the chain wave waits for block 0 anyway: fetch what finishing needs
                if (fused) {
                    olo = nolo;
                    ohi = nohi;
                    pre[0] = npre[0];
                    pre[1] = npre[1];
                } else {
                    const uint4* od = reinterpret_cast<const uint4*>(a.slots + 32ull * m1.x);
                    olo = od[0];
                    ohi = od[1];
                    if (m1.y < m1.z) pre[0] = a.cons[m1.y];
                    if (m1.y + 1 < m1.z) pre[1] = a.cons[m1.y + 1];
                }
                if (nfu) {
                    const uint4* od = reinterpret_cast<const uint4*>(a.slots + 32ull * nm1.x);
                    nolo = od[0];
                    nohi = od[1];
                    if (nm1.y < nm1.z) npre[0] = a.cons[nm1.y];
                    if (nm1.y + 1 < nm1.z) npre[1] = a.cons[nm1.y + 1];
                    if (nm1.w != ~0u) {
                        nnm0 = a.meta[2ull * nm1.w];
                        nnm1 = a.meta[2ull * nm1.w + 1];
                    }
                }
            }
            if (kW == 3 && wave == 2 && nfu && nm1.w != ~0u) {  // the expander needs m0.y of every job too
                nnm0 = a.meta[2ull * nm1.w];
                nnm1 = a.meta[2ull * nm1.w + 1];
            }
            for (uint32_t it = 0; it < maxnb + lag; ++it) {
                if (wave == 1) {
                    if (it < m0.y) {  // block it of this lane's job -> buffer it & 1
                        uint32_t w[16];
                        cur.block(a, it, ring, w);
                        if (kW == 2) {
                            kw_expand_store(w, reinterpret_cast<uint4*>(&kw[((it & 1) * 64 + lane) * kPcRow]));
                        } else {
                            uint4* row = reinterpret_cast<uint4*>(&wbuf[((it & 1) * 64 + lane) * kWRow]);
#pragma unroll
                            for (int q = 0; q < 4; ++q)
                                row[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
                        }
                    }
                    if (it == 0 && nfu) {
                        const uint4* nT = reinterpret_cast<const uint4*>(a.tmpl) + 4ull * nm0.x;
                        nt[0] = nT[0]; nt[1] = nT[1]; nt[2] = nT[2]; nt[3] = nT[3];
                        if (nm0.y > 1) {
                            nt[4] = nT[4]; nt[5] = nT[5]; nt[6] = nT[6]; nt[7] = nT[7];
                        }
                        nr = a.holes[nm0.z];
                        if (nm1.w != ~0u) {
                            nnm0 = a.meta[2ull * nm1.w];
                            nnm1 = a.meta[2ull * nm1.w + 1];
                        }
                    }
                } else if (kW == 3 && wave == 2) {
                    if (it >= 1 && it - 1 < m0.y) {  // expand block it-1: wbuf -> kw, buffer (it-1) & 1
                        const uint32_t bb = (it - 1) & 1;
                        const uint4* row = reinterpret_cast<const uint4*>(&wbuf[(bb * 64 + lane) * kWRow]);
                        uint32_t w[16];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const uint4 v = row[q];
                            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
                        }
                        kw_expand_store(w, reinterpret_cast<uint4*>(&kw[(bb * 64 + lane) * kPcRow]));
                    }
                } else if (wave == 0 && it >= lag && it - lag < m0.y) {  // block it-lag from buffer (it-lag) & 1
                    compress_kw(st, reinterpret_cast<const uint4*>(&kw[(((it - lag) & 1) * 64 + lane) * kPcRow]));
                }
                lds_barrier();
                RF_STAMP(sk); ++sk;
            }
            // Hand-over first, frontier second: the chain wave stores the digest
            // and passes a fused target's digest through s_dig / s_next, then
            // runs the frontier atomics (each a returning HBM round trip) while
            // the producer already assembles and expands the target's block 0.
            // No second barrier: s_next / s_dig are rewritten only at the next
            // job's finish, after the block loop's barriers, and the producer
            // reads them before its first one.
            bool changed = false;
            if (wave == 0) {
                uint32_t next = ~0u;
                if (has) {
                    changed = finish_job_pre(a, m1, st, olo, ohi);
                    if (changed && m1.w != ~0u) {
                        next = m1.w;
                        s_dig[lane][0] = make_uint4(bswap32(st.h[0]), bswap32(st.h[1]), bswap32(st.h[2]),
                                                    bswap32(st.h[3]));
                        s_dig[lane][1] = make_uint4(bswap32(st.h[4]), bswap32(st.h[5]), bswap32(st.h[6]),
                                                    bswap32(st.h[7]));
                    }
                }
                s_next[lane] = next;
            }
            RF_STAMP(sk); ++sk;
            lds_barrier();
            const uint32_t nx = s_next[lane];
            if (wave == 0) {
                uint32_t cb = 0, ce = 0;
                if (has) {
                    a.dirty[p] = 0u;
                    cb = m1.y;
                    // the fusion target's edge is the last of the range
                    ce = !changed ? m1.y : (m1.w != ~0u ? m1.z - 1 : m1.z);
                }
                propagate_pre(a, cb, ce, pre);
                const uint64_t fb = __ballot(nx != ~0u);
                if (lane == 0 && fb) atomicAdd(fused_part(a), (uint32_t)__popcll(fb));  // fused jobs hashed
            }
            fslot = has ? m1.x : ~0u;
            has = nx != ~0u;
            p = has ? nx : 0u;
        }
    }
}
#endif  // RF_DIAG

// k2_level_pl: k2_level_pc with two chain waves running the two-lane lagged
// chain (lag_chain.h RF_L2_*: 9 instructions per round instead of
// compress_kw's 14; ~1.2 instead of ~1.9 us per block).  A workgroup still
// takes 64 jobs: chain wave c holds jobs 32c..32c+31 (job j's e-lane and its
// row_half_mirror a-lane), the producer (kW = 2) or assembler + expander (kW
// = 3) waves hold one job per lane as before.  The chain runs every block
// step for all its lanes (a lane past its job's last block hashes stale rows
// and is ignored): a job's digest is its chaining value after group 0 of
// block nb (the k1_sha256_octo rule), combined into the e-lane with one
// mirror move per word.  Block counts differ between the waves' job sets,
// so the iteration count comes from LDS: s_nbx[j] = the fused target's block
// count, published with s_next at the hand-over and max-reduced by every
// wave (six shuffles; an LDS atomicMax into one word measured 10 us per step
// slower: 32 lanes per wave serialise on it).
// stamps (RF_K2_STAMPS): workgroup 0's chain wave 0 (row 0) and producer (row 1)
// Stamps go to LDS and are copied out at the kernel's end: a global store per
// stamp counts in vmcnt and turned the next vmcnt wait of the wave into a wait
// for the store's acknowledgement (phases looked ~0.5-1 us longer than they are).
#define RF_STAMP_PL(k)                                                                                \
    do {                                                                                              \
        if (kDiag && a.stamps && blockIdx.x == 0 && lane == 0 && (wave == 0 || wave == kProd) && (k) < 64)    \
            s_stamp[wave != 0][(k)] = __builtin_amdgcn_s_memrealtime();                              \
    } while (0)

// Streamed hand-over (kStream, kW = 2): no per-block barrier.  Blocks get
// workgroup-wide ids (consecutive over the launch; both waves count them the
// same way) and live in a ring of three LDS row buffers, id % 3.  The
// producer publishes a block's K+W rows in 16-word chunks -- s_flag[buffer]
// = 4 id + chunks written -- and the chain waits for exactly the chunk its
// next LDS read needs, so a fused job's block 0 starts right after its
// assembly, not after its whole expansion.  s_cons[c] = 1 + the last id
// chain wave c finished; the producer writes id only once both are >= id - 2.
// While the chain hashes a job's last block the producer is idle: it then
// builds the fusion target's block 1 (id + 1 of the next job) when that block
// is template-only (the fused hole ends in block 0: every 1000align link), so
// the next link's chain runs its blocks 0 and 1 back to back.
// Flags are written after s_waitcnt lgkmcnt(0) (the rows are in LDS) and
// polled with s_sleep; no global-memory wait is involved.
// Flag accesses are explicit ds_read/ds_write: a volatile access through the
// (generic) flag pointer compiles to a FLAT load/store, which counts in vmcnt
// as well, and every poll then waited for all the wave's HBM loads in flight
// (s_waitcnt vmcnt(0) lgkmcnt(0)).  The low 32 bits of a generic pointer into
// LDS are its LDS offset.
__device__ __forceinline__ uint32_t lds_ld(const volatile uint32_t* p) {
    uint32_t v;
    __asm__ volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(v)
                     : "v"((uint32_t)reinterpret_cast<uintptr_t>(p))
                     : "memory");
    return v;
}
__device__ __forceinline__ void lds_st(volatile uint32_t* p, uint32_t v) {
    __asm__ volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)reinterpret_cast<uintptr_t>(p)), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t lds_poll(volatile uint32_t* flag, uint32_t need, uint32_t known) {
    while ((int32_t)(known - need) < 0) {
        known = __builtin_amdgcn_readfirstlane(lds_ld(flag));
        if ((int32_t)(known - need) < 0) __builtin_amdgcn_s_sleep(1);
    }
    __asm__ volatile("" ::: "memory");
    return known;
}
__device__ __forceinline__ void lds_publish(volatile uint32_t* flag, uint32_t v, uint32_t lane) {
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(flag, v);
}
// As lds_publish for the chunk before the last one.  A partial count
// (lgkmcnt(4): "the four younger row writes may still be out") would let the
// drain overlap the next expansion, but it silently relies on the compiler
// emitting exactly four LDS writes per chunk and no SMEM load in between
// (SMEM also counts in lgkmcnt and returns out of order), so the wait is full.
__device__ __forceinline__ void lds_publish_prev(volatile uint32_t* flag, uint32_t v, uint32_t lane) {
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(flag, v);
}

// K+W[16c .. 16c+15] of a block into its row (kw_expand_store in chunks; w
// is the rolling 16-word schedule window, as there)
template <bool kStore = true>
__device__ __forceinline__ void kw_expand_chunk(uint32_t (&w)[16], uint4* row, int c) {
    constexpr uint32_t K[64] = RF_SHA_K;
#pragma unroll
    for (int t4 = 4 * c; t4 < 4 * c + 4; ++t4) {
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = 4 * t4 + u;
            uint32_t wt;
            if (t < 16) {
                wt = w[t];
            } else {
                wt = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
                w[t & 15] = wt;
            }
            v[u] = K[t] + wt;
        }
        if (kStore) row[t4] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// Block 0 of a fused job on the CHAIN wave (k2_level_pl, cb0): both lanes of
// the job (e-lane, a-lane: row_half_mirror partners) hold W[0..15] and
// expand W[16..63] together -- the e-lane sigma1(W[t-2]) + W[t-7], the a-lane
// sigma0(W[t-15]) + W[t-16], summed across the pair by one DPP add -- and the
// pair stores K+W into the job's row.  ~9 instructions per word instead of the
// producer's ~12, and no hand-over: the chain starts the rounds right after.
// kQ4 < 16 (split block 0): only K+W[0 .. 4 kQ4) -- the producer expands the rest.
template <int kQ4 = 16>
__device__ __forceinline__ void chain_expand_b0(uint32_t (&w)[16], bool elane, uint4* row) {
    constexpr uint32_t K[64] = RF_SHA_K;
    const uint32_t r1 = elane ? 17u : 7u, r2 = elane ? 19u : 18u, r3 = elane ? 10u : 3u;
    const uint32_t E = elane ? ~0u : 0u;  // selects by mask (one bitop3), never by address
#pragma unroll
    for (int t4 = 0; t4 < kQ4; ++t4) {
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = 4 * t4 + u;
            uint32_t wt;
            if (t < 16) {
                wt = w[t];
            } else {
                const uint32_t x = __builtin_amdgcn_bitop3_b32(E, w[(t - 2) & 15], w[(t - 15) & 15], 0xCA);
                const uint32_t y = __builtin_amdgcn_bitop3_b32(E, w[(t - 7) & 15], w[t & 15], 0xCA);
                const uint32_t h = xor3(__builtin_amdgcn_alignbit(x, x, r1), __builtin_amdgcn_alignbit(x, x, r2),
                                        x >> r3) + y;
                wt = h + (uint32_t)__builtin_amdgcn_mov_dpp((int)h, 0x141, 0xf, 0xf, true);  // + partner's half
                w[t & 15] = wt;
            }
            v[u] = K[t] + wt;
        }
        row[t4] = make_uint4(v[0], v[1], v[2], v[3]);  // both lanes: identical values, no EXEC change
    }
}

// Workgroup-uniform max of a lane value that is usually small (block counts):
// count up with ballots -- a compare and a scalar branch per step -- instead
// of six dependent ds_bpermute shuffles; shuffles above 64.
__device__ __forceinline__ uint32_t wave_max_small(uint32_t x) {
    uint32_t m = 0;
    while (m < 64 && __any(x > m)) ++m;
    if (m == 64) {
        for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
        m = x;
    }
    return __builtin_amdgcn_readfirstlane(m);
}

__device__ __forceinline__ uint32_t lf_job(const LevelArgs& a, uint32_t* ring, uint32_t ii, bool iv = false);
__device__ __forceinline__ void count_fused(const LevelArgs& a, uint32_t hashed);

// kJ = 64 jobs per workgroup (two chain waves), or 32 (one chain wave: the
// half workgroup, for levels a little wider than one 64-job workgroup per
// CU -- three fit a CU, each chain wave on a SIMD of its own)
template <uint32_t kW, bool kStream, uint32_t kJ = 64>
__global__ __launch_bounds__(64 * (kJ / 32 + kW - 1)) void k2_level_pl(LevelArgs a) {
    static_assert(kW == 2 || kW == 3, "producer (+ expander)");
    static_assert(!kStream || kW == 2, "streamed hand-over: producer + chain only");
    static_assert(kJ == 64 || (kJ == 32 && kW == 2 && !kStream), "the half workgroup: chain + producer");
    constexpr uint32_t lag = kW - 1;
    constexpr uint32_t kCW = kJ / 32;                  // chain waves
    constexpr uint32_t kProd = kCW, kExp = kCW + 1;    // wave roles: 0 .. kCW - 1 chain
    constexpr uint32_t kThreads = 64 * (kCW + kW - 1);
    constexpr uint32_t kBufs = kStream ? 3 : 2;  // row buffers of kJ rows
    // + the a-lanes' k row (kBufs kJ) and a junk row the half workgroup's
    // producer lanes without a job write their split chunks to
    constexpr uint32_t kOnes = kBufs * kJ, kJunk = kOnes + 1;
    __shared__ __attribute__((aligned(16))) uint32_t kw[(kBufs * kJ + 2) * kPcRow];
    __shared__ __attribute__((aligned(16))) uint32_t wbuf[kW == 3 ? 2 * 64 * kWRow : 4];
    __shared__ uint32_t ring_all[64 * kRing];
    __shared__ uint4 s_dig[64][2];
    __shared__ uint32_t s_next[64];
    __shared__ uint32_t s_flag[3], s_cons[2];
    __shared__ uint32_t s_nbx[64];  // fused targets' block counts (the next iteration's max)
    __shared__ uint4 s_pp[64][2];   // cb0: a finished job's {id, consumer range, valid}, first two edges
    __shared__ uint4 s_nnm[64][2];  // cb0 = 2: the fusion target's own target's record, from the producer
    // W[0..15] per job, staged by the chain: stream cb0, and the split block 0
    __shared__ uint32_t s_w0[kW == 2 ? 64 * 17 : 1];
    __shared__ uint32_t s_split;  // split block 0: (split + 1) sid + c once the producer's c-th chunk is in
    __shared__ uint32_t s_cw[2];                      // ... block id + 1 staged, per chain wave
    __shared__ uint32_t s_hq[64 * kHq];               // the producer's hole chunks (ChunkCursor)
    __shared__ unsigned long long s_stamp[2][64];
    __shared__ uint32_t s_runs[2 * kRunWords];
    static_assert(kThreads * kRing <= (kBufs * kJ + 2) * kPcRow, "the sink lanes' rings live in kw");
    stage_runs(a, s_runs);
    if (a.sink_wg && blockIdx.x >= a.sink_wg) {
        // the attached sink list (and with ovf the own list's overflow), one
        // job per lane, below the chains' priority: these lanes fill the
        // issue slots the latency form's waves leave idle instead of taking
        // CUs from its workgroups
        // (RF_K2_OVF=2: overflow lanes at the chains' priority, A/B)
        if (a.ovf == 2) __builtin_amdgcn_s_setprio(3);
        WgStamp ws;
        ws.begin(a);
        __syncthreads();
        const LaunchList ll(a, s_runs);
        constexpr uint32_t nt = kThreads;
        const uint32_t g2 = gridDim.x - a.sink_wg;
        const uint32_t lo = a.ovf ? min(ll.n1, a.sink_wg * kJ) : ll.n1;
        uint32_t hashed = 0;
        for (uint32_t base = lo + (blockIdx.x - a.sink_wg) * nt; base < ll.n; base += g2 * nt) {
            if (threadIdx.x == 0) ws.jobs += min(nt, ll.n - base);
            const uint32_t i = base + threadIdx.x;
            hashed += lf_job(a, &kw[threadIdx.x * kRing], i < ll.n ? ll.at(a, i) : ~0u);
        }
        count_fused(a, hashed);
        ws.end(a);
        return;
    }
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t* ring = &ring_all[lane * kRing];
    // chain lanes: half-row position hp; e-lanes hp & 4 == 0, partner 7 - hp
    const uint32_t hp = lane & 15;
    const bool elane = (hp & 4) == 0;
    const uint32_t ep = elane ? hp : ((hp & 8) | (7 - (hp & 7)));
    const uint32_t jl = wave < kCW ? 32 * wave + 8 * (lane >> 4) + ((ep & 3) | ((ep >> 3) << 2)) : lane;
    uint32_t* const ones = &kw[kOnes * kPcRow];
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        ones[lane] = lane ? 1u : 0u;
        if (lane < kPcRow - 64) ones[64 + lane] = 1u;
    }
    if (wave == 1 && kCW > 1) __builtin_amdgcn_s_setprio(3);
    if (threadIdx.x == 0) {
        s_flag[0] = s_flag[1] = s_flag[2] = 0;
        s_cons[0] = s_cons[1] = 0;
        s_cw[0] = s_cw[1] = 0;
        s_split = 0;
    }
    if (kDiag && a.stamps && threadIdx.x < 128) s_stamp[threadIdx.x >> 6][threadIdx.x & 63] = 0;
    lds_barrier();
    // streamed: next block id, flags seen, a pre-built block 1 of the next job
    uint32_t gb = 0, known = 0, known_c0 = 0, known_c1 = 0, pre_id = ~0u;
    // (producer) a pre-built block the next job did not use -- it had one
    // block, or there was none -- must not stay published: its id is the next
    // job's block 0 (or later), whose rows are not written yet
    auto drop_pre = [&]() {
        if (pre_id != ~0u && pre_id >= gb) lds_publish(&s_flag[pre_id % 3], 4 * pre_id, lane);
        pre_id = ~0u;
    };
    // Σ amounts of the lane's half (Σ1: 6 11 25 on e-lanes, Σ0: 2 13 22 on a-lanes)
    const uint32_t sh1 = elane ? 6u : 2u, sh2 = elane ? 11u : 13u, sh3 = elane ? 25u : 22u;
    const uint32_t M = elane ? 0u : ~0u;
    const uint32_t one = 1u, zero = 0u;
    constexpr uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    zero_other_counts(a);
    WgStamp ws;
    ws.begin(a);
    const LaunchList ll(a, s_runs);  // (staged before the barrier above)
    // (lane workgroups: the list's tail is theirs)
    const uint32_t n = !a.sink_wg ? ll.n : a.ovf ? min(ll.n1, a.sink_wg * kJ) : ll.n1;
    const uint32_t gstride = a.sink_wg ? a.sink_wg : gridDim.x;
    // One copy of the loop per wave role (chain / producer / expander), each
    // with only its own state: the register allocator then sizes the kernel
    // for the largest role instead of the sum of all roles' live values, and
    // a role's waits no longer cover the other roles' loads in flight.  Every
    // role runs the same barrier sequence (its control comes from LDS).
    auto body = [&](auto rc) {
        constexpr uint32_t R = decltype(rc)::value;
        constexpr bool kChain = R < kCW, kIsProd = R == kProd, kIsExp = R == kExp;
        // split passes so far (every role counts them alike: the flag values)
        uint32_t sid = 0, known_sp = 0;
        for (uint32_t base = blockIdx.x * kJ; base < n; base += gstride * kJ) {
            if (threadIdx.x == 0) ws.jobs += min(kJ, n - base);
            const uint32_t i = base + jl;
            bool has = jl < kJ && i < n;  // (half workgroup: producer lanes kJ.. have none)
            const uint32_t ii = has ? ll.at(a, i) : 0u;  // (list position, when has)
            uint32_t p = has ? a.list[ii] : 0u;
            // the listed job's record (append_jobs wrote it beside the list)
            uint4 lm0 = make_uint4(0, 0, 0, 0), lm1 = lm0;
            if (has) {
                lm0 = a.lmeta[2ull * ii];
                lm1 = a.lmeta[2ull * ii + 1];
            }
            uint32_t fslot = ~0u;
            uint32_t maxnb;
            {
                const uint32_t il = base + lane;
                maxnb = wave_max_small(lane < kJ && il < n ? a.lmeta[2ull * ll.at(a, il)].y : 0u);
            }
            uint4 nm0 = make_uint4(0, 0, 0, 0), nm1 = nm0, nolo = nm0, nohi = nm0, nnm0 = nm0, nnm1 = nm0;
            uint4 nt[8];
            uint2 nr = make_uint2(0, 0);
            // split block 0: the job's block 1 was built during the job before it
            // (producer, per lane), and the pass's row-buffer parity: block b of
            // the pass is in buffer (b + xp) & 1 (every role, workgroup-uniform)
            bool pre1 = false;
            uint32_t xp = 0;
            uint2 npre[2] = {make_uint2(0, 0), make_uint2(0, 0)};
            uint4 nmlo = make_uint4(IV[0], IV[1], IV[2], IV[3]), nmhi = make_uint4(IV[4], IV[5], IV[6], IV[7]);
            uint32_t sk = 0;
            // cb0 (kW == 2, barrier hand-over): from the second pass on every job
            // is a fusion target whose block 0 the chain wave builds itself --
            // W[0..15] (wb0) read back from the producer's ring at the previous
            // job's finish, after the chain OR-ed the new digest into its hole
            // (nrc: the target's hole record, fetched a job ahead)
            constexpr bool kCB = kW == 2 && !kStream;
            uint32_t pass = 0;
            bool pend = false;  // (producer) s_pp holds the last finished jobs, not yet propagated
            // cb0 = 2: the chain fetches only the fusion target's old digest
            // and first two reverse edges; its template (the producer's ring)
            // and its own target's record (s_nnm) come from the producer, and
            // its start state is the IV (its hole is at byte 2: no constant
            // leading block)
            const bool handoff = kCB && a.cb0 == 2 && a.handoff;

            // cb0: the frontier atomics of a finished job run on the producer
            // (idle in a pass's last iteration), not on the chain's critical path
            auto producer_propagate = [&]() {
                const uint4 q = s_pp[lane][0], e = s_pp[lane][1];
                const bool v = lane < kJ && q.w != 0;  // (half workgroup: lanes kJ.. hold no job)
                if (v) a.dirty[q.x] = 0u;
                const uint2 pe[2] = {make_uint2(e.x, e.y), make_uint2(e.z, e.w)};
                propagate_pre(a, v ? q.y : 0u, v ? q.z : 0u, pe);
                pend = false;
            };
            // kW = 3: as with cb0, a finished job's frontier atomics run on the
            // producer in its idle last iteration of the next pass, not on the
            // chain's critical path (RF_K2_DBG_NOEXP=6: on the chain, A/B)
            const bool pp3 = kW == 3 && !kStream && dbg_mode(a) != 6;
            uint32_t wb0[16];
    #pragma unroll
            for (int q = 0; q < 16; ++q) wb0[q] = lane + q;  // (pass 0's warm-up expands these)
            uint2 nrc = make_uint2(0, 0);
            uint4 ntc[4];  // cb0 = 2: the fusion target's template block 0, fetched a job ahead
            while (maxnb) {
                RF_STAMP_PL(sk); ++sk;
                const bool cb0 = kCB && a.cb0 && pass > 0;  // workgroup-uniform
                // split block 0 (cb0 = 2 with precomputed block-1 rows): the
                // chain expands K+W[16..31] only and the producer K+W[32..63]
                // of block 0 from the W[0..15] the chain staged, beside
                // copying block 1's precomputed rows
                const bool split = kCB && a.cb0 == 2 && a.split && pass > 0;
                // this pass's last iteration builds the fusion targets' block 1
                // into the buffer its own last block leaves free
                const bool build1 = kCB && a.cb0 == 2 && a.split;
                // streamed hand-over with a register-built block 0: the chain
                // writes chunk 0 (K+W[0..15]) itself and stages W[0..15] for the
                // producer, which expands chunks 1-3 while the chain runs rounds 0-15
                const bool sc = kStream && a.cb0 == 2 && pass > 0;
                const bool fused = fslot != ~0u;
                // a job is fused in every lane that has one after the first pass
                const bool wfused = __any(fused);
                uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
                if (has) {
                    if (fused) {
                        m0 = nm0;
                        m1 = nm1;
                        nm0 = nnm0;
                        nm1 = nnm1;
                    } else {
                        m0 = lm0;
                        m1 = lm1;
                    }
                }
                const bool nfu = has && m1.w != ~0u;
                if (nfu && !fused) {
                    nm0 = a.meta[2ull * m1.w];
                    nm1 = a.meta[2ull * m1.w + 1];
                    // (chain: as below -- the wait in the branch, not at the join;
                    // the chain idles in a pass-0 job's first iteration anyway)
                    if (kChain && !RF_K2_JOIN_WAIT) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                }
                ChunkCursor cur;
                cur.hq = &s_hq[lane * kHq];
                uint4 olo = make_uint4(0, 0, 0, 0), ohi = olo;
                uint2 pre[2] = {make_uint2(0, 0), make_uint2(0, 0)};
                if (!kStream && dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                if (kIsProd && has) {
                    cur.fslot = fslot;
                    if (cb0 || sc) {
                        cur.begin_chain(m0, reinterpret_cast<const uint4*>(a.tmpl));
                    } else if (fused) {
                        cur.flo = s_dig[lane][0];
                        cur.fhi = s_dig[lane][1];
                        cur.begin_pre(m0, reinterpret_cast<const uint4*>(a.tmpl), nt, nr, ring);
                    } else {
                        cur.begin(a, m0, ring);
                    }
                }
                // the job's initial chaining value H (IV, or the midstate after its
                // constant leading blocks): the fused target's was fetched a job ahead
                uint4 hlo = make_uint4(IV[0], IV[1], IV[2], IV[3]), hhi = make_uint4(IV[4], IV[5], IV[6], IV[7]);
                if (kChain && has) {
                    if (fused) {
                        olo = nolo;
                        ohi = nohi;
                        pre[0] = npre[0];
                        pre[1] = npre[1];
                        hlo = nmlo;
                        hhi = nmhi;
                    } else {
                        const uint4* od = reinterpret_cast<const uint4*>(a.slots + 32ull * m1.x);
                        olo = od[0];
                        ohi = od[1];
                        if (m1.y < m1.z) pre[0] = a.cons[m1.y];
                        if (m1.y + 1 < m1.z) pre[1] = a.cons[m1.y + 1];
                        if (a.mid) {
                            hlo = a.mid[2ull * p];
                            hhi = a.mid[2ull * p + 1];
                        }
                        // Wait for these loads here, inside the branch: at the join
                        // below the compiler placed a vmcnt(0) that every pass ran,
                        // and on a fused pass it waited for the previous job's digest
                        // store and atomics (vmcnt counts stores on gfx9): ~1-4 us
                        // on each link's block 0 (stamps, pass 1 5.4 us vs 1.7).
                        if (!RF_K2_JOIN_WAIT) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                    }
                }
                if (kIsExp && nfu && nm1.w != ~0u) {
                    nnm0 = a.meta[2ull * nm1.w];
                    nnm1 = a.meta[2ull * nm1.w + 1];
                }
                // the chain's lagged state: as after a block whose raw state is zero
                // with chaining value H (lag_chain.h / k1_sha256_duo, there H = IV)
                uint32_t Hr0 = elane ? hhi.x : hlo.x, Hr1 = elane ? hhi.y : hlo.y;
                uint32_t Hr2 = elane ? hhi.z : hlo.z, Hr3 = elane ? hhi.w : hlo.w;
                uint32_t Pa = 0, Pb = 0, Pc = 0, Pd = 0;
                uint32_t Z = elane ? hhi.w + hlo.w : 0u, Y = 0;
                uint32_t c63 = 0, c64 = elane ? hlo.z : 0u - hhi.x, c65 = elane ? hlo.y : 0u - hlo.w;
                // the fusion target's records, issued only after the state above
                // is built from this job's: a wait for this job's loads must not
                // also wait for these (they are used one job later).  The empty
                // asm pins the order (the compiler otherwise sinks the state's
                // selects below the loads and waits for everything, vmcnt(0)).
                __asm__ volatile("" ::"v"(Hr0), "v"(Hr1), "v"(Hr2), "v"(Hr3), "v"(Z), "v"(c64), "v"(c65) : "memory");
                if (kChain && has && nfu) {
                    const uint4* od = reinterpret_cast<const uint4*>(a.slots + 32ull * nm1.x);
                    nolo = od[0];
                    nohi = od[1];
                    if (handoff) {  // (the reverse edges the producer propagates with, as without handoff)
                        if (nm1.y < nm1.z) npre[0] = a.cons[nm1.y];
                        if (nm1.y + 1 < nm1.z) npre[1] = a.cons[nm1.y + 1];
                    }
                }
                if (kChain && has && nfu && !handoff) {
                    if (kW == 2) {
                        nrc = fused_hole(a, nm0.z);
                        if (a.cb0 == 2) {
                            const uint4* nT = reinterpret_cast<const uint4*>(a.tmpl) + 4ull * nm0.x;
                            ntc[0] = nT[0]; ntc[1] = nT[1]; ntc[2] = nT[2]; ntc[3] = nT[3];
                        }
                    }
                    if (nm1.y < nm1.z) npre[0] = a.cons[nm1.y];
                    if (nm1.y + 1 < nm1.z) npre[1] = a.cons[nm1.y + 1];
                    if (nm1.w != ~0u) {
                        nnm0 = a.meta[2ull * nm1.w];
                        nnm1 = a.meta[2ull * nm1.w + 1];
                    }
                    if (a.mid && !a.fuse_pos2) {  // (a fuse_pos2 target starts from the IV)
                        nmlo = a.mid[2ull * m1.w];
                        nmhi = a.mid[2ull * m1.w + 1];
                    }
                }
                if (kChain && dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }  // (the next target's loads issued)
                uint32_t t0, t1, t2, t3;
                uint32_t D0 = 0, D1 = 0, D2 = 0, D3 = 0;
                bool spl0 = false;  // (chain) the block step below is a split block 0
                const uint32_t nbl = m0.y;  // this lane's job's blocks (0: no job)
                // one block step of the chain over block b's rows (group 0 first
                // finishes block b-1: feed-forward, the a-half's last two rounds)
                // b: the job's block (capture rule), bufb: its row buffer (kStream:
                // the global block gb, whose chunks it waits for)
                auto chain_block = [&](uint32_t b, uint32_t bufb, bool full, bool own0 = false) {
                    const uint32_t bi = kStream ? bufb % 3 : (bufb & 1);
                    if (kStream && full && !own0) known = lds_poll(&s_flag[bi], 4 * bufb + 1, 4 * bufb);
                    if (kStream && full && dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                    const uint32_t row_off = ((bi * kJ + jl) * kPcRow) * 4, ones_off = kOnes * kPcRow * 4;
                    const uint4* r4 = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(kw) +
                                                                     ((M & ones_off) | (~M & row_off)));
                    uint4 v = r4[0], vn = r4[1];
                    {
                        const uint32_t k1 = v.y + c64, k2 = v.z + c65;
                        asm volatile(RF_L2_GROUP0
                                     : RF_LAG_STATE, RF_L2_TMP, RF_LAG_H,
                                       [c63] "=&v"(c63), [c64] "+v"(c64), [c65] "+v"(c65)
                                     : RF_L2_IN(k1, k2, v.w, vn.x), [kw0] "v"(v.x), [one] "v"(one),
                                       [zero] "v"(zero));
                    }
                    if (b == nbl) {  // the job's final chaining value
                        D0 = Hr0; D1 = Hr1; D2 = Hr2; D3 = Hr3;
                    }
                    if (!full) return;
                    v = vn;
                    vn = r4[2];
    #pragma unroll
                    for (int g = 1; g < 16; ++g) {
                        uint4 vnn = vn;
                        if (kStream && (g == 2 || g == 6 || g == 10)) {  // r4[g + 2] opens chunk (g + 2) / 4
                            known = lds_poll(&s_flag[bi], 4 * bufb + (g + 2) / 4 + 1, known);
                            if (dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                        }
                        // split block 0: r4[g + 2] opens the producer's chunk (g + 2) / 4
                        // (split 1: chunks 2, 3; split 2: chunks 1-3)
                        if (!kStream && spl0 && (g == 6 || g == 10 || (g == 2 && a.split == 2)))
                            known_sp = lds_poll(&s_split, (a.split + 1) * sid + (g + 2) / 4 - (a.split == 2 ? 0u : 1u),
                                                known_sp);
                        if (g < 14) vnn = r4[g + 2];
                        const uint32_t k4 = g == 15 ? c63 : vn.x;
                        asm volatile(RF_L2_GROUP : RF_LAG_STATE, RF_L2_TMP : RF_L2_IN(v.y, v.z, v.w, k4));
                        v = vn;
                        vn = vnn;
                    }
                };
                if constexpr (kStream) {
                    if (kIsProd) {
                        for (uint32_t b = 0; b < maxnb; ++b, ++gb) {
                            if (gb == pre_id) continue;  // built during the previous job, flag published
                            if (gb >= 3) {  // buffer gb % 3: both chain waves past block gb - 3
                                known_c0 = lds_poll(&s_cons[0], gb - 2, known_c0);
                                known_c1 = lds_poll(&s_cons[1], gb - 2, known_c1);
                            }
                            if (dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                            const bool mine = b < m0.y;
                            uint32_t w[16];
                            volatile uint32_t* fl = &s_flag[gb % 3];
                            uint4* row = reinterpret_cast<uint4*>(&kw[((gb % 3) * 64 + lane) * kPcRow]);
                            if (sc && b == 0) {
                                // the chain wrote chunk 0 and staged W[0..15]: expand 1-3
                                (void)lds_poll(&s_cw[0], gb + 1, 0u);
                                (void)lds_poll(&s_cw[1], gb + 1, 0u);
    #pragma unroll
                                for (int q = 0; q < 16; ++q) w[q] = s_w0[lane * 17 + q];
    #pragma unroll
                                for (int c = 1; c < 4; ++c) {
                                    if (mine) kw_expand_chunk(w, row, c);
                                    lds_publish(fl, 4 * gb + c + 1, lane);
                                }
                            } else {
                                if (mine) cur.block(a, b, ring, w, wfused);
    #pragma unroll
                                for (int c = 0; c < 4; ++c) {
                                    if (mine) kw_expand_chunk(w, row, c);
                                    if (c == 0)  // the chain starts on it: publish at once
                                        lds_publish(fl, 4 * gb + 1, lane);
                                    else if (c >= 2)  // chunk c - 1, its writes drained behind chunk c's
                                        lds_publish_prev(fl, 4 * gb + c, lane);
                                    if (dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                                }
                                lds_publish(fl, 4 * gb + 4, lane);
                            }
                            if (b == 0 && nfu) {
                                const uint4* nT = reinterpret_cast<const uint4*>(a.tmpl) + 4ull * nm0.x;
                                nt[0] = nT[0]; nt[1] = nT[1]; nt[2] = nT[2]; nt[3] = nT[3];
                                if (nm0.y > 1) {
                                    nt[4] = nT[4]; nt[5] = nT[5]; nt[6] = nT[6]; nt[7] = nT[7];
                                }
                                nr = fused_hole(a, nm0.z);
                                if (nm1.w != ~0u) {
                                    nnm0 = a.meta[2ull * nm1.w];
                                    nnm1 = a.meta[2ull * nm1.w + 1];
                                }
                            }
                            RF_STAMP_PL(sk); ++sk;
                        }
                        // idle until the hand-over: build the fusion targets' block 1
                        // (the next job's second id) if every lane whose target has
                        // a block 1 can -- it holds no hole (the fused digest ends
                        // in block 0) and the target has exactly two blocks
                        const bool need = nfu && nm0.y >= 2;
                        const bool can = nm0.y == 2 && nr.x + 32 <= 64;
                        if (a.cb0 == 2 && nfu && nm0.y > 1) {
                            const uint4 b1[4] = {nt[4], nt[5], nt[6], nt[7]};
                            ring_put(ring, 16, b1);
                        }
                        drop_pre();
                        if (__any(need) && __all(!need || can)) {
                            const uint32_t id1 = gb + 1;
                            known_c0 = lds_poll(&s_cons[0], id1 - 2, known_c0);
                            known_c1 = lds_poll(&s_cons[1], id1 - 2, known_c1);
                            uint4* row = reinterpret_cast<uint4*>(&kw[((id1 % 3) * 64 + lane) * kPcRow]);
                            if (need) {
                                uint32_t w[16] = {nt[4].x, nt[4].y, nt[4].z, nt[4].w, nt[5].x, nt[5].y, nt[5].z, nt[5].w,
                                                  nt[6].x, nt[6].y, nt[6].z, nt[6].w, nt[7].x, nt[7].y, nt[7].z, nt[7].w};
    #pragma unroll
                                for (int q = 0; q < 16; ++q) w[q] = bswap32(w[q]);
    #pragma unroll
                                for (int c = 0; c < 4; ++c) kw_expand_chunk(w, row, c);
                            }
                            lds_publish(&s_flag[id1 % 3], 4 * id1 + 4, lane);
                            pre_id = id1;
                        }
                    } else {
                        for (uint32_t b = 0; b < maxnb; ++b, ++gb) {
                            const bool own0 = sc && b == 0;
                            if (own0) {  // chunk 0 into the row, W[0..15] staged for the producer
                                constexpr uint32_t K[16] = {0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u,
                                                            0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
                                                            0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u,
                                                            0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u};
                                uint4* row = reinterpret_cast<uint4*>(&kw[((gb % 3) * 64 + jl) * kPcRow]);
    #pragma unroll
                                for (int q = 0; q < 4; ++q)
                                    row[q] = make_uint4(K[4 * q] + wb0[4 * q], K[4 * q + 1] + wb0[4 * q + 1],
                                                        K[4 * q + 2] + wb0[4 * q + 2], K[4 * q + 3] + wb0[4 * q + 3]);
    #pragma unroll
                                for (int q = 0; q < 16; ++q) s_w0[jl * 17 + q] = wb0[q];
                                lds_publish(&s_cw[wave], gb + 1, lane);
                            }
                            chain_block(b, gb, true, own0);
                            lds_publish(&s_cons[wave], gb + 1, lane);
                            RF_STAMP_PL(sk); ++sk;
                        }
                    }
                } else {
                const uint32_t iters = cb0 ? maxnb : maxnb + lag;
                for (uint32_t it = 0; it < iters; ++it) {
                    if (kIsProd) {
                        const uint32_t pb = cb0 ? it + 1 : it;  // the block this iteration builds
                        // split: block 0's K+W[32..63] from the W[0..15] the chain
                        // staged (chunk 1 only rolls the window: K+W[16..31] are the
                        // chain's); block 1 was built during the job before
                        const bool tab = split && it == 0 && has && pre1;
                        if (split && it == 0) {
                            uint32_t w[16];
    #pragma unroll
                            for (int q = 0; q < 16; ++q) w[q] = s_w0[lane * 17 + q];
                            if (dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                            uint4* row0 = reinterpret_cast<uint4*>(&kw[(lane < kJ ? (xp & 1) * kJ + lane : kJunk) * kPcRow]);
                            const uint32_t fb = (a.split + 1) * sid;  // this pass's flag values: fb + 1 ..
                            if (a.split == 2) {  // chunks 1-3 (the chain wrote chunk 0 only)
                                kw_expand_chunk(w, row0, 1);
                                lds_publish(&s_split, fb + 1, lane);
                                kw_expand_chunk(w, row0, 2);
                                lds_publish(&s_split, fb + 2, lane);
                            } else {  // chunks 2, 3 (chunk 1 only rolls the window)
                                kw_expand_chunk<false>(w, row0, 1);
                                kw_expand_chunk(w, row0, 2);
                                lds_publish(&s_split, fb + 1, lane);
                            }
                            if (dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                            kw_expand_chunk(w, row0, 3);
                            lds_publish(&s_split, fb + a.split + 1, lane);
                            if (dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                            if (tab) cur.skip(1, ring);  // (a longer target's block 2 on from the cursor)
                            // the last pass's frontier atomics here, where the chain's
                            // rounds of block 0 leave the producer time, not in the
                            // last iteration, which builds the next block 1
                            if (pend) producer_propagate();
                            if (dbg_mode(a) == 2) { RF_STAMP_PL(sk); ++sk; }
                        }
                        if (pb < m0.y && !tab && !((dbg_mode(a) == 3 && pb >= 1) || dbg_mode(a) == 4)) {
                            uint32_t w[16];
                            cur.block(a, pb, ring, w, wfused);
                            // (RF_K2_STAMPS=3: every block's assembly end on the producer)
                            if ((dbg_mode(a) == 2 && it == 0) || dbg_mode(a) == 8) { RF_STAMP_PL(sk); ++sk; }
                            if (kW == 2) {
                                kw_expand_store(w, reinterpret_cast<uint4*>(&kw[(((pb + xp) & 1) * kJ + lane) * kPcRow]));
                            } else {
                                uint4* row = reinterpret_cast<uint4*>(&wbuf[((it & 1) * 64 + lane) * kWRow]);
    #pragma unroll
                                for (int q = 0; q < 4; ++q)
                                    row[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
                            }
                        }
                        if (it == 0 && nfu) {
                            const uint4* nT = reinterpret_cast<const uint4*>(a.tmpl) + 4ull * nm0.x;
                            nt[0] = nT[0]; nt[1] = nT[1]; nt[2] = nT[2]; nt[3] = nT[3];
                            if (nm0.y > 1) {
                                nt[4] = nT[4]; nt[5] = nT[5]; nt[6] = nT[6]; nt[7] = nT[7];
                            }
                            nr = fused_hole(a, nm0.z);
                            if (nm1.w != ~0u) {
                                nnm0 = a.meta[2ull * nm1.w];
                                nnm1 = a.meta[2ull * nm1.w + 1];
                            }
                        }

                        // idle in the last iteration (every block of the pass built):
                        // the fusion target's template blocks 0 and 1 into the ring,
                        // for the chain to OR the digest into at the hand-over
                        if (((kCB && a.cb0) || pp3) && it + 1 == iters && pend) producer_propagate();
                        if (kCB && a.cb0 && it + 1 == iters && nfu) {
                            const uint4 b0[4] = {nt[0], nt[1], nt[2], nt[3]}, b1[4] = {nt[4], nt[5], nt[6], nt[7]};
                            ring_put(ring, 0, b0);
                            if (nm0.y > 1) ring_put(ring, 16, b1);
                            if (handoff) {
                                s_nnm[lane][0] = nnm0;
                                s_nnm[lane][1] = nnm1;
                            }
                        }
                        // split: the fusion target's block 1 (template only: its one
                        // hole ends in block 0) into the buffer this pass's last
                        // block leaves free -- the next pass's block-1 buffer
                        if (build1 && it + 1 == iters) {
                            pre1 = nfu && nm0.y >= 2;
                            if (pre1) {
                                uint32_t w[16] = {nt[4].x, nt[4].y, nt[4].z, nt[4].w, nt[5].x, nt[5].y, nt[5].z, nt[5].w,
                                                  nt[6].x, nt[6].y, nt[6].z, nt[6].w, nt[7].x, nt[7].y, nt[7].z, nt[7].w};
    #pragma unroll
                                for (int q = 0; q < 16; ++q) w[q] = bswap32(w[q]);
                                kw_expand_store(w, reinterpret_cast<uint4*>(&kw[(((maxnb + xp) & 1) * kJ + lane) * kPcRow]));
                            }
                        }
                    } else if (kIsExp) {
                        if (it >= 1 && it - 1 < m0.y && !((dbg_mode(a) == 3 && it >= 2) || dbg_mode(a) == 4)) {
                            const uint32_t bb = (it - 1) & 1;
                            const uint4* row = reinterpret_cast<const uint4*>(&wbuf[(bb * 64 + lane) * kWRow]);
                            uint32_t w[16];
    #pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const uint4 v = row[q];
                                w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
                            }
                            kw_expand_store(w, reinterpret_cast<uint4*>(&kw[(bb * 64 + lane) * kPcRow]));
                        }
                    } else if (kChain) {
                        // One call site each for the expansion and the block step, so
                        // pass 0 (producer-built rows) and the cb0 passes run the same
                        // code.  Every launch starts with a cold instruction cache:
                        // the first cb0 pass used to fetch ~9 KB of new code (its own
                        // inlined block step and the expansion) and took ~4.5 us
                        // longer than the later links.  In pass 0's first iteration
                        // the chain only waits for the producer's first row, so it
                        // runs the expansion there once on dummy words into the
                        // other row buffer (the producer writes it only after the
                        // barrier): the code is then cached when the links start.
                        const bool exb = it == 0 && (cb0 || (kCB && a.cb0 && pass == 0 && dbg_mode(a) != 5));
                        if (exb) {
                            uint4* row = reinterpret_cast<uint4*>(&kw[((cb0 ? (xp & 1) * kJ : kJ) + jl) * kPcRow]);
                            if (!kStream && a.split == 2)  // (pass 0: warms the code the split passes run)
                                chain_expand_b0<4>(wb0, elane, row);
                            else if (!kStream && a.split)
                                chain_expand_b0<8>(wb0, elane, row);
                            else
                                chain_expand_b0(wb0, elane, row);
                        }
                        if (dbg_mode(a) == 2 && it == 0) { RF_STAMP_PL(sk); ++sk; }
                        if (cb0 || it >= lag) {
                            const uint32_t cbk = cb0 ? it : it - lag;
                            spl0 = split && it == 0;
                            chain_block(cbk, cbk + xp, true);
                        }
                        if (dbg_mode(a) == 2 && it == 0) { RF_STAMP_PL(sk); ++sk; }
                    }
                    lds_barrier();
                    RF_STAMP_PL(sk); ++sk;
                }
                }
                bool changed = false;
                const bool own = kChain && has && elane;
                if (kChain) {
                    // The fusion target's prefetched records (issued at this job's
                    // start, blocks ago: arrived) are made to count as arrived here,
                    // before the digest store and frontier atomics: vmcnt also counts
                    // those, so a wait for the records at the next job's start would
                    // otherwise be a vmcnt(0) that waits for the store's HBM ack.
                    __asm__ volatile("" ::"v"(nolo.x), "v"(nolo.y), "v"(nolo.z), "v"(nolo.w), "v"(nohi.x), "v"(nohi.y),
                                     "v"(nohi.z), "v"(nohi.w), "v"(npre[0].x), "v"(npre[0].y), "v"(npre[1].x),
                                     "v"(npre[1].y), "v"(nmlo.x), "v"(nmlo.y), "v"(nmlo.z), "v"(nmlo.w));
                    __asm__ volatile("" ::"v"(nmhi.x), "v"(nmhi.y), "v"(nmhi.z), "v"(nmhi.w), "v"(nnm0.x), "v"(nnm0.y),
                                     "v"(nnm0.z), "v"(nnm0.w), "v"(nnm1.x), "v"(nnm1.y), "v"(nnm1.z), "v"(nnm1.w),
                                     "v"(nm0.x), "v"(nm0.y), "v"(nm0.z), "v"(nm0.w));
                    __asm__ volatile("" ::"v"(nm1.x), "v"(nm1.y), "v"(nm1.z), "v"(nm1.w));
                    chain_block(maxnb, kStream ? gb : maxnb + xp, false);  // group 0 of block maxnb: the longest jobs' final value
                    // the a-lane's half (H0..H3) into its e-lane (H4..H7 there)
                    ShaState st;
                    st.h[0] = __builtin_amdgcn_mov_dpp((int)D0, 0x141, 0xf, 0xf, true);
                    st.h[1] = __builtin_amdgcn_mov_dpp((int)D1, 0x141, 0xf, 0xf, true);
                    st.h[2] = __builtin_amdgcn_mov_dpp((int)D2, 0x141, 0xf, 0xf, true);
                    st.h[3] = __builtin_amdgcn_mov_dpp((int)D3, 0x141, 0xf, 0xf, true);
                    st.h[4] = D0; st.h[5] = D1; st.h[6] = D2; st.h[7] = D3;
                    uint32_t next = ~0u, nbn = 0;
                    if (own) {
                        changed = finish_job_pre(a, m1, st, olo, ohi);
                        if (changed && m1.w != ~0u) {
                            next = m1.w;
                            nbn = nm0.y;
                            const uint32_t D[8] = {bswap32(st.h[0]), bswap32(st.h[1]), bswap32(st.h[2]),
                                                   bswap32(st.h[3]), bswap32(st.h[4]), bswap32(st.h[5]),
                                                   bswap32(st.h[6]), bswap32(st.h[7])};
                            if (kCB && a.cb0 == 1) {  // into the target's block 0 (and 1), in the producer's ring
                                or_digest(&ring_all[jl * kRing], nrc.x, D);
                            } else if (!(kW == 2 && a.cb0 == 2)) {
                                s_dig[jl][0] = make_uint4(D[0], D[1], D[2], D[3]);
                                s_dig[jl][1] = make_uint4(D[4], D[5], D[6], D[7]);
                            }
                        }
                    }
                    if (kCB && a.cb0 == 1) {  // both lanes of the job: the target's W[0..15]
    #pragma unroll
                        for (int q = 0; q < 16; ++q) wb0[q] = bswap32(ring_all[jl * kRing + q]);
                    } else if (kW == 2 && a.cb0 == 2) {
                        // the digest's big-endian words H0..H7 in both lanes (the
                        // e-lane holds H4..7, its a-lane H0..3, each the other's
                        // half by the mirror moves above), then block 0 = the
                        // template with H at byte 2: W0 = T0 | H0 >> 16, Wk =
                        // H(k-1):Hk >> 16, W8 = H7 << 16 | T8
                        const uint32_t E = elane ? ~0u : 0u;
                        uint32_t H[8];
                        H[0] = __builtin_amdgcn_bitop3_b32(E, st.h[0], D0, 0xCA);
                        H[1] = __builtin_amdgcn_bitop3_b32(E, st.h[1], D1, 0xCA);
                        H[2] = __builtin_amdgcn_bitop3_b32(E, st.h[2], D2, 0xCA);
                        H[3] = __builtin_amdgcn_bitop3_b32(E, st.h[3], D3, 0xCA);
                        H[4] = __builtin_amdgcn_bitop3_b32(E, D0, st.h[0], 0xCA);
                        H[5] = __builtin_amdgcn_bitop3_b32(E, D1, st.h[1], 0xCA);
                        H[6] = __builtin_amdgcn_bitop3_b32(E, D2, st.h[2], 0xCA);
                        H[7] = __builtin_amdgcn_bitop3_b32(E, D3, st.h[3], 0xCA);
                        if (handoff) {  // the target's template block 0, in the producer's ring
    #pragma unroll
                            for (int q = 0; q < 16; ++q) wb0[q] = bswap32(ring_all[jl * kRing + q]);
                            nnm0 = s_nnm[jl][0];
                            nnm1 = s_nnm[jl][1];
                        } else {
                            const uint32_t T[16] = {ntc[0].x, ntc[0].y, ntc[0].z, ntc[0].w, ntc[1].x, ntc[1].y,
                                                    ntc[1].z, ntc[1].w, ntc[2].x, ntc[2].y, ntc[2].z, ntc[2].w,
                                                    ntc[3].x, ntc[3].y, ntc[3].z, ntc[3].w};
    #pragma unroll
                            for (int q = 0; q < 16; ++q) wb0[q] = bswap32(T[q]);
                        }
                        wb0[0] |= H[0] >> 16;
    #pragma unroll
                        for (int q = 1; q < 8; ++q) wb0[q] = __builtin_amdgcn_alignbit(H[q - 1], H[q], 16);
                        wb0[8] |= H[7] << 16;
                        if (!kStream && a.split && elane)  // the next split pass's producer expands from these
    #pragma unroll
                            for (int q = 0; q < 16; ++q) s_w0[jl * 17 + q] = wb0[q];
                    }
                    if (elane) {
                        s_next[jl] = next;
                        s_nbx[jl] = nbn;
                        if ((kCB && a.cb0) || pp3) {
                            s_pp[jl][0] = make_uint4(p, m1.y, !changed ? m1.y : (m1.w != ~0u ? m1.z - 1 : m1.z),
                                                     own ? 1u : 0u);
                            s_pp[jl][1] = make_uint4(pre[0].x, pre[0].y, pre[1].x, pre[1].y);
                        }
                    }
                }
                RF_STAMP_PL(sk); ++sk;
                lds_barrier();
                RF_STAMP_PL(sk); ++sk;
                const uint32_t nx = jl < kJ ? s_next[jl] : ~0u;
                // split: the next pass's block 1 sits in the buffer this pass's
                // last block (maxnb - 1) left free, so its block b goes to
                // buffer (b + xp') & 1 with (1 + xp') & 1 = (maxnb + xp) & 1
                if (build1) xp = (maxnb + xp + 1) & 1;
                maxnb = wave_max_small(lane < kJ ? s_nbx[lane] : 0u);
                if (kChain) {
                    if (!(kCB && a.cb0) && !pp3) {
                        uint32_t cb = 0, ce = 0;
                        if (own) {
                            a.dirty[p] = 0u;
                            cb = m1.y;
                            ce = !changed ? m1.y : (m1.w != ~0u ? m1.z - 1 : m1.z);
                        }
                        propagate_pre(a, cb, ce, pre);
                    }
                    const uint64_t fb = __ballot(own && nx != ~0u);
                    if (lane == 0 && fb) atomicAdd(fused_part(a), (uint32_t)__popcll(fb));
                }
                if (kIsProd && ((kCB && a.cb0) || pp3)) pend = true;

                fslot = has ? m1.x : ~0u;
                has = nx != ~0u;
                p = has ? nx : 0u;
                if (split) ++sid;
                ++pass;
            }
            if (kStream && kIsProd) drop_pre();
            if (kIsProd && (kCB || kW == 3) && pend) producer_propagate();  // the last pass's jobs
        }
    };
    if (wave < kCW) {
        body(std::integral_constant<uint32_t, 0>{});
    } else if (wave == kProd) {
        body(std::integral_constant<uint32_t, kProd>{});
    } else {
        if constexpr (kW == 3) body(std::integral_constant<uint32_t, kExp>{});
    }
    if (kDiag && a.stamps && blockIdx.x == 0 && (wave == 0 || wave == kProd))
        a.stamps[128 * a.lvl + 64 * (wave != 0) + lane] = s_stamp[wave != 0][lane];
    ws.end(a);
}

// Load time: the chaining value after each job's constant leading blocks.
__global__ __launch_bounds__(256) void k2_midstates(const uint8_t* __restrict__ tmpl,
                                                    const uint32_t* __restrict__ start,
                                                    const uint32_t* __restrict__ lead, uint32_t n,
                                                    uint4* __restrict__ mid) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        ShaState st;
        st.init();
        const uint4* T = reinterpret_cast<const uint4*>(tmpl) + 4ull * start[i];
        for (uint32_t b = 0; b < lead[i]; ++b) {
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 v = T[4 * b + q];
                w[4 * q] = bswap32(v.x); w[4 * q + 1] = bswap32(v.y);
                w[4 * q + 2] = bswap32(v.z); w[4 * q + 3] = bswap32(v.w);
            }
            sha256_compress(st, w);
        }
        mid[2ull * i] = make_uint4(st.h[0], st.h[1], st.h[2], st.h[3]);
        mid[2ull * i + 1] = make_uint4(st.h[4], st.h[5], st.h[6], st.h[7]);
    }
}

// A fused job's operands, fetched a job ahead: its first two template blocks
// (tt), its one hole record (rr), its old digest (ol, oh) and its start state
// (hl, hh: the midstate, or untouched = IV).
__device__ __forceinline__ void fetch_fused_ops(const LevelArgs& a, uint32_t q, const uint4& q0, const uint4& q1,
                                                uint4 (&tt)[8], uint2& rr, uint4& ol, uint4& oh, uint4& hl,
                                                uint4& hh, bool jf) {
    const uint4* T = reinterpret_cast<const uint4*>(a.tmpl) + 4ull * q0.x;
    tt[0] = T[0]; tt[1] = T[1]; tt[2] = T[2]; tt[3] = T[3];
    if (q0.y > 1) {
        tt[4] = T[4]; tt[5] = T[5]; tt[6] = T[6]; tt[7] = T[7];
    }
    rr = fused_hole(a, q0.z, jf);
    const uint4* od = reinterpret_cast<const uint4*>(a.slots + 32ull * q1.x);
    ol = od[0];
    oh = od[1];
    if (a.mid && !fused_iv(a, jf)) {
        hl = a.mid[2ull * q];
        hh = a.mid[2ull * q + 1];
    }
}

// Hashes, one lane per chain, the fused chain that starts at job p (~0u: the
// lane has none): p's records m0/m1, its operands (fetch_fused_ops: t, r,
// olo/ohi, hlo/hhi) and its fusion target's records nm0/nm1 are in
// registers, and its one hole reads slot fslot, whose new digest flo/fhi is
// handed over in registers.  Each job whose digest changed hands it to its
// fusion target; a job's other consumers are queued (propagate) -- unless
// kProp is false (k3_mark_slots' split form: another wave queued them).
// Returns the jobs this lane hashed.  Called by every lane of the wave.
template <bool kProp = true>
__device__ __forceinline__ uint32_t hash_fused_chain(const LevelArgs& a, uint32_t* ring, uint32_t p, uint4 m0,
                                                     uint4 m1, uint4 nm0, uint4 nm1, uint4 (&t)[8], uint2 r,
                                                     uint4 olo, uint4 ohi, uint4 hlo, uint4 hhi, uint32_t fslot,
                                                     uint4 flo, uint4 fhi) {
    constexpr uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    const uint4* T4 = reinterpret_cast<const uint4*>(a.tmpl);
    uint32_t hashed = 0;
    while (__any(p != ~0u)) {
        uint32_t cb = 0, cz = 0, nx = ~0u;
        if (p != ~0u) {
            const bool nf = m1.w != ~0u;
            uint4 nt[8], nolo = olo, nohi = ohi;
            uint4 nhlo = make_uint4(IV[0], IV[1], IV[2], IV[3]), nhhi = make_uint4(IV[4], IV[5], IV[6], IV[7]);
            uint2 nr = r;
            uint4 nnm0 = nm0, nnm1 = nm1;
            if (nf) {
                fetch_fused_ops(a, m1.w, nm0, nm1, nt, nr, nolo, nohi, nhlo, nhhi, true);
                if (nm1.w != ~0u) {
                    nnm0 = a.meta[2ull * nm1.w];
                    nnm1 = a.meta[2ull * nm1.w + 1];
                }
            }
            MatCursor cur;
            cur.fslot = fslot;
            cur.flo = flo;
            cur.fhi = fhi;
            cur.begin_pre(m0, T4, t, r, ring);
            cur.q0.r.y = fslot;  // (its one hole reads the handed-over slot; fused_hole)
            ShaState st;
            st.h[0] = hlo.x; st.h[1] = hlo.y; st.h[2] = hlo.z; st.h[3] = hlo.w;
            st.h[4] = hhi.x; st.h[5] = hhi.y; st.h[6] = hhi.z; st.h[7] = hhi.w;
            for (uint32_t b = 0; b < cur.nb; ++b) {
                uint32_t w[16];
                cur.block(a, b, ring, w, true);
                sha256_compress(st, w);
            }
            // The next job's operands (issued at this job's start: arrived) are
            // made to count as arrived here, before the digest store and the
            // frontier atomics: vmcnt also counts stores, and the compiler's wait
            // for them after the store was a vmcnt(0) -- a store acknowledgement
            // on every job of the chain (as in k2_level_pl).
            if (!RF_K2_JOIN_WAIT) {
                __asm__ volatile("" ::"v"(nt[0].x), "v"(nt[0].y), "v"(nt[0].z), "v"(nt[0].w), "v"(nt[1].x), "v"(nt[1].y),
                                 "v"(nt[1].z), "v"(nt[1].w), "v"(nt[2].x), "v"(nt[2].y), "v"(nt[2].z), "v"(nt[2].w),
                                 "v"(nt[3].x), "v"(nt[3].y), "v"(nt[3].z), "v"(nt[3].w));
                __asm__ volatile("" ::"v"(nt[4].x), "v"(nt[4].y), "v"(nt[4].z), "v"(nt[4].w), "v"(nt[5].x), "v"(nt[5].y),
                                 "v"(nt[5].z), "v"(nt[5].w), "v"(nt[6].x), "v"(nt[6].y), "v"(nt[6].z), "v"(nt[6].w),
                                 "v"(nt[7].x), "v"(nt[7].y), "v"(nt[7].z), "v"(nt[7].w));
                __asm__ volatile("" ::"v"(nolo.x), "v"(nolo.y), "v"(nolo.z), "v"(nolo.w), "v"(nohi.x), "v"(nohi.y),
                                 "v"(nohi.z), "v"(nohi.w), "v"(nhlo.x), "v"(nhlo.y), "v"(nhlo.z), "v"(nhlo.w),
                                 "v"(nhhi.x), "v"(nhhi.y), "v"(nhhi.z), "v"(nhhi.w));
                __asm__ volatile("" ::"v"(nnm0.x), "v"(nnm0.y), "v"(nnm0.z), "v"(nnm0.w), "v"(nnm1.x), "v"(nnm1.y),
                                 "v"(nnm1.z), "v"(nnm1.w), "v"(nr.x), "v"(nr.y));
            }
            const bool ch = finish_job_pre(a, m1, st, olo, ohi);
            ++hashed;
            cb = m1.y;
            cz = !ch ? m1.y : (nf ? m1.z - 1 : m1.z);  // the fusion target's edge is the range's last
            if (ch && nf) {
                nx = m1.w;
                fslot = m1.x;
                flo = make_uint4(bswap32(st.h[0]), bswap32(st.h[1]), bswap32(st.h[2]), bswap32(st.h[3]));
                fhi = make_uint4(bswap32(st.h[4]), bswap32(st.h[5]), bswap32(st.h[6]), bswap32(st.h[7]));
                m0 = nm0;
                m1 = nm1;
#pragma unroll
                for (int q = 0; q < 8; ++q) t[q] = nt[q];
                r = nr;
                olo = nolo;
                ohi = nohi;
                hlo = nhlo;
                hhi = nhhi;
                nm0 = nnm0;
                nm1 = nnm1;
            }
        }
        if constexpr (kProp) propagate(a, cb, cz);
        p = nx;
    }
    return hashed;
}

// Adds the wave's fused-chain job counts to its fused part (jobs hashed outside
// the level lists, k3_step_end / rf_graph_recompute's total).
__device__ __forceinline__ void count_fused(const LevelArgs& a, uint32_t hashed) {
    for (int o = 32; o > 0; o >>= 1) hashed += __shfl_xor(hashed, o, 64);
    if (__lane_id() == 0 && hashed) atomicAdd(fused_part(a), hashed);
}

// A changed input slot s (digest nlo/nhi, already stored; cp0/cp1 its
// reverse-edge range): its consumers join their levels' lists, except the
// slot-fused one, which this lane hashes at once (one-lane SHA-256, the new
// digest handed over in registers) and follows through its fusion chain like
// the level kernels do -- never queued, so a level whose queueable jobs are
// all slot-fused is not launched (configs[2]: every leaf OpVal and its
// Coerce; before, a mark kernel, a launch gap and a level kernel whose list ->
// record -> hole -> digest loads started cold).  Each job of the chain starts
// with its record, first two template blocks, hole record, old digest and
// start state in registers: they and the next job's record are fetched while
// the job before it is hashed.  Called by every lane of the wave.
// MarkStamp (diagnostic builds): a lane's phase times, reduced per wave.
struct MarkStamp {
#ifdef RF_DIAG
    unsigned long long t0 = 0;
    uint32_t d[4] = {0, 0, 0, 0};
    __device__ __forceinline__ MarkStamp* sink(const LevelArgs& a) { return a.stamps ? this : nullptr; }
    __device__ __forceinline__ void begin() { t0 = __builtin_amdgcn_s_memrealtime(); }
    __device__ __forceinline__ void lap(int k) { d[k] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0); }
    // workgroups 0..31 of k3_mark_slots: {start, max over lanes of each lap}
    // into stamps row L (the level rows' stamps are [L][128])
    __device__ __forceinline__ void end(const LevelArgs& a) {
        if (!a.stamps || blockIdx.x >= 32) return;
        for (int k = 0; k < 4; ++k)
            for (int o = 32; o > 0; o >>= 1) d[k] = max(d[k], (uint32_t)__shfl_xor((int)d[k], o, 64));
        if (threadIdx.x == 0) {
            unsigned long long* r = a.stamps + 128ull * a.n_levels + 4 * blockIdx.x;
            r[0] = t0;
            r[1] = d[0] | ((unsigned long long)d[1] << 32);
            r[2] = d[2] | ((unsigned long long)d[3] << 32);
            r[3] = 1;
        }
    }
#else
    __device__ __forceinline__ MarkStamp* sink(const LevelArgs&) { return nullptr; }
    __device__ __forceinline__ void begin() {}
    __device__ __forceinline__ void lap(int) {}
    __device__ __forceinline__ void end(const LevelArgs&) {}
#endif
};

template <bool kProp = true>
__device__ __forceinline__ void mark_input_slot_from(const LevelArgs& a, uint32_t* ring, uint32_t s, const uint4& nlo,
                                                     const uint4& nhi, uint32_t c, uint32_t ce, uint32_t p, uint4 m0,
                                                     uint4 m1, MarkStamp* ms = nullptr) {
    constexpr uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    // the job's operands (fetched a job ahead after the first)
    uint4 nm0 = make_uint4(0, 0, 0, 0), nm1 = nm0, olo = nm0, ohi = nm0;
    uint4 hlo = make_uint4(IV[0], IV[1], IV[2], IV[3]), hhi = make_uint4(IV[4], IV[5], IV[6], IV[7]);
    uint4 t[8];
    uint2 r = make_uint2(~0u, 0u);
    if (p != ~0u) {
        fetch_fused_ops(a, p, m0, m1, t, r, olo, ohi, hlo, hhi, false);  // (slot-fused: its record)
        if (m1.w != ~0u) {
            nm0 = a.meta[2ull * m1.w];
            nm1 = a.meta[2ull * m1.w + 1];
        }
    }
    const uint32_t hashed =
        hash_fused_chain<kProp>(a, ring, p, m0, m1, nm0, nm1, t, r, olo, ohi, hlo, hhi, s, nlo, nhi);
    if (ms) ms->lap(1);
    // the slot's other consumers
    propagate(a, c, ce);
    if (ms) ms->lap(2);
    count_fused(a, hashed);
    if (ms) {
        vm_drain();
        ms->lap(3);
    }
}

// The same from the slot's reverse-edge range cp0/cp1 (no plan: the
// slot-fused job is the range's first edge, its record one more load away).
__device__ __forceinline__ void mark_input_slot(const LevelArgs& a, uint32_t* ring, bool changed, uint32_t s,
                                                const uint4& nlo, const uint4& nhi, uint32_t cp0, uint32_t cp1) {
    uint32_t c = changed ? cp0 : 0u, ce = changed ? cp1 : 0u, p = ~0u;
    uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
    const uint2 f = a.cons[c < ce ? c : 0u];
    if (c < ce && (f.y & kSlotFused)) {
        p = f.x;
        ++c;
        m0 = a.meta[2ull * p];
        m1 = a.meta[2ull * p + 1];
    }
    mark_input_slot_from(a, ring, s, nlo, nhi, c, ce, p, m0, m1);
}

// A slot's plan entry (GraphDev::plan) beside its old digest: {c, ce, p} and
// p's record, loaded in the round trip that reads the slot.
struct SlotPlan {
    uint4 v, m0, m1;
    __device__ __forceinline__ void load(const LevelArgs& a, uint32_t s) {
        const uint4* P = a.plan + 3ull * s;
        v = P[0];
        m0 = P[1];
        m1 = P[2];
    }
};

// Hashes, one lane per chain, the fused chain that starts at job p (~0u:
// none) with records m0/m1 and its one hole reading slot fslot, whose new
// digest flo/fhi is handed over in registers -- as hash_fused_chain, without
// fetching each next job's operands a job ahead (the throughput forms: other
// waves of the SIMD cover the round trips, and the registers the look-ahead
// needs would cost a wave per SIMD).  Returns the jobs this lane hashed.
// Called by every lane of the wave.
// jf: p is fused to a job (lf_job), not to an input slot (the mark kernel):
// its hole record need not be loaded (fused_hole); the chain's later jobs are.
__device__ __forceinline__ uint32_t hash_fused_chain_lean(const LevelArgs& a, uint32_t* ring, uint32_t p, uint4 m0,
                                                          uint4 m1, uint32_t fslot, uint4 flo, uint4 fhi, bool jf) {
    uint32_t hashed = 0;
    while (__any(p != ~0u)) {
        uint32_t cb = 0, cz = 0, nx = ~0u;
        if (p != ~0u) {
            // issued at the job's start, used at its end: its old digest and
            // its fusion target's record (two round trips off each link)
            const uint4* od = reinterpret_cast<const uint4*>(a.slots + 32ull * m1.x);
            const uint4 olo = od[0], ohi = od[1];
            const bool nf = m1.w != ~0u;
            uint4 nm0 = make_uint4(0, 0, 0, 0), nm1 = nm0;
            if (nf) {
                nm0 = a.meta[2ull * m1.w];
                nm1 = a.meta[2ull * m1.w + 1];
            }
            // the start state first: the template's wait in begin_fused then
            // covers it, so the block loop holds no load of the preheader's
            // (a midstate load issued after the template made the compiler put a
            // vmcnt(0) at the top of every block -- a full round trip on the
            // block b+2 template it had just issued)
            ShaState st;
            if (fused_iv(a, jf))
                st.init();  // (no constant leading blocks: no midstate load)
            else
                init_state(a, p, st);
            MatCursor cur;
            cur.fslot = fslot;
            cur.flo = flo;
            cur.fhi = fhi;
            cur.begin_fused(a, m0, ring, jf);
            jf = true;
            for (uint32_t b = 0; b < cur.nb; ++b) {
                uint32_t w[16];
                cur.block(a, b, ring, w, true);
                sha256_compress(st, w);
            }
            const bool ch = finish_job_pre(a, m1, st, olo, ohi);
            ++hashed;
            cb = m1.y;
            cz = !ch ? m1.y : (nf ? m1.z - 1 : m1.z);  // the fusion target's edge is the range's last
            if (ch && nf) {
                nx = m1.w;
                fslot = m1.x;
                flo = make_uint4(bswap32(st.h[0]), bswap32(st.h[1]), bswap32(st.h[2]), bswap32(st.h[3]));
                fhi = make_uint4(bswap32(st.h[4]), bswap32(st.h[5]), bswap32(st.h[6]), bswap32(st.h[7]));
                m0 = nm0;
                m1 = nm1;
            }
        }
        propagate(a, cb, cz);
        p = nx;
    }
    return hashed;
}

// k3_mark_slots' append wave (wave 1) for one changed slot (changed, plan
// pl): the slot's other consumers, then each job of its fused chain's
// consumers but its fusion target's edge (the range's last), walking the
// chain by its records -- the next job's record loaded before the current
// job's appends.  Called by every lane of the wave.
__device__ __forceinline__ void queue_chain_consumers(const LevelArgs& a, bool changed, const SlotPlan& pl) {
    uint32_t p = changed ? pl.v.z : ~0u;
    uint4 m1 = pl.m1;
    propagate(a, changed ? pl.v.x : 0u, changed ? pl.v.y : 0u);
    while (__any(p != ~0u)) {
        uint32_t cb = 0, cz = 0, nx = ~0u;
        uint4 nm1 = m1;
        if (p != ~0u) {
            const bool nf = m1.w != ~0u;
            cb = m1.y;
            cz = nf ? m1.z - 1 : m1.z;
            if (nf) {
                nx = m1.w;
                nm1 = a.meta[2ull * nx + 1];
            }
        }
        propagate(a, cb, cz);
        p = nx;
        m1 = nm1;
    }
}

constexpr uint32_t kMarkBlock = 64;
// change sets from GraphDev::cfg_thru_mark slots (RF_K2_THRU_MARK_DEFAULT =
// 98,304) mark in k3_mark_slots_lf (the resident waves of k3_mark_slots, two
// per SIMD at 240 VGPRs, hold 131k lanes)

// set_slots: write input digests; a changed slot queues (or hashes) its consumers.
#ifndef RF_MARK_SPLIT
#define RF_MARK_SPLIT 1  // (A/B builds: 0 = one wave a workgroup, the slot's other consumers after its chain)
#endif
// k3_mark_slots' waves per workgroup: wave 0 hashes the 64 slots' fused
// chains, wave 1 queues every consumer the slots and their chains' jobs
// reach (reverse edges, dirty bits and list appends: dependent round trips
// that followed each job's hash in the chain's lane), told which slots
// changed through LDS.  A chain's jobs have one hole each, their
// predecessor's digest (the first: the slot's), so each job's digest changes
// with its input -- short of a SHA-256 collision, where the consumers queued
// ahead are re-hashed to the same digests: extra work, never a different
// digest.
constexpr uint32_t kMarkWaves = (RF_MARK_SPLIT && RF_SLOT_PLAN) ? 2u : 1u;

__global__ __launch_bounds__(kMarkBlock * kMarkWaves) void k3_mark_slots(const uint32_t* __restrict__ sl,
                                                                         const uint8_t* __restrict__ dig, uint32_t n,
                                                                         LevelArgs a) {
    __shared__ uint32_t ring_all[kMarkBlock * kRing];
    __shared__ unsigned long long s_ch[2];
    const uint32_t wave = kMarkWaves > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0u;
    const uint32_t lane = threadIdx.x & (kMarkBlock - 1);
    uint32_t* ring = &ring_all[lane * kRing];
    MarkStamp ms;
    ms.begin();
    uint32_t it = 0;
    for (uint32_t base = blockIdx.x * kMarkBlock; base < n; base += gridDim.x * kMarkBlock, ++it) {
        const uint32_t i = base + lane;
        bool changed = false;
        uint32_t s = 0, cp0 = 0, cp1 = 0;
        uint4 nlo = make_uint4(0, 0, 0, 0), nhi = nlo;
        SlotPlan pl;
        pl.v = make_uint4(0, 0, ~0u, 0);
        pl.m0 = pl.m1 = nlo;
        if (i < n) {
            s = sl[i];
            if constexpr (RF_SLOT_PLAN) {
                pl.load(a, s);  // with the digests, not after the compare
            } else {
                cp0 = a.cons_ptr[s];
                cp1 = a.cons_ptr[s + 1];
            }
            if (wave == 0) {
                const uint4* src = reinterpret_cast<const uint4*>(dig + 32ull * i);
                uint4* dst = reinterpret_cast<uint4*>(a.slots + 32ull * s);
                nlo = src[0];
                nhi = src[1];
                const uint4 olo = dst[0], ohi = dst[1];
                changed = (olo.x != nlo.x) | (olo.y != nlo.y) | (olo.z != nlo.z) | (olo.w != nlo.w) |
                          (ohi.x != nhi.x) | (ohi.y != nhi.y) | (ohi.z != nhi.z) | (ohi.w != nhi.w);
                if (changed) {
                    dst[0] = nlo;
                    dst[1] = nhi;
                }
            }
        }
#ifdef RF_DIAG
        if (a.stamps) {
            __asm__ volatile("" ::"v"(pl.v.x), "v"(pl.m0.x), "v"(pl.m1.x), "v"(cp0));
            ms.lap(0);  // the slot's loads arrived (compare done)
        }
#endif
        if constexpr (kMarkWaves > 1) {
            if (wave == 0) {
                const unsigned long long ch = __ballot(changed);
                if (lane == 0) s_ch[it & 1] = ch;
            }
            __syncthreads();
            if (wave == 1) {  // the consumers, beside the chains
                queue_chain_consumers(a, (s_ch[it & 1] >> lane) & 1ull, pl);
                continue;
            }
            mark_input_slot_from<false>(a, ring, s, nlo, nhi, 0u, 0u, changed ? pl.v.z : ~0u, pl.m0, pl.m1,
                                        ms.sink(a));
        } else if constexpr (RF_SLOT_PLAN) {
            mark_input_slot_from(a, ring, s, nlo, nhi, changed ? pl.v.x : 0u, changed ? pl.v.y : 0u,
                                 changed ? pl.v.z : ~0u, pl.m0, pl.m1, ms.sink(a));
        } else {
            mark_input_slot(a, ring, changed, s, nlo, nhi, cp0, cp1);
        }
    }
    if (wave == 0) ms.end(a);
}

// Throughput form of an incremental level (chosen per level and step when
// the change set fills the chip, launch_graph_level): one lane per listed
// job, 256-thread workgroups, no producer / chain split -- every lane of
// every wave hashes (one-lane rounds, the schedule in registers).  A listed
// job's fused chain is followed in its lane by hash_fused_chain_lean (one
// hole, its digest handed over in registers, no look-ahead: 168 VGPRs, three
// waves per SIMD; the look-ahead form needed 251 and two, and measured 2 %
// slower on the 100M step).  k2_level_pl's two-lane chains shorten a link's
// latency but keep only 64 jobs per 192-thread workgroup resident (two per
// CU), so once a level's list is several times the resident set the step is
// bound by rounds of resident workgroups x link latency (configs[3]'s
// 100M-node DAG on one GPU), and this form is faster.
// One listed job per lane, the throughput form's body (k2_level_lf, and the
// sink list riding on an octo-form launch): list entry ii (~0u: none) is
// hashed in the lane, its fused chain followed in the lane; every lane of the
// wave calls it (propagate's appends are per wave).  Returns the fused jobs
// the lane hashed.
__device__ __forceinline__ uint32_t lf_job(const LevelArgs& a, uint32_t* ring, uint32_t ii, bool iv) {
    uint32_t p = ~0u;
    uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
    if (ii != ~0u) {
        p = a.list[ii];
        m0 = a.lmeta[2ull * ii];
        m1 = a.lmeta[2ull * ii + 1];
    }
    uint32_t cb = 0, cz = 0, nx = ~0u, fslot = ~0u;
    uint4 flo = make_uint4(0, 0, 0, 0), fhi = flo, nm0 = flo, nm1 = flo;
    if (p != ~0u) {
        ShaState st;
        if (iv)
            st.init();  // (its level has no constant leading blocks: LevelArgs::lead0)
        else
            init_state(a, p, st);  // (before the cursor's loads: see hash_fused_chain_lean)
        MatCursor cur;
        cur.begin(a, m0, ring);
        for (uint32_t b = 0; b < cur.nb; ++b) {
            uint32_t w[16];
            cur.block(a, b, ring, w);
            sha256_compress(st, w);
        }
        const bool ch = finish_job(a, m1, st);
        a.dirty[p] = 0u;
        const bool nf = m1.w != ~0u;
        cb = m1.y;
        cz = !ch ? m1.y : (nf ? m1.z - 1 : m1.z);
        if (ch && nf) {
            nx = m1.w;
            fslot = m1.x;
            flo = make_uint4(bswap32(st.h[0]), bswap32(st.h[1]), bswap32(st.h[2]), bswap32(st.h[3]));
            fhi = make_uint4(bswap32(st.h[4]), bswap32(st.h[5]), bswap32(st.h[6]), bswap32(st.h[7]));
            nm0 = a.meta[2ull * nx];
            nm1 = a.meta[2ull * nx + 1];
        }
    }
    propagate(a, cb, cz);
    return hash_fused_chain_lean(a, ring, nx, nm0, nm1, fslot, flo, fhi, true);
}

#ifndef RF_LF_PRIO
#define RF_LF_PRIO 0  // (A/B builds: 1 = sink workgroups at low issue priority, 2 = also the third wave a SIMD)
#endif
constexpr uint32_t kLfPrio = RF_LF_PRIO;
#ifndef RF_LF_WAVES
#define RF_LF_WAVES 3  // (A/B builds: waves a SIMD the throughput form is compiled for)
#endif
// Start delay of the throughput form's second and third resident workgroups
// on a CU, in 10-ns ticks per round (A/B builds: -DRF_LF_STAGGER=0 off).  A
// SIMD's waves run the same chains in step and waited for their loads
// together (the 100M Exec level: ~37 % of the critical SIMDs' issue slots
// idle with three waves on them); staggered by 3 us a round, 100M 0.7-1 %
// faster, per-sample 1 % (same box, profiles/r06/ab_stagger*); 7 us: neutral.
#ifndef RF_LF_STAGGER
#define RF_LF_STAGGER 300
#endif
__global__ __launch_bounds__(kLevelBlock, RF_LF_WAVES) void k2_level_lf(LevelArgs a) {  // (3 waves a SIMD: <= 168 VGPRs)
    __shared__ uint32_t ring_all[kLevelBlock * kRing];
    __shared__ uint32_t s_runs[2 * kRunWords];
    uint32_t* ring = &ring_all[threadIdx.x * kRing];
    if (RF_LF_STAGGER) {
        // the waves a SIMD holds run the same chains in step, so they wait for
        // their loads at the same time; start the CU's second and third
        // workgroups later
        const uint32_t r = blockIdx.x / a.n_cu;
        if (r) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)RF_LF_STAGGER * r) __builtin_amdgcn_s_sleep(8);
        }
    }
    stage_runs(a, s_runs);
    zero_other_counts(a);
    WgStamp ws;
    ws.begin(a);
    __syncthreads();
    const LaunchList ll(a, s_runs);
    const uint32_t n = ll.n;
    uint32_t hashed = 0;
    for (uint32_t base = blockIdx.x * kLevelBlock; base < n; base += gridDim.x * kLevelBlock) {
        if (threadIdx.x == 0) ws.jobs += min(kLevelBlock, n - base);
        if (kLfPrio) {
            // issue priority by what the workgroup holds: the level's own
            // (long) jobs high, the attached sinks (short, slack until the
            // long ones end) low; with kLfPrio 2 also own-list workgroups past
            // two a CU (the third wave on a SIMD) medium
            const bool own = base < ll.n1;
            const uint32_t pr = !own ? 0u : (kLfPrio == 2 && blockIdx.x >= 2 * a.n_cu) ? 1u : 2u;
            if (pr == 0) __builtin_amdgcn_s_setprio(0);
            else if (pr == 1) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(2);
        }
        const uint32_t i = base + threadIdx.x;
        hashed += lf_job(a, ring, i < n ? ll.at(a, i) : ~0u, (i < ll.n1 ? a.lead0 : a.lead0_2) != 0);
    }
    count_fused(a, hashed);
    ws.end(a);
}

// k3_mark_slots for change sets that fill the chip (GraphDev::thru form
// choice, at least cfg_thru_mark slots): the slot-fused chains without the
// look-ahead (hash_fused_chain_lean), so three waves fit a SIMD instead of
// two and a 100M-node DAG's 141k changed slots run in one round of resident
// waves.
__global__ __launch_bounds__(kMarkBlock) void k3_mark_slots_lf(const uint32_t* __restrict__ sl,
                                                               const uint8_t* __restrict__ dig, uint32_t n,
                                                               LevelArgs a) {
    __shared__ uint32_t ring_all[kMarkBlock * kRing];
    uint32_t* ring = &ring_all[threadIdx.x * kRing];
    uint32_t hashed = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        bool changed = false;
        uint32_t s = 0, c = 0, ce = 0;
        uint4 nlo = make_uint4(0, 0, 0, 0), nhi = nlo;
        SlotPlan pl;
        pl.v = make_uint4(0, 0, ~0u, 0);
        pl.m0 = pl.m1 = nlo;
        if (i < n) {
            s = sl[i];
            const uint4* src = reinterpret_cast<const uint4*>(dig + 32ull * i);
            uint4* dst = reinterpret_cast<uint4*>(a.slots + 32ull * s);
            nlo = src[0];
            nhi = src[1];
            if constexpr (RF_SLOT_PLAN) {
                pl.load(a, s);
                c = pl.v.x;
                ce = pl.v.y;
            } else {
                c = a.cons_ptr[s];
                ce = a.cons_ptr[s + 1];
            }
            const uint4 olo = dst[0], ohi = dst[1];
            changed = (olo.x != nlo.x) | (olo.y != nlo.y) | (olo.z != nlo.z) | (olo.w != nlo.w) |
                      (ohi.x != nhi.x) | (ohi.y != nhi.y) | (ohi.z != nhi.z) | (ohi.w != nhi.w);
            if (changed) {
                dst[0] = nlo;
                dst[1] = nhi;
            }
        }
        if (!changed) c = ce = 0;
        uint32_t p = ~0u;
        uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
        if constexpr (RF_SLOT_PLAN) {
            p = changed ? pl.v.z : ~0u;
            m0 = pl.m0;
            m1 = pl.m1;
        } else {
            const uint2 f = a.cons[c < ce ? c : 0u];
            if (c < ce && (f.y & kSlotFused)) {
                p = f.x;
                ++c;
                m0 = a.meta[2ull * p];
                m1 = a.meta[2ull * p + 1];
            }
        }
        hashed += hash_fused_chain_lean(a, ring, p, m0, m1, s, nlo, nhi, false);
        propagate(a, c, ce);  // the slot's other consumers
    }
    if (dbg_mode(a) != 16) count_fused(a, hashed);
}

// ---- the octo form: levels of few long jobs (GraphDev kLvlOct) ---------------
// k2_level_pl keeps 64 jobs per workgroup on two-lane chains (9 VALU a round)
// fed by a producer that assembles one block a step through a hole pipeline;
// on a level of a few hundred 18-block, 32-hole merge jobs (the merge tree
// above the fill level) the chip is nearly idle and that pipeline's chunk
// transitions set the pace: 1.3-1.7 us a block (the 8-rank piece's merge
// levels: 33 + 32 + 28 us, profiles/r03/s3/wg_c4r8.log).  Here a workgroup
// takes 8 jobs.  Every hole's digest is final when the level starts (level-
// synchronous), so the producer wave stages each job's WHOLE material in LDS
// first -- template blocks and hole records, then the holes' digests, each
// batch of loads issued back to back: two dependent HBM round trips for the 8
// jobs -- and then expands 8 blocks of each job per step (one lane per (job,
// block), double-buffered rows); the chain wave runs K1's octo chain (8 lanes
// a job, the duo's 8-instruction round: lag_chain.h RF_OCT_*).  Jobs have no
// fusion target, at most kOctMaxBlocks blocks and kOctMaxHoles holes
// (rf_graph_load's kLvlOct analysis).  An attached sink list (LaunchList)
// runs in the workgroups from a.oct_wg on, one job per lane as k2_level_lf
// (lf_job, the ring in the kw array): the octo workgroups come first in
// dispatch order, the short sinks fill the CUs the few long jobs leave idle.
constexpr uint32_t kOctStage = kOctMaxBlocks * 16 + 4;  // words per job's staged material (16-B aligned)

// OR digest D (8 LE words) into the linear material stage m at byte `pos`
// (or_digest without the ring wrap).
__device__ __forceinline__ void or_digest_lin(uint32_t* m, uint32_t pos, const uint32_t (&D)[8]) {
    const uint32_t x = pos >> 2, sh = 32 - 8 * (pos & 3);
    uint32_t prev = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const uint32_t cur = k < 8 ? D[k] : 0u;
        const uint32_t v = (uint32_t)((((uint64_t)cur << 32) | prev) >> sh);
        if (v) atomicOr(&m[x + k], v);
        prev = cur;
    }
}

__global__ __launch_bounds__(128) void k2_level_oct(LevelArgs a) {
    // two buffers of 8 blocks x 8 jobs K+W rows (row j * 8 + f), then the
    // a-lanes' k row (as k1_sha256_octo); the 8 jobs' staged materials
    __shared__ __attribute__((aligned(16))) uint32_t kw[129 * kPcRow];
    __shared__ __attribute__((aligned(16))) uint32_t mat[8 * kOctStage];
    __shared__ uint32_t s_runs[2 * kRunWords];
    static_assert(128 * kRing <= 129 * kPcRow, "the sink lanes' rings live in kw");
    stage_runs(a, s_runs);
    __syncthreads();
    const LaunchList ll(a, s_runs);
    if (blockIdx.x >= a.oct_wg) {  // the attached sink list, one job per lane
        WgStamp ws;
        ws.begin(a);
        const uint32_t g2 = gridDim.x - a.oct_wg;
        uint32_t hashed = 0;
        for (uint32_t base = ll.n1 + (blockIdx.x - a.oct_wg) * 128; base < ll.n; base += g2 * 128) {
            if (threadIdx.x == 0) ws.jobs += min(128u, ll.n - base);
            const uint32_t i = base + threadIdx.x;
            hashed += lf_job(a, &kw[threadIdx.x * kRing], i < ll.n ? ll.at(a, i) : ~0u);
        }
        count_fused(a, hashed);
        ws.end(a);
        return;
    }
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t f = lane >> 3;  // the lane's job of the group (both waves)
    uint32_t* const ones = &kw[128 * kPcRow];
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        ones[lane] = lane ? 1u : 0u;
        if (lane < kPcRow - 64) ones[64 + lane] = 1u;
    }
    const bool elane = (lane & 4) == 0;
    const uint32_t q3 = lane & 3;
    const uint32_t shq = elane ? (q3 == 1 ? 11u : q3 == 2 ? 25u : 6u) : (q3 == 1 ? 13u : q3 == 2 ? 22u : 2u);
    const uint32_t M = elane ? 0u : ~0u;
    const uint32_t one = 1u, zero = 0u;
    constexpr uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    zero_other_counts(a);
    WgStamp ws;
    ws.begin(a);
    const uint32_t n = ll.n1;
    const uint4* T4 = reinterpret_cast<const uint4*>(a.tmpl);
    for (uint32_t base = blockIdx.x * 8; base < n; base += a.oct_wg * 8) {
        if (threadIdx.x == 0) ws.jobs += min(8u, n - base);
        const uint32_t i = base + f;
        const bool has = i < n;
        uint32_t p = 0;
        uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
        if (has) {
            const uint32_t ii = ll.at(a, i);
            p = a.list[ii];
            m0 = a.lmeta[2ull * ii];
            m1 = a.lmeta[2ull * ii + 1];
        }
        const uint32_t nb = min(m0.y, kOctMaxBlocks);  // (0 without a job; the clamp only guards the stage)
        uint32_t maxnb = nb;
        for (int o = 8; o < 64; o <<= 1) maxnb = max(maxnb, (uint32_t)__shfl_xor((int)maxnb, o, 64));
        maxnb = __builtin_amdgcn_readfirstlane(maxnb);
        // (producer) K+W rows of blocks 8c .. 8c+7 of each job into buffer c & 1
        auto expand = [&](uint32_t c) {
            const uint32_t j = lane & 7, b = 8 * c + j;
            if (b < nb) {
                const uint4* src = reinterpret_cast<const uint4*>(&mat[f * kOctStage + 16 * b]);
                uint32_t w[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint4 v = src[q];
                    w[4 * q] = bswap32(v.x); w[4 * q + 1] = bswap32(v.y);
                    w[4 * q + 2] = bswap32(v.z); w[4 * q + 3] = bswap32(v.w);
                }
                kw_expand_store(w, reinterpret_cast<uint4*>(&kw[((c & 1) * 64 + j * 8 + f) * kPcRow]));
            }
        };
        // (chain) the job's start state and old digest, fetched now, used at the end
        uint4 hlo = make_uint4(IV[0], IV[1], IV[2], IV[3]), hhi = make_uint4(IV[4], IV[5], IV[6], IV[7]);
        uint4 olo = make_uint4(0, 0, 0, 0), ohi = olo;
        if (wave == 0) {
            if (has && a.mid) {
                hlo = a.mid[2ull * p];
                hhi = a.mid[2ull * p + 1];
            }
            if (has) {
                const uint4* od = reinterpret_cast<const uint4*>(a.slots + 32ull * m1.x);
                olo = od[0];
                ohi = od[1];
            }
        } else {
            // 1. the 8 jobs' templates and hole records (one lane per hole)
            uint4 tv[8][2];
            uint2 hr[8];
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const uint32_t tb = __builtin_amdgcn_readlane(m0.x, 8 * g);
                const uint32_t bg = min(__builtin_amdgcn_readlane(m0.y, 8 * g), kOctMaxBlocks);
                const uint32_t hb = __builtin_amdgcn_readlane(m0.z, 8 * g);
                const uint32_t he = __builtin_amdgcn_readlane(m0.w, 8 * g);
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const uint32_t q = lane + 64 * k;
                    tv[g][k] = q < 4 * bg ? T4[4ull * tb + q] : make_uint4(0, 0, 0, 0);
                }
                hr[g] = hb + lane < he ? a.holes[hb + lane] : make_uint2(~0u, 0u);
            }
            // 2. the holes' digests
            uint4 dlo[8], dhi[8];
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const uint4* src = reinterpret_cast<const uint4*>(a.slots + 32ull * (hr[g].x != ~0u ? hr[g].y : 0u));
                dlo[g] = src[0];
                dhi[g] = src[1];
            }
            // 3. templates into the stage, then each digest OR-ed into its zero hole
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const uint32_t bg = min(__builtin_amdgcn_readlane(m0.y, 8 * g), kOctMaxBlocks);
                uint4* st = reinterpret_cast<uint4*>(&mat[g * kOctStage]);
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const uint32_t q = lane + 64 * k;
                    if (q < 4 * bg) st[q] = tv[g][k];
                }
            }
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                if (hr[g].x <= kOctMaxBlocks * 64 - 32) {
                    const uint32_t D[8] = {dlo[g].x, dlo[g].y, dlo[g].z, dlo[g].w, dhi[g].x, dhi[g].y, dhi[g].z, dhi[g].w};
                    or_digest_lin(&mat[g * kOctStage], hr[g].x, D);
                }
            }
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            expand(0);
        }
        __syncthreads();  // chunk 0's rows
        uint32_t Hr0 = elane ? hhi.x : hlo.x, Hr1 = elane ? hhi.y : hlo.y;
        uint32_t Hr2 = elane ? hhi.z : hlo.z, Hr3 = elane ? hhi.w : hlo.w;
        uint32_t Pa = 0, Pb = 0, Pc = 0, Pd = 0;
        uint32_t Z = elane ? hhi.w + hlo.w : 0u, Y = 0;
        uint32_t c63 = 0, c64 = elane ? hlo.z : 0u - hhi.x, c65 = elane ? hlo.y : 0u - hlo.w;
        uint32_t t0, t1, t3;
        uint32_t D0 = 0, D1 = 0, D2 = 0, D3 = 0;
        uint4 v = make_uint4(0, 0, 0, 0), vn = v;
        for (uint32_t c = 0; 8 * c < maxnb; ++c) {
            if (wave == 1) {
                if (8 * (c + 1) < maxnb) expand(c + 1);
            } else {
                const uint32_t cnt = min(8u, maxnb - 8 * c);
                // e-lanes read their job's rows, a-lanes the ones row
                const uint32_t ones_off = 128 * kPcRow * 4, buf_off = ((c & 1) * 64 + f) * kPcRow * 4;
                const uint4* r4 = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(kw) +
                                                                 ((M & ones_off) | (~M & buf_off)));
                v = r4[0];
                vn = r4[1];
                for (uint32_t j = 0; j < cnt; ++j) {
                    const uint32_t nrow_off = buf_off + (j + 1 < cnt ? j + 1 : j) * 8 * kPcRow * 4;
                    const uint4* r4n = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(kw) +
                                                                      ((M & ones_off) | (~M & nrow_off)));
                    uint4 vnn = r4[2];
                    {
                        const uint32_t k1 = v.y + c64, k2 = v.z + c65;
                        asm volatile(RF_OCT_GROUP0
                                     : RF_LAG_STATE, RF_LAG_TMP, RF_LAG_H, [c63] "=&v"(c63), [c64] "+v"(c64),
                                       [c65] "+v"(c65)
                                     : RF_LAG_IN(k1, k2, v.w, vn.x), [kw0] "v"(v.x), [one] "v"(one), [zero] "v"(zero));
                    }
                    if (8 * c + j == nb) {  // the job's final chaining value
                        D0 = Hr0; D1 = Hr1; D2 = Hr2; D3 = Hr3;
                    }
                    v = vn;
                    vn = vnn;
#pragma unroll
                    for (int g = 1; g < 16; ++g) {
                        vnn = g < 14 ? r4[g + 2] : r4n[g - 14];
                        const uint32_t k4 = g == 15 ? c63 : vn.x;
                        asm volatile(RF_OCT_GROUP : RF_LAG_STATE, RF_LAG_TMP : RF_LAG_IN(v.y, v.z, v.w, k4));
                        v = vn;
                        vn = vnn;
                    }
                    r4 = r4n;
                }
            }
            __syncthreads();
        }
        if (wave == 0) {
            {  // group 0 of block maxnb: the longest jobs' final value
                const uint32_t k1 = v.y + c64, k2 = v.z + c65;
                asm volatile(RF_OCT_GROUP0
                             : RF_LAG_STATE, RF_LAG_TMP, RF_LAG_H, [c63] "=&v"(c63), [c64] "+v"(c64), [c65] "+v"(c65)
                             : RF_LAG_IN(k1, k2, v.w, vn.x), [kw0] "v"(v.x), [one] "v"(one), [zero] "v"(zero));
            }
            if (nb == maxnb) {
                D0 = Hr0; D1 = Hr1; D2 = Hr2; D3 = Hr3;
            }
            // lane 8f (e) holds H4..H7, lane 8f + 4 (a) H0..H3
            ShaState st;
            st.h[0] = (uint32_t)__shfl((int)D0, (int)lane + 4, 64);
            st.h[1] = (uint32_t)__shfl((int)D1, (int)lane + 4, 64);
            st.h[2] = (uint32_t)__shfl((int)D2, (int)lane + 4, 64);
            st.h[3] = (uint32_t)__shfl((int)D3, (int)lane + 4, 64);
            st.h[4] = D0; st.h[5] = D1; st.h[6] = D2; st.h[7] = D3;
            const bool own = has && (lane & 7) == 0;
            bool changed = false;
            if (own) {
                changed = finish_job_pre(a, m1, st, olo, ohi);
                a.dirty[p] = 0u;
            }
            // no fusion target (kLvlOct): every consumer of a changed digest is queued
            propagate(a, own && changed ? m1.y : 0u, own && changed ? m1.z : 0u);
        }
    }
    ws.end(a);
}

// ---- partitioned DAG exchange (partition.cpp) --------------------------------
// Exports whose digest changed since last sent: their bit (bit0 + i) in the
// boundary bitset, the snapshot updated, the digest into the send block.
__global__ __launch_bounds__(256) void k_part_pack(const uint32_t* __restrict__ export_slot, uint32_t n,
                                                   const uint8_t* __restrict__ slots, uint8_t* snap, uint8_t* send,
                                                   uint32_t* bits, uint32_t bit0) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* src = reinterpret_cast<const uint4*>(slots + 32ull * export_slot[i]);
    uint4* sn = reinterpret_cast<uint4*>(snap + 32ull * i);
    const uint4 lo = src[0], hi = src[1], olo = sn[0], ohi = sn[1];
    const bool changed = (olo.x != lo.x) | (olo.y != lo.y) | (olo.z != lo.z) | (olo.w != lo.w) |
                         (ohi.x != hi.x) | (ohi.y != hi.y) | (ohi.z != hi.z) | (ohi.w != hi.w);
    if (changed) {
        const uint32_t b = bit0 + i;
        atomicOr(&bits[b >> 5], 1u << (b & 31));
        sn[0] = lo;
        sn[1] = hi;
    }
    uint4* dst = reinterpret_cast<uint4*>(send + 32ull * i);
    dst[0] = lo;
    dst[1] = hi;
}

// flag[0] = any bit set in the (OR-reduced) bitset; flag[1] = any of this
// rank's imports has its bit set (else its next superstep has nothing to do).
__global__ __launch_bounds__(256) void k_part_any(const uint64_t* __restrict__ bits, uint64_t nwords,
                                                  const uint32_t* __restrict__ import_bid, uint32_t n_import,
                                                  uint32_t* flag) {
    uint64_t v = 0;
    for (uint64_t i = threadIdx.x; i < nwords; i += blockDim.x) v |= bits[i];
    const int any = __syncthreads_or(v != 0);
    bool mine = false;
    if (any) {
        const uint32_t* b32 = reinterpret_cast<const uint32_t*>(bits);
        for (uint32_t i = threadIdx.x; i < n_import && !mine; i += blockDim.x) {
            const uint32_t b = import_bid[i];
            mine = (b32[b >> 5] >> (b & 31)) & 1u;
        }
    }
    const int my = __syncthreads_or(mine);
    if (threadIdx.x == 0) {
        flag[0] = any ? 1u : 0u;
        flag[1] = my ? 1u : 0u;
    }
}

// Imports whose boundary bit is set: the gathered digest into the slot; a
// changed slot queues its local consumers (as k3_mark_slots).
__global__ __launch_bounds__(kMarkBlock) void k_part_apply(const uint32_t* __restrict__ import_slot,
                                                           const uint32_t* __restrict__ import_bid, uint32_t n,
                                                           const uint32_t* __restrict__ bits,
                                                           const uint8_t* __restrict__ gather, LevelArgs a) {
    __shared__ uint32_t ring_all[kMarkBlock * kRing];
    uint32_t* ring = &ring_all[threadIdx.x * kRing];
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        bool changed = false;
        uint32_t s = 0, cp0 = 0, cp1 = 0;
        uint4 nlo = make_uint4(0, 0, 0, 0), nhi = nlo;
        SlotPlan pl;
        pl.v = make_uint4(0, 0, ~0u, 0);
        pl.m0 = pl.m1 = nlo;
        if (i < n) {
            const uint32_t b = import_bid[i];
            if (!bits || ((bits[b >> 5] >> (b & 31)) & 1u)) {  // null bits: every import (fixed rounds)
                s = import_slot[i];
                const uint4* src = reinterpret_cast<const uint4*>(gather + 32ull * b);
                uint4* dst = reinterpret_cast<uint4*>(a.slots + 32ull * s);
                nlo = src[0];
                nhi = src[1];
                if constexpr (RF_SLOT_PLAN) {
                    pl.load(a, s);
                } else {
                    cp0 = a.cons_ptr[s];
                    cp1 = a.cons_ptr[s + 1];
                }
                const uint4 olo = dst[0], ohi = dst[1];
                changed = (olo.x != nlo.x) | (olo.y != nlo.y) | (olo.z != nlo.z) | (olo.w != nlo.w) |
                          (ohi.x != nhi.x) | (ohi.y != nhi.y) | (ohi.z != nhi.z) | (ohi.w != nhi.w);
                if (changed) {
                    dst[0] = nlo;
                    dst[1] = nhi;
                }
            }
        }
        if constexpr (RF_SLOT_PLAN)
            mark_input_slot_from(a, ring, s, nlo, nhi, changed ? pl.v.x : 0u, changed ? pl.v.y : 0u,
                                 changed ? pl.v.z : ~0u, pl.m0, pl.m1);
        else
            mark_input_slot(a, ring, changed, s, nlo, nhi, cp0, cp1);
    }
}

// GraphDev::plan from the records: per slot its reverse-edge range past the
// slot-fused consumer (flagged first in the range at load), that consumer
// and its record.
__global__ __launch_bounds__(256) void k_slot_plan(const uint32_t* __restrict__ cons_ptr,
                                                   const uint2* __restrict__ cons, const uint4* __restrict__ meta,
                                                   uint32_t S, uint4* __restrict__ plan) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < S; s += gridDim.x * blockDim.x) {
        uint32_t c = cons_ptr[s], p = ~0u;
        const uint32_t ce = cons_ptr[s + 1];
        uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;
        if (c < ce) {
            const uint2 f = cons[c];
            if (f.y & kSlotFused) {
                p = f.x;
                ++c;
                m0 = meta[2ull * p];
                m1 = meta[2ull * p + 1];
            }
        }
        plan[3ull * s] = make_uint4(c, ce, p, 0u);
        plan[3ull * s + 1] = m0;
        plan[3ull * s + 2] = m1;
    }
}

// End of a recompute: record what each level hashed, reset the lists.
__global__ void k3_step_end(uint32_t* counts, uint32_t* last, const uint32_t* __restrict__ ls, uint32_t L,
                            int full) {
    // counts[L] + the fused parts: jobs hashed inside fused chains (never queued)
    for (uint32_t l = threadIdx.x; l < L; l += blockDim.x) {
        uint32_t c = counts[l];  // (the A/B build's one cursor a level)
        for (uint32_t k = 0; k < kListShards; ++k) c += counts[list_shard_off(L) + k * cursor_lp(L) + l];
        last[l] = full ? ls[l + 1] - ls[l] : c;
        counts[l] = 0;
    }
    if (threadIdx.x == 0) {
        uint32_t f = counts[L];
        for (uint32_t k = 0; k < kFusedParts; ++k) f += counts[L + 1 + kPartStride * k];
        last[L] = full ? 0u : f;
    }
    __syncthreads();
    for (uint32_t l = L + threadIdx.x; l < counts_half_words(L); l += blockDim.x) counts[l] = 0;
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

static uint32_t grid_mark(uint64_t items) {
    uint64_t g = (items + kMarkBlock - 1) / kMarkBlock;
    return (uint32_t)(g < 1 ? 1 : g > 16384 ? 16384 : g);
}

// The level-kernel arguments the mark / apply kernels hash slot-fused jobs with.
static LevelArgs mark_level_args(const GraphDev& g) {
    LevelArgs a{0, 0, 0, 0, 0, g.meta, g.holes, g.cons, g.lvl_start_dev, g.n_levels,
                g.tmpl, g.slots, g.dirty, g.list, g.counts, nullptr, g.mid, g.cons_ptr, g.lmeta, 0, 0, nullptr, nullptr};
    a.fuse_pos2 = g.fuse_pos2 ? 1u : 0u;
    a.sf_pos = g.sf_pos;
#ifdef RF_DIAG
    if (g.dbg_mark == 1) a.dbg_twice = 16;  // (diagnostic build: k3_mark_slots_lf skips its count)
    a.stamps = g.stamps;                     // (k3_mark_slots: MarkStamp into row L)
#endif
    a.plan = g.plan;
    return a;
}

hipError_t launch_slot_plan(const GraphDev& g, hipStream_t s) {
    if (!g.n_slots) return hipSuccess;
    hipLaunchKernelGGL(k_slot_plan, dim3(grid_for(g.n_slots, 8192)), dim3(256), 0, s, g.cons_ptr, g.cons, g.meta,
                       g.n_slots, g.plan);
    return hipGetLastError();
}

hipError_t launch_graph_mark_slots(GraphDev& g, const uint32_t* slots, const uint8_t* digests,
                                   uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    g.last_mark_lf = n >= g.cfg_thru_mark ? 1u : 0u;
    // the lean form from g.cfg_thru_mark slots (default RF_K2_THRU_MARK_DEFAULT; fixed per
    // graph, rf_graph_set_forms)
    if (n >= g.cfg_thru_mark)
        hipLaunchKernelGGL(k3_mark_slots_lf, dim3(grid_mark(n)), dim3(kMarkBlock), 0, s, slots, digests, n,
                           mark_level_args(g));
    else
        hipLaunchKernelGGL(k3_mark_slots, dim3(grid_mark(n)), dim3(kMarkBlock * kMarkWaves), 0, s, slots, digests, n,
                           mark_level_args(g));
    return hipGetLastError();
}

// The mark kernel as a graph kernel node (rf_graph_update_recompute_async):
// its launch parameters for this batch, argument values in `args`.
void graph_mark_params(const GraphDev& g, const uint32_t* slots, const uint8_t* digests, uint32_t n,
                       MarkArgs* args, hipKernelNodeParams* p) {
    static_assert(sizeof(MarkArgs::a) >= sizeof(LevelArgs), "MarkArgs::a holds the mark kernel's LevelArgs");
    args->sl = slots;
    args->dig = digests;
    args->n = n;
    const LevelArgs a = mark_level_args(g);
    memcpy(args->a, &a, sizeof(a));
    void* v[4] = {&args->sl, &args->dig, &args->n, args->a};
    for (int i = 0; i < 4; ++i) args->ptrs[i] = v[i];
    p->func = reinterpret_cast<void*>(k3_mark_slots);
    p->gridDim = dim3(n ? grid_mark(n) : 1);  // an empty batch still runs (and marks nothing)
    p->blockDim = dim3(kMarkBlock * kMarkWaves);
    p->sharedMemBytes = 0;
    p->kernelParams = args->ptrs;
    p->extra = nullptr;
}

const void* graph_mark_kernel() { return reinterpret_cast<const void*>(k3_mark_slots); }

// Whether an incremental plain step runs level lvl in the throughput form
// (k2_level_lf): min(its jobs, the step's marked input slots) reaches the
// threshold of its kind (GraphDev::thru_slots / thru_slots_wide).
bool graph_level_lf(const GraphDev& g, uint32_t lvl) {
    const uint64_t n = g.lvl_start[lvl + 1] - g.lvl_start[lvl];
    return std::min<uint64_t>(n, g.step_marked) >=
           ((g.inc_level[lvl] & kLvlForm) == 2 ? g.thru_slots_wide : g.thru_slots);
}

// Half workgroups (k2_level_pl<2, false, 32>) for a latency-form level of
// short jobs estimated at 64-96 chains per CU (RF_K2_HALF=0: never, A/B)
bool graph_level_half(const GraphDev& g, uint32_t lvl) {
    static const bool half_ok = RF_DIAG_KNOB("RF_K2_HALF", 1) != 0;
    static const bool one_lane = RF_DIAG_KNOB("RF_K2_CHAIN", 9) == 14;
    const uint64_t est = std::min<uint64_t>(g.lvl_start[lvl + 1] - g.lvl_start[lvl], g.step_marked);
    return half_ok && !one_lane && (g.inc_level[lvl] & kLvlForm) == 1 && !(g.inc_level[lvl] & kLvlOct) &&
           !g.stream_handover && g.n_cu && est > 64ull * g.n_cu && est <= 96ull * g.n_cu && !graph_level_lf(g, lvl);
}

hipError_t launch_graph_level(const GraphDev& g, uint32_t lvl, int full, hipStream_t s, uint32_t* zero_counts,
                              uint32_t sink_lvl) {
    const uint32_t b = g.lvl_start[lvl], e = g.lvl_start[lvl + 1];
    if (e <= b) return hipSuccess;
    // RF_DBG_HASH2: hash twice (k2_level); RF_K2_STAMPS=2: per-chunk stamps (k2_level_pl)
    // RF_K2_DBG_NOEXP=3|4 (timing diagnostic, WRONG digests): the producer
    // skips assembling + expanding blocks >= 1 (3) or every block (4); =5
    // (A/B, digests right): no instruction-cache warm-up in k2_level_pl's pass 0;
    // =6 (A/B): k2_level_pl<3>'s frontier atomics on the chain, not the producer
    // (diagnostic build only) RF_DBG_HASH2 -> 1, RF_K2_STAMPS=2|3 -> 2|8,
    // else RF_K2_DBG_NOEXP (3|4: WRONG digests, a timing probe)
    static const uint32_t dbg2 = RF_DIAG_KNOB("RF_DBG_HASH2", 0) ? 1u
                                 : RF_DIAG_KNOB("RF_K2_STAMPS", 0) == 2 ? 2u
                                 : RF_DIAG_KNOB("RF_K2_STAMPS", 0) == 3 ? 8u
                                                                       : (uint32_t)RF_DIAG_KNOB("RF_K2_DBG_NOEXP", 0);
    // RF_K2_CB0=0: fused jobs' block 0 built by the producer (A/B), else by the chain
    static const uint32_t cb0 = RF_DIAG_KNOB("RF_K2_CB0", 1) == 0 ? 0u : 1u;
    // RF_K2_REV=0: the list in append order (A/B)
    static const uint32_t rev = RF_DIAG_KNOB("RF_K2_REV", 1) == 0 ? 0u : 1u;
    LevelArgs a{b, e, lvl, full, dbg2, g.meta, g.holes, g.cons, g.lvl_start_dev, g.n_levels,
                g.tmpl, g.slots, g.dirty, g.list, g.counts, g.stamps, g.mid, g.cons_ptr, g.lmeta,
                g.hole_in_b0 && cb0 ? (g.fuse_pos2 ? 2u : 1u) : 0u, full ? 0u : rev, zero_counts,
                full ? nullptr : g.wgst};
    a.split = (!full && a.cb0 == 2) ? g.split_b0 : 0u;
    a.n_cu = g.n_cu ? g.n_cu : 256u;
    a.fuse_pos2 = g.fuse_pos2 ? 1u : 0u;
    a.sf_pos = g.sf_pos;
    a.lead0 = lvl < g.lvl_lead0.size() ? g.lvl_lead0[lvl] : 0u;
    a.lead0_2 = sink_lvl < g.lvl_lead0.size() ? g.lvl_lead0[sink_lvl] : 0u;
    static const uint32_t handoff = RF_DIAG_KNOB("RF_K2_HANDOFF", 1) == 0 ? 0u : 1u;  // (0: the chain fetches them itself)
    a.handoff = handoff;
    // incremental: the dirty count is only known on device; 1024 blocks (4
    // per CU, all resident) cover any level's list with a grid-stride loop
    static const uint32_t inc_cap = (uint32_t)RF_DIAG_KNOB("RF_INC_GRID", 1024);
    if (!full) {
        if (!(g.inc_level[lvl] & kLvlForm)) return hipSuccess;  // every job of the level is a fusion target
        // an attached sink list: its jobs after the level's own, same launch
        // (the grid sized for both)
        const uint32_t n2 = sink_lvl != ~0u ? g.lvl_start[sink_lvl + 1] - g.lvl_start[sink_lvl] : 0u;
        if (sink_lvl != ~0u) {
            a.s2 = g.lvl_start[sink_lvl];
            a.lvl2 = sink_lvl;
        }
        // grid cap (RF_K2_GRID): workgroups past the dirty count exit at once,
        // but each still costs a dispatch before the kernel can end
        static const uint64_t wg_cap = (uint64_t)RF_DIAG_KNOB("RF_K2_GRID", 2048);
        uint64_t wg = (e - b + n2 + 63) / 64;
        if (wg > wg_cap) wg = wg_cap;
        // RF_K2_CHAIN=14: the one-lane chain (k2_level_pc), for A/B runs
        static const bool one_lane = RF_DIAG_KNOB("RF_K2_CHAIN", 9) == 14;
        // a level of few long jobs (kLvlOct): the octo form, 8 jobs a
        // workgroup, then an attached sink list's workgroups (128 jobs each)
        if ((g.inc_level[lvl] & kLvlOct) && !one_lane) {
            a.oct_wg = std::min<uint32_t>((e - b + 7) / 8, 1024u);
            const uint32_t sg = std::min<uint32_t>((n2 + 127) / 128, 1024u);
            hipLaunchKernelGGL(k2_level_oct, dim3(a.oct_wg + sg), dim3(128), 0, s, a);
            return hipGetLastError();
        }
        const bool wide = (g.inc_level[lvl] & kLvlForm) == 2;
        // g.stream_handover (RF_K2_STREAM=1 at load): the streamed hand-over
        // (measured no faster on configs[2]: the producer serializes a fused
        // job's blocks 0 and 1); default per-block barriers
        const bool no_stream = !g.stream_handover;
        // RF_K2_PAD_KB: dynamic LDS per workgroup on top of the static arrays
        // (A/B: enough to keep a second workgroup off the CU, so no wave
        // shares a SIMD with another workgroup's prioritised chain wave)
        static const uint32_t pad = (uint32_t)RF_DIAG_KNOB("RF_K2_PAD_KB", 0) * 1024u;
        if (one_lane && sink_lvl != ~0u) {  // (k2_level_pc takes no attached list: the sink level after it)
            if (hipError_t err = launch_graph_level(g, lvl, 0, s, zero_counts)) return err;
            return launch_graph_level(g, sink_lvl, 0, s);
        }
        if (graph_level_lf(g, lvl)) {
            // the throughput form: 256 lanes per workgroup, four resident per
            // CU, grid-stride over the device-side count
            static const uint64_t lf_cap = (uint64_t)RF_DIAG_KNOB("RF_K2_LF_GRID", 1024);
            uint64_t lg = (e - b + n2 + kLevelBlock - 1) / kLevelBlock;
            if (lg > lf_cap) lg = lf_cap;
            hipLaunchKernelGGL(k2_level_lf, dim3((uint32_t)lg), dim3(kLevelBlock), 0, s, a);
            return hipGetLastError();
        }
        // the latency form with an attached sink list: the level's own list
        // in its workgroups, the sinks one per lane in low-priority
        // workgroups after them (RF_K2_SINK_LANES=0: sinks as listed jobs, A/B)
        static const bool sink_lanes = RF_DIAG_KNOB("RF_K2_SINK_LANES", 1) != 0;
        // the overflow of a latency-form level a little wider than the chip
        // (estimated from the step's marked slots: more than one 64-job
        // workgroup per CU) -- one workgroup per CU takes 64 chains, the rest
        // run one per lane in workgroups after them, instead of a second
        // workgroup on a few CUs whose chain waves then share SIMDs (the
        // 8-rank piece's Exec level: 274 workgroups, 18 CUs doubled, 104 us
        // against 77 alone).  RF_K2_OVF=0: off (A/B), 2: the lanes at the
        // chains' priority.
        const uint32_t ovf_lanes = g.ovf_mode;  // (RF_K2_OVF, read at load)
        const uint32_t nt = wide ? 256u : 192u;
        const uint64_t est = std::min<uint64_t>(e - b, g.step_marked);
        // half workgroups (32 jobs, one chain wave: three fit a CU, each chain
        // on its own SIMD) for a latency-form level estimated at more than one
        // 64-job workgroup per CU but at most three 32-job ones (the 8-rank
        // piece's Exec level: 17.5k chains) -- instead of a second 64-job
        // workgroup on some CUs, whose four chain waves then share SIMDs.
        // RF_K2_HALF=0: off (A/B)
        if (graph_level_half(g, lvl)) {
            if (!g.split_half) a.split = 0;
            uint64_t hg = (e - b + 31) / 32;
            if (hg > wg_cap) hg = wg_cap;
            uint64_t grid = hg;
            if (sink_lvl != ~0u && sink_lanes) {
                a.sink_wg = (uint32_t)hg;
                grid += std::min<uint64_t>((n2 + 127) / 128, 1024u);
            }
            hipLaunchKernelGGL((k2_level_pl<2, false, 32>), dim3((uint32_t)grid), dim3(128), pad, s, a);
            return hipGetLastError();
        }
        if (!one_lane && ovf_lanes && g.n_cu && est > 64ull * g.n_cu) {
            a.sink_wg = g.n_cu;
            a.ovf = ovf_lanes;
            wg = a.sink_wg + std::min<uint64_t>((e - b - 64ull * g.n_cu + n2 + nt - 1) / nt, 1024u);
        } else if (!one_lane && sink_lvl != ~0u && sink_lanes) {
            a.sink_wg = (uint32_t)std::min<uint64_t>((e - b + 63) / 64, wg_cap);
            wg = a.sink_wg + std::min<uint64_t>((n2 + nt - 1) / nt, 1024u);
        }
#ifdef RF_DIAG  // (the measured-dead forms: the one-lane chain, the streamed hand-over)
        if (one_lane && wide)
            hipLaunchKernelGGL(k2_level_pc<3>, dim3((uint32_t)wg), dim3(192), pad, s, a);
        else if (one_lane)
            hipLaunchKernelGGL(k2_level_pc<2>, dim3((uint32_t)wg), dim3(128), pad, s, a);
        else if (!no_stream && !wide)
            hipLaunchKernelGGL((k2_level_pl<2, true>), dim3((uint32_t)wg), dim3(192), pad, s, a);
        else
#endif
        if (wide)
            hipLaunchKernelGGL((k2_level_pl<3, false>), dim3((uint32_t)wg), dim3(256), pad, s, a);
        else
            hipLaunchKernelGGL((k2_level_pl<2, false>), dim3((uint32_t)wg), dim3(192), pad, s, a);
        (void)no_stream;
        return hipGetLastError();
    }
    const uint32_t grid = grid_for(e - b, full ? 16384u : inc_cap);
    hipLaunchKernelGGL(k2_level, dim3(grid), dim3(kLevelBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_graph_midstates(const uint8_t* tmpl, const uint32_t* start, const uint32_t* lead, uint32_t n,
                                  uint4* mid, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k2_midstates, dim3(grid_for(n, 16384)), dim3(256), 0, s, tmpl, start, lead, n, mid);
    return hipGetLastError();
}

hipError_t launch_part_pack(const uint32_t* export_slot, uint32_t n, const uint8_t* slots, uint8_t* snap,
                            uint8_t* send, uint32_t* bits, uint32_t bit0, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_part_pack, dim3((n + 255) / 256), dim3(256), 0, s, export_slot, n, slots, snap, send, bits,
                       bit0);
    return hipGetLastError();
}

hipError_t launch_part_any(const uint64_t* bits, uint64_t nwords, const uint32_t* import_bid, uint32_t n_import,
                           uint32_t* flag, hipStream_t s) {
    hipLaunchKernelGGL(k_part_any, dim3(1), dim3(256), 0, s, bits, nwords, import_bid, n_import, flag);
    return hipGetLastError();
}

hipError_t launch_part_apply(const GraphDev& g, const uint32_t* import_slot, const uint32_t* import_bid, uint32_t n,
                             const uint32_t* bits, const uint8_t* gather, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_part_apply, dim3(grid_mark(n)), dim3(kMarkBlock), 0, s, import_slot, import_bid, n,
                       bits, gather, mark_level_args(g));
    return hipGetLastError();
}

hipError_t launch_graph_step_end(const GraphDev& g, int full, hipStream_t s) {
    hipLaunchKernelGGL(k3_step_end, dim3(1), dim3(256), 0, s, g.counts, g.counts_last, g.lvl_start_dev,
                       g.n_levels, full);
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
