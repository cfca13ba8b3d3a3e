// engine.h -- internal declarations shared by the HIP translation units and
// the C-ABI implementation (capi.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "diag.h"

namespace rf {

// ---- K1: batched SHA-256 -------------------------------------------------
// Lane-per-message kernel with a sharded dynamic work queue.
struct LanesArgs {
    const uint8_t* arena;
    const uint64_t* offs;   // [n] byte offsets (16-B aligned)
    const uint64_t* lens;   // [n]
    const uint32_t* order;  // [n_order] message ids in processing order (largest first)
    uint32_t n_order;
    uint32_t n_shards;      // queue shards; message q belongs to shard q % n_shards
    uint32_t* heads;        // [n_shards] next position per shard (pre-set)
    uint8_t* out;           // [n][32]
};
hipError_t launch_sha_lanes(const LanesArgs& a, uint32_t grid, hipStream_t s);
uint32_t sha_lanes_block();

// Wave-per-message kernel for long messages (critical path of skewed sets).
struct SoloArgs {
    const uint8_t* arena;
    const uint64_t* offs;
    const uint64_t* lens;
    const uint32_t* order;  // [n_order] message ids
    uint32_t n_order;
    uint8_t* out;
};
// duo: the round chain on two lanes (k1_sha256_duo); else one lane (k1_sha256_solo)
hipError_t launch_sha_solo(const SoloArgs& a, bool duo, hipStream_t s);
// Lane per message with a producer wave beside the chain wave (small sets).
hipError_t launch_sha_pair(const SoloArgs& a, hipStream_t s);
// Eight messages per wave on the duo's two-lane chain (small sets).
hipError_t launch_sha_octo(const SoloArgs& a, hipStream_t s);

// Streaming SHA-256 (rf_sha_streams): segment i = nblocks[i] whole blocks at
// arena + offs[i] (16-B aligned) fed into midstate mid[8i..8i+7] in place.
struct ResumeArgs {
    const uint8_t* arena;
    const uint64_t* offs;
    const uint64_t* nblocks;
    uint32_t* mid;
    uint32_t n;
};
hipError_t launch_sha_resume(const ResumeArgs& a, hipStream_t s);

// out32[ids[i]] = digs32[i] (the host leg's digests into the plan's output).
hipError_t launch_scatter_digests(uint8_t* out32, const uint32_t* ids, const uint8_t* digs32, uint64_t n,
                                  hipStream_t s);

// Checks that the gfx950 code object of this library loads on the device.
hipError_t probe_kernels();

hipError_t launch_place_ids(uint8_t* arena, const uint64_t* mat_off, const uint32_t* entry, uint64_t n,
                            const uint8_t* ids32, hipStream_t s);
hipError_t launch_gen_fill(uint8_t* arena, const uint64_t* offs, const uint64_t* lens, uint64_t n,
                           uint64_t seed, uint64_t arena_bytes, hipStream_t s);

// ---- K2/K3: digest DAG -----------------------------------------------------
// GraphDev::inc_level flags.  The sink level (kLvlSink, the last level) holds
// the queueable jobs nothing reads (physical cache keys) whose inputs are
// final by the fill level (kLvlFill); its list is attached to the launch of
// the last level from kLvlSinkMin (the highest level a sink's inputs need
// below it) to the fill level that runs in the throughput form -- the sinks
// fill the SIMDs a wide level's waves leave idle -- else to the fill level's
// launch.
constexpr uint8_t kLvlForm = 3, kLvlSinkMin = 0x20, kLvlFill = 0x40, kLvlSink = 0x80;
// kLvlOct: a level of few long jobs (form 2, at most kOctMaxLevel jobs, each
// with no fusion target, <= kOctMaxBlocks blocks and <= kOctMaxHoles holes)
// runs in the octo form (k2_level_oct): 8 jobs per workgroup, each job's whole
// material staged in LDS, K1's 8-instruction octo chain
constexpr uint8_t kLvlOct = 0x10;
constexpr uint32_t kOctMaxBlocks = 32, kOctMaxHoles = 64, kOctMaxLevel = 4096;
// The fused-job count (jobs hashed inside fused chains, never queued) is
// added by every chain wave; one counter took every wave's atomic in turn at
// the memory side (~19 ns each: the 100M step's lean mark kernel, 2,200
// waves, waited 41 us for them).  It is spread over kFusedParts counters
// kPartStride words apart after each cursor half's L + 1 level counts, and
// folded into [L] where it is read (k3_step_end, graph_read_counts).
constexpr uint32_t kFusedParts = 64, kPartStride = 32, kCountsExtra = kFusedParts * kPartStride;
// A level's append cursors sit Lp words apart (Lp = L rounded up to 32
// words: a level's cursors on lines of their own).
__host__ __device__ constexpr uint32_t cursor_lp(uint32_t L) { return (L + 31) / 32 * 32; }
// The level lists' append cursors, kListShards per level: level l's list
// region [lvl_start[l], lvl_start[l+1]) is cut by job id into kListShards
// runs of 2^sh jobs (list_shard_shift), and a job joins the run its own id
// falls in -- so a run never overflows (a job is listed at most once a step)
// and the waves appending to one level spread their atomics over the runs'
// cursors instead of taking one cursor in turn at the memory side (~19 ns
// each: the 100M step's lean mark kernel, 2,200 waves appending to the Exec
// level).  Shard k of level l at list_shard_off(L) + k * Lp + l (a level's
// cursors on lines of their own).
#ifndef RF_SLOT_PLAN
#define RF_SLOT_PLAN 1  // the mark kernels' per-slot plan (GraphDev::plan; A/B builds: 0 = off)
#endif
#ifndef RF_LIST_SHARDS
#define RF_LIST_SHARDS 16  // (a power of two; A/B builds: 1 = one run a level, 0 = round 4's lists)
#endif
constexpr bool kLegacyLists = RF_LIST_SHARDS == 0;  // one cursor, no staged runs (A/B)
constexpr uint32_t kListShards = RF_LIST_SHARDS ? RF_LIST_SHARDS : 1;
__host__ __device__ constexpr uint32_t list_shard_off(uint32_t L) {
    return L + 1 + kCountsExtra;
}
__host__ __device__ constexpr uint32_t counts_half_words(uint32_t L) {
    return list_shard_off(L) + kListShards * cursor_lp(L);
}
// log2 of a level's run length: the least sh with ceil(C / 2^sh) <= kListShards
__host__ __device__ inline uint32_t list_shard_shift(uint32_t C) {
    const uint32_t q = (C + kListShards - 1) / kListShards;
    return q <= 1 ? 0u : 32u - (uint32_t)__builtin_clz(q - 1);
}
struct GraphDev {
    uint32_t n_jobs = 0, n_slots = 0, n_levels = 0;
    // jobs in internal (level) order
    // job record, 32 B, one pair of 16-B loads per job:
    //   meta[2j]   = {template offset / 64, blocks, hole_begin, hole_end}
    //   meta[2j+1] = {out slot, consumer_begin, consumer_end, fusion target or ~0}
    //   (the fusion target's reverse edge is the last of the range)
    uint4* meta = nullptr;           // [2J]
    uint2* holes = nullptr;          // [H] {byte position, slot}
    uint32_t* cons_ptr = nullptr;    // [S+1] slot -> consumer jobs (internal ids)
    // [3S] the mark kernels' per-slot plan, built at load / restore from the
    // records above (launch_slot_plan): plan[3s] = {first reverse edge after
    // the slot-fused one, reverse-edge end, slot-fused job or ~0, 0},
    // plan[3s+1..2] = that job's record -- a changed input slot reaches its
    // slot-fused job's template, hole and old digest in one dependent load
    // instead of three (cons_ptr -> cons -> meta)
    uint4* plan = nullptr;
    uint2* cons = nullptr;           // [C] {consumer job, its level}
    uint8_t* tmpl = nullptr;         // padded templates, zero at the holes (read-only)
    uint8_t* slots = nullptr;        // [S][32] digest table
    uint32_t* dirty = nullptr;       // [J] queued-this-step flag per internal id (a word each)
    uint32_t* list = nullptr;        // [J] per-level work lists (level l at lvl_start[l])
    uint4* lmeta = nullptr;          // [2J] each listed job's record, at its list position
    uint32_t* counts = nullptr;      // [L+1] list lengths (append cursors); [L] + the parts after it = fused jobs hashed
    uint32_t* counts_last = nullptr; // [L+1] jobs hashed per level by the last recompute; [L] fused
    // Plain-launch incremental steps alternate between two halves of the
    // cursor array (counts = the half the next step appends to and reads,
    // counts_other = the previous step's, zeroed by this step's first level
    // kernel), so no step-end kernel is needed.
    uint32_t* counts_other = nullptr;
    uint32_t* lvl_start_dev = nullptr; // [L+1]
    std::vector<uint32_t> lvl_start; // host copy [L+1]
    // [L] per level: bits kLvlForm = 1 (has jobs that can be queued, i.e. not
    // all fusion targets) or 2 (those average >= RF_K2_WIDE blocks), 0 = never
    // launched by an incremental step; plus the sink-list flags below
    std::vector<uint8_t> inc_level;
    // plain incremental steps: the sink level's list runs attached to another
    // level's launch (graph_enqueue), not as a level of its own -- unless a
    // partition import feeds one of its jobs (rf_graph_set_part)
    bool sink_attach_ok = true;
    // every job's first hole starts in block 0 of its (midstate-trimmed)
    // template, so a fusion target's block 0 can be built by the chain wave
    // (k2_level_pl cb0); false only for the RF_K2_NO_MIDSTATE A/B load
    bool hole_in_b0 = true;
    // every fusion target's hole is at material byte 2 (right after its WD
    // prefix: no Universe), so the chain assembles its block 0 in registers
    bool fuse_pos2 = true;
    // every slot-fused job (an input slot's one-hole consumer, hashed by the
    // mark kernels) without constant leading blocks and with its hole at this
    // byte: its record and midstate are not loaded; ~0u: loaded (the default,
    // and after a checkpoint restore)
    uint32_t sf_pos = ~0u;
    // per level: 1 = no job of it has constant leading blocks (no midstate
    // load for its listed jobs, k2_level_lf); empty after a restore (loaded)
    std::vector<uint8_t> lvl_lead0;
    // RF_K2_STREAM=1 at load: the streamed hand-over variant of k2_level_pl
    // (opt-in, measured slower; kept correct by a forced-mode GPU test)
    bool stream_handover = false;
    // The next plain incremental step's level-kernel forms, set per step by
    // graph_enqueue: a level runs k2_level_lf (one lane per listed job, the
    // throughput form) instead of k2_level_pl when min(its jobs, step_marked)
    // >= thru_slots -- step_marked = the input slots marked for the step (an
    // upper bound of the chains that can reach the level), the level's size
    // the other bound (merge-tree levels stay in the latency form)
    uint64_t step_marked = 0, thru_slots = ~0ull, thru_slots_wide = ~0ull;  // (wide: inc_level 2)
    uint32_t n_cu = 0;      // the device's CUs (latency-form overflow lanes, k2_level_pl)
    uint32_t ovf_mode = 0;  // overflow lanes: 0 off, 1 on, 2 at the chains' priority (RF_K2_OVF, at load)
    // The thresholds themselves, fixed per graph: defaults (or RF_K2_THRU /
    // RF_K2_THRU_WIDE read once when the graph is loaded or restored), or
    // rf_graph_set_forms; cfg_thru_mark: the mark kernel's lean form
    // (k3_mark_slots_lf) from this many changed slots
    uint64_t cfg_thru = 0, cfg_thru_wide = 0, cfg_thru_mark = 0;
    // what the last plain step / mark launch chose (rf_graph_stats)
    uint32_t last_levels_lf = 0, last_mark_lf = 0, last_levels_oct = 0, last_levels_half = 0;
    uint32_t last_sink_attach = ~0u;  // the level whose launch took the sink list last step (~0u: none)
    uint32_t sink_at = 2;             // where the sink list may run (RF_K2_SINK_AT at load; graph_enqueue)
    unsigned long long* stamps = nullptr;  // diagnostic phase stamps [L][128] (RF_K2_STAMPS)
    unsigned long long* wgst = nullptr;    // diagnostic per-workgroup records [L][2048][4] (RF_K2_WGSTAMPS)
    // [2J] each job's initial chaining value (IV, or the midstate after the
    // constant blocks its template starts with -- the record's template
    // offset and block count already skip them); null when no job has any
    uint4* mid = nullptr;
    // split block 0 (k2_level_pl cb0 = 2): the producer expands the upper
    // half of a fusion target's block 0 and builds its template-only block 1
    // during the job before it; set at load / restore (RF_K2_SPLIT=0: off)
    uint32_t split_b0 = 0;  // 1: the producer expands K+W[32..63]; 2: K+W[16..63]
    // split block 0 in the 32-job workgroups too (RF_K2_SPLIT_HALF=1 at load;
    // off by default: the 8-rank piece 0.2997 -> 0.2973 ms without it,
    // profiles/r04/sw3)
    uint32_t split_half = 0;
    uint32_t dbg_mark = 0;  // diagnostic (RF_K2_DBG_MARK=1 at load): the lean mark kernel skips its fused-job count (stats wrong, digests right)
};
// Midstates of the jobs' leading constant blocks, hashed once at load: job i
// (internal order) hashes lead[i] blocks of its template from block
// start[i] (64-B units) into mid[2i..2i+1] (state words); IV when lead[i] = 0.
hipError_t launch_graph_midstates(const uint8_t* tmpl, const uint32_t* start, const uint32_t* lead, uint32_t n,
                                  uint4* mid, hipStream_t s);
// The per-slot plan (GraphDev::plan) of a graph whose meta / cons_ptr / cons
// are on the device.
hipError_t launch_slot_plan(const GraphDev& g, hipStream_t s);
hipError_t launch_graph_mark_slots(GraphDev& g, const uint32_t* slots, const uint8_t* digests,
                                   uint32_t n, hipStream_t s);
// k3_mark_slots as a graph kernel node: argument values + node parameters
struct MarkArgs {
    const uint32_t* sl;
    const uint8_t* dig;
    uint32_t n;
    alignas(16) unsigned char a[320];  // the kernel's LevelArgs (k2_graph.hip), by value
    void* ptrs[4];
};
void graph_mark_params(const GraphDev& g, const uint32_t* slots, const uint8_t* digests, uint32_t n,
                       MarkArgs* args, hipKernelNodeParams* p);
const void* graph_mark_kernel();
hipError_t launch_graph_level(const GraphDev& g, uint32_t level, int full, hipStream_t s,
                              uint32_t* zero_counts = nullptr, uint32_t sink_lvl = ~0u);
bool graph_level_lf(const GraphDev& g, uint32_t lvl);
bool graph_level_half(const GraphDev& g, uint32_t lvl);
hipError_t launch_graph_step_end(const GraphDev& g, int full, hipStream_t s);
hipError_t launch_gather_slots(const uint8_t* slots, const uint32_t* idx, uint32_t n, uint8_t* out,
                               hipStream_t s);
// Partitioned DAG exchange: pack changed exports (bits at bit0 + i), test the
// reduced bitset, apply changed imports (queues their local consumers).
hipError_t launch_part_pack(const uint32_t* export_slot, uint32_t n, const uint8_t* slots, uint8_t* snap,
                            uint8_t* send, uint32_t* bits, uint32_t bit0, hipStream_t s);
hipError_t launch_part_any(const uint64_t* bits, uint64_t nwords, const uint32_t* import_bid, uint32_t n_import,
                           uint32_t* flag, hipStream_t s);
hipError_t launch_part_apply(const GraphDev& g, const uint32_t* import_slot, const uint32_t* import_bid, uint32_t n,
                             const uint32_t* bits, const uint8_t* gather, hipStream_t s);

// K3 reachability (Eval.dirty): one frontier level; bits = marked set,
// next/n_next = the newly marked nodes (n_next zeroed by the caller).
hipError_t launch_reach_step(const uint32_t* front, uint32_t n_front, const uint64_t* cons_ptr, const uint32_t* cons,
                             uint32_t* bits, uint32_t* next, uint32_t* n_next, hipStream_t s);

hipError_t launch_or_reduce(const uint64_t* gathered, uint64_t nwords, int nranks, uint64_t* out,
                            hipStream_t s);

// ---- K4: bloom probe ---------------------------------------------------------
struct BloomDev {
    uint64_t m = 1, k = 1, length = 0, nwords = 0;
    uint64_t* words = nullptr;
    uint64_t* len_dev = nullptr;  // device copy of length (grows on add)
};
hipError_t launch_bloom_probe(const BloomDev& b, const uint8_t* d32, uint64_t n, uint8_t* out,
                              hipStream_t s);
hipError_t launch_bloom_add(const BloomDev& b, const uint8_t* d32, uint64_t n, hipStream_t s);
// Repository.Collect: dead[n] flags, tile_count[bloom_collect_tiles(n)]
// scratch; out_idx receives the dead indices ascending; nb2 = {n_dead,
// dead_bytes} (u64, i64), zeroed by the caller.
uint64_t bloom_collect_tiles(uint64_t n);
hipError_t launch_bloom_collect(const BloomDev& b, const uint8_t* d32, const int64_t* sizes, uint64_t n,
                                uint8_t* dead, uint32_t* tile_count, uint64_t* out_idx, uint64_t* nb2,
                                hipStream_t s);

// ---- K5: digest-keyed hash table (Canonicalize's flowMap) --------------------
uint32_t dedup_table_slots(uint32_t n);
// canon[i] = min{j : dig[j] == dig[i]}; table [dedup_table_slots(n)] and
// slot_of [n] are scratch; *n_unique = |{i : canon[i] == i}|.
// clear_table = false: the caller has already filled the table with ~0
hipError_t launch_dedup(const uint8_t* dig, uint32_t n, uint32_t* table, uint32_t* slot_of, uint32_t* canon,
                        uint32_t* n_unique, hipStream_t s, bool clear_table = true);
hipError_t launch_fill_u32(uint32_t* p, uint32_t v, uint64_t n, hipStream_t s);

// HBM assoc (assoc.Assoc with test/testutil/assoc.go semantics)
struct AssocView {
    uint32_t* tag;
    uint4* keys;
    uint4* vals;
    uint32_t mask;
    uint32_t* count;
};
hipError_t launch_assoc_insert(const AssocView& t, uint32_t kind, const uint8_t* keys, const uint32_t* canon,
                               uint32_t n, uint32_t* slot_of, hipStream_t s);
hipError_t launch_assoc_round(const AssocView& t, const uint32_t* rem, const uint32_t* n_rem, uint32_t n_max,
                              const uint32_t* canon, unsigned long long* cls, uint32_t round,
                              const uint32_t* slot_of, const uint8_t* expect, const uint8_t* vals,
                              int32_t* status, uint32_t* next, uint32_t* n_next, hipStream_t s);
hipError_t launch_assoc_get(const AssocView& t, uint32_t kind, const uint8_t* keys, uint64_t n, uint8_t* vals,
                            uint8_t* found, hipStream_t s);
hipError_t launch_assoc_select(const uint8_t* found, const uint8_t* vals, const uint64_t* key_ptr, uint64_t n,
                              int32_t* which, uint8_t* out, hipStream_t s);
hipError_t launch_assoc_abbrev(const AssocView& t, uint32_t kind, uint32_t cap, const uint8_t* qkeys,
                               const uint8_t* nhex, uint32_t q, uint32_t* matches, uint32_t* hit_slot,
                               hipStream_t s);
hipError_t launch_iota(uint32_t* out, uint32_t n, hipStream_t s);
hipError_t launch_assoc_rehash(const AssocView& from, uint32_t cap_from, const AssocView& to, hipStream_t s);

}  // namespace rf
