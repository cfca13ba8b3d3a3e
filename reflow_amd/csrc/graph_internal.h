// graph_internal.h -- internal: the object behind rf_graph* (digest DAG on
// one device), shared by capi.cpp (load, recompute) and partition.cpp
// (multi-GPU pieces).  Not part of the public ABI.
#pragma once
#include <vector>

#include "ctx.h"
#include "engine.h"

// A loaded piece's place in a partitioned DAG (partition.cpp).
struct GraphPart {
    int nranks = 1, rank = 0;
    uint32_t max_export = 0, n_export = 0, n_import = 0;
    bool any_import = true;   // some rank imports (else one exchange ends a step)
    uint32_t rounds = 0;      // > 0: fixed-round protocol (rf_graph_part::rounds)
    uint64_t nwords = 0;      // u64 words of the boundary bitset (nranks * max_export bits)
    DevBuf d_export_slot, d_import_slot, d_import_bid;
    DevBuf d_snap;            // [n_export][32] export digests as last sent
    DevBuf d_send;            // [max_export][32]
    DevBuf d_gather;          // [nranks][max_export][32]
    DevBuf d_bits, d_bits_g;  // boundary bitset; gathered copies (host transport OR)
    DevBuf d_flag;
    HostBuf h_buf;            // host transport staging
    uint64_t last_supersteps = 0;
    // Fixed-round protocol on a rank with imports and every export produced
    // below the lowest level that reads an import: that level and the ones
    // above wait for the exchange (one hash of the import readers per step
    // instead of one before and one after it); ~0u: no deferral
    uint32_t defer_lvl = ~0u;
};

struct rf_graph {
    rf_ctx* ctx = nullptr;
    rf::GraphDev g;
    std::vector<int64_t> producer;   // slot -> external job or -1
    std::vector<uint32_t> ext2int;   // external job id -> internal
    bool initialized = false;
    DevBuf b_stamps, b_mid, b_wgst, b_plan;
    DevBuf b_meta, b_holes, b_cons_ptr, b_cons_job, b_tmpl, b_slots, b_dirty, b_list, b_lmeta, b_counts,
        b_counts_last, b_lvl_start, b_tmp_idx, b_tmp_dig;
    uint64_t total_blocks = 0, hole_count = 0, tmpl_bytes = 0, last_recomputed = 0;
    uint32_t max_level_jobs = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipGraphExec_t exec_inc = nullptr, exec_full = nullptr;
    // mark + incremental levels as one graph (rf_graph_update_recompute_async);
    // the template graph is kept: its mark node's parameters change per call
    hipGraph_t graph_upd = nullptr;
    hipGraphExec_t exec_upd = nullptr;
    hipGraphNode_t upd_mark = nullptr;
    bool timed = false;
    bool time_next = false;  // record e0/e1 around the next plain recompute (synchronous callers)
    // input slots written since the last incremental step (set_slots,
    // set_slots_device, update; a partition's imports before a post-exchange
    // pass that is a step of its own): picks that step's level-kernel forms
    // (graph_enqueue); rf_graph_save refuses while it is non-zero
    uint64_t marked = 0;
    uint32_t* last_counts = nullptr;  // device cursors of the last recompute (counts_last, or a plain step's half)
    GraphPart* part = nullptr;  // multi-GPU partition (rf_graph_set_part), else null
};


// lvl_lo / lvl_hi / swap: plain incremental steps only (graph_enqueue)
int graph_recompute_locked(rf_graph* gr, int full, hipStream_t s, uint32_t lvl_lo = 0, uint32_t lvl_hi = ~0u,
                           bool swap = true);
bool graph_plain_steps();  // incremental steps are plain launches (not RF_K2_GRAPH=1)
void graph_forms_from_env(rf::GraphDev& G);  // form thresholds at load / restore
uint32_t graph_split_on();
int graph_read_counts(rf_graph* gr, hipStream_t s, std::vector<uint32_t>& counts);
uint32_t graph_ovf_cus(const rf_ctx* ctx, uint32_t* mode);  // RF_K2_OVF_CU / RF_K2_OVF                        // RF_K2_SPLIT (default on)
int graph_device_alloc(rf_graph* gr, uint32_t J, uint32_t S, uint32_t L, uint64_t H, uint64_t tmpl_bytes);
int graph_build_plan(rf_graph* gr);  // GraphDev::plan, after the records are on the device
void graph_part_release(rf_graph* gr);
