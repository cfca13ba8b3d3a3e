// partition_split.cpp -- the host splitter of a partitioned digest DAG
// (SURVEY §8(e)): rf_graph_split gives one rank its piece of a global job
// graph -- its jobs renumbered, the slots it reads from other ranks as
// imports, the slots other ranks read from it as exports, and the boundary
// ids the superstep exchange uses (partition.cpp).  Host-only (no HIP): it
// also builds into the sanitizer test (make asan).
#include <string.h>

#include <algorithm>
#include <memory>
#include <vector>

#include "errors.h"

using rf::fail;

// ---------------------------------------------------------------------------
// host splitter
struct rf_graph_piece {
    std::vector<uint32_t> out_slot, tmpl_len, hole_pos, hole_slot;
    std::vector<uint64_t> tmpl_off, hole_ptr;
    const uint8_t* blob = nullptr;
    uint64_t blob_len = 0;
    std::vector<uint32_t> global_of_local;  // local slot -> global slot
    std::vector<uint32_t> export_slot, import_slot, import_bid;
    uint32_t max_export = 0;
    int nranks = 1, rank = 0;
    bool any_import = false;
    uint32_t rounds = 0;  // the most rank-boundary crossings on any path
};

// The most rank-boundary crossings on any path of the global job graph: an
// edge producer p -> consumer k crosses when p is owned (not replicated) and
// k is hashed elsewhere (another rank, or every rank).  Kahn order over the
// jobs; RF_EINVAL on a cycle.
static int max_crossings(const rf_graph_desc* d, const int32_t* owner, const std::vector<int64_t>& producer,
                         uint32_t* out) {
    const uint32_t J = d->n_jobs, S = d->n_slots;
    const uint64_t H = J ? d->hole_ptr[J] : 0;
    std::vector<uint64_t> cptr(S + 1, 0);
    for (uint64_t h = 0; h < H; ++h) cptr[d->hole_slot[h] + 1]++;
    for (uint32_t s = 0; s < S; ++s) cptr[s + 1] += cptr[s];
    std::vector<uint32_t> cjob(H), indeg(J, 0), cross(J, 0);
    {
        std::vector<uint64_t> fill(cptr.begin(), cptr.end() - 1);
        for (uint32_t k = 0; k < J; ++k)
            for (uint64_t h = d->hole_ptr[k]; h < d->hole_ptr[k + 1]; ++h) {
                cjob[fill[d->hole_slot[h]]++] = k;
                if (producer[d->hole_slot[h]] >= 0) indeg[k]++;
            }
    }
    std::vector<uint32_t> q;
    q.reserve(J);
    for (uint32_t j = 0; j < J; ++j)
        if (!indeg[j]) q.push_back(j);
    uint32_t best = 0;
    for (size_t i = 0; i < q.size(); ++i) {
        const uint32_t p = q[i], s = d->out_slot[p];
        best = std::max(best, cross[p]);
        for (uint64_t c = cptr[s]; c < cptr[s + 1]; ++c) {
            const uint32_t k = cjob[c];
            const uint32_t x = cross[p] + ((owner[p] >= 0 && owner[k] != owner[p]) ? 1u : 0u);
            cross[k] = std::max(cross[k], x);
            if (--indeg[k] == 0) q.push_back(k);
        }
    }
    if (q.size() != J) return fail(RF_EINVAL, "job graph has a cycle");
    *out = best;
    return RF_OK;
}

extern "C" int rf_graph_split(const rf_graph_desc* d, int nranks, int rank, const int32_t* owner,
                              rf_graph_piece** out) {
    ARG(d && owner && out, "null argument");
    ARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank");
    *out = nullptr;
    const uint32_t J = d->n_jobs, S = d->n_slots;
    ARG(J == 0 || (d->out_slot && d->tmpl_off && d->tmpl_len && d->hole_ptr), "null job arrays");
    const uint64_t H = J ? d->hole_ptr[J] : 0;
    ARG(H == 0 || (d->hole_pos && d->hole_slot), "null hole arrays");
    std::vector<int64_t> producer(S, -1);
    for (uint32_t j = 0; j < J; ++j) {
        ARG(owner[j] >= -1 && owner[j] < nranks, "owner out of range (-1 = every rank)");
        if (d->out_slot[j] >= S) return fail(RF_EINVAL, "job %u: out_slot out of range", j);
        if (producer[d->out_slot[j]] >= 0) return fail(RF_EINVAL, "slot %u written twice", d->out_slot[j]);
        producer[d->out_slot[j]] = j;
        for (uint64_t h = d->hole_ptr[j]; h < d->hole_ptr[j + 1]; ++h)
            if (d->hole_slot[h] >= S) return fail(RF_EINVAL, "job %u: hole slot out of range", j);
    }
    // exports of every rank (deterministic order: by slot), so boundary ids agree
    std::vector<std::vector<uint32_t>> exports(nranks);
    {
        std::vector<uint8_t> is_export(S, 0);
        for (uint32_t k = 0; k < J; ++k)
            for (uint64_t h = d->hole_ptr[k]; h < d->hole_ptr[k + 1]; ++h) {
                const int64_t p = producer[d->hole_slot[h]];
                if (p < 0 || owner[p] < 0) continue;  // input, or replicated: no exchange
                // read on a rank that does not hash it: every rank if k is replicated
                if (owner[k] != owner[p]) is_export[d->hole_slot[h]] = 1;
            }
        for (uint32_t s = 0; s < S; ++s)
            if (is_export[s]) exports[owner[producer[s]]].push_back(s);
    }
    auto* pc = new rf_graph_piece();
    std::unique_ptr<rf_graph_piece> guard(pc);
    pc->nranks = nranks;
    pc->rank = rank;
    for (const auto& e : exports) pc->max_export = std::max<uint32_t>(pc->max_export, (uint32_t)e.size());
    std::vector<uint32_t> bid_of(S, ~0u);
    for (int r = 0; r < nranks; ++r)
        for (uint32_t i = 0; i < exports[r].size(); ++i) bid_of[exports[r][i]] = (uint32_t)r * pc->max_export + i;
    // local jobs (global order) and the slots they touch, renumbered densely
    std::vector<uint32_t> local_of(S, ~0u);
    std::vector<uint8_t> used(S, 0);
    std::vector<uint32_t> jobs;
    for (uint32_t j = 0; j < J; ++j)
        if (owner[j] == -1 || owner[j] == rank) {
            jobs.push_back(j);
            used[d->out_slot[j]] = 1;
            for (uint64_t h = d->hole_ptr[j]; h < d->hole_ptr[j + 1]; ++h) used[d->hole_slot[h]] = 1;
        }
    for (uint32_t s = 0; s < S; ++s)
        if (used[s]) {
            local_of[s] = (uint32_t)pc->global_of_local.size();
            pc->global_of_local.push_back(s);
        }
    pc->hole_ptr.push_back(0);
    for (uint32_t j : jobs) {
        pc->out_slot.push_back(local_of[d->out_slot[j]]);
        pc->tmpl_off.push_back(d->tmpl_off[j]);
        pc->tmpl_len.push_back(d->tmpl_len[j]);
        for (uint64_t h = d->hole_ptr[j]; h < d->hole_ptr[j + 1]; ++h) {
            pc->hole_pos.push_back(d->hole_pos[h]);
            pc->hole_slot.push_back(local_of[d->hole_slot[h]]);
        }
        pc->hole_ptr.push_back(pc->hole_pos.size());
    }
    pc->blob = d->blob;
    pc->blob_len = d->blob_len;
    for (uint32_t s : exports[rank]) pc->export_slot.push_back(local_of[s]);
    pc->any_import = false;
    for (uint32_t k = 0; k < J && !pc->any_import; ++k)  // does any rank import anything?
        for (uint64_t h = d->hole_ptr[k]; h < d->hole_ptr[k + 1]; ++h) {
            const int64_t p = producer[d->hole_slot[h]];
            if (p >= 0 && owner[p] >= 0 && owner[k] != owner[p]) {
                pc->any_import = true;
                break;
            }
        }
    if (int rc = max_crossings(d, owner, producer, &pc->rounds)) return rc;
    // imports: slots this piece reads that another rank's job produces
    for (uint32_t ls = 0; ls < pc->global_of_local.size(); ++ls) {
        const uint32_t s = pc->global_of_local[ls];
        const int64_t p = producer[s];
        if (p >= 0 && owner[p] >= 0 && owner[p] != rank) {
            pc->import_slot.push_back(ls);
            pc->import_bid.push_back(bid_of[s]);
        }
    }
    *out = guard.release();
    return RF_OK;
}

extern "C" void rf_graph_piece_free(rf_graph_piece* pc) { delete pc; }

extern "C" int rf_graph_piece_desc(const rf_graph_piece* pc, rf_graph_desc* o) {
    ARG(pc && o, "null argument");
    o->n_jobs = (uint32_t)pc->out_slot.size();
    o->n_slots = (uint32_t)pc->global_of_local.size();
    o->out_slot = pc->out_slot.data();
    o->tmpl_off = pc->tmpl_off.data();
    o->tmpl_len = pc->tmpl_len.data();
    o->hole_ptr = pc->hole_ptr.data();
    o->hole_pos = pc->hole_pos.data();
    o->hole_slot = pc->hole_slot.data();
    o->blob = pc->blob;
    o->blob_len = pc->blob_len;
    return RF_OK;
}

extern "C" int rf_graph_piece_part(const rf_graph_piece* pc, rf_graph_part* o) {
    ARG(pc && o, "null argument");
    o->nranks = pc->nranks;
    o->rank = pc->rank;
    o->max_export = pc->max_export;
    o->n_export = (uint32_t)pc->export_slot.size();
    o->export_slot = pc->export_slot.data();
    o->n_import = (uint32_t)pc->import_slot.size();
    o->import_slot = pc->import_slot.data();
    o->import_bid = pc->import_bid.data();
    o->any_import = pc->any_import ? 1 : 0;
    o->rounds = pc->rounds;
    return RF_OK;
}

extern "C" int rf_graph_piece_slots(const rf_graph_piece* pc, const uint32_t** global_of_local, uint32_t* n) {
    ARG(pc && global_of_local && n, "null argument");
    *global_of_local = pc->global_of_local.data();
    *n = (uint32_t)pc->global_of_local.size();
    return RF_OK;
}

// ---------------------------------------------------------------------------
// a loaded piece's partition and the superstep recompute
