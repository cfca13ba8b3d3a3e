// partition.cpp -- one digest DAG over many GPUs: the
// partition attached to a loaded piece (rf_graph_set_part) and the superstep
// recompute across ranks (rf_graph_recompute_part).  The host splitter that
// makes a rank's piece of a global job graph is partition_split.cpp.
//
// Protocol (bulk-synchronous supersteps, no global level agreement needed):
//   1. every rank recomputes its piece (K3 frontier + K2 levels);
//   2. each rank sets, in a bitset over all ranks' export slots (boundary id
//      = owner rank * max_export + export index), the bits of its exports
//      whose digest changed since they were last sent; the bitsets are
//      OR-reduced over the ranks (RCCL has no bitwise OR: all-gather + a
//      local OR kernel, rf_comm_allreduce_or);
//   3. no bit set anywhere: done.  Else every rank all-gathers the export
//      digests, writes each changed import into its slot and queues the
//      slot's local consumers (k3_mark_slots' compare-and-queue), and the
//      next superstep recomputes them.
// The global graph is a DAG, so this reaches the same digests as a
// single-rank recompute; a partition by 1000align sample (the shared
// reference-index chain replicated) has no imports and ends after one
// exchange.  Transport: an rf_comm (RCCL over xGMI, device buffers) or a host
// all-gather callback (gloo in tests / ranks sharing a GPU).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <vector>

#include "ctx.h"
#include "engine.h"
#include "graph_internal.h"

using namespace rf;

// ---------------------------------------------------------------------------
// the host splitter (rf_graph_split, rf_graph_piece_*): partition_split.cpp

void graph_part_release(rf_graph* gr) {
    GraphPart* P = gr->part;
    if (!P) return;
    for (DevBuf* b : {&P->d_export_slot, &P->d_import_slot, &P->d_import_bid, &P->d_snap, &P->d_send, &P->d_gather,
                      &P->d_bits, &P->d_bits_g, &P->d_flag})
        b->release();
    P->h_buf.release();
    delete P;
    gr->part = nullptr;
}

extern "C" int rf_graph_set_part(rf_graph* gr, const rf_graph_part* p) {
    ARG(gr && p, "null argument");
    ARG(p->nranks >= 1 && p->rank >= 0 && p->rank < p->nranks, "bad rank");
    ARG(p->n_export <= p->max_export, "n_export > max_export");
    ARG(p->n_export == 0 || p->export_slot, "null export_slot");
    ARG(p->n_import == 0 || (p->import_slot && p->import_bid), "null import arrays");
    ARG((uint64_t)p->nranks * p->max_export < (1ull << 32), "boundary too large");
    for (uint32_t i = 0; i < p->n_export; ++i) {
        if (p->export_slot[i] >= gr->g.n_slots) return fail(RF_EINVAL, "export slot %u out of range", p->export_slot[i]);
        if (gr->producer[p->export_slot[i]] < 0)
            return fail(RF_EINVAL, "export slot %u is not produced by this piece", p->export_slot[i]);
    }
    for (uint32_t i = 0; i < p->n_import; ++i) {
        if (p->import_slot[i] >= gr->g.n_slots) return fail(RF_EINVAL, "import slot %u out of range", p->import_slot[i]);
        if (gr->producer[p->import_slot[i]] >= 0)
            return fail(RF_EINVAL, "import slot %u is produced by this piece", p->import_slot[i]);
        if (p->import_bid[i] >= (uint64_t)p->nranks * p->max_export || p->import_bid[i] / p->max_export == (uint32_t)p->rank)
            return fail(RF_EINVAL, "import %u: boundary id %u is not another rank's export", i, p->import_bid[i]);
    }
    rf_ctx* ctx = gr->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    //  a change set marked on a recomputed graph was queued for
    // the plain step's levels; attach a part between steps, never inside one
    // (a graph never recomputed only wrote its inputs: its next step is full)
    if (gr->initialized && gr->marked)
        return fail(RF_EPRECONDITION, "set_part: input slots set since the last recompute");
    graph_part_release(gr);
    auto* P = new GraphPart();
    gr->part = P;
    P->nranks = p->nranks;
    P->rank = p->rank;
    P->max_export = p->max_export;
    P->n_export = p->n_export;
    P->n_import = p->n_import;
    P->any_import = p->any_import != 0;
    P->rounds = p->rounds;
    P->nwords = ((uint64_t)p->nranks * p->max_export + 63) / 64;
    auto up = [&](DevBuf& b, const void* src, size_t bytes) -> hipError_t {
        hipError_t e = b.ensure(std::max<size_t>(bytes, 64));
        return e != hipSuccess || !bytes ? e : sync_copy(ctx, b.p, src, bytes, hipMemcpyHostToDevice);
    };
    const uint64_t blk = 32ull * std::max<uint32_t>(p->max_export, 1);
    hipError_t e;
    if ((e = up(P->d_export_slot, p->export_slot, 4ull * p->n_export)) != hipSuccess ||
        (e = up(P->d_import_slot, p->import_slot, 4ull * p->n_import)) != hipSuccess ||
        (e = up(P->d_import_bid, p->import_bid, 4ull * p->n_import)) != hipSuccess ||
        (e = P->d_snap.ensure(32ull * std::max<uint32_t>(p->n_export, 1))) != hipSuccess ||
        (e = P->d_send.ensure(blk)) != hipSuccess || (e = P->d_gather.ensure(blk * p->nranks)) != hipSuccess ||
        (e = P->d_bits.ensure(8 * std::max<uint64_t>(P->nwords, 1))) != hipSuccess ||
        (e = P->d_bits_g.ensure(8 * std::max<uint64_t>(P->nwords, 1) * p->nranks)) != hipSuccess ||
        (e = P->d_flag.ensure(64)) != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? RF_ENOMEM : RF_EDEVICE, "partition alloc: %s", hipGetErrorString(e));
    // nothing sent yet: every export counts as changed at the first exchange
    HIPC(sync_memset(ctx, P->d_snap.p, 0, 32ull * std::max<uint32_t>(p->n_export, 1)));
    // An import read by a job of the sink level (GraphDev kLvlSink): that
    // level then runs as a level of its own, after the exchange passes'
    // levels, not attached to an earlier launch
    {
        GraphDev& G = gr->g;
        uint32_t sink = ~0u;
        for (uint32_t l = 0; l < G.n_levels; ++l)
            if (G.inc_level[l] & kLvlSink) sink = l;
        G.sink_attach_ok = true;
        for (uint32_t i = 0; sink != ~0u && i < p->n_import && G.sink_attach_ok; ++i) {
            uint32_t cp[2];
            HIPC(sync_copy(ctx, cp, gr->b_cons_ptr.as<uint32_t>() + p->import_slot[i], 8, hipMemcpyDeviceToHost));
            if (cp[1] <= cp[0]) continue;
            std::vector<uint32_t> ce(2ull * (cp[1] - cp[0]));
            HIPC(sync_copy(ctx, ce.data(), gr->b_cons_job.as<uint32_t>() + 2ull * cp[0], 4 * ce.size(),
                           hipMemcpyDeviceToHost));
            for (size_t k = 1; k < ce.size(); k += 2)
                if ((ce[k] & 0x7fffffffu) == sink) G.sink_attach_ok = false;
        }
    }
    // Deferral (fixed rounds, plain steps): the lowest level reading an import
    // and the highest level producing an export.  If every export is final
    // before any import is read, the levels from the lowest import reader up
    // wait for the exchange -- a step then hashes each import reader once
    // (configs[3]'s global root on rank 0: 1+1 hashes of 5 blocks and five
    // empty level launches fewer).  RF_PART_DEFER=0: off (A/B).
    if (P->rounds && P->nranks > 1 && P->n_import && RF_DIAG_KNOB("RF_PART_DEFER", 1) != 0) {
        const GraphDev& G = gr->g;
        uint32_t lmin = ~0u;
        for (uint32_t i = 0; i < p->n_import; ++i) {
            uint32_t cp[2];
            HIPC(sync_copy(ctx, cp, gr->b_cons_ptr.as<uint32_t>() + p->import_slot[i], 8, hipMemcpyDeviceToHost));
            if (cp[1] <= cp[0]) continue;
            std::vector<uint32_t> ce(2ull * (cp[1] - cp[0]));
            HIPC(sync_copy(ctx, ce.data(), gr->b_cons_job.as<uint32_t>() + 2ull * cp[0], 4 * ce.size(),
                           hipMemcpyDeviceToHost));
            for (size_t k = 1; k < ce.size(); k += 2) lmin = std::min(lmin, ce[k] & 0x7fffffffu);  // (kSlotFused)
        }
        uint32_t emax = 0;
        for (uint32_t i = 0; i < p->n_export; ++i) {
            const uint32_t j = gr->ext2int[(size_t)gr->producer[p->export_slot[i]]];
            const uint32_t l = (uint32_t)(std::upper_bound(G.lvl_start.begin(), G.lvl_start.end(), j) -
                                          G.lvl_start.begin()) - 1;
            emax = std::max(emax, l + 1);
        }
        if (lmin != ~0u && emax <= lmin) P->defer_lvl = lmin;
    }
    return RF_OK;
}

// OR of the ranks' boundary bitsets, in place in d_bits.
static int part_or(rf_graph* gr, rf_comm* comm, rf_host_allgather_fn fn, void* user, hipStream_t s) {
    GraphPart* P = gr->part;
    const uint64_t nb = 8 * P->nwords;
    if (P->nranks == 1 || !nb) return RF_OK;
    if (comm) return rf_comm_allreduce_or(comm, P->d_bits.p, P->nwords, s);
    HIPC(P->h_buf.ensure(nb * (P->nranks + 1)));
    uint64_t* h = reinterpret_cast<uint64_t*>(P->h_buf.bytes());
    HIPC(hipMemcpyAsync(h, P->d_bits.p, nb, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (fn(user, h, h + P->nwords, nb)) return fail(RF_EDEVICE, "host all-gather (boundary bitset) failed");
    for (int r = 0; r < P->nranks; ++r)
        for (uint64_t w = 0; w < P->nwords; ++w) h[w] |= h[P->nwords * (r + 1) + w];
    HIPC(hipMemcpyAsync(P->d_bits.p, h, nb, hipMemcpyHostToDevice, s));
    HIPC(hipStreamSynchronize(s));
    return RF_OK;
}

// All-gather of the export blocks ([max_export][32] per rank) into d_gather.
static int part_gather(rf_graph* gr, rf_comm* comm, rf_host_allgather_fn fn, void* user, hipStream_t s) {
    GraphPart* P = gr->part;
    const uint64_t blk = 32ull * P->max_export;
    if (!blk) return RF_OK;
    if (P->nranks == 1) {
        HIPC(hipMemcpyAsync(P->d_gather.p, P->d_send.p, blk, hipMemcpyDeviceToDevice, s));
        return RF_OK;
    }
    if (comm) return rf_comm_allgather(comm, P->d_send.p, P->d_gather.p, blk, s);
    HIPC(P->h_buf.ensure(blk * (P->nranks + 1)));
    uint8_t* h = P->h_buf.bytes();
    HIPC(hipMemcpyAsync(h, P->d_send.p, blk, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (fn(user, h, h + blk, blk)) return fail(RF_EDEVICE, "host all-gather (boundary digests) failed");
    HIPC(hipMemcpyAsync(P->d_gather.p, h + blk, blk * P->nranks, hipMemcpyHostToDevice, s));
    HIPC(hipStreamSynchronize(s));
    return RF_OK;
}

static int part_counts(rf_graph* gr, hipStream_t s, uint64_t* tot) {
    std::vector<uint32_t> counts;
    if (int rc = graph_read_counts(gr, s, counts)) return rc;
    for (uint32_t c : counts) *tot += c;
    return RF_OK;
}

// Fixed-round protocol (rf_graph_part::rounds > 0): the splitter knows the
// most boundary crossings R on any path, so a change settles after R
// exchanges.  Each round gathers EVERY export digest (no changed-since-sent
// bitset, no OR-reduce, no "anything left?" readback), and k_part_apply
// writes the imports whose digest differs from the slot's and queues (or
// hashes, slot fusion) their consumers.  A rank without imports has nothing
// to recompute after its first pass.  With an rf_comm and no count readback
// nothing here waits on the host: kernels and RCCL calls queue on the stream.
static int recompute_rounds(rf_graph* gr, rf_comm* comm, rf_host_allgather_fn fn, void* user, int full,
                            uint64_t* out_recomputed, hipStream_t s) {
    GraphPart* P = gr->part;
    uint64_t tot = 0;
    // deferred levels (GraphPart::defer_lvl): the local pass stops below them
    // and leaves the step open (no cursor swap: their queued jobs stay listed),
    // the post-exchange passes start at them
    const bool defer = P->defer_lvl != ~0u && !full && gr->initialized && graph_plain_steps();
    const uint32_t lo = defer ? P->defer_lvl : 0u;
    if (int rc = graph_recompute_locked(gr, full, s, 0, defer ? lo : ~0u, !defer)) return rc;
    if (out_recomputed && !defer)  // (deferred: the post pass counts the whole step, same cursor half)
        if (int rc = part_counts(gr, s, &tot)) return rc;
    for (uint32_t r = 0; r < P->rounds; ++r) {
        if (P->n_export)
            HIPC(launch_gather_slots(gr->g.slots, P->d_export_slot.as<uint32_t>(), P->n_export,
                                     P->d_send.as<uint8_t>(), s));
        if (int rc = part_gather(gr, comm, fn, user, s)) return rc;
        if (!P->n_import) continue;
        HIPC(launch_part_apply(gr->g, P->d_import_slot.as<uint32_t>(), P->d_import_bid.as<uint32_t>(), P->n_import,
                               nullptr, P->d_gather.as<uint8_t>(), s));
        // the imports are this pass's marked input slots (an upper bound:
        // only changed ones queue anything) -- except in a deferred step,
        // whose passes must pick the same forms (the sink list's launch)
        if (!defer) gr->marked += P->n_import;
        if (int rc = graph_recompute_locked(gr, 0, s, lo)) return rc;
        if (out_recomputed)
            if (int rc = part_counts(gr, s, &tot)) return rc;
    }
    P->last_supersteps = 1 + P->rounds;
    if (out_recomputed) *out_recomputed = tot;
    return RF_OK;
}

extern "C" int rf_graph_recompute_part(rf_graph* gr, rf_comm* comm, rf_host_allgather_fn fn, void* user, int full,
                                       uint64_t* out_recomputed) {
    ARG(gr && gr->part, "graph has no partition (rf_graph_set_part)");
    GraphPart* P = gr->part;
    ARG(P->nranks == 1 || comm || fn, "several ranks need an rf_comm or a host all-gather");
    rf_ctx* ctx = gr->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    hipStream_t s = ctx->stream;
    if (P->rounds && P->nranks > 1) return recompute_rounds(gr, comm, fn, user, full, out_recomputed, s);
    uint64_t tot = 0, steps = 0;
    bool run = true;  // this rank has new inputs for the superstep
    for (;;) {
        if (run) {
            if (int rc = graph_recompute_locked(gr, steps == 0 ? full : 0, s)) return rc;
            if (out_recomputed)
                if (int rc = part_counts(gr, s, &tot)) return rc;
        }
        ++steps;
        if (!P->nwords) break;  // no rank exports anything: the pieces are independent
        HIPC(hipMemsetAsync(P->d_bits.p, 0, 8 * P->nwords, s));
        HIPC(launch_part_pack(P->d_export_slot.as<uint32_t>(), P->n_export, gr->g.slots, P->d_snap.as<uint8_t>(),
                              P->d_send.as<uint8_t>(), P->d_bits.as<uint32_t>(), (uint32_t)P->rank * P->max_export, s));
        if (int rc = part_or(gr, comm, fn, user, s)) return rc;
        if (P->any_import) {  // a changed import may change exports again: one more superstep
            uint32_t flag[2] = {0, 0};
            HIPC(launch_part_any(P->d_bits.as<uint64_t>(), P->nwords, P->d_import_bid.as<uint32_t>(), P->n_import,
                                 P->d_flag.as<uint32_t>(), s));
            HIPC(hipMemcpyAsync(flag, P->d_flag.p, 8, hipMemcpyDeviceToHost, s));
            HIPC(hipStreamSynchronize(s));
            if (!flag[0]) break;
            run = flag[1] != 0;
        }
        if (int rc = part_gather(gr, comm, fn, user, s)) return rc;
        if (!P->any_import) break;  // exports observed, nobody consumes them
        if (run) {
            HIPC(launch_part_apply(gr->g, P->d_import_slot.as<uint32_t>(), P->d_import_bid.as<uint32_t>(),
                                   P->n_import, P->d_bits.as<uint32_t>(), P->d_gather.as<uint8_t>(), s));
            gr->marked += P->n_import;  // (upper bound of the next superstep's changed inputs)
        }
    }
    P->last_supersteps = steps;
    if (out_recomputed) *out_recomputed = tot;
    return RF_OK;
}

extern "C" int rf_graph_part_gathered(rf_graph* gr, const void** d_digests32, uint64_t* n, uint64_t* supersteps) {
    ARG(gr && gr->part, "graph has no partition");
    if (d_digests32) *d_digests32 = gr->part->d_gather.p;
    if (n) *n = (uint64_t)gr->part->nranks * gr->part->max_export;
    if (supersteps) *supersteps = gr->part->last_supersteps;
    return RF_OK;
}
