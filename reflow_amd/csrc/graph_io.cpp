// graph_io.cpp -- checkpoint / resume of a loaded digest DAG: rf_graph_save
// writes the lowered device form (job records, holes, reverse edges, padded
// templates, midstates, level layout) together with the current slot digests;
// rf_graph_restore brings it back onto a device ready for incremental steps,
// without the lowering, the level / fusion analysis, the midstate hashing or a
// full recompute.
//
// Reference: memoization is Reflow's resume mechanism: a run's
// State is marshalled after every runner step (runner/runner.go:51-85) and
// the local executor restores its execs from manifests
// (local/executor.go:122-200); the digests themselves are recomputed per Eval
// (flow.go:653-664).  Here the digests ARE the state a resumed run needs, so
// they are persisted with the graph they belong to, and a later process
// applies only what changed since.
//
// File: a 128-B header, the sections in a fixed order (each a u64 length and
// its bytes), then one SHA-256 per 64 MiB chunk of each section, the SHA-256
// of header || chunk digests, and an end marker.  The chunk digests are
// computed on the host leg's threads (SHA-NI); a mismatch on restore is
// RF_EINTEGRITY (errors.Integrity, repository/file/repository.go:160-162).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "graph_internal.h"

using namespace rf;

namespace {

constexpr char kMagic[8] = {'R', 'F', 'G', 'R', 'A', 'P', 'H', '1'};
constexpr char kEnd[8] = {'R', 'F', 'G', 'R', 'E', 'N', 'D', '1'};
// 1 (round 4) and 3 share one layout; 2 (round 5) appended four sections
// of the since-removed flow step (jlv, cout_rng, cout, dstart), which a
// restore reads, checks against the checksums and drops
constexpr uint32_t kVersion = 3;
constexpr uint64_t kChunk = 64ull << 20;   // checksum granule
constexpr uint64_t kStage = 256ull << 20;  // D2H / H2D staging (4 chunks)

enum : uint32_t { kHoleInB0 = 1, kFusePos2 = 2, kHasMid = 4, kInitialized = 8 };

struct Header {
    char magic[8];
    uint32_t version, flags;
    uint32_t n_jobs, n_slots, n_levels, max_level_jobs;
    uint64_t n_holes, tmpl_bytes, total_blocks, chunk;
    uint64_t n_sections;
    uint64_t n_cout;  // version 2 only: the flow step's chain-out edges (its "cout" section: 8 B each); else 0
    uint8_t reserved[128 - 8 - 6 * 4 - 6 * 8];
};
static_assert(sizeof(Header) == 128, "header layout");

// One section of the file: host bytes, or a device buffer moved through the
// pinned stage, or (neither) a version-2 section a restore reads and drops.
struct Section {
    const char* name;
    uint64_t bytes;
    void* host = nullptr;  // host memory (save: source; restore: destination)
    void* dev = nullptr;   // device memory
};

std::vector<Section> sections(rf_graph* gr, std::vector<uint32_t>& lvl, std::vector<uint8_t>& inc,
                              std::vector<uint32_t>& ext2int, bool has_mid, uint32_t version = kVersion,
                              uint64_t n_cout = 0) {
    const GraphDev& G = gr->g;
    const uint64_t J = G.n_jobs, S = G.n_slots, L = G.n_levels, H = gr->hole_count;
    std::vector<Section> v = {
        {"lvl_start", 4 * (L + 1), lvl.data()},
        {"inc_level", L, inc.data()},
        {"ext2int", 4 * J, ext2int.data()},
        {"meta", 32 * J, nullptr, gr->b_meta.p},
        {"holes", 8 * H, nullptr, gr->b_holes.p},
        {"cons_ptr", 4 * (S + 1), nullptr, gr->b_cons_ptr.p},
        {"cons_job", 8 * H, nullptr, gr->b_cons_job.p},
        {"tmpl", gr->tmpl_bytes, nullptr, gr->b_tmpl.p},
        {"slots", 32 * S, nullptr, gr->b_slots.p},
    };
    if (has_mid) v.push_back({"mid", 32 * J, nullptr, gr->b_mid.p});
    if (version == 2)
        for (Section x : {Section{"jlv", 8 * J}, Section{"cout_rng", 8 * J}, Section{"cout", 8 * n_cout},
                          Section{"dstart", 4 * (L + 1)}})
            v.push_back(x);
    return v;
}

// SHA-256 of each kChunk granule of buf[0, n) into out (in order), on the
// host pool when there is one.
void hash_chunks(rf_ctx* ctx, const uint8_t* buf, uint64_t n, uint8_t* out) {
    const uint64_t nc = (n + kChunk - 1) / kChunk;
    HostPool* pool = ctx_pool(ctx);
    if (!pool || nc < 2) {
        for (uint64_t c = 0; c < nc; ++c) host_sha256(buf + c * kChunk, std::min(kChunk, n - c * kChunk), out + 32 * c);
        return;
    }
    std::atomic<uint64_t> next{0};
    pool->run([&](unsigned) {
        for (uint64_t c; (c = next.fetch_add(1)) < nc;)
            host_sha256(buf + c * kChunk, std::min(kChunk, n - c * kChunk), out + 32 * c);
    });
}

// Consistency checks of a file being restored, section by section, before
// any of it reaches a kernel: every index a kernel follows stays inside its
// array, and the structure the kernels assume holds (a file whose checksums
// match may still come from anywhere).  Sections arrive in file order
// (lvl_start, inc_level, ext2int, meta, holes, cons_ptr, cons_job, ...), the
// device ones in pieces [o, o + n) that keep records whole (kStage).
struct Validator {
    const Header& h;
    const std::vector<uint32_t>& lvl;      // level layout (host section, complete before the device ones)
    const std::vector<uint8_t>& inc;       // per-level flags (host section, ditto)
    std::vector<uint32_t>& out_slot;       // internal job -> out slot (from the records)
    uint32_t lv = 0;                       // meta cursor: the level of the next record
    std::vector<uint8_t> one_hole;         // internal job has exactly one hole
    std::vector<uint8_t> produced;         // slot is some job's output
    std::vector<uint32_t> cons_ptr;        // host copy: slot -> its reverse-edge range
    uint64_t slot = 0;                     // cons_job cursor: the slot whose range holds the next edge
    // fusion targets: job t fused behind j must have exactly one
    // hole reading j's out slot -- at byte 2 when the file says kFusePos2 (the
    // chain builds its block 0 in registers, from the IV: no midstate) --
    // else a file with valid checksums restores into wrong digests
    std::vector<uint32_t> exp_slot;                   // target -> its producer's out slot (~0: not a target)
    std::vector<std::pair<uint64_t, uint32_t>> tgt_holes;  // (the target's hole index, expected slot), ascending
    size_t tgt_cur = 0;

    // after the structure sections: every fusion target's hole was seen
    int done() const {
        if (tgt_cur != tgt_holes.size()) return fail(RF_EINTEGRITY, "graph restore: fusion target holes missing");
        return RF_OK;
    }

    Validator(const Header& hh, const std::vector<uint32_t>& l, const std::vector<uint8_t>& in, std::vector<uint32_t>& os)
        : h(hh), lvl(l), inc(in), out_slot(os) {}

    // a host section, once complete
    int host_done(const char* name, const std::vector<uint32_t>* ext2int) {
        if (!strcmp(name, "lvl_start")) {
            if (lvl[0] != 0 || lvl[h.n_levels] != h.n_jobs)
                return fail(RF_EINTEGRITY, "graph restore: bad level layout");
            for (uint32_t l = 0; l < h.n_levels; ++l)
                if (lvl[l] > lvl[l + 1]) return fail(RF_EINTEGRITY, "graph restore: bad level layout");
        } else if (!strcmp(name, "ext2int")) {  // a permutation of the internal ids
            std::vector<uint8_t> seen(h.n_jobs, 0);
            for (uint32_t i : *ext2int) {
                if (i >= h.n_jobs || seen[i]) return fail(RF_EINTEGRITY, "graph restore: job numbering damaged");
                seen[i] = 1;
            }
        }
        return RF_OK;
    }

    int piece(const char* name, const uint8_t* p, uint64_t n, uint64_t o) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
        const uint64_t J = h.n_jobs, S = h.n_slots, H = h.n_holes, TB = h.tmpl_bytes / 64;
        if (!strcmp(name, "meta")) {
            if (o == 0) one_hole.assign(J, 0), produced.assign(S, 0), exp_slot.assign(J, ~0u);
            for (uint64_t r = 0; r < n / 32; ++r) {
                const uint32_t* m = w + 8 * r;
                if ((uint64_t)m[0] + m[1] > TB || m[2] > m[3] || m[3] > H || m[4] >= S || m[5] > m[6] || m[6] > H ||
                    (m[7] != 0xffffffffu && m[7] >= J))
                    return fail(RF_EINTEGRITY, "graph restore: job record %llu out of range",
                                (unsigned long long)(o / 32 + r));
                const uint64_t j = o / 32 + r;
                // a level run in the octo form stages each job whole in LDS
                while (lv < h.n_levels && lvl[lv + 1] <= j) ++lv;
                if (lv < h.n_levels && (inc[lv] & kLvlOct) &&
                    (m[1] > kOctMaxBlocks || m[3] - m[2] > kOctMaxHoles || m[7] != 0xffffffffu))
                    return fail(RF_EINTEGRITY, "graph restore: job record %llu exceeds its level's form",
                                (unsigned long long)j);
                out_slot[j] = m[4];
                one_hole[j] = m[3] - m[2] == 1;
                produced[m[4]] = 1;
                if (exp_slot[j] != ~0u) {  // j is a fusion target (its producer's record came first)
                    if (m[3] - m[2] != 1) return fail(RF_EINTEGRITY, "graph restore: fusion target %llu has %u holes",
                                                     (unsigned long long)j, m[3] - m[2]);
                    tgt_holes.push_back({m[2], exp_slot[j]});
                }
                if (m[7] != 0xffffffffu) {
                    if (m[7] <= j || exp_slot[m[7]] != ~0u)
                        return fail(RF_EINTEGRITY, "graph restore: fusion target of job %llu inconsistent",
                                    (unsigned long long)j);
                    exp_slot[m[7]] = m[4];
                }
            }
        } else if (!strcmp(name, "holes")) {
            for (uint64_t r = 0; r < n / 8; ++r) {
                const uint64_t hi = o / 8 + r;
                if (w[2 * r + 1] >= S || w[2 * r] >= (1u << 24))
                    return fail(RF_EINTEGRITY, "graph restore: hole %llu out of range", (unsigned long long)hi);
                if (tgt_cur < tgt_holes.size() && tgt_holes[tgt_cur].first == hi) {
                    if (w[2 * r + 1] != tgt_holes[tgt_cur].second || ((h.flags & 2u) && w[2 * r] != 2))  // (kFusePos2)
                        return fail(RF_EINTEGRITY, "graph restore: fusion target hole %llu inconsistent",
                                    (unsigned long long)hi);
                    ++tgt_cur;
                }
            }
        } else if (!strcmp(name, "cons_ptr")) {
            if (o == 0) cons_ptr.reserve(S + 1);
            for (uint64_t r = 0; r < n / 4; ++r) {
                if (w[r] > H || (!cons_ptr.empty() && w[r] < cons_ptr.back()))
                    return fail(RF_EINTEGRITY, "graph restore: reverse-edge index out of range");
                cons_ptr.push_back(w[r]);
            }
            if (o + n == 4 * (S + 1) && (cons_ptr.size() != S + 1 || cons_ptr[0] != 0 || cons_ptr[S] != H))
                return fail(RF_EINTEGRITY, "graph restore: reverse-edge index out of range");
        } else if (!strcmp(name, "cons_job")) {
            // edge e = {consumer x, its level y | kSlotFused}: x must lie in
            // level y (append_jobs writes list[lvl_start[y] + count] and its
            // record there), and the slot-fused flag may mark only the first
            // edge of an input slot's range, pointing at a one-hole job (the
            // mark kernel hashes that job with the slot's digest in its hole)
            for (uint64_t r = 0; r < n / 8; ++r) {
                const uint64_t e = o / 8 + r;
                while (slot < S && cons_ptr[slot + 1] <= e) ++slot;
                const uint32_t x = w[2 * r], y = w[2 * r + 1] & 0x7fffffffu;
                const bool fused = (w[2 * r + 1] & 0x80000000u) != 0;
                if (x >= J || y >= h.n_levels || x < lvl[y] || x >= lvl[y + 1] || slot >= S ||
                    (fused && (e != cons_ptr[slot] || produced[slot] || !one_hole[x])))
                    return fail(RF_EINTEGRITY, "graph restore: reverse edge %llu inconsistent", (unsigned long long)e);
            }
        } else if (!strcmp(name, "mid")) {
            // a kFusePos2 fusion target starts from the IV (k2_level_pl hands
            // its block 0 over in registers and never loads its midstate)
            static const uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                           0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
            for (uint64_t r = 0; r < n / 32; ++r) {
                const uint64_t j = o / 32 + r;
                if ((h.flags & 2u) && exp_slot[j] != ~0u && memcmp(w + 8 * r, IV, 32) != 0)
                    return fail(RF_EINTEGRITY, "graph restore: fusion target %llu has a midstate", (unsigned long long)j);
            }
        }
        return RF_OK;
    }
};

struct Stage {  // pinned staging, released on every path
    HostBuf b;
    ~Stage() { b.release(); }
};

struct File {
    FILE* f = nullptr;
    ~File() {
        if (f) fclose(f);
    }
};

}  // namespace

extern "C" int rf_graph_save(rf_graph* gr, const char* path) {
    ARG(gr && path && *path, "null argument");
    rf_ctx* ctx = gr->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    // The file holds slot digests, not the change set pending between a
    // set_slots and the recompute that consumes it (the queued flags and
    // per-level lists): a slot set but not yet propagated would be saved
    // with stale consumers and restored with nothing queued.  Refuse.
    if (gr->marked) return fail(RF_EPRECONDITION, "graph save: input slots set since the last recompute");
    DevGuard dg(ctx->device);
    // steps queued on callers' streams must be complete before the state is read
    HIPC(hipDeviceSynchronize());
    GraphDev& G = gr->g;
    std::vector<uint32_t> lvl(G.lvl_start.begin(), G.lvl_start.end());
    std::vector<uint8_t> inc(G.inc_level.begin(), G.inc_level.end());
    std::vector<uint32_t> ext2int(gr->ext2int.begin(), gr->ext2int.end());
    const bool has_mid = G.mid != nullptr;
    std::vector<Section> secs = sections(gr, lvl, inc, ext2int, has_mid);
    Header h{};
    memcpy(h.magic, kMagic, 8);
    h.version = kVersion;
    h.flags = (G.hole_in_b0 ? kHoleInB0 : 0) | (G.fuse_pos2 ? kFusePos2 : 0) | (has_mid ? kHasMid : 0) |
              (gr->initialized ? kInitialized : 0);
    h.n_jobs = G.n_jobs;
    h.n_slots = G.n_slots;
    h.n_levels = G.n_levels;
    h.max_level_jobs = gr->max_level_jobs;
    h.n_holes = gr->hole_count;
    h.tmpl_bytes = gr->tmpl_bytes;
    h.total_blocks = gr->total_blocks;
    h.chunk = kChunk;
    h.n_sections = secs.size();
    const std::string tmp = std::string(path) + ".tmp";
    File out;
    if (!(out.f = fopen(tmp.c_str(), "wb"))) return fail(RF_EIO, "graph save: cannot create %s", tmp.c_str());
    auto put = [&](const void* p, uint64_t n) { return fwrite(p, 1, n, out.f) == n; };
    if (!put(&h, sizeof h)) return fail(RF_EIO, "graph save: write failed");
    Stage st;
    HostBuf& stage = st.b;
    HIPC(stage.ensure(kStage));
    std::vector<uint8_t> digests;
    for (const Section& sc : secs) {
        if (!put(&sc.bytes, 8)) return fail(RF_EIO, "graph save: write failed");
        for (uint64_t o = 0; o < sc.bytes; o += kStage) {
            const uint64_t n = std::min(kStage, sc.bytes - o);
            const uint8_t* src;
            if (sc.dev) {
                HIPC(sync_copy(ctx, stage.p, static_cast<const uint8_t*>(sc.dev) + o, n, hipMemcpyDeviceToHost));
                src = stage.bytes();
            } else {
                src = static_cast<const uint8_t*>(sc.host) + o;
            }
            const size_t d0 = digests.size();
            digests.resize(d0 + 32 * ((n + kChunk - 1) / kChunk));
            hash_chunks(ctx, src, n, digests.data() + d0);
            if (!put(src, n)) return fail(RF_EIO, "graph save: write failed (%s)", sc.name);
        }
    }
    std::vector<uint8_t> all(sizeof h + digests.size());
    memcpy(all.data(), &h, sizeof h);
    if (!digests.empty()) memcpy(all.data() + sizeof h, digests.data(), digests.size());
    uint8_t root[32];
    host_sha256(all.data(), all.size(), root);
    const uint64_t nd = digests.size() / 32;
    if (!put(&nd, 8) || !put(digests.data(), digests.size()) || !put(root, 32) || !put(kEnd, 8))
        return fail(RF_EIO, "graph save: write failed");
    if (fflush(out.f) != 0 || fsync(fileno(out.f)) != 0) return fail(RF_EIO, "graph save: flush failed");
    fclose(out.f);
    out.f = nullptr;
    if (rename(tmp.c_str(), path) != 0) return fail(RF_EIO, "graph save: cannot rename to %s", path);
    return RF_OK;
}

extern "C" int rf_graph_restore(rf_ctx* ctx, const char* path, rf_graph** out) {
    ARG(ctx && path && out, "null argument");
    *out = nullptr;
    File in;
    if (!(in.f = fopen(path, "rb"))) return fail(RF_EIO, "graph restore: cannot open %s", path);
    auto get = [&](void* p, uint64_t n) { return fread(p, 1, n, in.f) == n; };
    Header h;
    if (!get(&h, sizeof h) || memcmp(h.magic, kMagic, 8) != 0)
        return fail(RF_EINVAL, "graph restore: %s is not a graph checkpoint", path);
    if (h.version < 1 || h.version > kVersion || h.chunk != kChunk)
        return fail(RF_EINVAL, "graph restore: checkpoint version %u not supported", h.version);
    const uint64_t n_sec = ((h.flags & kHasMid) ? 10u : 9u) + (h.version == 2 ? 4u : 0u);
    if (h.n_sections != n_sec || h.n_jobs > (1u << 31) || h.n_levels > h.n_jobs + 1 ||
        (h.version == 2 ? h.n_cout >= 0xffffffffull : h.n_cout != 0))
        return fail(RF_EINTEGRITY, "graph restore: corrupt header");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard dg(ctx->device);
    auto* gr = new rf_graph();
    std::unique_ptr<rf_graph, void (*)(rf_graph*)> guard(gr, [](rf_graph* x) { rf_graph_destroy(x); });
    gr->ctx = ctx;
    gr->hole_count = h.n_holes;
    gr->tmpl_bytes = h.tmpl_bytes;
    gr->total_blocks = h.total_blocks;
    gr->max_level_jobs = h.max_level_jobs;
    GraphDev& G = gr->g;
    G.hole_in_b0 = (h.flags & kHoleInB0) != 0;
    G.fuse_pos2 = (h.flags & kFusePos2) != 0;
    G.stream_handover = RF_DIAG_KNOB("RF_K2_STREAM", 0) == 1;
    graph_forms_from_env(G);
    G.n_cu = graph_ovf_cus(ctx, &G.ovf_mode);
    if (int rc = graph_device_alloc(gr, h.n_jobs, h.n_slots, h.n_levels, h.n_holes, h.tmpl_bytes)) return rc;
    const bool has_mid = (h.flags & kHasMid) != 0;
    if (has_mid) {
        HIPC(gr->b_mid.ensure(std::max<size_t>(32ull * h.n_jobs, 64)));
        G.mid = gr->b_mid.as<uint4>();
    }
    std::vector<uint32_t> lvl(h.n_levels + 1);
    std::vector<uint8_t> inc(h.n_levels);
    std::vector<uint32_t> ext2int(h.n_jobs);
    std::vector<Section> secs = sections(gr, lvl, inc, ext2int, has_mid, h.version, h.n_cout);
    std::vector<uint32_t> out_slot(h.n_jobs);  // internal job -> out slot (from the records)
    Validator val(h, lvl, inc, out_slot);
    Stage st;
    HostBuf& stage = st.b;
    HIPC(stage.ensure(kStage));
    std::vector<uint8_t> digests;
    for (const Section& sc : secs) {
        uint64_t n_sec = 0;
        if (!get(&n_sec, 8) || n_sec != sc.bytes)
            return fail(RF_EINTEGRITY, "graph restore: section %s truncated or resized", sc.name);
        for (uint64_t o = 0; o < sc.bytes; o += kStage) {
            const uint64_t n = std::min(kStage, sc.bytes - o);
            uint8_t* dst = sc.host ? static_cast<uint8_t*>(sc.host) + o : stage.bytes();
            if (!get(dst, n)) return fail(RF_EINTEGRITY, "graph restore: section %s truncated", sc.name);
            const size_t d0 = digests.size();
            digests.resize(d0 + 32 * ((n + kChunk - 1) / kChunk));
            hash_chunks(ctx, dst, n, digests.data() + d0);
            // the indices and structure the kernels follow are checked before
            // the piece reaches the device (kStage keeps records whole)
            if (int rc = val.piece(sc.name, dst, n, o)) return rc;
            if (sc.dev) HIPC(sync_copy(ctx, static_cast<uint8_t*>(sc.dev) + o, dst, n, hipMemcpyHostToDevice));
        }
        if (sc.host)
            if (int rc = val.host_done(sc.name, &ext2int)) return rc;
    }
    if (int rc = val.done()) return rc;
    uint64_t nd = 0;
    uint8_t root[32], want[32], end[8];
    if (!get(&nd, 8) || nd != digests.size() / 32) return fail(RF_EINTEGRITY, "graph restore: checksum list damaged");
    std::vector<uint8_t> stored(32 * nd);
    if (!get(stored.data(), stored.size()) || !get(want, 32) || !get(end, 8) || memcmp(end, kEnd, 8) != 0)
        return fail(RF_EINTEGRITY, "graph restore: trailer truncated");
    std::vector<uint8_t> all(sizeof h + stored.size());
    memcpy(all.data(), &h, sizeof h);
    if (!stored.empty()) memcpy(all.data() + sizeof h, stored.data(), stored.size());
    host_sha256(all.data(), all.size(), root);
    if (memcmp(root, want, 32) != 0 || stored != digests)
        return fail(RF_EINTEGRITY, "graph restore: %s does not match its checksums", path);
    // host-side state: level layout (checked as it arrived; its device copy
    // every level kernel reads), and slot -> producing (external) job
    HIPC(sync_copy(ctx, gr->b_lvl_start.p, lvl.data(), 4ull * (h.n_levels + 1), hipMemcpyHostToDevice));
    G.lvl_start.assign(lvl.begin(), lvl.end());
    G.inc_level.assign(inc.begin(), inc.end());
    gr->ext2int = std::move(ext2int);
    gr->producer.assign(h.n_slots, -1);
    for (uint32_t j = 0; j < h.n_jobs; ++j) {
        const uint32_t i = gr->ext2int[j];
        if (i >= h.n_jobs || out_slot[i] >= h.n_slots) return fail(RF_EINTEGRITY, "graph restore: bad job record");
        gr->producer[out_slot[i]] = j;
    }
    G.split_b0 = G.hole_in_b0 && G.fuse_pos2 ? graph_split_on() : 0u;  // (as rf_graph_load)
    if (int rc = graph_build_plan(gr)) return rc;
    gr->initialized = (h.flags & kInitialized) != 0;
    guard.release();
    *out = gr;
    return RF_OK;
}
