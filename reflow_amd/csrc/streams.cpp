// streams.cpp -- streaming SHA-256 behind the C-ABI (rf_sha_streams_*) and
// the integrity checks (rf_sha_streams_verify, rf_sha256_verify).
//
// Reference: Digester.NewWriter() returns an io.Writer whose state carries
// across Write calls (grailbio/base/digest over crypto/sha256, flow.go:36);
// Repository.Put hashes an io.Reader as it copies it (repository/file/
// repository.go:237-264), s3's Put through a TeeReader (repository/s3/s3.go:
// 120-147), and ReadFrom / WriteTo re-digest a transfer and fail with
// errors.Integrity on a mismatch (repository/file/repository.go:126-166).
//
// Many streams, batched: a Write batch hands chunks for any streams; per
// stream the carried partial block plus its chunks give whole blocks (hashed
// from the stream's midstate) and a new partial block.  The whole-block
// segments are split like a K1 plan: the largest go to the host leg (SHA-NI,
// zero-copy from the caller's chunks), the rest to k1_sha256_resume (lane per
// segment; the bytes packed into a pinned stage and uploaded), by a makespan
// model.  Digest pads the carried block on the same path.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <numeric>
#include <vector>

#include "ctx.h"
#include "engine.h"

using namespace rf;

namespace {
constexpr uint32_t kIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                             0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

struct Piece {
    const uint8_t* p;
    uint64_t len;
};

// One stream's share of a batch: its carried bytes, then its pieces in order.
struct Seg {
    uint64_t stream;
    uint64_t bytes;  // carry + pieces
    uint64_t nb;     // whole blocks hashed now
    uint32_t p0, p1; // pieces [p0, p1) of the batch's piece list
    bool host;
};
}  // namespace

struct rf_sha_streams {
    rf_ctx* ctx = nullptr;
    uint64_t n = 0;
    uint32_t flags = 0;
    std::vector<uint32_t> mid;    // [n][8] midstates (host copy is authoritative)
    std::vector<uint8_t> carry;   // [n][64] partial block
    std::vector<uint32_t> clen;   // [n]
    std::vector<uint64_t> total;  // [n] bytes written since the last digest
    // a feed that failed part-way (a HIP error after the host leg absorbed
    // its segments) leaves midstates, carries and lengths out of step: every
    // later call on the set fails
    bool failed = false;
    DevBuf d_arena, d_mid, d_offs, d_nb;
    HostBuf h_stage, h_mid;
};

extern "C" int rf_sha_streams_open(rf_ctx* ctx, uint64_t n, uint32_t flags, rf_sha_streams** out) {
    ARG(ctx && out, "null argument");
    ARG(n >= 1 && n <= (1ull << 32), "streams: 1 <= n <= 2^32");
    ARG(!((flags & RF_SHA_ALL_HOST) && (flags & RF_SHA_NO_HOST)), "RF_SHA_ALL_HOST with RF_SHA_NO_HOST");
    ARG((flags & ~(RF_SHA_ALL_HOST | RF_SHA_NO_HOST)) == 0, "streams take only RF_SHA_ALL_HOST / RF_SHA_NO_HOST");
    auto* S = new rf_sha_streams();
    S->ctx = ctx;
    S->n = n;
    S->flags = flags;
    S->mid.resize(8 * n);
    for (uint64_t i = 0; i < n; ++i) memcpy(&S->mid[8 * i], kIV, sizeof kIV);
    S->carry.assign(64 * n, 0);
    S->clen.assign(n, 0);
    S->total.assign(n, 0);
    *out = S;
    return RF_OK;
}

extern "C" void rf_sha_streams_close(rf_sha_streams* S) {
    if (!S) return;
    DevGuard g(S->ctx->device);
    for (DevBuf* b : {&S->d_arena, &S->d_mid, &S->d_offs, &S->d_nb}) b->release();
    S->h_stage.release();
    S->h_mid.release();
    delete S;
}

// Host leg or GPU for each segment: the h largest (by bytes) to the host
// slots (one 1-way SHA-NI chain per stream: the chunks are hashed in place),
// the rest to k1_sha256_resume, whose cost is the pack + upload of its bytes
// plus max(longest segment's chain at 3.2 us/block, blocks at chip rate).
static void split_segments(std::vector<Seg>& segs, unsigned threads, uint32_t flags) {
    const uint64_t n = segs.size();
    for (Seg& s : segs) s.host = false;
    if (!n || (flags & RF_SHA_NO_HOST) || threads == 0) return;
    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return segs[a].nb > segs[b].nb; });
    uint64_t h = n;
    if (!(flags & RF_SHA_ALL_HOST)) {
        const double rate = host_sha_rate(1), link = 25e9, pack = 8e9, blk_rate = 35e12 / 1464.0;
        std::vector<double> suf_bytes(n + 1, 0), suf_nb(n + 1, 0);
        for (uint64_t i = n; i-- > 0;) {
            suf_bytes[i] = suf_bytes[i + 1] + (double)segs[order[i]].nb * 64;
            suf_nb[i] = suf_nb[i + 1] + (double)segs[order[i]].nb;
        }
        std::vector<double> load(threads, 0.0);
        double best = 1e300, maxload = 0;
        for (uint64_t x = 0; x <= n; ++x) {
            if (x) {
                std::pop_heap(load.begin(), load.end(), std::greater<double>());
                load.back() += (double)segs[order[x - 1]].nb * 64 / rate + 5e-6;
                maxload = std::max(maxload, load.back());
                std::push_heap(load.begin(), load.end(), std::greater<double>());
            }
            const double host_t = x ? maxload + 50e-6 : 0.0;
            const double gpu_t = x < n ? 30e-6 + suf_bytes[x] / pack + suf_bytes[x] / link +
                                             std::max((double)segs[order[x]].nb * 3.2e-6, suf_nb[x] / blk_rate)
                                       : 0.0;
            const double m = std::max(host_t, gpu_t);
            if (m < best) {
                best = m;
                h = x;
            }
        }
    }
    for (uint64_t i = 0; i < h; ++i) segs[order[i]].host = true;
}

// Bytes [from, to) of the segment's virtual concatenation carry ++ pieces.
static void seg_copy(const rf_sha_streams* S, const Seg& s, const std::vector<Piece>& pieces, uint64_t from,
                     uint64_t to, uint8_t* dst) {
    uint64_t pos = 0;
    auto take = [&](const uint8_t* p, uint64_t len) {
        const uint64_t a = std::max(from, pos), b = std::min(to, pos + len);
        if (a < b) memcpy(dst + (a - from), p + (a - pos), b - a);
        pos += len;
    };
    take(&S->carry[64 * s.stream], S->clen[s.stream]);
    for (uint32_t k = s.p0; k < s.p1 && pos < to; ++k) take(pieces[k].p, pieces[k].len);
}

// Feeds every segment: whole blocks into its stream's midstate, the rest
// into its carried block.  Caller holds ctx->mu.
static int streams_feed(rf_sha_streams* S, std::vector<Seg>& segs, const std::vector<Piece>& pieces) {
    rf_ctx* ctx = S->ctx;
    HostPool* pool = (S->flags & RF_SHA_NO_HOST) ? nullptr : ctx_pool(ctx);
    if ((S->flags & RF_SHA_ALL_HOST) && !pool)
        return fail(RF_EINVAL, "streams opened with RF_SHA_ALL_HOST but the host leg is off");
    split_segments(segs, pool ? pool->size() : 0, S->flags);
    // GPU segments: pack whole blocks (64-B aligned), midstates, run, read back
    std::vector<uint32_t> gpu;
    uint64_t stage_bytes = 0;
    for (uint32_t i = 0; i < segs.size(); ++i)
        if (!segs[i].host && segs[i].nb) {
            gpu.push_back(i);
            stage_bytes += 64 * segs[i].nb;
        }
    std::stable_sort(gpu.begin(), gpu.end(), [&](uint32_t a, uint32_t b) { return segs[a].nb > segs[b].nb; });
    if (!gpu.empty()) {
        const uint64_t g = gpu.size();
        HIPC(S->h_stage.ensure(stage_bytes + 64));
        HIPC(S->h_mid.ensure(32 * g + 16 * g));
        HIPC(S->d_arena.ensure(stage_bytes + 64));
        HIPC(S->d_mid.ensure(32 * g));
        HIPC(S->d_offs.ensure(8 * g));
        HIPC(S->d_nb.ensure(8 * g));
        uint32_t* hm = reinterpret_cast<uint32_t*>(S->h_mid.bytes());
        uint64_t* hoff = reinterpret_cast<uint64_t*>(S->h_mid.bytes() + 32 * g);
        uint64_t* hnb = hoff + g;
        uint64_t pos = 0;
        for (uint64_t k = 0; k < g; ++k) {
            const Seg& s = segs[gpu[k]];
            seg_copy(S, s, pieces, 0, 64 * s.nb, S->h_stage.bytes() + pos);
            memcpy(hm + 8 * k, &S->mid[8 * s.stream], 32);
            hoff[k] = pos;
            hnb[k] = s.nb;
            pos += 64 * s.nb;
        }
        hipStream_t st = ctx->stream;
        HIPC(hipMemcpyAsync(S->d_arena.p, S->h_stage.p, stage_bytes, hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(S->d_mid.p, hm, 32 * g, hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(S->d_offs.p, hoff, 8 * g, hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(S->d_nb.p, hnb, 8 * g, hipMemcpyHostToDevice, st));
        ResumeArgs ra{S->d_arena.as<uint8_t>(), S->d_offs.as<uint64_t>(), S->d_nb.as<uint64_t>(),
                      S->d_mid.as<uint32_t>(), (uint32_t)g};
        HIPC(launch_sha_resume(ra, st));
        HIPC(hipMemcpyAsync(hm, S->d_mid.p, 32 * g, hipMemcpyDeviceToHost, st));
        // host-leg segments run while the GPU works (disjoint streams)
    }
    std::vector<uint32_t> host;
    for (uint32_t i = 0; i < segs.size(); ++i)
        if (segs[i].host) host.push_back(i);
    if (!host.empty()) {
        std::stable_sort(host.begin(), host.end(), [&](uint32_t a, uint32_t b) { return segs[a].bytes > segs[b].bytes; });
        std::atomic<uint64_t> next{0};
        pool->run([&](unsigned) {
            for (uint64_t q; (q = next.fetch_add(1)) < host.size();) {
                const Seg& s = segs[host[q]];
                for (uint32_t k = s.p0; k < s.p1; ++k)
                    host_sha_absorb(&S->mid[8 * s.stream], &S->carry[64 * s.stream], &S->clen[s.stream],
                                    pieces[k].p, pieces[k].len);
            }
        });
    }
    if (!gpu.empty()) {
        HIPC(hipStreamSynchronize(ctx->stream));
        const uint32_t* hm = reinterpret_cast<const uint32_t*>(S->h_mid.bytes());
        for (uint64_t k = 0; k < gpu.size(); ++k) {
            const Seg& s = segs[gpu[k]];
            memcpy(&S->mid[8 * s.stream], hm + 8 * k, 32);
        }
    }
    // GPU (and block-less) segments: the bytes past their whole blocks become the carry
    for (Seg& s : segs) {
        if (s.host) continue;
        uint8_t tail[64];
        const uint64_t rest = s.bytes - 64 * s.nb;
        seg_copy(S, s, pieces, 64 * s.nb, s.bytes, tail);
        memcpy(&S->carry[64 * s.stream], tail, rest);
        S->clen[s.stream] = (uint32_t)rest;
    }
    return RF_OK;
}

extern "C" int rf_sha_streams_write(rf_sha_streams* S, const uint64_t* ids, const uint8_t* const* chunks,
                                    const uint64_t* lens, uint64_t n) {
    ARG(S && (n == 0 || (ids && chunks && lens)), "null argument");
    if (!n) return RF_OK;
    for (uint64_t i = 0; i < n; ++i) {
        if (ids[i] >= S->n) return fail(RF_EINVAL, "stream id %llu >= %llu", (unsigned long long)ids[i],
                                        (unsigned long long)S->n);
        ARG(chunks[i] || lens[i] == 0, "null chunk with nonzero length");
    }
    // every read and update of the per-stream state happens under the
    // context lock (a concurrent rf_sha_streams_digest resets clen / total)
    std::lock_guard<std::mutex> lk(S->ctx->mu);
    if (S->failed) return fail(RF_EDEVICE, "stream set failed in an earlier call");
    // group the chunks by stream, batch order within a stream (Write order)
    std::vector<uint64_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0ull);
    std::stable_sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return ids[a] < ids[b]; });
    std::vector<Piece> pieces;
    std::vector<Seg> segs;
    std::vector<uint64_t> added;  // per segment: the bytes this batch writes
    pieces.reserve(n);
    for (uint64_t q = 0; q < n;) {
        const uint64_t s = ids[idx[q]];
        Seg g{s, S->clen[s], 0, (uint32_t)pieces.size(), 0, false};
        uint64_t add = 0;
        for (; q < n && ids[idx[q]] == s; ++q) {
            if (!lens[idx[q]]) continue;
            pieces.push_back(Piece{chunks[idx[q]], lens[idx[q]]});
            g.bytes += lens[idx[q]];
            add += lens[idx[q]];
        }
        g.p1 = (uint32_t)pieces.size();
        g.nb = g.bytes / 64;
        segs.push_back(g);
        added.push_back(add);
    }
    DevGuard dg(S->ctx->device);
    if (int rc = streams_feed(S, segs, pieces)) {
        S->failed = true;
        return rc;
    }
    // lengths are committed only with the midstates they describe
    for (size_t k = 0; k < segs.size(); ++k) S->total[segs[k].stream] += added[k];
    return RF_OK;
}

// Pads each stream's carried block (FIPS 180-4: 0x80, zeros, the bit length
// big-endian) and hashes it on the same legs; out32 = the final state,
// big-endian; the streams restart empty.
static int streams_final(rf_sha_streams* S, const uint64_t* ids, uint64_t n, uint8_t* out32) {
    std::vector<uint8_t> pad(128 * n, 0);
    std::vector<Piece> pieces(n);
    std::vector<Seg> segs(n);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t s = ids[i];
        const uint32_t c = S->clen[s];
        uint8_t* b = &pad[128 * i];
        memcpy(b, &S->carry[64 * s], c);
        b[c] = 0x80;
        const uint64_t nb = c + 9 <= 64 ? 1 : 2, bits = S->total[s] * 8;
        for (int k = 0; k < 8; ++k) b[64 * nb - 1 - k] = (uint8_t)(bits >> (8 * k));
        S->clen[s] = 0;
        pieces[i] = Piece{b, 64 * nb};
        segs[i] = Seg{s, 64 * nb, nb, (uint32_t)i, (uint32_t)i + 1, false};
    }
    if (int rc = streams_feed(S, segs, pieces)) return rc;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t s = ids[i];
        for (int k = 0; k < 8; ++k) {
            const uint32_t v = S->mid[8 * s + k];
            out32[32 * i + 4 * k] = (uint8_t)(v >> 24);
            out32[32 * i + 4 * k + 1] = (uint8_t)(v >> 16);
            out32[32 * i + 4 * k + 2] = (uint8_t)(v >> 8);
            out32[32 * i + 4 * k + 3] = (uint8_t)v;
        }
        memcpy(&S->mid[8 * s], kIV, sizeof kIV);
        S->total[s] = 0;
    }
    return RF_OK;
}

static int check_distinct(const rf_sha_streams* S, const uint64_t* ids, uint64_t n) {
    std::vector<uint64_t> v(ids, ids + n);
    std::sort(v.begin(), v.end());
    for (uint64_t i = 0; i < n; ++i) {
        if (v[i] >= S->n) return fail(RF_EINVAL, "stream id %llu out of range", (unsigned long long)v[i]);
        if (i && v[i] == v[i - 1]) return fail(RF_EINVAL, "stream id %llu twice in one digest batch",
                                                (unsigned long long)v[i]);
    }
    return RF_OK;
}

extern "C" int rf_sha_streams_digest(rf_sha_streams* S, const uint64_t* ids, uint64_t n, uint8_t* out32) {
    ARG(S && (n == 0 || (ids && out32)), "null argument");
    if (!n) return RF_OK;
    if (int rc = check_distinct(S, ids, n)) return rc;
    std::lock_guard<std::mutex> lk(S->ctx->mu);
    if (S->failed) return fail(RF_EDEVICE, "stream set failed in an earlier call");
    DevGuard dg(S->ctx->device);
    if (int rc = streams_final(S, ids, n, out32)) {
        S->failed = true;
        return rc;
    }
    return RF_OK;
}

extern "C" int rf_sha_streams_len(rf_sha_streams* S, uint64_t id, uint64_t* len) {
    ARG(S && len, "null argument");
    ARG(id < S->n, "stream id out of range");
    std::lock_guard<std::mutex> lk(S->ctx->mu);
    *len = S->total[id];
    return RF_OK;
}

extern "C" int rf_sha_streams_verify(rf_sha_streams* S, const uint64_t* ids, const uint8_t* want32, uint64_t n,
                                     int32_t* status) {
    ARG(S && (n == 0 || (ids && want32 && status)), "null argument");
    if (!n) return RF_OK;
    std::vector<uint8_t> got(32 * n);
    if (int rc = rf_sha_streams_digest(S, ids, n, got.data())) return rc;
    bool bad = false;
    for (uint64_t i = 0; i < n; ++i) {
        status[i] = memcmp(&got[32 * i], want32 + 32 * i, 32) ? RF_EINTEGRITY : RF_OK;
        bad |= status[i] != RF_OK;
    }
    return bad ? fail(RF_EINTEGRITY, "digest mismatch (errors.Integrity)") : RF_OK;
}

extern "C" int rf_sha256_verify(rf_ctx* ctx, const uint8_t* const* msgs, const uint64_t* lens, uint64_t n,
                                const uint8_t* want32, int32_t* status) {
    ARG(ctx && (n == 0 || (msgs && lens && want32 && status)), "null argument");
    if (!n) return RF_OK;
    std::vector<uint8_t> got(32 * n);
    if (int rc = rf_sha256_batch(ctx, msgs, lens, n, got.data())) return rc;
    bool bad = false;
    for (uint64_t i = 0; i < n; ++i) {
        status[i] = memcmp(&got[32 * i], want32 + 32 * i, 32) ? RF_EINTEGRITY : RF_OK;
        bad |= status[i] != RF_OK;
    }
    return bad ? fail(RF_EINTEGRITY, "digest mismatch (errors.Integrity)") : RF_OK;
}
