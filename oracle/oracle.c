/*
 * oracle.c -- CPU restatement of Reflow's memoization hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (reflow_amd/, the
 * C-ABI library libreflow_hip.so) links, loads or calls this file.  It is
 * used only by tests/ (as the parity checker), by __graft_entry__.smoke()
 * (as the checker) and by bench.py's cpu_baseline leg (as the timed CPU
 * port).  It is never the thing measured on the GPU and never a fallback.
 *
 * Restated algorithms (reference = LDuderino/reflow @ v0, /root/reference):
 *   - SHA-256 (FIPS 180-4).  The reference uses Go crypto/sha256 through
 *     reflow.Digester = digest.Digester(crypto.SHA256)  (flow.go:36) and
 *     streams whole files into it (repository/file/repository.go:50-63).
 *   - digest.WriteDigest framing (grailbio/base/digest, not vendored):
 *     0x00 0x05 || 32 hash bytes  (pinned by the goldens).
 *   - MurmurHash3 x64_128, seed 0, streaming semantics of
 *     vendor/github.com/spaolacci/murmur3/murmur128.go:56-171, murmur.go:34-59.
 *   - Bloom filter probe/add of vendor/github.com/willf/bloom/bloom.go:
 *     baseHashes :94-104, location :107-115, Add :144-150, Test :182-190,
 *     with bitset.Test/Set of vendor/github.com/willf/bitset/bitset.go:143-156.
 *   - bloomlive.T.Contains keys = WriteDigest(d) (internal/bloomlive/bloomlive.go:30-36).
 *
 * Pinned by: reference golden digests (flow_test.go:33-34, executor_test.go:77,
 * syntax/digest_test.go:25, values/digest_test.go:28) through
 * oracle/reflow_oracle.py, FIPS-180 known answers, and the SMHasher
 * MurmurHash3_x64_128 verification value 0x6384BA69.  Bloom bit locations
 * have no reference known-answer test ("parity unpinned" beyond the
 * SMHasher pin of murmur3 and the restated arithmetic), see DESIGN.md.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

/* ------------------------------------------------------------------ */
/* SHA-256, portable scalar (FIPS 180-4 §6.2)                          */
/* ------------------------------------------------------------------ */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_compress(uint32_t st[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
        w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) |
               ((uint32_t)blk[4 * t + 2] << 8) | (uint32_t)blk[4 * t + 3];
    for (int t = 16; t < 64; ++t) {
        uint32_t s0 = ROR(w[t - 15], 7) ^ ROR(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ROR(w[t - 2], 17) ^ ROR(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int t = 0; t < 64; ++t) {
        uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[t] + w[t];
        uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void orc_sha256(const uint8_t *msg, uint64_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint64_t full = len / 64;
    for (uint64_t i = 0; i < full; ++i) sha256_compress(st, msg + 64 * i);
    uint8_t tail[128];
    uint64_t rem = len - 64 * full;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, msg + 64 * full, rem);
    tail[rem] = 0x80;
    uint64_t tl = (rem + 9 <= 64) ? 64 : 128;
    uint64_t bits = len * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_compress(st, tail);
    if (tl == 128) sha256_compress(st, tail + 64);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* Batched form used by the CPU baseline: message i = arena[offs[i] .. +lens[i]).
 * Work is split over nthreads pthreads in a round-robin over messages, the CPU
 * analogue of local/executor.go:522-538 (errgroup, DigestLimiter=60). */
typedef struct {
    const uint8_t *arena; const uint64_t *offs, *lens; uint64_t n; uint8_t *out;
    int tid, nth;
} sha_job;

static void *sha_worker(void *p) {
    sha_job *j = (sha_job *)p;
    for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nth)
        orc_sha256(j->arena + j->offs[i], j->lens[i], j->out + 32 * i);
    return NULL;
}

void orc_sha256_batch(const uint8_t *arena, const uint64_t *offs, const uint64_t *lens,
                      uint64_t n, uint8_t *out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256];
    sha_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (sha_job){arena, offs, lens, n, out, t, nthreads};
        pthread_create(&th[t], NULL, sha_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------ */
/* Synthetic content generator (shared spec with the device generator) */
/* word q of stream s = mix64(s + (q+1)*0x9E3779B97F4A7C15), LE bytes. */
/* This is splitmix64 in its counter form.              */
/* ------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

void orc_fill_stream(uint64_t seed, uint8_t *dst, uint64_t len) {
    uint64_t q = 0;
    for (; 8 * q + 8 <= len; ++q) {
        uint64_t v = mix64(seed + (q + 1) * 0x9E3779B97F4A7C15ULL);
        memcpy(dst + 8 * q, &v, 8);
    }
    if (8 * q < len) {
        uint64_t v = mix64(seed + (q + 1) * 0x9E3779B97F4A7C15ULL);
        memcpy(dst + 8 * q, &v, len - 8 * q);
    }
}

typedef struct {
    uint64_t seed; uint8_t *arena; const uint64_t *offs, *lens; uint64_t n; int tid, nth;
} fill_job;

static void *fill_worker(void *p) {
    fill_job *j = (fill_job *)p;
    for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nth)
        orc_fill_stream(j->seed ^ i, j->arena + j->offs[i], j->lens[i]);
    return NULL;
}

/* SHA-256 of stream `seed` of `len` bytes without materialising it: 1 MiB
 * chunks generated and compressed in turn (configs[1] files reach 2 GiB). */
void orc_stream_sha256(uint64_t seed, uint64_t len, uint8_t out[32]) {
    enum { CH = 1 << 20 };
    static __thread uint8_t *buf = NULL;
    if (!buf) buf = (uint8_t *)malloc(CH + 128);
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint64_t done = 0;
    for (;;) {
        const uint64_t n = len - done < CH ? len - done : CH;
        for (uint64_t q = 0; 8 * q < n; ++q) {
            uint64_t v = mix64(seed + (done / 8 + q + 1) * 0x9E3779B97F4A7C15ULL);
            memcpy(buf + 8 * q, &v, 8);
        }
        if (n == CH) {
            for (uint64_t b = 0; b < CH / 64; ++b) sha256_compress(st, buf + 64 * b);
            done += CH;  /* len a multiple of CH: the next pass pads an empty tail */
            continue;
        }
        /* last (partial) chunk: whole blocks, then the padded tail */
        const uint64_t full = n / 64, rem = n - 64 * full;
        for (uint64_t b = 0; b < full; ++b) sha256_compress(st, buf + 64 * b);
        uint8_t tail[128];
        memset(tail, 0, sizeof tail);
        if (rem) memcpy(tail, buf + 64 * full, rem);
        tail[rem] = 0x80;
        const uint64_t tl = (rem + 9 <= 64) ? 64 : 128, bits = len * 8;
        for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
        sha256_compress(st, tail);
        if (tl == 128) sha256_compress(st, tail + 64);
        break;
    }
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

typedef struct {
    uint64_t seed; const uint64_t *lens; uint64_t n; uint8_t *out; int tid, nth;
} stream_job;

static void *stream_worker(void *p) {
    stream_job *j = (stream_job *)p;
    for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nth)
        orc_stream_sha256(j->seed ^ i, j->lens[i], j->out + 32 * i);
    return NULL;
}

/* out[i] = SHA-256 of message i = stream (seed ^ i) of lens[i] bytes. */
void orc_stream_sha256_batch(uint64_t seed, const uint64_t *lens, uint64_t n, uint8_t *out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    stream_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (stream_job){seed, lens, n, out, t, nthreads};
        pthread_create(&th[t], NULL, stream_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* message i = stream (seed ^ i), the layout rf_gen_fill produces on device. */
void orc_fill_batch(uint64_t seed, uint8_t *arena, const uint64_t *offs, const uint64_t *lens,
                    uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    fill_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (fill_job){seed, arena, offs, lens, n, t, nthreads};
        pthread_create(&th[t], NULL, fill_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------ */
/* Digest-DAG evaluation (CPU port of Flow.Digest / PhysicalDigest):    */
/* jobs given as rf_graph_desc arrays, evaluated in the caller's        */
/* topological order: copy the material, write WD digests of the        */
/* referenced slots into the holes, SHA-256 into the output slot.       */
/* This is the recursive WriteDigest of flow.go:675-750 with the memo   */
/* of :653-658, one SHA-256 per job, single thread like Canonicalize.   */
/* ------------------------------------------------------------------ */
void orc_graph_eval(uint64_t n_jobs, const uint64_t *order, const uint32_t *out_slot,
                    const uint64_t *tmpl_off, const uint32_t *tmpl_len, const uint64_t *hole_ptr,
                    const uint32_t *hole_pos, const uint32_t *hole_slot, const uint8_t *blob,
                    uint8_t *slots32) {
    uint8_t *buf = NULL;
    size_t cap = 0;
    for (uint64_t q = 0; q < n_jobs; ++q) {
        const uint64_t j = order ? order[q] : q;
        const uint32_t len = tmpl_len[j];
        if (len > cap) {
            cap = len * 2 + 64;
            buf = (uint8_t *)realloc(buf, cap);
        }
        memcpy(buf, blob + tmpl_off[j], len);
        for (uint64_t h = hole_ptr[j]; h < hole_ptr[j + 1]; ++h)
            memcpy(buf + hole_pos[h], slots32 + 32ull * hole_slot[h], 32);
        orc_sha256(buf, len, slots32 + 32ull * out_slot[j]);
    }
    free(buf);
}

/* ------------------------------------------------------------------ */
/* Incremental recompute (the CPU port of rf_graph_set_slots +          */
/* rf_graph_recompute): after input slots change, their consumers are   */
/* re-hashed in topological order; a job whose digest did not change    */
/* does not dirty its own consumers (early cut-off).  The reference has */
/* no incremental form -- Flow.Digest is memoized per *Flow node and    */
/* every Eval recomputes every digest (flow.go:653-664, 814-843) -- so  */
/* this is the CPU statement of the same dirty-closure work the GPU     */
/* path does, used as the checker of its dirty counts and as the        */
/* single-thread CPU leg of configs[2].  The caller keeps the arrays.   */
/* ------------------------------------------------------------------ */
typedef struct {
    uint64_t n_jobs, n_slots;
    const uint32_t *out_slot, *tmpl_len, *hole_pos, *hole_slot;
    const uint64_t *tmpl_off, *hole_ptr;
    const uint8_t *blob;
    uint32_t *topo;      /* topological position of each job */
    uint64_t *cptr;      /* slot -> consumer jobs (CSR)      */
    uint32_t *cjob;
    uint8_t *queued;     /* job already in the heap          */
    uint32_t *heap;      /* min-heap of topo positions       */
    uint32_t *job_at;    /* topo position -> job             */
    uint8_t *buf;
    uint64_t cap;
    uint64_t last_blocks; /* SHA-256 blocks hashed by the last update */
} orc_graph;

orc_graph *orc_graph_new(uint64_t n_jobs, uint64_t n_slots, const uint32_t *out_slot, const uint64_t *tmpl_off,
                         const uint32_t *tmpl_len, const uint64_t *hole_ptr, const uint32_t *hole_pos,
                         const uint32_t *hole_slot, const uint8_t *blob) {
    orc_graph *g = (orc_graph *)calloc(1, sizeof *g);
    g->n_jobs = n_jobs; g->n_slots = n_slots; g->out_slot = out_slot; g->tmpl_off = tmpl_off;
    g->tmpl_len = tmpl_len; g->hole_ptr = hole_ptr; g->hole_pos = hole_pos; g->hole_slot = hole_slot;
    g->blob = blob;
    const uint64_t H = n_jobs ? hole_ptr[n_jobs] : 0;
    g->cptr = (uint64_t *)calloc(n_slots + 1, 8);
    g->cjob = (uint32_t *)malloc(4 * (H + 1));
    for (uint64_t h = 0; h < H; ++h) g->cptr[hole_slot[h] + 1]++;
    for (uint64_t s = 0; s < n_slots; ++s) g->cptr[s + 1] += g->cptr[s];
    uint64_t *fill = (uint64_t *)malloc(8 * (n_slots + 1));
    memcpy(fill, g->cptr, 8 * (n_slots + 1));
    for (uint64_t j = 0; j < n_jobs; ++j)
        for (uint64_t h = hole_ptr[j]; h < hole_ptr[j + 1]; ++h) g->cjob[fill[hole_slot[h]]++] = (uint32_t)j;
    /* Kahn over jobs: in-degree = holes whose slot some job writes */
    int64_t *producer = (int64_t *)malloc(8 * (n_slots + 1));
    for (uint64_t s = 0; s < n_slots; ++s) producer[s] = -1;
    for (uint64_t j = 0; j < n_jobs; ++j) producer[out_slot[j]] = (int64_t)j;
    uint32_t *indeg = (uint32_t *)calloc(n_jobs + 1, 4);
    for (uint64_t j = 0; j < n_jobs; ++j)
        for (uint64_t h = hole_ptr[j]; h < hole_ptr[j + 1]; ++h)
            if (producer[hole_slot[h]] >= 0) indeg[j]++;
    g->job_at = (uint32_t *)malloc(4 * (n_jobs + 1));
    g->topo = (uint32_t *)malloc(4 * (n_jobs + 1));
    uint64_t qh = 0, qt = 0;
    for (uint64_t j = 0; j < n_jobs; ++j)
        if (!indeg[j]) g->job_at[qt++] = (uint32_t)j;
    while (qh < qt) {
        const uint32_t j = g->job_at[qh++];
        const uint32_t s = out_slot[j];
        for (uint64_t c = g->cptr[s]; c < g->cptr[s + 1]; ++c)
            if (--indeg[g->cjob[c]] == 0) g->job_at[qt++] = g->cjob[c];
    }
    for (uint64_t i = 0; i < qt; ++i) g->topo[g->job_at[i]] = (uint32_t)i;
    free(fill); free(producer); free(indeg);
    g->queued = (uint8_t *)calloc(n_jobs + 1, 1);
    g->heap = (uint32_t *)malloc(4 * (n_jobs + 1));
    return g;
}

void orc_graph_free(orc_graph *g) {
    if (!g) return;
    free(g->cptr); free(g->cjob); free(g->job_at); free(g->topo); free(g->queued); free(g->heap); free(g->buf);
    free(g);
}

static void heap_push(uint32_t *h, uint64_t *n, uint32_t v) {
    uint64_t i = (*n)++;
    while (i && h[(i - 1) / 2] > v) { h[i] = h[(i - 1) / 2]; i = (i - 1) / 2; }
    h[i] = v;
}

static uint32_t heap_pop(uint32_t *h, uint64_t *n) {
    const uint32_t top = h[0], v = h[--(*n)];
    uint64_t i = 0;
    for (;;) {
        uint64_t c = 2 * i + 1;
        if (c >= *n) break;
        if (c + 1 < *n && h[c + 1] < h[c]) ++c;
        if (h[c] >= v) break;
        h[i] = h[c]; i = c;
    }
    h[i] = v;
    return top;
}

/* Write n changed input slots into slots32 and re-derive their dependents;
 * returns the number of jobs hashed. */
uint64_t orc_graph_update(orc_graph *g, uint8_t *slots32, const uint32_t *changed, const uint8_t *digests32,
                          uint64_t n) {
    uint64_t hn = 0, hashed = 0;
    g->last_blocks = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t s = changed[i];
        memcpy(slots32 + 32ull * s, digests32 + 32 * i, 32);
        for (uint64_t c = g->cptr[s]; c < g->cptr[s + 1]; ++c) {
            const uint32_t k = g->cjob[c];
            if (!g->queued[k]) { g->queued[k] = 1; heap_push(g->heap, &hn, g->topo[k]); }
        }
    }
    uint8_t d[32];
    while (hn) {
        const uint32_t j = g->job_at[heap_pop(g->heap, &hn)];
        g->queued[j] = 0;
        const uint32_t len = g->tmpl_len[j];
        if (len > g->cap) { g->cap = 2 * (uint64_t)len + 64; g->buf = (uint8_t *)realloc(g->buf, g->cap); }
        memcpy(g->buf, g->blob + g->tmpl_off[j], len);
        for (uint64_t h = g->hole_ptr[j]; h < g->hole_ptr[j + 1]; ++h)
            memcpy(g->buf + g->hole_pos[h], slots32 + 32ull * g->hole_slot[h], 32);
        orc_sha256(g->buf, len, d);
        ++hashed;
        g->last_blocks += ((uint64_t)len + 9 + 63) / 64;
        uint8_t *o = slots32 + 32ull * g->out_slot[j];
        if (!memcmp(o, d, 32)) continue;  /* early cut-off */
        memcpy(o, d, 32);
        const uint32_t s = g->out_slot[j];
        for (uint64_t c = g->cptr[s]; c < g->cptr[s + 1]; ++c) {
            const uint32_t k = g->cjob[c];
            if (!g->queued[k]) { g->queued[k] = 1; heap_push(g->heap, &hn, g->topo[k]); }
        }
    }
    return hashed;
}

uint64_t orc_graph_last_blocks(const orc_graph *g) { return g->last_blocks; }

/* Full recompute in topological order (every job once). */
void orc_graph_full(orc_graph *g, uint8_t *slots32) {
    for (uint64_t q = 0; q < g->n_jobs; ++q) {
        const uint32_t j = g->job_at[q];
        const uint32_t len = g->tmpl_len[j];
        if (len > g->cap) { g->cap = 2 * (uint64_t)len + 64; g->buf = (uint8_t *)realloc(g->buf, g->cap); }
        memcpy(g->buf, g->blob + g->tmpl_off[j], len);
        for (uint64_t h = g->hole_ptr[j]; h < g->hole_ptr[j + 1]; ++h)
            memcpy(g->buf + g->hole_pos[h], slots32 + 32ull * g->hole_slot[h], 32);
        orc_sha256(g->buf, len, slots32 + 32ull * g->out_slot[j]);
    }
}

/* ------------------------------------------------------------------ */
/* Job-local check of a whole slot table (the parity checker at sizes   */
/* the serial evaluators above cannot reach in seconds): every job's    */
/* output slot must equal SHA-256 of its material with the table's own  */
/* digests in its holes -- flow.go:675-750's WriteDigest of one node    */
/* from its deps' memoised digests (:653-658).  With every input slot   */
/* at its assigned value this is parity of the whole table with the     */
/* full evaluation, by induction over a topological order, whatever     */
/* path (incremental or full) produced it.  Jobs are split over         */
/* nthreads pthreads in chunks of 4096; returns the number of           */
/* mismatching jobs and *first = the lowest one (~0 if none).           */
/* ------------------------------------------------------------------ */
typedef struct {
    uint64_t n_jobs; const uint32_t *out_slot, *tmpl_len, *hole_pos, *hole_slot;
    const uint64_t *tmpl_off, *hole_ptr; const uint8_t *blob, *slots32;
    int tid, nth; uint64_t bad, first;
} check_job;

static void *check_worker(void *p) {
    check_job *c = (check_job *)p;
    enum { CHUNK = 4096 };
    uint8_t *buf = NULL, d[32];
    uint64_t cap = 0;
    c->bad = 0; c->first = ~0ull;
    for (uint64_t lo = (uint64_t)c->tid * CHUNK; lo < c->n_jobs; lo += (uint64_t)c->nth * CHUNK) {
        const uint64_t hi = lo + CHUNK < c->n_jobs ? lo + CHUNK : c->n_jobs;
        for (uint64_t j = lo; j < hi; ++j) {
            const uint32_t len = c->tmpl_len[j];
            if (len > cap) { cap = 2 * (uint64_t)len + 64; buf = (uint8_t *)realloc(buf, cap); }
            memcpy(buf, c->blob + c->tmpl_off[j], len);
            for (uint64_t h = c->hole_ptr[j]; h < c->hole_ptr[j + 1]; ++h)
                memcpy(buf + c->hole_pos[h], c->slots32 + 32ull * c->hole_slot[h], 32);
            orc_sha256(buf, len, d);
            if (memcmp(d, c->slots32 + 32ull * c->out_slot[j], 32)) {
                if (!c->bad || j < c->first) c->first = j;
                ++c->bad;
            }
        }
    }
    free(buf);
    return NULL;
}

uint64_t orc_graph_check(uint64_t n_jobs, const uint32_t *out_slot, const uint64_t *tmpl_off,
                         const uint32_t *tmpl_len, const uint64_t *hole_ptr, const uint32_t *hole_pos,
                         const uint32_t *hole_slot, const uint8_t *blob, const uint8_t *slots32, int nthreads,
                         uint64_t *first) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    check_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (check_job){n_jobs, out_slot, tmpl_len, hole_pos, hole_slot, tmpl_off, hole_ptr, blob, slots32,
                              t, nthreads, 0, ~0ull};
        pthread_create(&th[t], NULL, check_worker, &jobs[t]);
    }
    uint64_t bad = 0, f = ~0ull;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        bad += jobs[t].bad;
        if (jobs[t].bad && jobs[t].first < f) f = jobs[t].first;
    }
    if (first) *first = f;
    return bad;
}

/* ------------------------------------------------------------------ */
/* MurmurHash3 x64_128, seed 0 (murmur128.go:56-171)                   */
/* ------------------------------------------------------------------ */
static const uint64_t C1 = 0x87c37b91114253d5ULL, C2 = 0x4cf5ad432745937fULL;
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33; return k;
}
static inline uint64_t ld64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

void orc_mm3_128(const uint8_t *data, uint64_t len, uint32_t seed, uint64_t out[2]) {
    uint64_t h1 = seed, h2 = seed;
    uint64_t nb = len / 16;
    for (uint64_t i = 0; i < nb; ++i) {
        uint64_t k1 = ld64(data + 16 * i), k2 = ld64(data + 16 * i + 8);
        k1 *= C1; k1 = rotl64(k1, 31); k1 *= C2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= C2; k2 = rotl64(k2, 33); k2 *= C1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t *t = data + 16 * nb;
    uint64_t k1 = 0, k2 = 0;
    switch (len & 15) {
    case 15: k2 ^= (uint64_t)t[14] << 48; /* fallthrough */
    case 14: k2 ^= (uint64_t)t[13] << 40; /* fallthrough */
    case 13: k2 ^= (uint64_t)t[12] << 32; /* fallthrough */
    case 12: k2 ^= (uint64_t)t[11] << 24; /* fallthrough */
    case 11: k2 ^= (uint64_t)t[10] << 16; /* fallthrough */
    case 10: k2 ^= (uint64_t)t[9] << 8;   /* fallthrough */
    case 9:  k2 ^= (uint64_t)t[8];
             k2 *= C2; k2 = rotl64(k2, 33); k2 *= C1; h2 ^= k2; /* fallthrough */
    case 8:  k1 ^= (uint64_t)t[7] << 56;  /* fallthrough */
    case 7:  k1 ^= (uint64_t)t[6] << 48;  /* fallthrough */
    case 6:  k1 ^= (uint64_t)t[5] << 40;  /* fallthrough */
    case 5:  k1 ^= (uint64_t)t[4] << 32;  /* fallthrough */
    case 4:  k1 ^= (uint64_t)t[3] << 24;  /* fallthrough */
    case 3:  k1 ^= (uint64_t)t[2] << 16;  /* fallthrough */
    case 2:  k1 ^= (uint64_t)t[1] << 8;   /* fallthrough */
    case 1:  k1 ^= (uint64_t)t[0];
             k1 *= C1; k1 = rotl64(k1, 31); k1 *= C2; h1 ^= k1;
    }
    h1 ^= len; h2 ^= len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    out[0] = h1; out[1] = h2;
}

/* ------------------------------------------------------------------ */
/* Bloom filter (willf/bloom v2.0.3, willf/bitset v1.1.2)              */
/* ------------------------------------------------------------------ */
/* baseHashes (bloom.go:94-104): (h1,h2)=mm3(data), (h3,h4)=mm3(data||0x01).
 * The streaming hasher keeps its state after Sum128, so the second pair is
 * the one-shot hash of the 1-byte-extended message. */
void orc_bloom_base_hashes(const uint8_t *data, uint64_t len, uint64_t h[4]) {
    uint8_t buf[256];
    uint8_t *p = len + 1 <= sizeof buf ? buf : (uint8_t *)malloc(len + 1);
    memcpy(p, data, len);
    p[len] = 1;
    orc_mm3_128(p, len, 0, h);
    orc_mm3_128(p, len + 1, 0, h + 2);
    if (p != buf) free(p);
}

/* location (bloom.go:107-110), before the "% m" of :113-115. */
uint64_t orc_bloom_location(const uint64_t h[4], uint64_t i) {
    return h[i % 2] + i * h[2 + (((i + (i % 2)) % 4) / 2)];
}

/* Test (bloom.go:182-190) with bitset.Test (bitset.go:143-149):
 * bit loc in word loc>>6, mask 1<<(loc&63); loc >= length ⇒ false. */
int orc_bloom_test(const uint64_t *words, uint64_t length, uint64_t m, uint64_t k,
                   const uint8_t *data, uint64_t len) {
    uint64_t h[4];
    orc_bloom_base_hashes(data, len, h);
    for (uint64_t i = 0; i < k; ++i) {
        uint64_t loc = orc_bloom_location(h, i) % m;
        if (loc >= length) return 0;
        if (!((words[loc >> 6] >> (loc & 63)) & 1)) return 0;
    }
    return 1;
}

/* Add (bloom.go:144-150), bitset.Set (bitset.go:151-156).  The caller sizes
 * words for max(length, m) bits; *length grows like extendSetMaybe. */
void orc_bloom_add(uint64_t *words, uint64_t *length, uint64_t m, uint64_t k,
                   const uint8_t *data, uint64_t len) {
    uint64_t h[4];
    orc_bloom_base_hashes(data, len, h);
    for (uint64_t i = 0; i < k; ++i) {
        uint64_t loc = orc_bloom_location(h, i) % m;
        if (loc >= *length) *length = loc + 1;
        words[loc >> 6] |= 1ULL << (loc & 63);
    }
}

/* bloomlive.T.Contains over a batch of 32-byte digests
 * (internal/bloomlive/bloomlive.go:30-36): key = 00 05 || digest. */
typedef struct {
    const uint64_t *words; uint64_t length, m, k; const uint8_t *d32; uint64_t n;
    uint8_t *out; int tid, nth;
} probe_job;

static void *probe_worker(void *p) {
    probe_job *j = (probe_job *)p;
    uint8_t key[34];
    key[0] = 0; key[1] = 5;
    for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nth) {
        memcpy(key + 2, j->d32 + 32 * i, 32);
        j->out[i] = (uint8_t)orc_bloom_test(j->words, j->length, j->m, j->k, key, 34);
    }
    return NULL;
}

void orc_bloomlive_contains_batch(const uint64_t *words, uint64_t length, uint64_t m, uint64_t k,
                                  const uint8_t *d32, uint64_t n, uint8_t *out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    probe_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (probe_job){words, length, m, k, d32, n, out, t, nthreads};
        pthread_create(&th[t], NULL, probe_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

void orc_bloomlive_add_batch(uint64_t *words, uint64_t *length, uint64_t m, uint64_t k,
                             const uint8_t *d32, uint64_t n) {
    uint8_t key[34];
    key[0] = 0; key[1] = 5;
    for (uint64_t i = 0; i < n; ++i) {
        memcpy(key + 2, d32 + 32 * i, 32);
        orc_bloom_add(words, length, m, k, key, 34);
    }
}
