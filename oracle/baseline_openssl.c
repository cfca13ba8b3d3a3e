/* baseline_openssl.c -- CPU BASELINE ONLY (test / bench infrastructure, never
 * linked into the product; see oracle.c's header for the rules).
 *
 * SHA-256 of a batch of messages with OpenSSL's libcrypto (SHA-NI on CPUs
 * that have it: the speed class of Go >= 1.21 crypto/sha256) on native
 * pthreads taking messages from a shared queue in the caller's order
 * (largest first: LPT).  It replaces the bench's Python ThreadPoolExecutor
 * over hashlib, whose per-message dispatch and GIL hand-offs understated the
 * host's rate 5-8x on configs[0]'s 4,096 x 256 KiB messages.
 *
 * The reference's own loop is local/executor.go:514-557 (one goroutine per
 * file, DigestLimiter = 60 at :41), each file hashed by
 * reflow.Digester = digest.Digester(crypto.SHA256) (flow.go:36).
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>

typedef struct {
    const uint8_t *arena;
    const uint64_t *offs, *lens, *order;
    uint64_t n;
    uint8_t *out;
    uint64_t next; /* shared queue position (atomic) */
    int fail;
} ossl_batch;

static void *ossl_worker(void *p) {
    ossl_batch *b = (ossl_batch *)p;
    EVP_MD_CTX *c = EVP_MD_CTX_new();
    const EVP_MD *md = EVP_sha256();
    for (;;) {
        const uint64_t q = __atomic_fetch_add(&b->next, 1, __ATOMIC_RELAXED);
        if (q >= b->n) break;
        const uint64_t i = b->order ? b->order[q] : q;
        unsigned int len = 0;
        if (!c || EVP_DigestInit_ex(c, md, NULL) != 1 ||
            EVP_DigestUpdate(c, b->arena + b->offs[i], (size_t)b->lens[i]) != 1 ||
            EVP_DigestFinal_ex(c, b->out + 32 * i, &len) != 1 || len != 32)
            __atomic_store_n(&b->fail, 1, __ATOMIC_RELAXED);
    }
    EVP_MD_CTX_free(c);
    return NULL;
}

/* out[32 i] = SHA-256(arena[offs[i] .. +lens[i]]) for every i; messages are
 * taken in `order` (NULL: 0..n-1) by nthreads threads.  Returns 0, or -1 if
 * libcrypto failed on any message. */
int orc_openssl_sha256_batch(const uint8_t *arena, const uint64_t *offs, const uint64_t *lens,
                             const uint64_t *order, uint64_t n, uint8_t *out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    ossl_batch b = {arena, offs, lens, order, n, out, 0, 0};
    pthread_t th[256];
    int started = 0;
    for (int t = 1; t < nthreads; ++t)
        if (pthread_create(&th[started], NULL, ossl_worker, &b) == 0) ++started;
    ossl_worker(&b);
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    return b.fail ? -1 : 0;
}

/* The install loop's CPU baseline (local/executor.go:514-557: each file read
 * and hashed by its own goroutine, <= 60 at a time; repository/file/
 * repository.go:50-63 io.Copy into the digester): every file read in 1 MiB
 * pieces and hashed with libcrypto, on nthreads native threads taking files
 * from one queue.  Returns 0, or -1 if a file could not be read. */
#include <stdio.h>
#include <stdlib.h>

typedef struct {
    const char *const *paths;
    uint64_t n;
    uint8_t *out;
    uint64_t next;
    int fail;
} ossl_files;

static void *ossl_file_worker(void *p) {
    ossl_files *b = (ossl_files *)p;
    EVP_MD_CTX *c = EVP_MD_CTX_new();
    const EVP_MD *md = EVP_sha256();
    const size_t piece = 1u << 20;
    unsigned char *buf = (unsigned char *)malloc(piece);
    for (;;) {
        const uint64_t i = __atomic_fetch_add(&b->next, 1, __ATOMIC_RELAXED);
        if (i >= b->n) break;
        FILE *f = fopen(b->paths[i], "rb");
        unsigned int len = 0;
        int ok = f && c && buf && EVP_DigestInit_ex(c, md, NULL) == 1;
        while (ok) {
            const size_t got = fread(buf, 1, piece, f);
            if (got && EVP_DigestUpdate(c, buf, got) != 1) ok = 0;
            if (got < piece) {
                if (ferror(f)) ok = 0;
                break;
            }
        }
        if (ok && (EVP_DigestFinal_ex(c, b->out + 32 * i, &len) != 1 || len != 32)) ok = 0;
        if (f) fclose(f);
        if (!ok) __atomic_store_n(&b->fail, 1, __ATOMIC_RELAXED);
    }
    free(buf);
    EVP_MD_CTX_free(c);
    return NULL;
}

int orc_openssl_sha256_files(const char *const *paths, uint64_t n, uint8_t *out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    ossl_files b = {paths, n, out, 0, 0};
    pthread_t th[256];
    int started = 0;
    for (int t = 1; t < nthreads; ++t)
        if (pthread_create(&th[started], NULL, ossl_file_worker, &b) == 0) ++started;
    ossl_file_worker(&b);
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    return b.fail ? -1 : 0;
}
