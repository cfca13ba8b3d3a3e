/*
 * reflow_hip.h -- C-ABI of the MI355X memoization engine (libreflow_hip.so).
 *
 * Drop-in boundary for Reflow's data-parallel memoization hot path
 * (reference: LDuderino/reflow @ v0, paths relative to /root/reference).
 * Every entry point is batched: the reference's per-call Go interfaces
 * (one io.Writer per file, one goroutine per cache lookup) are coalesced by
 * the host shim into device batches (INTEGRATION.md shows the cgo binding).
 *
 * Conventions
 *   - Plain pointers and sizes; no C++ or torch types cross this boundary.
 *   - Every function returns an rf_status (0 = RF_OK).  On failure
 *     rf_last_error() returns a thread-local message.  No exception crosses.
 *   - Host buffers are caller-owned and not retained after return (cgo rule).
 *     Device buffers passed to *_device functions are caller-owned HBM.
 *   - "stream" arguments are hipStream_t values passed as void* (NULL = the
 *     context's own stream).  *_device functions are asynchronous on it.
 *   - A digest is 32 raw SHA-256 bytes.  WD(d) = 0x00 0x05 || d (34 bytes) is
 *     the grailbio/base/digest.WriteDigest framing the reference hashes.
 *
 * The product path is the HIP path: if the gfx950 code object cannot be
 * loaded or no device is present, rf_init fails with RF_EDEVICE -- there is
 * no CPU fallback behind this ABI.  The one place host cores hash is the K1
 * planner's host leg (rf_set_host_threads): a scheduled part of a batch, not
 * a fallback -- the longest SHA-256 chains of a skewed batch, which a host
 * core with SHA-NI runs ~40x faster than one GPU wave, go to a pool of host
 * threads (the reference's <=60-goroutine digest pool, local/executor.go:41)
 * while the GPU kernels hash the rest.  It needs a device like every other
 * call, and rf_set_host_threads(ctx, 0) pins every message to the GPU.
 */
#ifndef REFLOW_HIP_H
#define REFLOW_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes; the shim maps them onto errors.Kind (errors/errors.go:39-76). */
typedef enum {
    RF_OK = 0,
    RF_EINVAL = 1,     /* errors.Invalid: malformed input, bad graph, cycle */
    RF_EIO = 2,        /* errors.Unavailable: reading an input file failed   */
    RF_EINTEGRITY = 3, /* errors.Integrity: digest mismatch on verify        */
    RF_EDEVICE = 4,    /* errors.Unavailable: HIP runtime / device failure   */
    RF_ENOMEM = 5,     /* errors.ResourcesExhausted: HBM or host allocation  */
    RF_ENOTFOUND = 6,  /* errors.NotExist                                     */
    RF_EPRECONDITION = 7 /* errors.Precondition: assoc compare-and-set failed */
} rf_status;

typedef struct rf_ctx rf_ctx;
typedef struct rf_sha_plan rf_sha_plan;
typedef struct rf_graph rf_graph;
typedef struct rf_bloom rf_bloom;
typedef struct rf_assoc rf_assoc;
typedef struct rf_install rf_install;

/* ---- context ----------------------------------------------------------- */
/* Bind a context to HIP device `device` (one process per GPU).  Replaces the
 * process-global reflow.Digester (flow.go:36) as the owner of device state. */
int rf_init(int device, rf_ctx **out);
void rf_destroy(rf_ctx *ctx);
const char *rf_last_error(void);
int rf_device_count(int *n);
/* Blocks until all work queued on the context's stream finished. */
int rf_sync(rf_ctx *ctx);
/* Version string, e.g. "reflow-hip 0.1 gfx950". */
const char *rf_version(void);

/* K1 host leg width: n >= 1 threads, 0 = none (every message on the GPU
 * kernels), -1 = default min(60, CPU share): 60 is the reference's
 * DigestLimiter (local/executor.go:41), the share the smaller of the affinity
 * mask and the cgroup cpu.max quota, divided by LOCAL_WORLD_SIZE (ranks per
 * node); RF_HOST_THREADS overrides the default.  Without the x86 SHA
 * extensions the host leg is off whatever n is. */
int rf_set_host_threads(rf_ctx *ctx, int n);
/* Host leg threads in effect, one core's measured SHA-NI rate (bytes/s; 0 if
 * unavailable) and whether the CPU has the SHA extensions. */
int rf_host_info(rf_ctx *ctx, int *threads, double *core_bytes_per_s, int *sha_ext);
/* The host leg's chains per thread (RF_HOST_WAYS, default 2: SHA-NI rounds
 * are latency-bound, two interleaved messages fill the issue slots) and one
 * thread's measured rate at that interleave (bytes/s) -- the per-thread peak
 * bench.py prices the host leg against. */
int rf_host_rate(rf_ctx *ctx, int *ways, double *thread_bytes_per_s);
/* The feed rate (bytes/s) the K1 planner prices the host leg's HBM-resident
 * bytes at: measured by the last plan run on this context whose host leg took
 * >= 1 GiB at the current width (*measured = 1; the leg's bytes over its wall
 * time, D2H copies and SHA-NI threads together), else the built-in PCIe Gen5
 * estimate (52 GB/s, *measured = 0).  Plans created after a measurement use
 * it: a caller calibrates with one RF_SHA_ALL_HOST run, then plans the split. */
int rf_host_link(rf_ctx *ctx, double *bytes_per_s, int *measured);

/* ---- device memory and timing -------------------------------------------
 * The engine owns its HIP runtime; callers (the cgo shim, bench.py, tests)
 * allocate HBM through these so no second runtime enters the process. */
int rf_malloc(rf_ctx *ctx, uint64_t bytes, void **out);
int rf_free(rf_ctx *ctx, void *p);
int rf_memcpy_h2d(rf_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int rf_memcpy_d2h(rf_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int rf_memset_d(rf_ctx *ctx, void *dst, int value, uint64_t bytes);
int rf_memcpy_d2d(rf_ctx *ctx, void *dst, const void *src, uint64_t bytes);
/* The context's hipStream_t. */
void *rf_stream(rf_ctx *ctx);
/* HIP-event timer on the context stream: start, then stop returns ms. */
int rf_timer_start(rf_ctx *ctx);
int rf_timer_stop(rf_ctx *ctx, float *ms);

/* ---- RCCL over xGMI (multi-GPU: one process per GPU) ----------------------
 * Bootstrap: rank 0 calls rf_comm_unique_id and ships the 128 bytes to the
 * other ranks out of band (bench.py uses torch.distributed/gloo on the CPU). */
typedef struct rf_comm rf_comm;
int rf_comm_unique_id(uint8_t id[128]);
int rf_comm_init(rf_ctx *ctx, int nranks, int rank, const uint8_t id[128], rf_comm **out);
void rf_comm_destroy(rf_comm *comm);
/* d_recv[r*bytes .. +bytes) = rank r's d_send (ncclAllGather). */
int rf_comm_allgather(rf_comm *comm, const void *d_send, void *d_recv, uint64_t bytes, void *stream);
/* In-place bitwise OR of nwords uint64 across ranks.  RCCL has no OR
 * reduction: all-gather of the packed words + a local OR kernel. */
int rf_comm_allreduce_or(rf_comm *comm, void *d_words, uint64_t nwords, void *stream);

/* ---- K1: batched SHA-256 (Digester.NewWriter/FromBytes, Repository.Put) --
 * Replaces the per-file io.Copy into Digester.NewWriter() at
 * repository/file/repository.go:50-63 (Install) and :237-264 (Put), driven by
 * the ≤60-goroutine loop of local/executor.go:514-557.  out32[i] = SHA256(msg i). */
int rf_sha256_batch(rf_ctx *ctx, const uint8_t *const *msgs, const uint64_t *lens, uint64_t n,
                    uint8_t *out32);

/* Same, messages given as one host arena + offsets. */
int rf_sha256_arena(rf_ctx *ctx, const uint8_t *arena, const uint64_t *offs, const uint64_t *lens,
                    uint64_t n, uint8_t *out32);

/* Device-resident form.  A plan is built once from host-side offsets and
 * lengths: it orders messages largest-first and splits them by a makespan
 * model over the legs -- the host leg (the largest messages, SHA-NI threads,
 * bytes streamed D2H in 8 MiB chunks), wave-per-message duo chains, and the
 * lane-per-message kernels; rf_sha_plan_run then digests messages already in
 * HBM.  The GPU legs are queued asynchronously on `stream`; with a host leg
 * the call is SYNCHRONOUS: it returns once the host threads are done (their
 * digests' upload and scatter into out queued on `stream`) -- ~1.3 s on
 * configs[1].  The context's mutex is released while the host threads hash,
 * so other calls on the context proceed meanwhile (calls that need the host
 * leg themselves wait for it); one run of a given plan at a time.
 * Requirements: offs[i] % 16 == 0.  out is n*32 bytes of device memory. */
int rf_sha_plan_create(rf_ctx *ctx, const uint64_t *offs, const uint64_t *lens, uint64_t n,
                       uint32_t flags, rf_sha_plan **out);
int rf_sha_plan_run(rf_sha_plan *plan, const void *d_arena, void *d_out32, void *stream);
typedef struct {
    uint64_t n_msgs, n_solo;     /* messages; messages run wave-per-message */
    uint64_t total_blocks;       /* Σ ceil((len+9)/64): algorithmic unit of K1 */
    uint64_t max_blocks;         /* critical path of the largest message       */
    uint64_t total_bytes;
    float last_ms_lanes, last_ms_solo, last_ms_total; /* HIP-event times of the last run */
    float last_ms_host;          /* wall time of the last run's host leg         */
    uint32_t host_threads;       /* host leg threads (0: no host leg)            */
    uint64_t n_host, host_bytes; /* messages / bytes on the host leg             */
} rf_sha_stats;
int rf_sha_plan_stats(rf_sha_plan *plan, rf_sha_stats *out);
void rf_sha_plan_destroy(rf_sha_plan *plan);
/* flags for rf_sha_plan_create */
#define RF_SHA_NO_SOLO 1u      /* every message lane-per-message */
#define RF_SHA_ALL_SOLO 2u     /* every message wave-per-message */
#define RF_SHA_ONE_LANE_CHAIN 4u /* wave-per-message kernel keeps the round chain on one lane */
#define RF_SHA_NO_PAIR 8u      /* small sets: lanes kernel instead of the producer/chain pair */
#define RF_SHA_NO_OCTO 16u     /* small sets: no eight-per-wave two-lane chains (pair or lanes) */
#define RF_SHA_ALL_HOST 32u    /* every message on the host leg (needs SHA-NI and host threads) */
#define RF_SHA_NO_HOST 64u     /* no host leg: every message on the GPU kernels */

/* ---- Streaming SHA-256 (Digester.NewWriter: an io.Writer whose state carries
 * across Write calls) for many streams at once -------------------------------
 * Repository.Put hashes an io.Reader as it copies it (repository/file/
 * repository.go:237-264; s3's Put through a TeeReader, repository/s3/s3.go:
 * 120-147): the shim feeds each upload's chunks here as they arrive, so no
 * upload is buffered whole.  Per stream the carried partial block plus its
 * chunks give whole blocks, hashed from the stream's midstate -- the largest
 * on the host leg (in place), the rest by k1_sha256_resume on the GPU, by a
 * makespan model like a K1 plan.  flags: 0, RF_SHA_ALL_HOST or
 * RF_SHA_NO_HOST (every segment on k1_sha256_resume). */
typedef struct rf_sha_streams rf_sha_streams;
int rf_sha_streams_open(rf_ctx *ctx, uint64_t n_streams, uint32_t flags, rf_sha_streams **out);
void rf_sha_streams_close(rf_sha_streams *s);
/* Write chunk i to stream ids[i]; chunks of one stream apply in batch order. */
int rf_sha_streams_write(rf_sha_streams *s, const uint64_t *ids, const uint8_t *const *chunks,
                         const uint64_t *lens, uint64_t n);
/* out32[i] = Digest() of stream ids[i] (distinct ids); the stream restarts empty. */
int rf_sha_streams_digest(rf_sha_streams *s, const uint64_t *ids, uint64_t n, uint8_t *out32);
/* Bytes written to stream id since its last digest (Put's returned size). */
int rf_sha_streams_len(rf_sha_streams *s, uint64_t id, uint64_t *len);
/* Integrity check (ReadFrom / WriteTo re-digest, repository/file/repository.go:
 * 126-166, 212): status[i] = RF_OK or RF_EINTEGRITY (digest of stream ids[i] vs
 * want32[i]); returns RF_EINTEGRITY if any differs (errors.Integrity).  The
 * streams restart empty. */
int rf_sha_streams_verify(rf_sha_streams *s, const uint64_t *ids, const uint8_t *want32, uint64_t n,
                          int32_t *status);
/* The same for whole messages: status[i] for SHA256(msg i) vs want32[i]. */
int rf_sha256_verify(rf_ctx *ctx, const uint8_t *const *msgs, const uint64_t *lens, uint64_t n,
                     const uint8_t *want32, int32_t *status);

/* Synthetic data generator (bench / tests): fills d_arena so that message i
 * is the splitmix64 counter stream with seed (seed ^ i). */
int rf_gen_fill(rf_ctx *ctx, void *d_arena, const uint64_t *d_offs, const uint64_t *d_lens,
                uint64_t n, uint64_t seed, uint64_t arena_bytes, void *stream);

/* ---- Fileset digest (Fileset.Digest/WriteDigest, executor.go:205-233) ----
 * n_sets filesets; set s owns groups [set_group[s], set_group[s+1]); group g
 * owns entries [group_entry[g], group_entry[g+1]).  A Map fileset is one
 * group; a List fileset contributes its (flattened, depth-first) Map leaves as
 * consecutive groups ("List wins if non-nil", executor.go:216-219).  Entries
 * within a group are sorted bytewise here (sort.Strings).  Material per group
 * = Σ path ‖ WD(id).  out32[s] = SHA256(material of set s). */
int rf_fileset_digest_batch(rf_ctx *ctx, uint64_t n_sets, const uint64_t *set_group,
                            const uint64_t *group_entry, const char *const *paths,
                            const uint32_t *path_lens, const uint8_t *ids32, uint8_t *out32);
/* As rf_fileset_digest_batch with the File IDs resident in HBM (d_ids32[e],
 * e.g. the out32 of an rf_sha_plan_run over the installed files): no ID
 * readback; the IDs are placed into the material on the device and only the
 * set digests return (Executor.install -> Fileset.Digest,
 * local/executor.go:514-557 + executor.go:205-233). */
int rf_fileset_digest_device(rf_ctx *ctx, uint64_t n_sets, const uint64_t *set_group,
                             const uint64_t *group_entry, const char *const *paths,
                             const uint32_t *path_lens, const void *d_ids32, uint8_t *out32);

/* ---- Executor.install: walk + read + digest a tree into a Fileset ----------
 * Replaces local/executor.go:514-557 (install: walker loop, <=60 concurrent
 * repo.Install calls, Fileset{Map} assembly) over internal/walker/walker.go:33-99
 * and repository/file/repository.go:50-63 (ID = SHA256(contents)).  Walk
 * semantics are the walker's: os.Stat follows symlinks, a path that does not
 * exist (ENOENT, e.g. a dangling link) is skipped, directory entries are
 * visited in bytewise-sorted, depth-first pre-order; every non-directory
 * entry is read and digested (one K1 batch per <= 8 GiB chunk).  Entry i has
 * relpath = filepath.Rel(root, path) ("." when root is a file), ID and Size =
 * the Stat size (executor.go:525).  A missing root gives n = 0 and the digest
 * of the empty Fileset.  Errors: RF_EIO for stat/readdir/open/read failures
 * (the walker's w.Err(), Install's error) and for a file whose size changed
 * between the walk and the read.  The optional symlink replacement of
 * executor.go:544-552 stays with the caller (it only uses the IDs returned).
 * rf_install_info: entry count, total relpath bytes, and
 * Fileset{Map: relpath -> File}.Digest() (executor.go:205-233).
 * rf_install_entries: caller-allocated paths (path_bytes), path_offs (n+1),
 * ids32 (32n), sizes (n), in walk order; any of them may be NULL. */
int rf_install_dir(rf_ctx *ctx, const char *root, rf_install **out);
int rf_install_info(const rf_install *in, uint64_t *n_entries, uint64_t *path_bytes,
                    uint8_t fileset_digest32[32]);
int rf_install_entries(const rf_install *in, char *paths, uint64_t *path_offs, uint8_t *ids32,
                       int64_t *sizes);
void rf_install_destroy(rf_install *in);
/* The walk alone, host-only (no device): internal/walker's Scan as install
 * uses it -- relpaths ("." for a file root) and Stat sizes of every
 * non-directory entry, bytewise-sorted depth-first pre-order, links
 * followed, vanished entries skipped.  rf_walk_entries: paths concatenated,
 * path_offs[n_entries + 1]. */
typedef struct rf_walk rf_walk;
int rf_walk_dir(const char *root, rf_walk **out);
int rf_walk_info(const rf_walk *w, uint64_t *n_entries, uint64_t *path_bytes);
int rf_walk_entries(const rf_walk *w, char *paths, uint64_t *path_offs, int64_t *sizes);
void rf_walk_free(rf_walk *w);

/* ---- Fileset values as JSON (the assoc value, eval.go:1141 -> marshal
 * eval.go:1961-1967 = json.Marshal + Repository.Put, repository.go:108-114) --
 * A fileset TREE: node i's List = nodes list_child[list_ptr[i] .. list_ptr[i+1])
 * (an empty range = nil or empty List: both omitted, `json:",omitempty"`);
 * node i's Map = entries [entry_ptr[i], entry_ptr[i+1]) with path bytes,
 * 32-B File ID and Size (executor.go:25-38).  JSON bytes follow Go 1.9/1.10
 * encoding/json: {"List":[...],"Fileset":{"<path>":{"ID":"sha256:<hex>","Size":N}}},
 * keys sorted bytewise, HTML-safe escaping, invalid UTF-8 -> �.  The ID's
 * text form is grailbio/base digest's String() (unvendored: parity unpinned). */
typedef struct {
    uint64_t n_nodes;
    const uint64_t *list_ptr;    /* [n_nodes+1] */
    const uint32_t *list_child;  /* [list_ptr[n_nodes]] */
    const uint64_t *entry_ptr;   /* [n_nodes+1] */
    const char *const *paths;    /* [entries] */
    const uint32_t *path_lens;   /* [entries] */
    const uint8_t *ids32;        /* [entries][32] */
    const int64_t *sizes;        /* [entries] */
} rf_fileset_tree;
/* json.Marshal of node `root` into out[cap]; *out_len = bytes needed (RF_EINVAL
 * if cap is short).  Host-only (no device needed). */
int rf_fileset_marshal_json(const rf_fileset_tree *t, uint32_t root, uint8_t *out, uint64_t cap,
                            uint64_t *out_len);
/* out32[i] = SHA256(json.Marshal(roots[i])): the value digests CacheWrite
 * stores (eval.go:1141-1151); the hashes run on K1. */
int rf_fileset_value_digest_batch(rf_ctx *ctx, const rf_fileset_tree *t, const uint32_t *roots,
                                  uint64_t n, uint8_t *out32);

/* ---- Coalescing concurrent callers (SURVEY §8(b) "Threading") -----------
 * The reference digests files in <=60 goroutines (local/executor.go:41,
 * 522-538) and looks cache keys up in a goroutine per node (eval.go:402-411);
 * called one request at a time, each would be its own tiny device batch.  A
 * coalescer is a queue any number of threads call into: the first caller
 * that finds no flush running becomes the flusher, waits up to max_wait_us
 * (or until max_batch requests are queued), and runs ONE batched call --
 * rf_sha256_batch, rf_bloom_probe or rf_assoc_get -- for everything queued;
 * requests arriving meanwhile form the next batch.  Blocking calls (a cgo
 * call per goroutine) and async tickets (submit, then poll or wait) share
 * it.  A failed batch returns its status to every request in it. */
enum { RF_COALESCE_SHA256 = 1, RF_COALESCE_PROBE = 2, RF_COALESCE_ASSOC_GET = 3 };
typedef struct rf_coalescer rf_coalescer;
typedef struct rf_coalesce_ticket rf_coalesce_ticket;
/* target: the rf_bloom (PROBE) or rf_assoc (ASSOC_GET, with assoc_kind);
 * NULL for SHA256. */
int rf_coalescer_open(rf_ctx *ctx, int kind, void *target, int assoc_kind, uint64_t max_batch,
                      uint64_t max_wait_us, rf_coalescer **out);
void rf_coalescer_close(rf_coalescer *c); /* completes what is queued */
int rf_coalesce_sha256(rf_coalescer *c, const uint8_t *msg, uint64_t len, uint8_t *out32);
int rf_coalesce_probe(rf_coalescer *c, const uint8_t *digest32, uint8_t *contains);
int rf_coalesce_assoc_get(rf_coalescer *c, const uint8_t *key32, uint8_t *val32, uint8_t *found);
/* Async: msg and out32 must stay valid until the ticket is done. */
int rf_coalesce_sha256_async(rf_coalescer *c, const uint8_t *msg, uint64_t len, uint8_t *out32,
                             rf_coalesce_ticket **out);
/* *done = 1 once out32 is written (returns its status); a poll that finds the
 * queue idle flushes it. */
int rf_coalesce_poll(rf_coalescer *c, rf_coalesce_ticket *t, int *done);
int rf_coalesce_wait(rf_coalescer *c, rf_coalesce_ticket *t);
void rf_coalesce_ticket_free(rf_coalescer *c, rf_coalesce_ticket *t); /* completes it first */
/* Batches flushed, requests served, largest batch. */
int rf_coalescer_stats(rf_coalescer *c, uint64_t *batches, uint64_t *requests, uint64_t *largest);

/* ---- K2/K3: incremental digest DAG (Flow.Digest / CacheKeys) ------------
 * The host lowers a Flow graph (flow.go:653-802) into hash JOBS over digest
 * SLOTS.  Job j hashes a byte template (its digest material, flow.go:675-750
 * or the physical material of :764-792) into slot out_slot[j]; the template
 * has "holes": hole h of job j places the 32 digest bytes of slot
 * hole_slot[h] at byte hole_pos[h] of the material (the host already wrote
 * the 0x00 0x05 WD prefix in front of each hole).  Slots written by no job
 * are inputs (e.g. File IDs).  Jobs must form a DAG over slots. */
typedef struct {
    uint32_t n_jobs, n_slots;
    const uint32_t *out_slot;    /* [n_jobs]                                    */
    const uint64_t *tmpl_off;    /* [n_jobs] byte offset of job j's template in blob */
    const uint32_t *tmpl_len;    /* [n_jobs] material length (bytes)            */
    const uint64_t *hole_ptr;    /* [n_jobs+1] CSR into hole_pos/hole_slot      */
    const uint32_t *hole_pos;    /* byte position of the 32 digest bytes         */
    const uint32_t *hole_slot;   /* slot whose digest fills the hole            */
    const uint8_t *blob;         /* templates                                   */
    uint64_t blob_len;
} rf_graph_desc;

/* Device footprint of a loaded graph: ~104 B a job (records, queued flags,
 * lists, midstates), 84 B a slot (digest, reverse-edge pointer, the mark
 * kernels' 48-B per-slot plan), 16 B a hole, and the templates padded to
 * 64-B blocks. */
int rf_graph_load(rf_ctx *ctx, const rf_graph_desc *desc, rf_graph **out);
void rf_graph_destroy(rf_graph *g);
/* Set input-slot digests (e.g. changed File IDs); marks their transitive
 * dependents dirty.  Setting a job's output slot is RF_EINVAL.  On a graph
 * never recomputed (fresh from rf_graph_load) the digests are only written:
 * its first recompute is a full one. */
int rf_graph_set_slots(rf_graph *g, const uint32_t *slots, const uint8_t *digests32, uint32_t n);
/* Device-resident form of set_slots (indices and digests in HBM). */
int rf_graph_set_slots_device(rf_graph *g, const void *d_slots, const void *d_digests32, uint32_t n,
                              void *stream);
/* Recompute dirty jobs level by level (K3 frontier + K2 node digests).
 * full != 0 recomputes every job.  Early cut-off: a job whose digest did not
 * change does not dirty its consumers.  *out_recomputed (may be NULL) receives
 * the number of jobs hashed (synchronises).
 * Each incremental level runs in one of two kernel forms, chosen per level
 * and step from the input slots marked since the last step (set_slots /
 * update): the two-lane latency form, or -- when min(level jobs, marked
 * slots) reaches 24,576 (65,536 for levels of long jobs) -- the lane-per-job
 * throughput form; change sets of >= 98,304 slots also mark in the
 * throughput form.  Results are identical.  The thresholds are fixed per
 * graph: the defaults below, RF_K2_THRU / RF_K2_THRU_WIDE (read once when the
 * graph is loaded or restored; RF_K2_THRU also sets the mark threshold), or
 * rf_graph_set_forms. */
int rf_graph_recompute(rf_graph *g, int full, uint64_t *out_recomputed);
#define RF_K2_THRU_DEFAULT 24576ull      /* levels of short jobs */
#define RF_K2_THRU_WIDE_DEFAULT 65536ull /* levels of long jobs (the per-sample OpK) */
#define RF_K2_THRU_MARK_DEFAULT 98304ull /* the mark kernel's lean form */
/* Kernel-form thresholds for this graph's next incremental steps (tuning and
 * A/B; results never depend on them): 0 = always the throughput form,
 * UINT64_MAX = never.  Not thread-safe against a step in flight on the
 * graph: call it between steps (the caller owns the graph, as for set_slots). */
int rf_graph_set_forms(rf_graph *g, uint64_t thru, uint64_t thru_wide, uint64_t thru_mark);
/* Canonicalize's hand-over when copies collapse (flow.go:814-843, the
 * flowMap's first copy wins, :881-907): g, just loaded from the copies'
 * job table with the duplicates' jobs dropped and every hole re-pointed at
 * its class's first copy (same slot numbering), takes src's whole slot table
 * -- src is the copies' graph, fully recomputed -- device to device, and is
 * ready for incremental steps without a full recompute (the state
 * rf_graph_restore leaves).  Both graphs of one context, equal n_slots, no
 * change set pending on either, src recomputed: RF_EINVAL /
 * RF_EPRECONDITION otherwise.  The caller vouches that src's digests are
 * what g's jobs compute (they are: every kept job is src's, reading slots of
 * equal digests). */
int rf_graph_adopt_slots(rf_graph *g, rf_graph *src);
/* Asynchronous form (no count readback). */
int rf_graph_recompute_async(rf_graph *g, int full, void *stream);
/* rf_graph_set_slots_device + rf_graph_recompute_async(g, 0, stream) in one
 * call.  By default that is the mark kernel and the step's plain level
 * launches (measured faster than a graph replay); with RF_K2_GRAPH=1 it is ONE
 * graph launch (the mark kernel the graph's first node, its parameters updated
 * per call on the host).  The first call on a fresh graph runs a full
 * recompute. */
int rf_graph_update_recompute_async(rf_graph *g, const void *d_slots, const void *d_digests32, uint32_t n,
                                    void *stream);
int rf_graph_get_slots(rf_graph *g, const uint32_t *slots, uint32_t n, uint8_t *out32);
/* Device-resident gather: d_out32[i] = slot d_slots[i] (e.g. boundary digests
 * for rf_comm_allgather).  Asynchronous on `stream`. */
int rf_graph_gather_device(rf_graph *g, const void *d_slots, uint32_t n, void *d_out32, void *stream);
typedef struct {
    uint32_t n_jobs, n_slots, n_levels, max_level_jobs;
    uint64_t total_blocks, hole_count, template_bytes;
    uint64_t last_recomputed;
    float last_ms; /* device time of the last synchronous rf_graph_recompute (asynchronous
                    * incremental steps record no events: RF_K2_EVENTS=1 does) */
    uint32_t last_levels_lf;  /* levels the last plain incremental step ran in the throughput form */
    uint32_t last_mark_lf;    /* the last set_slots batch marked in the throughput form (0/1) */
    uint32_t last_levels_oct; /* levels the last plain incremental step ran in the octo form */
    uint32_t split_block0;    /* fused links split block 0's schedule over chain and producer: 0 off, 1 / 2 (RF_K2_SPLIT) */
    uint32_t last_sink_attach; /* level whose launch ran the sink list in the last plain step (UINT32_MAX: none) */
    uint32_t last_levels_half; /* levels the last plain step ran in 32-job latency-form workgroups */
} rf_graph_stats;
/* Fills the whole struct above (its round-4 layout, unchanged since; a field
 * added later comes with a new, sized entry point rather than a change to
 * this one). */
int rf_graph_stats_get(rf_graph *g, rf_graph_stats *out);

/* ---- Checkpoint / resume of a loaded DAG ------------------------
 * Reference: a run's State is marshalled after every runner step
 * (runner/runner.go:51-85) and the local executor restores its execs from
 * manifests (local/executor.go:122-200); memoization is the resume mechanism.
 * rf_graph_save writes the graph's lowered device form (job records, holes,
 * reverse edges, padded templates, midstates, level layout) AND its current
 * slot digests to `path` (written to path.tmp, fsync'ed, renamed), with a
 * SHA-256 per 64 MiB chunk and one over them.  Steps queued on any stream
 * complete first (device synchronise).  rf_graph_restore loads such a file on
 * ctx's device: the graph is ready for incremental steps (set_slots +
 * recompute) at once -- no lowering, no level analysis, no full recompute.
 * A partition (rf_graph_set_part) is not part of the file: re-attach it.
 * Errors: RF_EIO (cannot create / open / write), RF_EINVAL (not a graph
 * checkpoint, or another version), RF_EINTEGRITY (truncated, the bytes do
 * not match their checksums, or the structure is inconsistent:
 * errors.Integrity), RF_EPRECONDITION from save when input slots were set
 * since the last recompute (the file holds digests, not a pending change
 * set: recompute first). */
int rf_graph_save(rf_graph *g, const char *path);
int rf_graph_restore(rf_ctx *ctx, const char *path, rf_graph **out);

/* ---- One DAG over many GPUs ---------------------------------
 * Each rank loads its PIECE of the global job graph (rf_graph_load on a local
 * desc: its own jobs plus replicated ones, slots renumbered locally) and
 * attaches its place in the partition: EXPORTS (local slots other ranks
 * read; export i of rank r has boundary id r * max_export + i, max_export the
 * same on every rank) and IMPORTS (local input slots fed from another rank's
 * boundary id).  rf_graph_recompute_part runs bulk-synchronous supersteps:
 * local recompute; an OR all-reduce of the bitset of exports changed since
 * they were last sent (RCCL has no bitwise OR: all-gather + local OR); an
 * all-gather of the export digests; changed imports written and their local
 * consumers queued; until no export changed (one exchange when no rank
 * imports, e.g. 1000align split by sample with the shared reference-index
 * chain replicated).  Transport: comm (RCCL over xGMI) or fn, a host
 * all-gather (recv[r*bytes ..] = rank r's send; 0 = ok) for ranks without
 * RCCL (tests on gloo, ranks sharing a GPU). */
typedef struct {
    int nranks, rank;
    uint32_t max_export;
    uint32_t n_export;
    const uint32_t *export_slot;
    uint32_t n_import;
    const uint32_t *import_slot;
    const uint32_t *import_bid;
    int any_import; /* some rank imports something (the same on every rank) */
    /* Exchange rounds per recompute, the same on every rank: the most
     * rank-boundary crossings on any path of the global graph (rf_graph_split;
     * 1 for configs[3]: sample roots -> the global root).  > 0 selects the
     * fixed-round protocol -- recompute, then `rounds` times: all-gather every
     * export digest, write the imports that differ (queueing their consumers)
     * and recompute -- with no OR-reduce and no host round trip, so with an
     * rf_comm and out_recomputed == NULL the whole call is asynchronous on the
     * context's stream.  0: the superstep protocol above (until no change). */
    uint32_t rounds;
} rf_graph_part;
typedef int (*rf_host_allgather_fn)(void *user, const void *send, void *recv, uint64_t bytes);
/* Attach (or replace) g's partition.  Between steps only: RF_EPRECONDITION
 * when input slots were set on a recomputed graph since its last recompute. */
int rf_graph_set_part(rf_graph *g, const rf_graph_part *p);
int rf_graph_recompute_part(rf_graph *g, rf_comm *comm, rf_host_allgather_fn fn, void *user, int full,
                            uint64_t *out_recomputed);
/* The last exchange's gathered export digests (device, [nranks*max_export][32],
 * boundary-id order) and the supersteps the last recompute took. */
int rf_graph_part_gathered(rf_graph *g, const void **d_digests32, uint64_t *n, uint64_t *supersteps);
/* Host-only splitter: rank `rank`'s piece of a global desc, owner[j] = the
 * rank that hashes job j (-1: every rank, e.g. the shared reference index).
 * The piece's desc arrays are owned by the piece (its blob is the global
 * blob, not copied); global_of_local maps its slots back. */
typedef struct rf_graph_piece rf_graph_piece;
int rf_graph_split(const rf_graph_desc *global, int nranks, int rank, const int32_t *owner, rf_graph_piece **out);
void rf_graph_piece_free(rf_graph_piece *p);
int rf_graph_piece_desc(const rf_graph_piece *p, rf_graph_desc *out);
int rf_graph_piece_part(const rf_graph_piece *p, rf_graph_part *out);
int rf_graph_piece_slots(const rf_graph_piece *p, const uint32_t **global_of_local, uint32_t *n);

/* Eval.dirty (eval.go:874-887) for every node of a Flow graph at once:
 * dirty[i] = 1 iff no_cache_extern and node i is an OpExtern (is_extern[i])
 * or one of its Deps is dirty -- Deps only ("dirty considers only visible
 * nodes": not MapFlow, Parent or continuations).  Eval.todo consults it under
 * NoCacheExtern to skip a node's cache lookup (eval.go:910).  Node i's deps
 * are deps[dep_ptr[i] .. dep_ptr[i+1]).  The closure runs on the GPU (K3
 * reachability over reverse edges, one launch per level); the reference's
 * per-node recursion has no memo. */
int rf_flow_dirty(rf_ctx *ctx, uint64_t n, const uint64_t *dep_ptr, const uint32_t *deps,
                  const uint8_t *is_extern, int no_cache_extern, uint8_t *dirty);

/* ---- K4: bloomlive / assoc probe (bloom.go:182-190, bloomlive.go:30-36) --
 * Filters cache-key lookups before Assoc.Get (eval.go:1202-1220) and serves
 * Liveset.Contains for Repository.Collect (repository/file/repository.go:304-327). */
/* words: bitset words (uint64, bit i in word i>>6); length = bitset length in bits. */
int rf_bloom_load(rf_ctx *ctx, uint64_t m, uint64_t k, const uint64_t *words, uint64_t nwords,
                  uint64_t length, rf_bloom **out);
/* Go JSON wire form {"m":M,"k":K,"b":"<base64url(BE64 len ‖ BE64 words)>"} (bloom.go:264-286). */
int rf_bloom_load_json(rf_ctx *ctx, const char *json, size_t len, rf_bloom **out);
/* The liveset's wire forms on the host alone (no device; what the loaders
 * above and the marshalers below use): parse into m, k, the bitset length
 * and its wordsNeeded(length) words (*n_words; RF_EINVAL with *n_words set
 * when cap_words is short), and format from host words (*out_len = bytes
 * needed, RF_EINVAL when cap is short).  Malformed or truncated input is
 * RF_EINVAL, never a read past len. */
int rf_bloom_parse_binary(const uint8_t *buf, size_t len, uint64_t *m, uint64_t *k, uint64_t *length,
                          uint64_t *words, uint64_t cap_words, uint64_t *n_words);
int rf_bloom_parse_json(const char *json, size_t len, uint64_t *m, uint64_t *k, uint64_t *length,
                        uint64_t *words, uint64_t cap_words, uint64_t *n_words);
int rf_bloom_format_binary(uint64_t m, uint64_t k, uint64_t length, const uint64_t *words, uint64_t n_words,
                           uint8_t *out, uint64_t cap, uint64_t *out_len);
int rf_bloom_format_json(uint64_t m, uint64_t k, uint64_t length, const uint64_t *words, uint64_t n_words,
                         uint8_t *out, uint64_t cap, uint64_t *out_len);
/* Go binary wire form BE64 m ‖ BE64 k ‖ BE64 len ‖ BE64 words (bloom.go:290-325). */
int rf_bloom_load_binary(rf_ctx *ctx, const uint8_t *buf, size_t len, rf_bloom **out);
/* New empty filter with m bits and k hashes (bloom.New, bloom.go:81-83). */
int rf_bloom_new(rf_ctx *ctx, uint64_t m, uint64_t k, rf_bloom **out);
void rf_bloom_destroy(rf_bloom *b);
/* out[i] = Contains(digest i): key = WD(d), all k bits set. */
int rf_bloom_probe(rf_bloom *b, const uint8_t *digests32, uint64_t n, uint8_t *out);
int rf_bloom_probe_device(rf_bloom *b, const void *d_digests32, uint64_t n, void *d_out,
                          void *stream);
/* Add WD(d) for each digest (eval.go:848-858 build side). */
int rf_bloom_add(rf_bloom *b, const uint8_t *digests32, uint64_t n);
int rf_bloom_add_device(rf_bloom *b, const void *d_digests32, uint64_t n, void *stream);
/* Read back m, k, length and the words (nwords = ceil(length/64) capacity). */
int rf_bloom_params(rf_bloom *b, uint64_t *m, uint64_t *k, uint64_t *length, uint64_t *nwords);
int rf_bloom_words(rf_bloom *b, uint64_t *words, uint64_t nwords);
/* Wire formats out (liveset build side, POST /collect body): Go MarshalJSON
 * {"m":M,"k":K,"b":"<base64.URLEncoding(BE64 len ‖ BE64 words)>"} (bloom.go:270-273,
 * bitset.go:693-702) and WriteTo BE64 m ‖ BE64 k ‖ bitset (bloom.go:290-301).
 * *out_len = bytes needed; RF_EINVAL if cap is short. */
int rf_bloom_marshal_json(rf_bloom *b, uint8_t *out, uint64_t cap, uint64_t *out_len);
int rf_bloom_marshal_binary(rf_bloom *b, uint8_t *out, uint64_t cap, uint64_t *out_len);
/* Repository.Collect (repository/file/repository.go:304-327) over n objects:
 * dead_idx[0 .. *n_dead) = the indices i, ascending, whose digest the liveset
 * does not contain (the objects Collect removes); *dead_bytes (may be NULL) =
 * the sum of their sizes (sizes may be NULL).  n < 2^32. */
int rf_bloom_collect(rf_bloom *b, const uint8_t *digests32, const int64_t *sizes, uint64_t n,
                     uint64_t *dead_idx, uint64_t *n_dead, int64_t *dead_bytes);
/* Device-resident form: d_counts2 receives {n_dead (u64), dead_bytes (i64)}. */
int rf_bloom_collect_device(rf_bloom *b, const void *d_digests32, const void *d_sizes, uint64_t n,
                            void *d_dead_idx, void *d_counts2, void *stream);

/* ---- K5: Canonicalize's flowMap (flow.go:814-843, flowMap.Get/Put :881-907) --
 * canon[i] = min{ j : digests[j] == digests[i] } over n node digests.  With
 * nodes numbered in the post-order of canonicalize's recursion (the order of
 * its m.Put calls) this is the flow the reference's first Put registers: the
 * canonical representative.  *n_unique = |{ i : canon[i] == i }|.  n <= 2^30. */
int rf_dedup_digests(rf_ctx *ctx, const uint8_t *digests32, uint32_t n, uint32_t *canon,
                     uint32_t *n_unique);
/* Device-resident form (digests e.g. gathered from rf_graph slots), on
 * `stream`.  *d_n_unique (uint32) gets the class count; its bit 31 set means
 * the batch hit the kernel's probe bound (65536 slots of linear probing at
 * load <= 1/2: not reachable for SHA-256 digests) and the result
 * must not be used -- rf_dedup_digests returns RF_EDEVICE for it. */
int rf_dedup_digests_device(rf_ctx *ctx, const void *d_digests32, uint32_t n, void *d_canon,
                            void *d_n_unique, void *stream);

/* ---- HBM assoc (assoc.Assoc, assoc/assoc.go:26-38) -----------------------
 * A digest -> digest map per kind in HBM with the semantics of the in-memory
 * assoc (test/testutil/assoc.go:34-56): the cache tier behind the probe, in
 * front of DynamoDB (assoc/dydbassoc).  Batched. */
int rf_assoc_new(rf_ctx *ctx, uint64_t capacity, rf_assoc **out);
void rf_assoc_destroy(rf_assoc *a);
/* Put, op i in batch order (ops on one key apply in index order): if
 * expect32 (may be NULL) row i is nonzero and the current value differs,
 * status[i] = RF_EPRECONDITION and nothing changes; else the value becomes
 * vals32[i] (all-zero deletes) and status[i] = RF_OK. */
int rf_assoc_put(rf_assoc *a, int kind, const uint8_t *expect32, const uint8_t *keys32,
                 const uint8_t *vals32, uint64_t n, int32_t *status);
/* Device-resident form (d_status: int32 per op); returns when applied. */
int rf_assoc_put_device(rf_assoc *a, int kind, const void *d_expect32, const void *d_keys32,
                        const void *d_vals32, uint64_t n, void *d_status);
/* Get: found[i] = 1 and vals32[i] = the value, or found[i] = 0 (NotExist,
 * vals32[i] zeroed). */
int rf_assoc_get(rf_assoc *a, int kind, const uint8_t *keys32, uint64_t n, uint8_t *vals32,
                 uint8_t *found);
int rf_assoc_get_device(rf_assoc *a, int kind, const void *d_keys32, uint64_t n, void *d_vals32,
                        void *d_found, void *stream);
/* Abbreviated keys (dydbassoc.go:111-147, ID4 index + Digest.Expands): key i
 * is given by its first nhex[i] hex digits (8..64) in keys32 row i.  status
 * RF_OK with the expanded key and its value, RF_ENOTFOUND, or RF_EINVAL when
 * more than one key matches. */
int rf_assoc_get_abbrev(rf_assoc *a, int kind, const uint8_t *keys32, const uint8_t *nhex, uint64_t n,
                        uint8_t *keys_out32, uint8_t *vals32, int32_t *status);
/* Eval.lookup's assoc step for a batch of nodes (eval.go:1172-1220), read
 * only: node i's cache keys (CacheKeys order, most to least concrete) are
 * keys32 rows [key_ptr[i], key_ptr[i+1]); all of them go in one Get batch (the
 * batching the TODO at eval.go:1199-1201 asks for).  which[i] = index within
 * the node of its first key with a value (vals32[i] = that value, the Fileset
 * id), or -1 (vals32[i] zeroed).  key_found / key_vals32 (either may be NULL):
 * per key, found and value -- the later candidates the caller tries when the
 * first fsid does not unmarshal (eval.go:1210-1218 moves on to the next key).
 * Nothing is written: read repair waits for the caller's checks
 * (rf_assoc_repair). */
int rf_assoc_lookup(rf_assoc *a, int kind, const uint8_t *keys32, const uint64_t *key_ptr, uint64_t n_nodes,
                    int32_t *which, uint8_t *vals32, uint8_t *key_found, uint8_t *key_vals32);
/* Read repair after the caller's checks (eval.go:1227-1258): node i takes part
 * iff which[i] >= 0 -- the key whose fsid unmarshalled and whose files all
 * exist (missing(), and not an empty value under RecomputeEmpty); the caller
 * sets which[i] = -1 for every other node.  Put(zero expect, key, vals32[i])
 * under every other key of the node (the reference's blind write-back), or,
 * with key_found (rf_assoc_lookup's) given, only under the keys that were
 * missing (precise read repair, the TODO at eval.go:1199-1201).  One Put
 * batch, node order then key order. */
int rf_assoc_repair(rf_assoc *a, int kind, const uint8_t *keys32, const uint64_t *key_ptr, uint64_t n_nodes,
                    const int32_t *which, const uint8_t *vals32, const uint8_t *key_found);
/* Occupied slots (live + deleted keys) and table capacity. */
int rf_assoc_stats(rf_assoc *a, uint64_t *occupied, uint64_t *capacity);

#ifdef __cplusplus
}
#endif
#endif /* REFLOW_HIP_H */
