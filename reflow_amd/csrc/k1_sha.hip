// k1_sha.hip -- K1: batched multi-message SHA-256 for gfx950.
//
// Replaces the per-file SHA-256 of repository/file/repository.go:50-63
// (Install: io.Copy into reflow.Digester.NewWriter()) that
// local/executor.go:514-557 runs in <=60 goroutines, and Repository.Put
// (repository/file/repository.go:237-264).  File.ID = SHA256(bytes).
//
// Two kernels, chosen per message by the host planner (capi.cpp):
//   k1_sha256_lanes  one LANE per message, 64 messages per wave, lanes pull new
//                    messages from a sharded work queue as they finish, so a
//                    wave never idles on its longest member.
//   k1_sha256_solo   one WAVE per long message: the 64 lanes expand the message
//                    schedule (K[t]+W[t]) of 64 consecutive blocks in parallel
//                    into LDS, then run the serial round chain reading those
//                    words by broadcast.  This cuts the per-block issue count of
//                    the critical chain from ~1464 to ~1000 instructions.  It
//                    runs at raised wave priority beside the lanes kernel.
// SHA-256 is Merkle-Damgard: one message's blocks are strictly serial and
// bit-exactness forbids tree hashing, so a skewed set is bounded below by its
// largest message (skew-aware roofline).
#include <cstdlib>

#include "engine.h"
#include "sha256_dev.h"
#include "lag_chain.h"

namespace rf {

constexpr uint32_t kLanesBlock = 256;
constexpr uint32_t kNone = 0xffffffffu;

__device__ __forceinline__ void store_digest(uint8_t* out, const ShaState& st) {
    uint4 lo, hi;
    lo.x = bswap32(st.h[0]); lo.y = bswap32(st.h[1]); lo.z = bswap32(st.h[2]); lo.w = bswap32(st.h[3]);
    hi.x = bswap32(st.h[4]); hi.y = bswap32(st.h[5]); hi.z = bswap32(st.h[6]); hi.w = bswap32(st.h[7]);
    reinterpret_cast<uint4*>(out)[0] = lo;
    reinterpret_cast<uint4*>(out)[1] = hi;
}

// Build the 16 big-endian words of block `blk` of message (p, len).
__device__ __forceinline__ void load_block(uint32_t (&w)[16], const uint8_t* p, uint64_t len,
                                           uint64_t blk) {
    const uint4* q = reinterpret_cast<const uint4*>(p + blk * 64u);
    const int64_t rem = (int64_t)len - (int64_t)(blk * 64u);
    if (rem >= 64) {
        const uint4 r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3];
        w[0] = bswap32(r0.x); w[1] = bswap32(r0.y); w[2] = bswap32(r0.z); w[3] = bswap32(r0.w);
        w[4] = bswap32(r1.x); w[5] = bswap32(r1.y); w[6] = bswap32(r1.z); w[7] = bswap32(r1.w);
        w[8] = bswap32(r2.x); w[9] = bswap32(r2.y); w[10] = bswap32(r2.z); w[11] = bswap32(r2.w);
        w[12] = bswap32(r3.x); w[13] = bswap32(r3.y); w[14] = bswap32(r3.z); w[15] = bswap32(r3.w);
    } else {
        // Tail: load only the 16-B chunks that hold message bytes; a chunk that
        // holds one valid byte lies inside that byte's aligned 16 B, never past
        // the allocation's last page.
        uint32_t raw[16];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            uint4 r = make_uint4(0, 0, 0, 0);
            if (rem > 16 * c) r = q[c];
            raw[4 * c] = r.x; raw[4 * c + 1] = r.y; raw[4 * c + 2] = r.z; raw[4 * c + 3] = r.w;
        }
        sha256_pad_words(w, raw, len, blk);
    }
}

// load_block split in two so a producer can have block b+1 in flight while it
// expands block b: the guarded 16-B loads, then byte swap / padding.
__device__ __forceinline__ void load_raw(uint4 (&r)[4], const uint8_t* p, uint64_t len, uint64_t blk) {
    const uint4* q = reinterpret_cast<const uint4*>(p + blk * 64u);
    const int64_t rem = (int64_t)len - (int64_t)(blk * 64u);
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = rem > 16 * c ? q[c] : make_uint4(0, 0, 0, 0);
}

__device__ __forceinline__ void raw_words(uint32_t (&w)[16], const uint4 (&r)[4], uint64_t len, uint64_t blk) {
    uint32_t raw[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        raw[4 * c] = r[c].x; raw[4 * c + 1] = r[c].y; raw[4 * c + 2] = r[c].z; raw[4 * c + 3] = r[c].w;
    }
    if ((int64_t)len - (int64_t)(blk * 64u) >= 64) {
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = bswap32(raw[i]);
    } else {
        sha256_pad_words(w, raw, len, blk);
    }
}

// Wave-cooperative dequeue: the lanes that need a message are counted with a
// ballot and served by ONE atomicAdd per wave on the wave's queue shard
// (message position q belongs to shard q % n_shards; LPT order is kept across
// shards).  Per-lane atomics on a shared counter serialise at ~0.1-0.3 us each
// (measured: 262k messages took 80 ms), the wave form costs one per wave.
// shard/tries are wave-uniform; an exhausted shard moves the whole wave on.
__device__ __forceinline__ uint32_t wave_fetch(const LanesArgs& a, bool need, uint32_t& shard,
                                               uint32_t& tries) {
    const uint32_t lane = __lane_id();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t got = kNone;
    uint64_t mask = __ballot(need);
    while (mask && tries < a.n_shards) {
        const uint32_t cnt = (uint32_t)__popcll(mask);
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)mask) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&a.heads[shard], cnt);
        base = __shfl(base, leader, 64);
        const bool mine = (mask >> lane) & 1ull;
        if (mine) {
            const uint64_t q = (uint64_t)(base + (uint32_t)__popcll(mask & lt)) * a.n_shards + shard;
            if (q < a.n_order) got = a.order[q];
        }
        mask = __ballot(mine && got == kNone);
        if (mask) {  // this shard ran dry for some lanes: the wave moves on
            shard = (shard + 1 == a.n_shards) ? 0u : shard + 1;
            ++tries;
        }
    }
    return got;
}

__global__ __launch_bounds__(kLanesBlock) void k1_sha256_lanes(LanesArgs a) {
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t shard = (gtid >> 6) % a.n_shards;
    uint32_t tries = 0;

    uint32_t id = wave_fetch(a, true, shard, tries);
    const uint8_t* p = nullptr;
    uint64_t len = 0, nb = 0, blk = 0;
    ShaState st;
    st.init();
    if (id != kNone) {
        p = a.arena + a.offs[id];
        len = a.lens[id];
        nb = sha256_nblocks(len);
    }
    while (__any(id != kNone)) {
        bool done = false;
        if (id != kNone) {
            uint32_t w[16];
            load_block(w, p, len, blk);
            sha256_compress(st, w);
            ++blk;
            if (blk == nb) {
                store_digest(a.out + 32ull * id, st);
                done = true;
            }
        }
        // wave-uniform point: one dequeue for every lane that finished
        const uint32_t nid = wave_fetch(a, done, shard, tries);
        if (done) {
            id = nid;
            st.init();
            blk = 0;
            if (id != kNone) {
                p = a.arena + a.offs[id];
                len = a.lens[id];
                nb = sha256_nblocks(len);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Solo: one wave per message.
// LDS: kw[blk][t] = K[t] + W_t for 64 blocks, rows padded to 68 words so a
// lane's 16-B stores of its own row spread over the banks; the chain reads a
// row with wave-uniform (broadcast) ds_read_b128.
constexpr uint32_t kRow = 68;

// Lane l of a wave writes row l = K[t] + W_t of block c + l (if it exists).
__device__ __forceinline__ void fill_kw_rows(uint32_t* kw, const uint8_t* p, uint64_t len, uint64_t nb,
                                             uint64_t c, uint32_t lane) {
    constexpr uint32_t K[64] = RF_SHA_K;
    const uint64_t b = c + lane;
    if (b >= nb) return;
    uint32_t w[16];
    load_block(w, p, len, b);
    uint32_t* row = &kw[lane * kRow];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
            w[t & 15] = wt;
        }
        row[t] = K[t] + wt;
    }
}

__global__ __launch_bounds__(64) void k1_sha256_solo(SoloArgs a) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ __attribute__((aligned(16))) uint32_t kw[64 * kRow];
    const uint32_t lane = threadIdx.x;
    for (uint32_t q = blockIdx.x; q < a.n_order; q += gridDim.x) {
        const uint32_t id = a.order[q];
        const uint8_t* p = a.arena + a.offs[id];
        const uint64_t len = a.lens[id];
        const uint64_t nb = sha256_nblocks(len);
        ShaState st;
        st.init();
        for (uint64_t c = 0; c < nb; c += 64) {
            fill_kw_rows(kw, p, len, nb, c, lane);
            __syncthreads();
            const uint32_t cnt = (uint32_t)((nb - c) < 64 ? (nb - c) : 64);
            for (uint32_t j = 0; j < cnt; ++j) {
                const uint4* r4 = reinterpret_cast<const uint4*>(&kw[j * kRow]);
                uint32_t a0 = st.h[0], b0 = st.h[1], c0 = st.h[2], d0 = st.h[3];
                uint32_t e0 = st.h[4], f0 = st.h[5], g0 = st.h[6], h0 = st.h[7];
#pragma unroll
                for (int t4 = 0; t4 < 16; ++t4) {
                    const uint4 v = r4[t4];
                    const uint32_t kv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const uint32_t t1 = add3v(h0 + kv[u], bsig1(e0), ch(e0, f0, g0));
                        h0 = g0; g0 = f0; f0 = e0; e0 = d0 + t1;
                        const uint32_t an = add3v(t1, bsig0(a0), maj(a0, b0, c0));
                        d0 = c0; c0 = b0; b0 = a0; a0 = an;
                    }
                }
                st.h[0] += a0; st.h[1] += b0; st.h[2] += c0; st.h[3] += d0;
                st.h[4] += e0; st.h[5] += f0; st.h[6] += g0; st.h[7] += h0;
            }
            __syncthreads();
        }
        if (lane == 0) store_digest(a.out + 32ull * id, st);
    }
}

// ---------------------------------------------------------------------------
// Duo: one wave per long message, the round chain split over two lanes and
// staggered by two rounds.
//
// Lanes with (lane & 8) == 0 ("e-lanes") run the e-half of round s; their
// partners lane^8 ("a-lanes") run the a-half of round s-2 in the same
// instruction stream.  With the state kept as the sequences e(r), a(r)
// (f = e(r-1), ..., d = a(r-3)) one round is
//   e-lanes: e(r+1) = Z + Σ1(e) + Ch(e,f,g),  Z = h + K+W(r) + d
//   a-lanes: a(r+1) = Z + Σ0(a) + Maj(a,b,c), Z = T1(r) = e(r+1) - d
// i.e. the same  R = Z + S + F  on both halves (Maj(a,b,c) = Ch(a^c, b, c)
// via sel = X0 ^ (X2 & M)).  S = Σ is spread over a quad of lanes: lane q
// of the quad rotates X0 by the q-th amount of its half (one v_alignbit with a
// per-lane amount) and two quad_perm DPP xors give all of them the xor of the
// three.  The Z of the next step needs one cross-lane value that is already a
// step old on both halves -- the partner's X0 (a(r-2) for the e-lane, e(r+2-2)
// for the a-lane, two rounds behind) -- so it is
//   Zt = (X2 ^ M) + k      e: g + K+W(r+1)     a: -c   (k = 1)
//   Z' = X0[lane^8] + Zt   one full-mask DPP add
// 8 VALU per round (9 with three v_alignbit per lane: 327 -> 297 ms per 16 MiB
// chain), every DPP source written >= 2 instructions earlier.  One wave issues
// one instruction per ~4-5 cycles whatever the dependences (tools/micro.py
// lat), so the instruction count per round is the chain's cost.
// Block boundaries: each half applies its own feed-forward (bank-masked DPP
// adds) when it reaches round 0 of the next block; the Z values that straddle the boundary read partner values from
// before the partner's feed-forward and get per-block corrections
// (c63/c64/c65 below).  A message starts from a zero raw state with
// chaining value IV, so block 0 takes the same path as every other block.
//
// Registers: the state rotates through four registers (the new X0 goes into
// the old X3's register), so after four steps the mapping is back in place;
// one asm block runs four steps and the compiler's pad after an asm block is
// paid once per four rounds.
// RF_LAG_* macros (step, feed-forward, block-boundary corrections): lag_chain.h

// Two waves: wave 0 runs the chain, wave 1 expands the next 64 blocks'
// K+W rows into the other half of a double buffer meanwhile (one barrier per
// 64 blocks), so the chain never waits for HBM or the message schedule.
__global__ __launch_bounds__(128) void k1_sha256_duo(SoloArgs a) {
    // two buffers of 64 K+W rows, then the a-lanes' k row: word 0 = 0
    // (block-start add), the rest 1 (Zt = -c)
    __shared__ __attribute__((aligned(16))) uint32_t kw[129 * kRow];
    // wave-uniform (SGPR) so the role branches below are scalar branches and
    // each wave meets exactly one barrier per chunk
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t* const ones = &kw[128 * kRow];
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        ones[lane] = lane ? 1u : 0u;
        if (lane < 4) ones[64 + lane] = 1u;
    }
    const bool elane = (lane & 8) == 0;
    // Σ over a quad: lane q (q = lane & 3 < 3) rotates by the q-th amount of
    // its half (Σ1: 6 11 25, Σ0: 2 13 22); two quad_perm DPP xors give every
    // lane of the quad the xor of all three (lane 3 of a quad is unused)
    const uint32_t q3 = lane & 3;
    const uint32_t shq = elane ? (q3 == 1 ? 11u : q3 == 2 ? 25u : 6u) : (q3 == 1 ? 13u : q3 == 2 ? 22u : 2u);
    const uint32_t M = elane ? 0u : ~0u;
    const uint32_t one = 1u, zero = 0u;
    for (uint32_t q = blockIdx.x; q < a.n_order; q += gridDim.x) {
        const uint32_t id = a.order[q];
        const uint8_t* p = a.arena + a.offs[id];
        const uint64_t len = a.lens[id];
        const uint64_t nb = sha256_nblocks(len);
        // Start as if after a block whose raw final state is zero with
        // chaining value IV: the feed-forward of block 0's group 0 then
        // produces the IV state and the corrections below are the general
        // ones for H = IV.
        uint32_t Hr0 = elane ? lag::IV[4] : lag::IV[0], Hr1 = elane ? lag::IV[5] : lag::IV[1];
        uint32_t Hr2 = elane ? lag::IV[6] : lag::IV[2], Hr3 = elane ? lag::IV[7] : lag::IV[3];
        uint32_t Pa = 0, Pb = 0, Pc = 0, Pd = 0;
        uint32_t Z = elane ? lag::IV[7] + lag::IV[3] : 0u, Y = 0;
        uint32_t c63 = 0;
        uint32_t c64 = elane ? lag::IV[2] : 0u - lag::IV[4];
        uint32_t c65 = elane ? lag::IV[1] : 0u - lag::IV[3];
        uint32_t t0, t1, t3;
        if (wave == 1) fill_kw_rows(kw, p, len, nb, 0, lane);
        __syncthreads();
        uint32_t buf = 0;
        for (uint64_t c = 0; c < nb; c += 64, buf ^= 1) {
            if (wave == 1) {
                if (c + 64 < nb) fill_kw_rows(&kw[(buf ^ 1) * 64 * kRow], p, len, nb, c + 64, lane);
            } else {
            const uint32_t cnt = (uint32_t)((nb - c) < 64 ? (nb - c) : 64);
            // e-lanes read row j of this buffer, a-lanes the ones row: a
            // bit-select of byte offsets (no per-lane branch)
            const uint32_t ones_off = 128 * kRow * 4, buf_off = buf * 64 * kRow * 4;
            const uint4* r4 = reinterpret_cast<const uint4*>(
                reinterpret_cast<const char*>(kw) + ((M & ones_off) | (~M & buf_off)));
            uint4 v = r4[0], vn = r4[1];
            for (uint32_t j = 0; j < cnt; ++j) {
                // the next row (clamped at the chunk end; its values are then
                // not used) -- its first 32 B are read during groups 14-15
                const uint32_t nrow_off = buf_off + (j + 1 < cnt ? j + 1 : j) * kRow * 4;
                const uint4* r4n = reinterpret_cast<const uint4*>(
                    reinterpret_cast<const char*>(kw) + ((M & ones_off) | (~M & nrow_off)));
                uint4 vnn = r4[2];
                {
                    // e-lanes enter the block at step 0, a-lanes at step 2
                    const uint32_t k1 = v.y + c64, k2 = v.z + c65;
                    asm volatile("s_nop 1\n\t" RF_LAG_FF("0x3", "a", "b", "c", "d")
                                 "v_add_u32 %[z], %[z], %[kw0]\n\t"
                                 RF_LAG_STEP("a", "b", "c", "d", "z", "y", "k1")
                                 RF_LAG_STEP("d", "a", "b", "c", "y", "z", "k2")
                                 RF_LAG_FF("0xc", "c", "d", "a", "b")
                                 RF_LAG_STEP("c", "d", "a", "b", "z", "y", "k3")
                                 RF_LAG_STEP("b", "c", "d", "a", "y", "z", "k4")
                                 RF_LAG_CORR
                                 : RF_LAG_STATE, RF_LAG_TMP, RF_LAG_H,
                                   [c63] "=&v"(c63), [c64] "+v"(c64), [c65] "+v"(c65)
                                 : RF_LAG_IN(k1, k2, v.w, vn.x), [kw0] "v"(v.x), [one] "v"(one),
                                   [zero] "v"(zero));
                }
                v = vn;
                vn = vnn;
#pragma unroll
                for (int g = 1; g < 16; ++g) {
                    // LDS reads run two groups ahead of the chain
                    vnn = g < 14 ? r4[g + 2] : r4n[g - 14];
                    const uint32_t k4 = g == 15 ? c63 : vn.x;
                    asm volatile(RF_LAG_GROUP : RF_LAG_STATE, RF_LAG_TMP : RF_LAG_IN(v.y, v.z, v.w, k4));
                    v = vn;
                    vn = vnn;
                }
                r4 = r4n;
            }
            }
            __syncthreads();
        }
        if (wave == 1) continue;
        // tail: the e-lanes are done (H += X, X untouched so the a-lanes' last
        // Z reads raw e(64)); the a-lanes run rounds 62 and 63, then H += X.
        asm volatile("s_nop 1\n\t" RF_LAG_FIN("0x3", "a", "b", "c", "d")
                     RF_LAG_STEP("a", "b", "c", "d", "z", "y", "k1")
                     RF_LAG_STEP("d", "a", "b", "c", "y", "z", "k2")
                     RF_LAG_FIN("0xc", "c", "d", "a", "b")
                     : RF_LAG_STATE, RF_LAG_TMP, RF_LAG_H
                     : RF_LAG_IN(one, one, one, one));
        // lane 8 (a-lane) holds H0..H3, lane 0 (e-lane) H4..H7
        if (lane == 0 || lane == 8) {
            uint4 o;
            o.x = bswap32(Hr0); o.y = bswap32(Hr1); o.z = bswap32(Hr2); o.w = bswap32(Hr3);
            reinterpret_cast<uint4*>(a.out + 32ull * id)[lane == 0 ? 1 : 0] = o;
        }
    }
}

// ---------------------------------------------------------------------------
// Octo: the duo's two-lane lagged chain for eight messages per wave (sets that
// leave the chip mostly idle, e.g. configs[0]'s 4096 files: 512 chain waves at
// 8 instructions per round instead of 64-message pair waves at 14).  Lanes
// 8f..8f+7 run message f: 8f..8f+3 the e-half, 8f+4..8f+7 the a-half.  Every
// lane of a quad ends a round with the full Σ (positions 0..2 rotate by the
// half's three amounts, position 3 repeats position 0's; quad_perm [1,2,0,1]
// then [2,0,1,2] xor them together), so the partner's X0 can come from the
// mirrored lane of the half-row (row_half_mirror: i <-> 7-i) and the halves'
// feed-forwards select banks 0x5 (e) / 0xa (a).
// The producer wave expands the K+W rows one lane per (message, block), in
// chunks of eight blocks per message, double-buffered; rows are block-major
// (message f's row of block j at (buf*8 + j)*8 + f) so the eight rows one
// ds_read_b128 reads sit 68 words apart, in disjoint banks.
// A message's digest is its chaining value after the group 0 of block nb --
// the block after its last, where both halves have applied the final
// feed-forward; the wave runs that group 0 for its longest message after the
// loop.  Shorter messages of the wave keep hashing rows nobody wrote (their
// lanes' results are never stored again).
// RF_OCT_* (the octo chain's step, group, group 0): lag_chain.h

// Producer lane l: block c + (l & 7) of message l >> 3 into its row of buffer kwb.
__device__ __forceinline__ void fill_oct_row(uint32_t* kwb, const uint8_t* p, uint64_t len, uint64_t nb,
                                             uint64_t c, uint32_t lane) {
    const uint32_t jj = lane & 7;
    const uint64_t b = c + jj;
    if (b >= nb) return;
    uint32_t w[16];
    load_block(w, p, len, b);
    kw_expand_store(w, reinterpret_cast<uint4*>(&kwb[(jj * 8 + (lane >> 3)) * kRow]));
}

constexpr uint32_t kOctChunk = 8;

__global__ __launch_bounds__(128) void k1_sha256_octo(SoloArgs a) {
    // two buffers of 8 blocks x 8 messages, then the a-lanes' k row
    __shared__ __attribute__((aligned(16))) uint32_t kw[129 * kRow];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t* const ones = &kw[128 * kRow];
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        ones[lane] = lane ? 1u : 0u;
        if (lane < 4) ones[64 + lane] = 1u;
    }
    const uint32_t f = lane >> 3;
    const bool elane = (lane & 4) == 0;
    const uint32_t q3 = lane & 3;
    const uint32_t shq = elane ? (q3 == 1 ? 11u : q3 == 2 ? 25u : 6u) : (q3 == 1 ? 13u : q3 == 2 ? 22u : 2u);
    const uint32_t M = elane ? 0u : ~0u;
    const uint32_t one = 1u, zero = 0u;
    const uint32_t n_groups = (a.n_order + 7) / 8;
    for (uint32_t q = blockIdx.x; q < n_groups; q += gridDim.x) {
        const uint32_t qi = 8 * q + f;
        const bool has = qi < a.n_order;
        const uint32_t id = has ? a.order[qi] : 0u;
        const uint64_t len = has ? a.lens[id] : 0;
        const uint8_t* p = a.arena + (has ? a.offs[id] : 0);
        const uint64_t nb = has ? sha256_nblocks(len) : 0;
        uint64_t maxnb = nb;
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t x = __shfl_xor(maxnb, o, 64);
            maxnb = x > maxnb ? x : maxnb;
        }
        uint32_t Hr0 = elane ? lag::IV[4] : lag::IV[0], Hr1 = elane ? lag::IV[5] : lag::IV[1];
        uint32_t Hr2 = elane ? lag::IV[6] : lag::IV[2], Hr3 = elane ? lag::IV[7] : lag::IV[3];
        uint32_t Pa = 0, Pb = 0, Pc = 0, Pd = 0;
        uint32_t Z = elane ? lag::IV[7] + lag::IV[3] : 0u, Y = 0;
        uint32_t c63 = 0;
        uint32_t c64 = elane ? lag::IV[2] : 0u - lag::IV[4];
        uint32_t c65 = elane ? lag::IV[1] : 0u - lag::IV[3];
        uint32_t t0, t1, t3;
        uint32_t D0 = 0, D1 = 0, D2 = 0, D3 = 0;
        uint4 v = make_uint4(0, 0, 0, 0), vn = v;
        if (wave == 1) fill_oct_row(kw, p, len, nb, 0, lane);
        __syncthreads();
        uint32_t buf = 0;
        for (uint64_t c = 0; c < maxnb; c += kOctChunk, buf ^= 1) {
            if (wave == 1) {
                if (c + kOctChunk < maxnb) fill_oct_row(&kw[(buf ^ 1) * 64 * kRow], p, len, nb, c + kOctChunk, lane);
            } else {
                const uint32_t cnt = (uint32_t)((maxnb - c) < kOctChunk ? (maxnb - c) : kOctChunk);
                // e-lanes read their message's rows, a-lanes the ones row
                const uint32_t ones_off = 128 * kRow * 4, buf_off = (buf * 64 + f) * kRow * 4;
                const uint4* r4 = reinterpret_cast<const uint4*>(
                    reinterpret_cast<const char*>(kw) + ((M & ones_off) | (~M & buf_off)));
                v = r4[0];
                vn = r4[1];
                for (uint32_t j = 0; j < cnt; ++j) {
                    const uint32_t nrow_off = buf_off + (j + 1 < cnt ? j + 1 : j) * 8 * kRow * 4;
                    const uint4* r4n = reinterpret_cast<const uint4*>(
                        reinterpret_cast<const char*>(kw) + ((M & ones_off) | (~M & nrow_off)));
                    uint4 vnn = r4[2];
                    {
                        const uint32_t k1 = v.y + c64, k2 = v.z + c65;
                        asm volatile(RF_OCT_GROUP0
                                     : RF_LAG_STATE, RF_LAG_TMP, RF_LAG_H,
                                       [c63] "=&v"(c63), [c64] "+v"(c64), [c65] "+v"(c65)
                                     : RF_LAG_IN(k1, k2, v.w, vn.x), [kw0] "v"(v.x), [one] "v"(one),
                                       [zero] "v"(zero));
                    }
                    if (c + j == nb) {  // message done: its final chaining value
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
        if (wave == 1) continue;
        {
            const uint32_t k1 = v.y + c64, k2 = v.z + c65;
            asm volatile(RF_OCT_GROUP0
                         : RF_LAG_STATE, RF_LAG_TMP, RF_LAG_H,
                           [c63] "=&v"(c63), [c64] "+v"(c64), [c65] "+v"(c65)
                         : RF_LAG_IN(k1, k2, v.w, vn.x), [kw0] "v"(v.x), [one] "v"(one), [zero] "v"(zero));
        }
        if (nb == maxnb) {
            D0 = Hr0; D1 = Hr1; D2 = Hr2; D3 = Hr3;
        }
        // lane 8f (e) holds H4..H7, lane 8f+4 (a) H0..H3
        if (has && (lane & 3) == 0) {
            uint4 o;
            o.x = bswap32(D0); o.y = bswap32(D1); o.z = bswap32(D2); o.w = bswap32(D3);
            reinterpret_cast<uint4*>(a.out + 32ull * id)[elane ? 1 : 0] = o;
        }
    }
}

// ---------------------------------------------------------------------------
// Pair: lane per message like k1_sha256_lanes, for sets too small to load the
// chip (<= one wave per SIMD), where a lane's chain is bound by its wave's
// issue rate: a producer wave loads/pads each message's next block and
// expands its schedule into a double-buffered LDS row (kw_expand_store), the
// chain wave runs the rounds from LDS (compress_kw: 14 instead of ~22
// instructions per round).  64 messages per workgroup (largest-first order,
// so a workgroup's messages have similar block counts), one barrier per block.
constexpr uint32_t kPairRow = 68;

__global__ __launch_bounds__(256) void k1_sha256_pair(SoloArgs a, uint32_t pw, uint32_t dbg) {
    __shared__ __attribute__((aligned(16))) uint32_t kw[2 * 64 * kPairRow];
    // wave 0 chain, wave pw producer, any other wave only meets the barriers
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wave = w0 == 0 ? 0u : w0 == pw ? 1u : 2u;
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = blockIdx.x * 64; base < a.n_order; base += gridDim.x * 64) {
        const uint32_t q = base + lane;
        const bool has = q < a.n_order;
        const uint32_t id = has ? a.order[q] : 0u;
        const uint64_t len = has ? a.lens[id] : 0;
        const uint8_t* p = a.arena + (has ? a.offs[id] : 0);
        const uint64_t nb = has ? sha256_nblocks(len) : 0;
        uint64_t maxnb = nb;
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t x = __shfl_xor(maxnb, o, 64);
            maxnb = x > maxnb ? x : maxnb;
        }
        ShaState st;
        st.init();
        uint4 r[4];
        if (wave == 1 && nb) load_raw(r, p, len, 0);
        for (uint64_t it = 0; it <= maxnb; ++it) {
            if (wave == 1) {
                if (it < nb && !(dbg & 1)) {
                    uint32_t w[16];
                    raw_words(w, r, len, it);
                    if (it + 1 < nb) load_raw(r, p, len, it + 1);  // in flight during the expansion
                    kw_expand_store(w, reinterpret_cast<uint4*>(&kw[((it & 1) * 64 + lane) * kPairRow]));
                }
            } else if (wave == 0 && it >= 1 && it - 1 < nb && !(dbg & 2)) {
                compress_kw(st, reinterpret_cast<const uint4*>(&kw[(((it - 1) & 1) * 64 + lane) * kPairRow]));
            }
            __syncthreads();
        }
        if (wave == 0 && has) store_digest(a.out + 32ull * id, st);
    }
}

// ---------------------------------------------------------------------------
// Synthetic content: word q of message i = mix64((seed ^ i) + (q+1)*G), LE.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_gen_fill(uint8_t* arena, const uint64_t* offs,
                                                  const uint64_t* lens, uint64_t n, uint64_t seed,
                                                  uint64_t nchunks) {
    constexpr uint64_t G = 0x9E3779B97F4A7C15ull;
    uint64_t cur = 0, cur_lo = 1, cur_hi = 0;  // empty range forces a search
    for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < nchunks;
         x += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t o = x * 16;
        if (!(o >= cur_lo && o < cur_hi)) {
            // last message with offs[i] <= o
            uint64_t lo = 0, hi = n;
            while (hi - lo > 1) {
                const uint64_t mid = (lo + hi) / 2;
                if (offs[mid] <= o) lo = mid; else hi = mid;
            }
            cur = lo;
            cur_lo = offs[lo];
            cur_hi = cur_lo + ((lens[lo] + 15) & ~15ull);
        }
        uint4 v = make_uint4(0, 0, 0, 0);
        if (n > 0 && o >= cur_lo && o < cur_hi) {
            const uint64_t rel = o - cur_lo;
            const uint64_t s = seed ^ cur;
            const uint64_t q = rel / 8;
            const uint64_t w0 = mix64(s + (q + 1) * G), w1 = mix64(s + (q + 2) * G);
            v = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
            const uint64_t len = lens[cur];
            if (rel + 16 > len) {  // zero bytes past the message end
                uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t valid = (int64_t)len - (int64_t)(rel + 4 * j);
                    if (valid <= 0) vv[j] = 0;
                    else if (valid < 4) vv[j] &= (1u << (8 * valid)) - 1;
                }
                v = make_uint4(vv[0], vv[1], vv[2], vv[3]);
            }
        }
        reinterpret_cast<uint4*>(arena)[x] = v;
    }
}

// Streaming: lane per segment, whole blocks from a carried midstate (the
// Writer state of Digester.NewWriter between Write calls).  Segments come
// largest first, so a wave's lanes run similar block counts.
__global__ __launch_bounds__(256) void k1_sha256_resume(ResumeArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    ShaState st;
    uint4* m4 = reinterpret_cast<uint4*>(a.mid + 8ull * i);
    const uint4 lo = m4[0], hi = m4[1];
    st.h[0] = lo.x; st.h[1] = lo.y; st.h[2] = lo.z; st.h[3] = lo.w;
    st.h[4] = hi.x; st.h[5] = hi.y; st.h[6] = hi.z; st.h[7] = hi.w;
    const uint4* q = reinterpret_cast<const uint4*>(a.arena + a.offs[i]);
    const uint64_t nb = a.nblocks[i];
    for (uint64_t b = 0; b < nb; ++b, q += 4) {
        const uint4 r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3];
        uint32_t w[16] = {bswap32(r0.x), bswap32(r0.y), bswap32(r0.z), bswap32(r0.w),
                          bswap32(r1.x), bswap32(r1.y), bswap32(r1.z), bswap32(r1.w),
                          bswap32(r2.x), bswap32(r2.y), bswap32(r2.z), bswap32(r2.w),
                          bswap32(r3.x), bswap32(r3.y), bswap32(r3.z), bswap32(r3.w)};
        sha256_compress(st, w);
    }
    m4[0] = make_uint4(st.h[0], st.h[1], st.h[2], st.h[3]);
    m4[1] = make_uint4(st.h[4], st.h[5], st.h[6], st.h[7]);
}

hipError_t launch_sha_resume(const ResumeArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k1_sha256_resume, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

// The host leg's digests into the plan's output rows: one 16-B half per lane.
__global__ __launch_bounds__(256) void k_scatter_digests(uint8_t* __restrict__ out, const uint32_t* __restrict__ ids,
                                                         const uint8_t* __restrict__ digs, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 2 * n) return;
    const uint64_t i = t >> 1, half = t & 1;
    reinterpret_cast<uint4*>(out + 32ull * ids[i])[half] = reinterpret_cast<const uint4*>(digs + 32 * i)[half];
}

hipError_t launch_scatter_digests(uint8_t* out32, const uint32_t* ids, const uint8_t* digs32, uint64_t n,
                                  hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t grid = (2 * n + 255) / 256;
    hipLaunchKernelGGL(k_scatter_digests, dim3((uint32_t)grid), dim3(256), 0, s, out32, ids, digs32, n);
    return hipGetLastError();
}

uint32_t sha_lanes_block() { return kLanesBlock; }

hipError_t probe_kernels() {
    hipFuncAttributes attr;
    return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&k1_sha256_lanes));
}

hipError_t launch_sha_lanes(const LanesArgs& a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(k1_sha256_lanes, dim3(grid), dim3(kLanesBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_sha_solo(const SoloArgs& a, bool duo, hipStream_t s) {
    if (a.n_order == 0) return hipSuccess;
    if (duo)
        hipLaunchKernelGGL(k1_sha256_duo, dim3(a.n_order), dim3(128), 0, s, a);
    else
        hipLaunchKernelGGL(k1_sha256_solo, dim3(a.n_order), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_sha_pair(const SoloArgs& a, hipStream_t s) {
    if (a.n_order == 0) return hipSuccess;
    uint32_t grid = (a.n_order + 63) / 64;
    if (grid > 4096) grid = 4096;
    // A pair workgroup reserves most of its CU's LDS so no other pair or duo
    // workgroup shares the CU: its chain wave then has a SIMD to itself (a
    // co-resident duo chain at s_setprio 3 took the issue slots: 1.9 -> 2.9 us
    // per block, and the planner's makespan model counts on 1.9).
    static const size_t reserve = 126 * 1024 - sizeof(uint32_t) * 2 * 64 * kPairRow;
    hipLaunchKernelGGL(k1_sha256_pair, dim3(grid), dim3(128), reserve, s, a, 1u, 0u);
    return hipGetLastError();
}

hipError_t launch_sha_octo(const SoloArgs& a, hipStream_t s) {
    if (a.n_order == 0) return hipSuccess;
    uint32_t grid = (a.n_order + 7) / 8;
    if (grid > 8192) grid = 8192;
    static const size_t reserve = (size_t)RF_DIAG_KNOB("RF_OCTO_LDS_KB", 0) * 1024;
    hipLaunchKernelGGL(k1_sha256_octo, dim3(grid), dim3(128), reserve, s, a);
    return hipGetLastError();
}

hipError_t launch_gen_fill(uint8_t* arena, const uint64_t* offs, const uint64_t* lens, uint64_t n,
                           uint64_t seed, uint64_t arena_bytes, hipStream_t s) {
    const uint64_t nchunks = arena_bytes / 16;
    uint64_t grid = (nchunks + 255) / 256;
    if (grid > 16384) grid = 16384;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_fill, dim3((uint32_t)grid), dim3(256), 0, s, arena, offs, lens, n,
                       seed, nchunks);
    return hipGetLastError();
}

// Fileset digest with device-resident File IDs: entry i's 32 ID bytes go to
// byte mat_off[i] of the material arena (one thread per byte; the material
// positions are unaligned: path lengths vary).
__global__ __launch_bounds__(256) void k_place_ids(uint8_t* __restrict__ arena, const uint64_t* __restrict__ mat_off,
                                                   const uint32_t* __restrict__ entry, uint64_t n,
                                                   const uint8_t* __restrict__ ids32) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 32 * n) return;
    const uint64_t i = t >> 5, b = t & 31;
    arena[mat_off[i] + b] = ids32[32ull * entry[i] + b];
}

hipError_t launch_place_ids(uint8_t* arena, const uint64_t* mat_off, const uint32_t* entry, uint64_t n,
                            const uint8_t* ids32, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t grid = (32 * n + 255) / 256;
    hipLaunchKernelGGL(k_place_ids, dim3((uint32_t)grid), dim3(256), 0, s, arena, mat_off, entry, n, ids32);
    return hipGetLastError();
}

}  // namespace rf
