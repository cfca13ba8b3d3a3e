// sha256_dev.h -- SHA-256 compression for gfx950 (CDNA4) VALU.
//
// Replaces Go crypto/sha256 as used through reflow.Digester
// (/root/reference/flow.go:36; streamed at repository/file/repository.go:56-61).
// FIPS 180-4 §6.2; bit-exact by construction, checked against oracle/oracle.c.
//
// Instruction selection (checked in the .s, see DESIGN.md "K1"):
//   ROTR      -> v_alignbit_b32 (x, x, n)
//   Σ/σ       -> 3 x v_alignbit / v_lshrrev + v_bitop3_b32 (xor3, table 0x96)
//   Ch, Maj   -> v_bitop3_b32 (tables 0xCA, 0xE8)
//   sums      -> v_add3_u32
//   BE loads  -> v_perm_b32 byte swap
// One 64-byte block costs ~1464 canonical int32 VALU ops.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rf {

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    return (m & a) | (~m & b);
}
// gfx950 has no v_xor3_b32; v_bitop3_b32 evaluates any 3-input truth table
// (S0 is the MSB of the table index, as in the 0xF0/0xCC/0xAA convention).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // e ? f : g
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority
}
__device__ __forceinline__ uint32_t bsig0(uint32_t a) { return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t e) { return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }

// v_add3_u32 pinned by inline asm where the scheduler otherwise splits the
// sum into 2-input adds to wait on a late operand (solo chain).
__device__ __forceinline__ uint32_t add3v(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

#define RF_SHA_K                                                                                   \
    {0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,     \
     0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,     \
     0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,     \
     0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,     \
     0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,     \
     0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,     \
     0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,     \
     0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,     \
     0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,     \
     0xc67178f2u}

struct ShaState {
    uint32_t h[8];
    __device__ __forceinline__ void init() {
        h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
        h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
    }
};

// Compress one block.  w[] holds the 16 big-endian message words and is
// overwritten by the rolling message schedule (no 64-entry W array: the
// window stays in 16 VGPRs).  Fully unrolled so every index is static.
__device__ __forceinline__ void sha256_compress(ShaState& s, uint32_t (&w)[16]) {
    constexpr uint32_t K[64] = RF_SHA_K;
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
    uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
            w[t & 15] = wt;
        }
        const uint32_t hk = h + K[t] + wt;                  // v_add3
        const uint32_t t1 = hk + bsig1(e) + ch(e, f, g);    // v_add3
        h = g; g = f; f = e; e = d + t1;
        const uint32_t an = t1 + bsig0(a) + maj(a, b, c);   // v_add3
        d = c; c = b; b = a; a = an;
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// Producer/chain split of one block (k2_level_pc, k1_sha256_pair): the
// producer expands the message schedule and stores K[t] + W[t] as 16 uint4
// into an LDS row; the chain runs the 64 rounds from that row, 14
// instructions per round (the schedule's ~8 per round moved off the chain).
__device__ __forceinline__ void kw_expand_store(uint32_t (&w)[16], uint4* row) {
    constexpr uint32_t K[64] = RF_SHA_K;
#pragma unroll
    for (int t4 = 0; t4 < 16; ++t4) {
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = 4 * t4 + u;
            uint32_t wt;
            if (t < 16) {
                wt = w[t];
            } else {
                wt = ssig1(w[(t - 2) & 15]) + w[(t - 7) & 15] + ssig0(w[(t - 15) & 15]) + w[t & 15];
                w[t & 15] = wt;
            }
            v[u] = K[t] + wt;
        }
        row[t4] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

__device__ __forceinline__ void compress_kw(ShaState& s, const uint4* row) {
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3];
    uint32_t e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int t4 = 0; t4 < 16; ++t4) {
        const uint4 v = row[t4];
        const uint32_t kv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t t1 = add3v(h + kv[u], bsig1(e), ch(e, f, g));
            h = g; g = f; f = e; e = d + t1;
            const uint32_t an = add3v(t1, bsig0(a), maj(a, b, c));
            d = c; c = b; b = a; a = an;
        }
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// Build the big-endian words of block `blk` of a message of `len` bytes whose
// raw little-endian-loaded words are raw[] (loaded from the block's address;
// bytes past the message end may hold anything).  Applies FIPS-180 padding:
// 0x80 after the last byte, zeros, 64-bit big-endian bit length in the last
// two words of the final block.  Branch-free per word.
__device__ __forceinline__ void sha256_pad_words(uint32_t (&w)[16], const uint32_t (&raw)[16],
                                                 uint64_t len, uint64_t blk) {
    const int64_t rem = (int64_t)len - (int64_t)(blk * 64u);  // bytes of message in this block
    const bool final_blk = rem <= 55;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int64_t v = rem - 4 * j;  // message bytes available in this word
        const uint32_t be = bswap32(raw[j]);
        uint32_t x;
        if (v >= 4) {
            x = be;
        } else if (v >= 0) {
            // keep the top v bytes, 0x80 at byte v (big-endian position)
            const uint32_t keep = v == 0 ? 0u : (0xffffffffu << (32 - 8 * (uint32_t)v));
            x = (be & keep) | (0x80u << (24 - 8 * (uint32_t)v));
        } else {
            x = 0u;
        }
        w[j] = x;
    }
    if (final_blk) {
        const uint64_t bits = len * 8u;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
    }
}

// Number of 64-byte blocks SHA-256 processes for a len-byte message.
__host__ __device__ __forceinline__ uint64_t sha256_nblocks(uint64_t len) { return (len + 9 + 63) / 64; }

}  // namespace rf
