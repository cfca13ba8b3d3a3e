// host_sha.cpp -- SHA-256 compression with the x86 SHA extensions for the
// planner's host leg (see host_sha.h).  Compiled by the host C++ compiler
// (no HIP); the SHA-NI function carries its own target attribute, so the
// rest of the library never assumes the instructions exist: the planner asks
// host_sha_available() first.
//
// Register layout of sha256rnds2: the eight state words live in two xmm
// registers, ABEF (lanes F,E,B,A from low to high) and CDGH (H,G,D,C); one
// rnds2 runs two rounds with the two low dwords of its message operand
// (K[t] + W[t] for rounds t, t+1).  Four message words per group; the
// schedule for words 16..63 is sha256msg1 (the sigma0 half), one alignr for
// W[t-7], and sha256msg2 (the sigma1 half).
#include "host_sha.h"

#include <cpuid.h>
#include <immintrin.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <vector>

namespace rf {

namespace {

alignas(16) const uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

constexpr uint32_t kIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                             0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

// Four rounds: group g of the message (words 4g..4g+3 in m).
#define RF_NI_ROUNDS(m, g)                                                             \
    do {                                                                               \
        __m128i kw_ = _mm_add_epi32((m), _mm_load_si128((const __m128i*)&kK[4 * (g)])); \
        cdgh = _mm_sha256rnds2_epu32(cdgh, abef, kw_);                                 \
        kw_ = _mm_shuffle_epi32(kw_, 0x0E);                                            \
        abef = _mm_sha256rnds2_epu32(abef, cdgh, kw_);                                 \
    } while (0)

// W[4g..4g+3] for g >= 4 from the four previous groups (m0 = group g-4,
// overwritten): W[t] = s1(W[t-2]) + W[t-7] + s0(W[t-15]) + W[t-16].
#define RF_NI_SCHED(m0, m1, m2, m3) \
    m0 = _mm_sha256msg2_epu32(_mm_add_epi32(_mm_sha256msg1_epu32(m0, m1), _mm_alignr_epi8(m3, m2, 4)), m3)

__attribute__((target("sha,sse4.1,ssse3"))) void ni_blocks(uint32_t st[8], const uint8_t* p, uint64_t nblocks) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st));        // A B C D
    __m128i cdgh = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st + 4));  // E F G H
    t = _mm_shuffle_epi32(t, 0xB1);                                             // B A D C
    cdgh = _mm_shuffle_epi32(cdgh, 0x1B);                                       // H G F E
    __m128i abef = _mm_alignr_epi8(t, cdgh, 8);                                 // F E B A
    cdgh = _mm_blend_epi16(cdgh, t, 0xF0);                                      // H G D C
    for (; nblocks; --nblocks, p += 64) {
        const __m128i abef0 = abef, cdgh0 = cdgh;
        __m128i m0 = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p)), bswap);
        __m128i m1 = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16)), bswap);
        __m128i m2 = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 32)), bswap);
        __m128i m3 = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 48)), bswap);
        RF_NI_ROUNDS(m0, 0);
        RF_NI_ROUNDS(m1, 1);
        RF_NI_ROUNDS(m2, 2);
        RF_NI_ROUNDS(m3, 3);
        for (int g = 4; g < 16; g += 4) {
            RF_NI_SCHED(m0, m1, m2, m3);
            RF_NI_ROUNDS(m0, g);
            RF_NI_SCHED(m1, m2, m3, m0);
            RF_NI_ROUNDS(m1, g + 1);
            RF_NI_SCHED(m2, m3, m0, m1);
            RF_NI_ROUNDS(m2, g + 2);
            RF_NI_SCHED(m3, m0, m1, m2);
            RF_NI_ROUNDS(m3, g + 3);
        }
        abef = _mm_add_epi32(abef, abef0);
        cdgh = _mm_add_epi32(cdgh, cdgh0);
    }
    t = _mm_shuffle_epi32(abef, 0x1B);         // A B E F
    cdgh = _mm_shuffle_epi32(cdgh, 0xB1);      // G H C D
    abef = _mm_blend_epi16(t, cdgh, 0xF0);     // A B C D
    cdgh = _mm_alignr_epi8(cdgh, t, 8);        // E F G H
    _mm_storeu_si128(reinterpret_cast<__m128i*>(st), abef);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(st + 4), cdgh);
}

#undef RF_NI_ROUNDS
#undef RF_NI_SCHED

// N interleaved chains: the same rounds and schedule as ni_blocks, each
// statement issued for every chain before the next, so N independent
// sha256rnds2 are in flight.  State kept in locals (written back once):
// through the caller's memory every round would add store-forwarding latency.
template <int N>
__attribute__((target("sha,sse4.1,ssse3"))) void ni_multi(uint32_t* const* st, const uint8_t* const* p,
                                                         uint64_t nblocks) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    __m128i abef[N], cdgh[N];
    const uint8_t* q[N];
#pragma GCC unroll 4
    for (int i = 0; i < N; ++i) {
        __m128i t = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(st[i])), 0xB1);
        __m128i c = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(st[i] + 4)), 0x1B);
        abef[i] = _mm_alignr_epi8(t, c, 8);
        cdgh[i] = _mm_blend_epi16(c, t, 0xF0);
        q[i] = p[i];
    }
    for (uint64_t b = 0; b < nblocks; ++b) {
        __m128i a0[N], c0[N], m[N][4];
#pragma GCC unroll 4
        for (int i = 0; i < N; ++i) {
            a0[i] = abef[i];
            c0[i] = cdgh[i];
#pragma GCC unroll 4
            for (int j = 0; j < 4; ++j)
                m[i][j] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(q[i] + 64 * b + 16 * j)),
                                           bswap);
        }
#pragma GCC unroll 16
        for (int g = 0; g < 16; ++g) {
#pragma GCC unroll 4
            for (int i = 0; i < N; ++i) {
                if (g >= 4) {
                    __m128i& x = m[i][g & 3];
                    x = _mm_sha256msg2_epu32(
                        _mm_add_epi32(_mm_sha256msg1_epu32(x, m[i][(g + 1) & 3]),
                                      _mm_alignr_epi8(m[i][(g + 3) & 3], m[i][(g + 2) & 3], 4)),
                        m[i][(g + 3) & 3]);
                }
                __m128i kw = _mm_add_epi32(m[i][g & 3], _mm_load_si128(reinterpret_cast<const __m128i*>(&kK[4 * g])));
                cdgh[i] = _mm_sha256rnds2_epu32(cdgh[i], abef[i], kw);
                kw = _mm_shuffle_epi32(kw, 0x0E);
                abef[i] = _mm_sha256rnds2_epu32(abef[i], cdgh[i], kw);
            }
        }
#pragma GCC unroll 4
        for (int i = 0; i < N; ++i) {
            abef[i] = _mm_add_epi32(abef[i], a0[i]);
            cdgh[i] = _mm_add_epi32(cdgh[i], c0[i]);
        }
    }
#pragma GCC unroll 4
    for (int i = 0; i < N; ++i) {
        const __m128i t = _mm_shuffle_epi32(abef[i], 0x1B);
        const __m128i c = _mm_shuffle_epi32(cdgh[i], 0xB1);
        _mm_storeu_si128(reinterpret_cast<__m128i*>(st[i]), _mm_blend_epi16(t, c, 0xF0));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(st[i] + 4), _mm_alignr_epi8(c, t, 8));
    }
}

}  // namespace

bool host_sha_available() {
    static const bool ok = [] {
        unsigned a = 0, b = 0, c = 0, d = 0;
        if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
        const bool sse41 = (c >> 19) & 1, ssse3 = (c >> 9) & 1;
        if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
        return sse41 && ssse3 && ((b >> 29) & 1);
    }();
    return ok;
}

void host_sha_init(uint32_t st[8]) { memcpy(st, kIV, sizeof kIV); }

// Portable compression for hosts without the SHA extensions (the host leg is
// then off -- host_sha_available() -- but checkpoint checksums still need it).
static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static void scalar_blocks(uint32_t st[8], const uint8_t* p, uint64_t nblocks) {
    for (; nblocks--; p += 64) {
        uint32_t w[64];
        for (int t = 0; t < 16; ++t)
            w[t] = (uint32_t)p[4 * t] << 24 | (uint32_t)p[4 * t + 1] << 16 | (uint32_t)p[4 * t + 2] << 8 | p[4 * t + 3];
        for (int t = 16; t < 64; ++t) {
            const uint32_t s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
            const uint32_t s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
            w[t] = w[t - 16] + s0 + w[t - 7] + s1;
        }
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
        for (int t = 0; t < 64; ++t) {
            const uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kK[t] + w[t];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            h = g;
            g = f;
            f = e;
            e = d + t1;
            d = c;
            c = b;
            b = a;
            a = t1 + t2;
        }
        st[0] += a;
        st[1] += b;
        st[2] += c;
        st[3] += d;
        st[4] += e;
        st[5] += f;
        st[6] += g;
        st[7] += h;
    }
}

void host_sha_blocks(uint32_t st[8], const uint8_t* p, uint64_t nblocks) {
    if (!nblocks) return;
    if (host_sha_available())
        ni_blocks(st, p, nblocks);
    else
        scalar_blocks(st, p, nblocks);
}

void host_sha_blocks_multi(int n, uint32_t* const* st, const uint8_t* const* p, uint64_t nblocks) {
    if (!nblocks) return;
    if (!host_sha_available()) {
        for (int i = 0; i < n; ++i) scalar_blocks(st[i], p[i], nblocks);
        return;
    }
    switch (n) {
        case 1: ni_blocks(st[0], p[0], nblocks); break;
        case 2: ni_multi<2>(st, p, nblocks); break;
        case 3: ni_multi<3>(st, p, nblocks); break;
        case 4: ni_multi<4>(st, p, nblocks); break;
        default: break;
    }
}

void host_sha_final(uint32_t st[8], const uint8_t* tail, uint64_t tail_len, uint64_t total_len,
                    uint8_t out32[32]) {
    uint8_t buf[128] = {0};
    if (tail_len) memcpy(buf, tail, tail_len);
    buf[tail_len] = 0x80;
    const uint64_t nb = tail_len + 9 <= 64 ? 1 : 2;
    const uint64_t bits = total_len * 8;
    for (int i = 0; i < 8; ++i) buf[64 * nb - 1 - i] = (uint8_t)(bits >> (8 * i));
    ni_blocks(st, buf, nb);
    for (int i = 0; i < 8; ++i) {
        out32[4 * i] = (uint8_t)(st[i] >> 24);
        out32[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out32[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out32[4 * i + 3] = (uint8_t)st[i];
    }
}

void host_sha256(const uint8_t* p, uint64_t len, uint8_t out32[32]) {
    uint32_t st[8];
    host_sha_init(st);
    const uint64_t nb = len / 64;
    host_sha_blocks(st, p, nb);
    host_sha_final(st, p + 64 * nb, len - 64 * nb, len, out32);
}

double host_sha_rate(int ways) {
    static double cache[5] = {-1, -1, -1, -1, -1};
    static std::mutex mu;
    if (ways < 1 || ways > 4) return 0.0;
    std::lock_guard<std::mutex> lk(mu);
    if (cache[ways] >= 0) return cache[ways];
    if (!host_sha_available()) return cache[ways] = 0.0;
    std::vector<uint8_t> buf(8u << 20);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 131u + (i >> 11));
    const uint64_t per = buf.size() / 64 / ways;
    uint32_t st[4][8];
    uint32_t* sp[4] = {st[0], st[1], st[2], st[3]};
    const uint8_t* pp[4];
    for (int i = 0; i < ways; ++i) pp[i] = buf.data() + 64 * per * i;
    double best = 1e30;
    for (int r = 0; r < 3; ++r) {
        for (int i = 0; i < ways; ++i) host_sha_init(st[i]);
        const auto t0 = std::chrono::steady_clock::now();
        host_sha_blocks_multi(ways, sp, pp, per);
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        best = std::min(best, dt);
    }
    volatile uint32_t sink = st[0][0];
    (void)sink;
    return cache[ways] = (double)(64 * per * ways) / best;
}

}  // namespace rf
