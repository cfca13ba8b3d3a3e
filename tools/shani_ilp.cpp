// shani_ilp.cpp -- diagnostic: SHA-NI blocks/s of one core with 1, 2 and 3
// independent messages interleaved (sha256rnds2 is latency-bound on a single
// chain: 32 dependent rnds2 per block).  Built with g++, host only.
#include <immintrin.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

alignas(16) static const uint32_t K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

template <int N>
__attribute__((target("sha,sse4.1,ssse3"))) void blocks(__m128i (&abef_io)[N], __m128i (&cdgh_io)[N],
                                                       const uint8_t* const (&p)[N], uint64_t nb) {
    __m128i abef[N], cdgh[N];
    for (int i = 0; i < N; ++i) {
        abef[i] = abef_io[i];
        cdgh[i] = cdgh_io[i];
    }
    const __m128i bs = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    for (uint64_t b = 0; b < nb; ++b) {
        __m128i a0[N], c0[N], m[N][4];
#pragma GCC unroll 4
        for (int i = 0; i < N; ++i) {
            a0[i] = abef[i];
            c0[i] = cdgh[i];
            for (int j = 0; j < 4; ++j)
                m[i][j] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p[i] + 64 * b + 16 * j)), bs);
        }
#pragma GCC unroll 16
        for (int g = 0; g < 16; ++g) {
#pragma GCC unroll 4
            for (int i = 0; i < N; ++i) {
                if (g >= 4) {
                    __m128i& x = m[i][g & 3];
                    x = _mm_sha256msg2_epu32(_mm_add_epi32(_mm_sha256msg1_epu32(x, m[i][(g + 1) & 3]),
                                                           _mm_alignr_epi8(m[i][(g + 3) & 3], m[i][(g + 2) & 3], 4)),
                                             m[i][(g + 3) & 3]);
                }
                __m128i kw = _mm_add_epi32(m[i][g & 3], _mm_load_si128((const __m128i*)&K[4 * g]));
                cdgh[i] = _mm_sha256rnds2_epu32(cdgh[i], abef[i], kw);
                kw = _mm_shuffle_epi32(kw, 0x0E);
                abef[i] = _mm_sha256rnds2_epu32(abef[i], cdgh[i], kw);
            }
        }
        for (int i = 0; i < N; ++i) {
            abef[i] = _mm_add_epi32(abef[i], a0[i]);
            cdgh[i] = _mm_add_epi32(cdgh[i], c0[i]);
        }
    }
    for (int i = 0; i < N; ++i) {
        abef_io[i] = abef[i];
        cdgh_io[i] = cdgh[i];
    }
}

template <int N>
double rate(const std::vector<uint8_t>& buf) {
    __m128i abef[N], cdgh[N];
    const uint8_t* p[N];
    const uint64_t per = buf.size() / N / 64;
    for (int i = 0; i < N; ++i) {
        abef[i] = _mm_set1_epi32(i + 1);
        cdgh[i] = _mm_set1_epi32(i + 7);
        p[i] = buf.data() + i * per * 64;
    }
    double best = 1e9;
    for (int r = 0; r < 5; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        blocks<N>(abef, cdgh, p, per);
        best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    volatile int sink = _mm_cvtsi128_si32(abef[0]);
    (void)sink;
    return per * 64.0 * N / best / 1e9;
}

int main() {
    std::vector<uint8_t> buf(48u << 20, 7);
    printf("1-way %.2f GB/s\n2-way %.2f GB/s\n3-way %.2f GB/s\n4-way %.2f GB/s\n", rate<1>(buf), rate<2>(buf),
           rate<3>(buf), rate<4>(buf));
}
