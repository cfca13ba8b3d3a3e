// k4_bloom.hip -- K4: batched bloomlive / assoc probe and build.
//
// Replaces bloomlive.T.Contains (/root/reference/internal/bloomlive/bloomlive.go:30-36)
// -> bloom.Test (vendor/github.com/willf/bloom/bloom.go:182-190) -> baseHashes
// (:94-104, murmur3 x64_128 seed 0, vendor/github.com/spaolacci/murmur3/
// murmur128.go:56-171) -> location (:107-115) -> bitset.Test
// (vendor/github.com/willf/bitset/bitset.go:143-149); and the build side
// bloom.Add (:144-150) used by eval.go:848-858.
//
// Key = WD(d) = 00 05 || d (34 bytes).  (h1,h2) = mm3(key), (h3,h4) =
// mm3(key || 0x01): both share the two 16-byte body blocks, so the body is
// mixed once and finalised twice.  loc_i = (h[i%2] + i*h[2+((i+i%2)%4)/2])
// mod m with an exact 64-bit Barrett reduction.  One lane per probe.
#include "engine.h"

namespace rf {

constexpr uint64_t kC1 = 0x87c37b91114253d5ull, kC2 = 0x4cf5ad432745937full;

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// Base hashes of WD(d) for a digest given as four little-endian u64 words.
__device__ __forceinline__ void base_hashes_wd(const uint64_t (&D)[4], uint64_t (&h)[4]) {
    const uint64_t key0 = 0x0500ull | (D[0] << 16);
    const uint64_t key1 = (D[0] >> 48) | (D[1] << 16);
    const uint64_t key2 = (D[1] >> 48) | (D[2] << 16);
    const uint64_t key3 = (D[2] >> 48) | (D[3] << 16);
    const uint64_t tail = D[3] >> 48;  // bytes d30 d31
    uint64_t h1 = 0, h2 = 0;
    const uint64_t ks[4] = {key0, key1, key2, key3};
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        uint64_t k1 = ks[2 * b], k2 = ks[2 * b + 1];
        k1 *= kC1; k1 = rotl64(k1, 31); k1 *= kC2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= kC2; k2 = rotl64(k2, 33); k2 *= kC1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        // tail of 2 bytes (len 34) or 3 bytes (len 35: || 0x01); k2 part empty
        uint64_t k1 = f == 0 ? tail : (tail | (1ull << 16));
        const uint64_t len = f == 0 ? 34 : 35;
        uint64_t a = h1, b = h2;
        k1 *= kC1; k1 = rotl64(k1, 31); k1 *= kC2; a ^= k1;
        a ^= len; b ^= len;
        a += b; b += a;
        a = fmix64(a); b = fmix64(b);
        a += b; b += a;
        h[2 * f] = a;
        h[2 * f + 1] = b;
    }
}

// x mod m, exact: mu = floor((2^64-1)/m) from the host; q underestimates
// floor(x/m) by at most 2.
__device__ __forceinline__ uint64_t mod_m(uint64_t x, uint64_t m, uint64_t mu) {
    const uint64_t q = __umul64hi(x, mu);
    uint64_t r = x - q * m;
    if (r >= m) r -= m;
    if (r >= m) r -= m;
    return r;
}

__device__ __forceinline__ uint64_t bloom_loc(const uint64_t (&h)[4], uint32_t i) {
    const uint64_t ii = i;
    return h[ii % 2] + ii * h[2 + (((ii + (ii % 2)) % 4) / 2)];
}

__device__ __forceinline__ void load_digest64(const uint8_t* d, uint64_t (&D)[4]) {
    const ulonglong2* p = reinterpret_cast<const ulonglong2*>(d);
    const ulonglong2 a = p[0], b = p[1];
    D[0] = a.x; D[1] = a.y; D[2] = b.x; D[3] = b.y;
}


// Fetch schedule: the k words are requested C at a time, and a key stops at
// the first chunk that holds a clear bit (bloom.Test's early exit, batched for
// memory-level parallelism).  The probe is bound by random 8-B gathers (one
// 64-B line each, ~55 G/s on MI355X, tools/micro.py gather), so the fewer
// words an absent key fetches, the faster; a present key always fetches k.
template <int C>
__global__ __launch_bounds__(256) void k4_bloom_probe(const uint64_t* __restrict__ words,
                                                      const uint64_t* __restrict__ len_dev,
                                                      uint64_t m, uint64_t mu, uint32_t k,
                                                      const uint8_t* __restrict__ d32, uint64_t n,
                                                      uint8_t* __restrict__ out) {
    const uint64_t length = *len_dev;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t D[4], h[4];
        load_digest64(d32 + 32 * i, D);
        base_hashes_wd(D, h);
        bool hit = true;
        for (uint32_t j0 = 0; j0 < k && hit; j0 += C) {
            uint64_t loc[C], w[C];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint32_t j = j0 + c;
                loc[c] = j < k ? mod_m(bloom_loc(h, j), m, mu) : 0;
                if (j < k && loc[c] >= length) hit = false;
            }
#pragma unroll
            for (int c = 0; c < C; ++c) w[c] = (hit && j0 + c < k) ? words[loc[c] >> 6] : ~0ull;
#pragma unroll
            for (int c = 0; c < C; ++c) hit = hit && ((w[c] >> (loc[c] & 63)) & 1ull);
        }
        out[i] = hit ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void k4_bloom_add(unsigned long long* __restrict__ words,
                                                    unsigned long long* __restrict__ len_dev,
                                                    uint64_t m, uint64_t mu, uint32_t k,
                                                    const uint8_t* __restrict__ d32, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t D[4], h[4];
        load_digest64(d32 + 32 * i, D);
        base_hashes_wd(D, h);
        uint64_t maxloc = 0;
        for (uint32_t j = 0; j < k; ++j) {
            const uint64_t loc = mod_m(bloom_loc(h, j), m, mu);
            atomicOr(&words[loc >> 6], 1ull << (loc & 63));
            maxloc = loc > maxloc ? loc : maxloc;
        }
        // bitset.Set grows length to loc+1 when loc >= length (bitset.go:151-156)
        atomicMax(len_dev, (unsigned long long)(maxloc + 1));
    }
}

// ---------------------------------------------------------------------------
// Repository.Collect (repository/file/repository.go:304-327): every object
// whose digest the liveset does not contain is removed.  Batched over n
// objects in three launches: (1) probe one tile of kTile objects per block,
// write a dead flag per object and the tile's dead count and bytes; (2) one
// block scans the tile counts; (3) each tile writes its dead indices at its
// scanned offset, in ascending order (the reference removes in walk order).
constexpr uint32_t kCollectBlock = 256, kCollectPer = 16, kTile = kCollectBlock * kCollectPer;

__device__ __forceinline__ bool bloom_contains(const uint64_t* __restrict__ words, uint64_t length,
                                               uint64_t m, uint64_t mu, uint32_t k, const uint8_t* d) {
    uint64_t D[4], h[4];
    load_digest64(d, D);
    base_hashes_wd(D, h);
    for (uint32_t j = 0; j < k; ++j) {
        const uint64_t loc = mod_m(bloom_loc(h, j), m, mu);
        if (loc >= length || !((words[loc >> 6] >> (loc & 63)) & 1ull)) return false;
    }
    return true;
}

__global__ __launch_bounds__(kCollectBlock) void k4_collect_mark(
    const uint64_t* __restrict__ words, const uint64_t* __restrict__ len_dev, uint64_t m, uint64_t mu,
    uint32_t k, const uint8_t* __restrict__ d32, const int64_t* __restrict__ sizes, uint64_t n,
    uint8_t* __restrict__ dead, uint32_t* __restrict__ tile_count, unsigned long long* __restrict__ bytes) {
    __shared__ uint32_t s_cnt[kCollectBlock / 64];
    __shared__ long long s_bytes[kCollectBlock / 64];
    const uint64_t length = *len_dev;
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    uint32_t cnt = 0;
    long long by = 0;
#pragma unroll 4
    for (uint32_t j = 0; j < kCollectPer; ++j) {
        const uint64_t i = base + (uint64_t)j * kCollectBlock + threadIdx.x;
        if (i < n) {
            const bool d = !bloom_contains(words, length, m, mu, k, d32 + 32 * i);
            dead[i] = d;
            cnt += d;
            if (d && sizes) by += sizes[i];
        }
    }
    // wave sums, then the block's
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_xor(cnt, o, 64);
        by += __shfl_xor(by, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        s_cnt[threadIdx.x >> 6] = cnt;
        s_bytes[threadIdx.x >> 6] = by;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t c = 0;
        long long b = 0;
        for (uint32_t w = 0; w < kCollectBlock / 64; ++w) {
            c += s_cnt[w];
            b += s_bytes[w];
        }
        tile_count[blockIdx.x] = c;
        if (b) atomicAdd(bytes, (unsigned long long)b);  // two's complement sum
    }
}

// Exclusive scan of the tile counts by one block, 1024 coalesced counts per
// pass (wave scans by shuffles, wave totals through LDS, a running carry);
// total -> *n_dead.
__global__ __launch_bounds__(1024) void k4_collect_scan(uint32_t* __restrict__ tile_count, uint64_t tiles,
                                                        unsigned long long* __restrict__ n_dead) {
    __shared__ uint32_t s_w[16];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long carry = 0;
    for (uint64_t b = 0; b < tiles; b += 1024) {
        const uint64_t t = b + threadIdx.x;
        const uint32_t c = t < tiles ? tile_count[t] : 0u;
        uint32_t x = c;  // inclusive wave scan
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) s_w[wave] = x;
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (uint32_t w = 0; w < 16; ++w) {
            before += w < wave ? s_w[w] : 0u;
            total += s_w[w];
        }
        if (t < tiles) tile_count[t] = (uint32_t)(carry + before + x - c);  // < 2^32: n < 2^32
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) *n_dead = carry;
}

__global__ __launch_bounds__(kCollectBlock) void k4_collect_scatter(const uint8_t* __restrict__ dead,
                                                                    const uint32_t* __restrict__ tile_off,
                                                                    uint64_t n, uint64_t* __restrict__ out) {
    __shared__ uint32_t s_w[kCollectBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint64_t run = tile_off[blockIdx.x];
    for (uint32_t j = 0; j < kCollectPer; ++j) {
        const uint64_t i = base + (uint64_t)j * kCollectBlock + threadIdx.x;
        const bool d = i < n && dead[i];
        const uint64_t bal = __ballot(d);
        if (lane == 0) s_w[wave] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (uint32_t w = 0; w < kCollectBlock / 64; ++w) {
            before += w < wave ? s_w[w] : 0;
            total += s_w[w];
        }
        if (d) out[run + before + (uint32_t)__popcll(bal & lt)] = i;
        run += total;
        __syncthreads();
    }
}

static uint64_t barrett_mu(uint64_t m) { return m ? (~0ull) / m : 0; }

hipError_t launch_bloom_collect(const BloomDev& b, const uint8_t* d32, const int64_t* sizes, uint64_t n,
                                uint8_t* dead, uint32_t* tile_count, uint64_t* out_idx,
                                uint64_t* n_dead_bytes2, hipStream_t s) {
    // n_dead_bytes2 = {n_dead, dead_bytes}, zeroed by the caller
    if (!n) return hipSuccess;
    const uint64_t tiles = (n + kTile - 1) / kTile;
    auto* nb = reinterpret_cast<unsigned long long*>(n_dead_bytes2);
    hipLaunchKernelGGL(k4_collect_mark, dim3((uint32_t)tiles), dim3(kCollectBlock), 0, s, b.words,
                       b.len_dev, b.m, barrett_mu(b.m), (uint32_t)b.k, d32, sizes, n, dead, tile_count,
                       nb + 1);
    hipLaunchKernelGGL(k4_collect_scan, dim3(1), dim3(1024), 0, s, tile_count, tiles, nb);
    hipLaunchKernelGGL(k4_collect_scatter, dim3((uint32_t)tiles), dim3(kCollectBlock), 0, s, dead,
                       tile_count, n, out_idx);
    return hipGetLastError();
}

uint64_t bloom_collect_tiles(uint64_t n) { return (n + kTile - 1) / kTile; }

static uint32_t grid_for(uint64_t items) {
    uint64_t g = (items + 255) / 256;
    if (g < 1) g = 1;
    if (g > 16384) g = 16384;
    return (uint32_t)g;
}

hipError_t launch_bloom_probe(const BloomDev& b, const uint8_t* d32, uint64_t n, uint8_t* out,
                              hipStream_t s) {
    if (!n) return hipSuccess;
    // one word at a time (tools/probe_sweep.py on MI355X, 1e9 probes, 1e8-key
    // filter: C=1 111.6 ms, 2: 117.0, 3: 123.8, 4: 131.0, all 10: 183.6)
    hipLaunchKernelGGL(k4_bloom_probe<1>, dim3(grid_for(n)), dim3(256), 0, s, b.words, b.len_dev, b.m,
                       barrett_mu(b.m), (uint32_t)b.k, d32, n, out);
    return hipGetLastError();
}

hipError_t launch_bloom_add(const BloomDev& b, const uint8_t* d32, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k4_bloom_add, dim3(grid_for(n)), dim3(256), 0, s,
                       reinterpret_cast<unsigned long long*>(b.words),
                       reinterpret_cast<unsigned long long*>(b.len_dev), b.m, barrett_mu(b.m),
                       (uint32_t)b.k, d32, n);
    return hipGetLastError();
}

}  // namespace rf
