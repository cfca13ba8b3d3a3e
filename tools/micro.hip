// micro.hip -- diagnostic microbenchmarks for K1 (not part of the product).
// Built by tools/micro.py into tools/_micro.so; one C entry per experiment,
// each returns the kernel time in ms (hipEvents) or a negative value.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../reflow_amd/csrc/sha256_dev.h"

using namespace rf;

// A: VALU only -- every lane compresses nblk blocks of register data.
__global__ __launch_bounds__(256) void k_compute(uint32_t nblk, uint32_t* out) {
    ShaState st;
    st.init();
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = threadIdx.x * 16 + j;
    for (uint32_t b = 0; b < nblk; ++b) {
        uint32_t x[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = w[j] ^ st.h[j & 7];
        sha256_compress(st, x);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = st.h[0] ^ st.h[7];
}

// B: lane-per-message with static assignment; message g at g*stride.
// layout 0: contiguous per message; layout 1: interleaved 64-B blocks
// (block b of lane g at (b*nlanes + g)*64).
__global__ __launch_bounds__(256) void k_loads(const uint8_t* arena, uint64_t stride, uint32_t nblk,
                                               uint32_t nlanes, int layout, int prefetch,
                                               uint32_t* out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nlanes) return;
    ShaState st;
    st.init();
    auto addr = [&](uint32_t b) -> const uint4* {
        if (layout == 0) return reinterpret_cast<const uint4*>(arena + g * stride + (uint64_t)b * 64);
        return reinterpret_cast<const uint4*>(arena + ((uint64_t)b * nlanes + g) * 64);
    };
    uint4 n0, n1, n2, n3;
    {
        const uint4* q = addr(0);
        n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3];
    }
    for (uint32_t b = 0; b < nblk; ++b) {
        const uint4 r0 = n0, r1 = n1, r2 = n2, r3 = n3;
        if (prefetch && b + 1 < nblk) {
            const uint4* q = addr(b + 1);
            n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3];
        }
        uint32_t w[16] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w,
                          r2.x, r2.y, r2.z, r2.w, r3.x, r3.y, r3.z, r3.w};
        sha256_compress(st, w);
        if (!prefetch && b + 1 < nblk) {
            const uint4* q = addr(b + 1);
            n0 = q[0]; n1 = q[1]; n2 = q[2]; n3 = q[3];
        }
    }
    out[g] = st.h[0];
}

static float time_launch(void (*fn)(void*), void* arg) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    fn(arg);  // warm
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    fn(arg);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    if (hipGetLastError() != hipSuccess) return -1.f;
    return ms;
}

struct CArgs { uint32_t grid, nblk; uint32_t* out; };
static void run_compute(void* p) {
    auto* a = (CArgs*)p;
    hipLaunchKernelGGL(k_compute, dim3(a->grid), dim3(256), 0, 0, a->nblk, a->out);
}

extern "C" float micro_compute(uint32_t grid, uint32_t nblk) {
    uint32_t* out;
    if (hipMalloc(&out, (size_t)grid * 256 * 4) != hipSuccess) return -2.f;
    CArgs a{grid, nblk, out};
    float ms = time_launch(run_compute, &a);
    hipFree(out);
    return ms;
}

struct LArgs { const uint8_t* arena; uint64_t stride; uint32_t nblk, nlanes; int layout, prefetch; uint32_t* out; };
static void run_loads(void* p) {
    auto* a = (LArgs*)p;
    hipLaunchKernelGGL(k_loads, dim3((a->nlanes + 255) / 256), dim3(256), 0, 0, a->arena, a->stride,
                       a->nblk, a->nlanes, a->layout, a->prefetch, a->out);
}

extern "C" float micro_loads(uint64_t stride, uint32_t nblk, uint32_t nlanes, int layout, int prefetch) {
    uint64_t bytes = layout == 0 ? (uint64_t)nlanes * stride + (uint64_t)nblk * 64 + 64
                                 : (uint64_t)nblk * nlanes * 64 + 64;
    uint8_t* arena;
    uint32_t* out;
    if (hipMalloc(&arena, bytes) != hipSuccess) return -2.f;
    if (hipMalloc(&out, (size_t)nlanes * 4) != hipSuccess) return -2.f;
    hipMemset(arena, 1, bytes);
    LArgs a{arena, stride, nblk, nlanes, layout, prefetch, out};
    float ms = time_launch(run_loads, &a);
    hipFree(arena);
    hipFree(out);
    return ms;
}
