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

// C: issue rate of single VALU opcodes: 8 independent chains per lane, each
// iteration 8 instructions, opcode selected by template (inline asm so the
// compiler keeps the exact instruction).
template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t iters, uint32_t* out) {
    uint32_t r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = threadIdx.x * 7 + j;
    const uint32_t c = blockIdx.x | 1;
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[j]) : "v"(c));
            if constexpr (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[j]));
            if constexpr (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(r[j]) : "v"(c));
            if constexpr (OP == 3) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(r[j]) : "v"(c));
            if constexpr (OP == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[j]) : "v"(c));
            if constexpr (OP == 5) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r[j]) : "v"(c));
            if constexpr (OP == 6) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(r[j]));
            if constexpr (OP == 7) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(r[j]) : "v"(c));
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) x ^= r[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

struct OArgs { int op; uint32_t grid, iters; uint32_t* out; };
static void run_op(void* p) {
    auto* a = (OArgs*)p;
    switch (a->op) {
    case 0: hipLaunchKernelGGL(k_op<0>, dim3(a->grid), dim3(256), 0, 0, a->iters, a->out); break;
    case 1: hipLaunchKernelGGL(k_op<1>, dim3(a->grid), dim3(256), 0, 0, a->iters, a->out); break;
    case 2: hipLaunchKernelGGL(k_op<2>, dim3(a->grid), dim3(256), 0, 0, a->iters, a->out); break;
    case 3: hipLaunchKernelGGL(k_op<3>, dim3(a->grid), dim3(256), 0, 0, a->iters, a->out); break;
    case 4: hipLaunchKernelGGL(k_op<4>, dim3(a->grid), dim3(256), 0, 0, a->iters, a->out); break;
    case 5: hipLaunchKernelGGL(k_op<5>, dim3(a->grid), dim3(256), 0, 0, a->iters, a->out); break;
    case 6: hipLaunchKernelGGL(k_op<6>, dim3(a->grid), dim3(256), 0, 0, a->iters, a->out); break;
    default: hipLaunchKernelGGL(k_op<7>, dim3(a->grid), dim3(256), 0, 0, a->iters, a->out); break;
    }
}

static float time_launch(void (*fn)(void*), void* arg);

extern "C" float micro_op(int op, uint32_t grid, uint32_t iters) {
    uint32_t* out;
    if (hipMalloc(&out, (size_t)grid * 256 * 4) != hipSuccess) return -2.f;
    OArgs a{op, grid, iters, out};
    float ms = time_launch(run_op, &a);
    hipFree(out);
    return ms;
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
