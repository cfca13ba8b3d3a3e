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

#define RF_E " row_ror:8 row_mask:0xf bank_mask:0x3"
#define RF_Q " quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x3"
#define RF_A " row_ror:8 row_mask:0xf bank_mask:0xc"
#define MDUO(x0, x1, x2, x3, sfx, e, q, aa)                                          \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[s1]\n\t"                          \
    "v_alignbit_b32 %[t1], %[" x0 "], %[" x0 "], %[s2]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" x0 "], %[" x0 "], %[s3]\n\t"                          \
    "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"                        \
    "v_bitop3_b32 %[t1], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t"                 \
    "v_bitop3_b32 %[t1], %[t1], %[" x1 "], %[" x2 "] bitop3:0xca\n\t"                \
    "v_add3_u32 %[t2], %[z], %[t0], %[t1]\n\t"                                       \
    "v_add_u32" sfx " %[" x3 "], %[" x3 "], %[t2]" e "\n\t"                          \
    "v_add_u32" sfx " %[z], %[" x2 "], %[k]" q "\n\t"                                \
    "v_add_u32" sfx " %[" x3 "], %[t2], %[t2]" aa "\n\t"

// lag-2 duo step: a-lanes run two rounds behind the e-lanes, so the
// cross-lane value is one step old and no instruction depends on the one
// right before it (9 VALU per round).
#define LAG2(x0, x1, x2, x3, z, zn)                                                 \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[s1]\n\t"                          \
    "v_alignbit_b32 %[t1], %[" x0 "], %[" x0 "], %[s2]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" x0 "], %[" x0 "], %[s3]\n\t"                          \
    "v_bitop3_b32 %[t3], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t"                 \
    "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"                        \
    "v_bitop3_b32 %[t3], %[t3], %[" x1 "], %[" x2 "] bitop3:0xca\n\t"                \
    "v_xad_u32 %[" zn "], %[" x2 "], %[m], %[k]\n\t"                                 \
    "v_add3_u32 %[" x3 "], %[" z "], %[t0], %[t3]\n\t"                               \
    "v_add_u32_dpp %[" zn "], %[" x0 "], %[" zn "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"

// orderings of the lag-2 step (OP 18..22)
#define LAGV1(x0, x1, x2, x3, z, zn) \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[s1]\n\t" \
    "v_bitop3_b32 %[t3], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t" \
    "v_alignbit_b32 %[t1], %[" x0 "], %[" x0 "], %[s2]\n\t" \
    "v_xad_u32 %[" zn "], %[" x2 "], %[m], %[k]\n\t" \
    "v_alignbit_b32 %[t2], %[" x0 "], %[" x0 "], %[s3]\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[" x1 "], %[" x2 "] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t" \
    "v_add_u32_dpp %[" zn "], %[" x0 "], %[" zn "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t" \
    "v_add3_u32 %[" x3 "], %[" z "], %[t0], %[t3]\n\t"

#define LAGV5(x0, x1, x2, x3, z, zn) \
    "v_xad_u32 %[" zn "], %[" x2 "], %[m], %[k]\n\t" \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[s1]\n\t" \
    "v_bitop3_b32 %[t3], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t" \
    "v_alignbit_b32 %[t1], %[" x0 "], %[" x0 "], %[s2]\n\t" \
    "v_alignbit_b32 %[t2], %[" x0 "], %[" x0 "], %[s3]\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[" x1 "], %[" x2 "] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t" \
    "v_add_u32_dpp %[" zn "], %[" x0 "], %[" zn "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t" \
    "v_add3_u32 %[" x3 "], %[" z "], %[t0], %[t3]\n\t"

#define LAGV6(x0, x1, x2, x3, z, zn) \
    "v_xad_u32 %[" zn "], %[" x2 "], %[m], %[k]\n\t" \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[s1]\n\t" \
    "v_bitop3_b32 %[t3], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t" \
    "v_alignbit_b32 %[t1], %[" x0 "], %[" x0 "], %[s2]\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[" x1 "], %[" x2 "] bitop3:0xca\n\t" \
    "v_alignbit_b32 %[t2], %[" x0 "], %[" x0 "], %[s3]\n\t" \
    "v_add_u32_dpp %[" zn "], %[" x0 "], %[" zn "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t" \
    "v_add3_u32 %[" x3 "], %[" z "], %[t0], %[t3]\n\t"

#define LAGV7(x0, x1, x2, x3, z, zn) \
    "v_xad_u32 %[" zn "], %[" x2 "], %[m], %[k]\n\t" \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[s1]\n\t" \
    "v_alignbit_b32 %[t1], %[" x0 "], %[" x0 "], %[s2]\n\t" \
    "v_bitop3_b32 %[t3], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t" \
    "v_alignbit_b32 %[t2], %[" x0 "], %[" x0 "], %[s3]\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[" x1 "], %[" x2 "] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t" \
    "v_add_u32_dpp %[" zn "], %[" x0 "], %[" zn "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t" \
    "v_add3_u32 %[" x3 "], %[" z "], %[t0], %[t3]\n\t"

#define LAGV8(x0, x1, x2, x3, z, zn) \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[s1]\n\t" \
    "v_alignbit_b32 %[t1], %[" x0 "], %[" x0 "], %[s2]\n\t" \
    "v_alignbit_b32 %[t2], %[" x0 "], %[" x0 "], %[s3]\n\t" \
    "v_bitop3_b32 %[t3], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t" \
    "v_xad_u32 %[" zn "], %[" x2 "], %[m], %[k]\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[" x1 "], %[" x2 "] bitop3:0xca\n\t" \
    "v_add_u32_dpp %[" zn "], %[" x0 "], %[" zn "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t" \
    "v_add3_u32 %[" x3 "], %[" z "], %[t0], %[t3]\n\t"

// issue cost per instruction type: 64 independent instructions (8 chains)
#define ICOST23(n) "v_alignbit_b32 %[r" n "], %[r" n "], %[r" n "], %[c]\n\t"
#define ICOST24(n) "v_alignbit_b32 %[r" n "], %[r" n "], %[r" n "], 7\n\t"
#define ICOST25(n) "v_bitop3_b32 %[r" n "], %[r" n "], %[c], %[e] bitop3:0x96\n\t"
#define ICOST26(n) "v_add3_u32 %[r" n "], %[r" n "], %[c], %[e]\n\t"
#define ICOST27(n) "v_xad_u32 %[r" n "], %[r" n "], %[c], %[e]\n\t"
#define ICOST28(n) "v_add_u32 %[r" n "], %[r" n "], %[c]\n\t"
#define ICOST29(n) "v_add_u32_dpp %[r" n "], %[c], %[r" n "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
#define ICOST30(n) "v_xor_b32 %[r" n "], %[r" n "], %[c]\n\t"
#define ICOST31(n) "v_add_u32_e64 %[r" n "], %[r" n "], %[c]\n\t"
#define ICOST32(n) "v_lshl_add_u32 %[r" n "], %[r" n "], 3, %[c]\n\t"
#define ICOST33(n) "v_add_u32 %[r" n "], %[r" n "], %[r" n "]\n\t"
#define ICOST34(n) "v_bitop3_b32 %[r" n "], %[r" n "], %[r" n "], %[c] bitop3:0x96\n\t"
#define ICOST35(n) "v_mov_b32 %[r" n "], %[c]\n\t"
#define SADD8 "s_add_u32 %[s0], %[s0], %[sc]\n\t" "s_add_u32 %[s1], %[s1], %[sc]\n\t" "s_add_u32 %[s2], %[s2], %[sc]\n\t" "s_add_u32 %[s3], %[s3], %[sc]\n\t" \
              "s_add_u32 %[s4], %[s4], %[sc]\n\t" "s_add_u32 %[s5], %[s5], %[sc]\n\t" "s_add_u32 %[s6], %[s6], %[sc]\n\t" "s_add_u32 %[s7], %[s7], %[sc]\n\t"
#define VS_MIX(n) "v_add_u32 %[r" n "], %[r" n "], %[c]\n\t" "s_add_u32 %[s" n "], %[s" n "], %[sc]\n\t"
#define VS_MIX3(n) "v_bitop3_b32 %[r" n "], %[r" n "], %[c], %[e] bitop3:0x96\n\t" "s_add_u32 %[s" n "], %[s" n "], %[sc]\n\t"
#define S8 [s0] "+s"(sq[0]), [s1] "+s"(sq[1]), [s2] "+s"(sq[2]), [s3] "+s"(sq[3]), [s4] "+s"(sq[4]), \
           [s5] "+s"(sq[5]), [s6] "+s"(sq[6]), [s7] "+s"(sq[7])
// D: single-wave latency: one dependent chain per lane (grid 1 x 64), so
// the time per instruction is the issue-to-dependent-issue latency.  OP 8/9
// run the duo round (10 instructions) with DPP / with plain adds.
template <int OP>
__global__ __launch_bounds__(64) void k_lat(uint32_t iters, uint32_t* out, uint64_t* cyc) {
    uint32_t r = threadIdx.x * 7 + 1, x1 = r * 3, x2 = r * 5, x3 = r * 9, z = r & 8 ? 0 : r;
    const uint32_t c = blockIdx.x | 1, s1 = threadIdx.x & 8 ? 2 : 6, s2 = threadIdx.x & 8 ? 13 : 11,
                   s3 = threadIdx.x & 8 ? 22 : 25, m = threadIdx.x & 8 ? ~0u : 0u;
    uint32_t t0, t1, t2, t3 = 0, zy = r;
    uint32_t q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = r + j;
    uint32_t sq[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sq[j] = __builtin_amdgcn_readfirstlane(iters + j);
    const uint32_t sc = __builtin_amdgcn_readfirstlane(iters * 3);
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j == 0) {
#define X8(i) i "\n\t" i "\n\t" i "\n\t" i "\n\t" i "\n\t" i "\n\t" i "\n\t" i "\n\t"
                if constexpr (OP == 0) asm volatile(X8("v_add_u32 %0, %0, %1") : "+v"(r) : "v"(c));
                if constexpr (OP == 1) asm volatile(X8("v_alignbit_b32 %0, %0, %0, 7") : "+v"(r));
                if constexpr (OP == 2) asm volatile(X8("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96") : "+v"(r) : "v"(c));
                if constexpr (OP == 3) asm volatile(X8("v_add3_u32 %0, %0, %1, %1") : "+v"(r) : "v"(c));
                if constexpr (OP == 4)
                    asm volatile(X8("v_add_u32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf") : "+v"(r) : "v"(c));
                if constexpr (OP == 5)
                    asm volatile(X8("v_add_u32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0x3") : "+v"(r) : "v"(c));
                if constexpr (OP == 6) asm volatile(X8("v_add_u32 %0, %1, %1") : "=v"(t0) : "v"(c));  // independent
                if constexpr (OP == 7) asm volatile(X8("v_add_u32 %0, %0, %1\n\ts_nop 0") : "+v"(r) : "v"(c));
#undef X8
            }
            if (OP == 8 && (j & 3) == 0)
                asm volatile(MDUO("a", "b", "c", "d", "_dpp", RF_E, RF_Q, RF_A)
                             MDUO("d", "a", "b", "c", "_dpp", RF_E, RF_Q, RF_A)
                             MDUO("c", "d", "a", "b", "_dpp", RF_E, RF_Q, RF_A)
                             MDUO("b", "c", "d", "a", "_dpp", RF_E, RF_Q, RF_A)
                             : [a] "+v"(r), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [z] "+v"(z),
                               [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
                             : [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [m] "v"(m), [k] "v"(c));
            if (OP == 9 && (j & 3) == 0)
                asm volatile(MDUO("a", "b", "c", "d", "", "", "", "")
                             MDUO("d", "a", "b", "c", "", "", "", "")
                             MDUO("c", "d", "a", "b", "", "", "", "")
                             MDUO("b", "c", "d", "a", "", "", "", "")
                             : [a] "+v"(r), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [z] "+v"(z),
                               [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
                             : [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [m] "v"(m), [k] "v"(c));
            if constexpr (OP >= 11 && OP <= 17) {
                if (j == 0) {
#define I8(ins) ins("0") ins("1") ins("2") ins("3") ins("4") ins("5") ins("6") ins("7")
#define IALIGN(n) "v_alignbit_b32 %[r" n "], %[r" n "], %[r" n "], 7\n\t"
#define IADD(n) "v_add_u32 %[r" n "], %[r" n "], %[c]\n\t"
#define IBOP(n) "v_bitop3_b32 %[r" n "], %[r" n "], %[c], %[e] bitop3:0x96\n\t"
#define IDPP(n) "v_add_u32_dpp %[r" n "], %[c], %[r" n "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
#define IBOPS(n) "v_bitop3_b32 %[r" n "], %[r" n "], %[r" n "], %[c] bitop3:0x96\n\t"
#define R8 [r0] "+v"(q[0]), [r1] "+v"(q[1]), [r2] "+v"(q[2]), [r3] "+v"(q[3]), [r4] "+v"(q[4]), \
           [r5] "+v"(q[5]), [r6] "+v"(q[6]), [r7] "+v"(q[7])
                    if constexpr (OP == 11) asm volatile(I8(IALIGN) : R8);
                    if constexpr (OP == 12) asm volatile(I8(IADD) : R8 : [c] "v"(c));
                    if constexpr (OP == 13) asm volatile(I8(IBOP) : R8 : [c] "v"(c), [e] "v"(s1));
                    if constexpr (OP == 14) asm volatile(I8(IDPP) : R8 : [c] "v"(c));
                    if constexpr (OP == 15) asm volatile(I8(IBOPS) : R8 : [c] "v"(c));
                    // explicit registers: c in bank 1, e in bank 2, r in banks 0/3 (16)
                    // or r in bank 1 with c (17)
                    if constexpr (OP == 16)
                        asm volatile(I8(IBOP) : [r0] "+{v40}"(q[0]), [r1] "+{v43}"(q[1]), [r2] "+{v44}"(q[2]),
                                     [r3] "+{v47}"(q[3]), [r4] "+{v48}"(q[4]), [r5] "+{v51}"(q[5]),
                                     [r6] "+{v52}"(q[6]), [r7] "+{v55}"(q[7])
                                     : [c] "{v61}"(c), [e] "{v62}"(s1));
                    if constexpr (OP == 17)
                        asm volatile(I8(IBOP) : [r0] "+{v41}"(q[0]), [r1] "+{v45}"(q[1]), [r2] "+{v49}"(q[2]),
                                     [r3] "+{v53}"(q[3]), [r4] "+{v57}"(q[4]), [r5] "+{v65}"(q[5]),
                                     [r6] "+{v69}"(q[6]), [r7] "+{v73}"(q[7])
                                     : [c] "{v61}"(c), [e] "{v62}"(s1));
                }
            }
            if (OP == 18 && (j & 3) == 0)
                asm volatile(LAGV1("a", "b", "c", "d", "z", "y") LAGV1("d", "a", "b", "c", "y", "z")
                             LAGV1("c", "d", "a", "b", "z", "y") LAGV1("b", "c", "d", "a", "y", "z")
                             : [a] "+v"(r), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [z] "+v"(z),
                               [y] "+v"(zy), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
                             : [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [m] "v"(m), [k] "v"(c));
            if (OP == 19 && (j & 3) == 0)
                asm volatile(LAGV5("a", "b", "c", "d", "z", "y") LAGV5("d", "a", "b", "c", "y", "z")
                             LAGV5("c", "d", "a", "b", "z", "y") LAGV5("b", "c", "d", "a", "y", "z")
                             : [a] "+v"(r), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [z] "+v"(z),
                               [y] "+v"(zy), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
                             : [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [m] "v"(m), [k] "v"(c));
            if (OP == 20 && (j & 3) == 0)
                asm volatile(LAGV6("a", "b", "c", "d", "z", "y") LAGV6("d", "a", "b", "c", "y", "z")
                             LAGV6("c", "d", "a", "b", "z", "y") LAGV6("b", "c", "d", "a", "y", "z")
                             : [a] "+v"(r), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [z] "+v"(z),
                               [y] "+v"(zy), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
                             : [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [m] "v"(m), [k] "v"(c));
            if (OP == 21 && (j & 3) == 0)
                asm volatile(LAGV7("a", "b", "c", "d", "z", "y") LAGV7("d", "a", "b", "c", "y", "z")
                             LAGV7("c", "d", "a", "b", "z", "y") LAGV7("b", "c", "d", "a", "y", "z")
                             : [a] "+v"(r), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [z] "+v"(z),
                               [y] "+v"(zy), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
                             : [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [m] "v"(m), [k] "v"(c));
            if (OP == 22 && (j & 3) == 0)
                asm volatile(LAGV8("a", "b", "c", "d", "z", "y") LAGV8("d", "a", "b", "c", "y", "z")
                             LAGV8("c", "d", "a", "b", "z", "y") LAGV8("b", "c", "d", "a", "y", "z")
                             : [a] "+v"(r), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [z] "+v"(z),
                               [y] "+v"(zy), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
                             : [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [m] "v"(m), [k] "v"(c));
            if constexpr (OP == 23)
                if (j == 0) asm volatile(I8(ICOST23) I8(ICOST23) I8(ICOST23) I8(ICOST23) I8(ICOST23) I8(ICOST23) I8(ICOST23) I8(ICOST23) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 24)
                if (j == 0) asm volatile(I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 25)
                if (j == 0) asm volatile(I8(ICOST25) I8(ICOST25) I8(ICOST25) I8(ICOST25) I8(ICOST25) I8(ICOST25) I8(ICOST25) I8(ICOST25) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 26)
                if (j == 0) asm volatile(I8(ICOST26) I8(ICOST26) I8(ICOST26) I8(ICOST26) I8(ICOST26) I8(ICOST26) I8(ICOST26) I8(ICOST26) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 27)
                if (j == 0) asm volatile(I8(ICOST27) I8(ICOST27) I8(ICOST27) I8(ICOST27) I8(ICOST27) I8(ICOST27) I8(ICOST27) I8(ICOST27) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 28)
                if (j == 0) asm volatile(I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 29)
                if (j == 0) asm volatile(I8(ICOST29) I8(ICOST29) I8(ICOST29) I8(ICOST29) I8(ICOST29) I8(ICOST29) I8(ICOST29) I8(ICOST29) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 30)
                if (j == 0) asm volatile(I8(ICOST30) I8(ICOST30) I8(ICOST30) I8(ICOST30) I8(ICOST30) I8(ICOST30) I8(ICOST30) I8(ICOST30) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 31)
                if (j == 0) asm volatile(I8(ICOST31) I8(ICOST31) I8(ICOST31) I8(ICOST31) I8(ICOST31) I8(ICOST31) I8(ICOST31) I8(ICOST31) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 32)
                if (j == 0) asm volatile(I8(ICOST32) I8(ICOST32) I8(ICOST32) I8(ICOST32) I8(ICOST32) I8(ICOST32) I8(ICOST32) I8(ICOST32) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 33)
                if (j == 0) asm volatile(I8(ICOST33) I8(ICOST33) I8(ICOST33) I8(ICOST33) I8(ICOST33) I8(ICOST33) I8(ICOST33) I8(ICOST33) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 34)
                if (j == 0) asm volatile(I8(ICOST34) I8(ICOST34) I8(ICOST34) I8(ICOST34) I8(ICOST34) I8(ICOST34) I8(ICOST34) I8(ICOST34) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 35)
                if (j == 0) asm volatile(I8(ICOST35) I8(ICOST35) I8(ICOST35) I8(ICOST35) I8(ICOST35) I8(ICOST35) I8(ICOST35) I8(ICOST35) : R8 : [c] "v"(c), [e] "v"(s1));
            if constexpr (OP == 36)
                if (j == 0) asm volatile(SADD8 SADD8 SADD8 SADD8 SADD8 SADD8 SADD8 SADD8 : S8 : [sc] "s"(sc) : "scc");
            if constexpr (OP == 37)
                if (j == 0) asm volatile(I8(VS_MIX) I8(VS_MIX) I8(VS_MIX) I8(VS_MIX) I8(VS_MIX) I8(VS_MIX) I8(VS_MIX) I8(VS_MIX)
                                         : R8, S8 : [c] "v"(c), [sc] "s"(sc) : "scc");
            if constexpr (OP == 38)
                if (j == 0) asm volatile(I8(VS_MIX3) I8(VS_MIX3) I8(VS_MIX3) I8(VS_MIX3) I8(VS_MIX3) I8(VS_MIX3) I8(VS_MIX3) I8(VS_MIX3)
                                         : R8, S8 : [c] "v"(c), [e] "v"(s1), [sc] "s"(sc) : "scc");
            // EXEC-masked copies of cost v_add vop2 / cost alignbit imm: does a
            // wave with only lanes 0..15 (or lane 0) active issue faster?
            if constexpr (OP == 39 || OP == 40 || OP == 41 || OP == 42) {
                if (j == 0 && threadIdx.x < ((OP == 39 || OP == 41) ? 16u : 1u)) {
                    if constexpr (OP == 39 || OP == 40)
                        asm volatile(I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) I8(ICOST28) : R8 : [c] "v"(c), [e] "v"(s1));
                    else
                        asm volatile(I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) I8(ICOST24) : R8 : [c] "v"(c), [e] "v"(s1));
                }
            }
            if (OP == 10 && (j & 3) == 0)
                asm volatile(LAG2("a", "b", "c", "d", "z", "y") LAG2("d", "a", "b", "c", "y", "z")
                             LAG2("c", "d", "a", "b", "z", "y") LAG2("b", "c", "d", "a", "y", "z")
                             : [a] "+v"(r), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [z] "+v"(z),
                               [y] "+v"(zy), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
                             : [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [m] "v"(m), [k] "v"(c));
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = sq[0] ^ sq[1] ^ sq[2] ^ sq[3] ^ sq[4] ^ sq[5] ^ sq[6] ^ sq[7] ^ r ^ x1 ^ x2 ^ x3 ^ z ^ t0 ^ zy ^ t3 ^ q[0] ^ q[1] ^ q[2] ^ q[3] ^ q[4] ^ q[5] ^ q[6] ^ q[7];
    if (threadIdx.x == 0) *cyc = c1 - c0;
}

struct LtArgs { int op; uint32_t iters; uint32_t* out; uint64_t* cyc; };
static void run_lat(void* p) {
    auto* a = (LtArgs*)p;
#define RF_LAT(N) case N: hipLaunchKernelGGL(k_lat<N>, dim3(1), dim3(64), 0, 0, a->iters, a->out, a->cyc); break;
    switch (a->op) { RF_LAT(0) RF_LAT(1) RF_LAT(2) RF_LAT(3) RF_LAT(4) RF_LAT(5) RF_LAT(6) RF_LAT(7) RF_LAT(8) RF_LAT(9) RF_LAT(10) RF_LAT(11) RF_LAT(12) RF_LAT(13) RF_LAT(14) RF_LAT(15) RF_LAT(16) RF_LAT(17) RF_LAT(18) RF_LAT(19) RF_LAT(20) RF_LAT(21) RF_LAT(22) RF_LAT(23) RF_LAT(24) RF_LAT(25) RF_LAT(26) RF_LAT(27) RF_LAT(28) RF_LAT(29) RF_LAT(30) RF_LAT(31) RF_LAT(32) RF_LAT(33) RF_LAT(34) RF_LAT(35) RF_LAT(36) RF_LAT(37) RF_LAT(38) RF_LAT(39) RF_LAT(40) RF_LAT(41) default: RF_LAT(42) }
#undef RF_LAT
}

static float time_launch(void (*fn)(void*), void* arg);

// Returns ms; *cycles = s_memtime delta of the timed launch.
extern "C" float micro_lat(int op, uint32_t iters, uint64_t* cycles) {
    uint32_t* out;
    uint64_t* cyc;
    if (hipMalloc(&out, 64 * 4) != hipSuccess || hipMalloc(&cyc, 8) != hipSuccess) return -2.f;
    LtArgs a{op, iters, out, cyc};
    float ms = time_launch(run_lat, &a);
    hipMemcpy(cycles, cyc, 8, hipMemcpyDeviceToHost);
    hipFree(out);
    hipFree(cyc);
    return ms;
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

// ---------------------------------------------------------------------------
// G: random 8-B gather ceiling (the K4 probe's access pattern without the
// hashing): each thread reads R words at pseudo-random positions of a table
// of nwords u64, all R requested before any is used (like the probe's
// phase 2), and streams a 32-B key per thread from `keys` (nt or default).
__device__ __forceinline__ uint64_t gmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

template <int R>
__global__ __launch_bounds__(256) void k_gather(const uint64_t* __restrict__ table, uint64_t nwords,
                                                const uint4* __restrict__ keys, int key_mode, uint64_t n,
                                                uint8_t* __restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t seed = i;
        if (key_mode == 1) {
            const uint4 a = keys[2 * i], b = keys[2 * i + 1];
            seed ^= ((uint64_t)a.x << 32 | a.y) ^ b.z;
        } else if (key_mode == 2) {
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            const v4u* kv = reinterpret_cast<const v4u*>(keys);
            const v4u a = __builtin_nontemporal_load(&kv[2 * i]);
            const v4u b = __builtin_nontemporal_load(&kv[2 * i + 1]);
            seed ^= ((uint64_t)a.x << 32 | a.y) ^ b.z;
        }
        uint64_t w[R];
#pragma unroll
        for (int j = 0; j < R; ++j) w[j] = table[__umul64hi(gmix(seed * R + j), nwords)];
        uint64_t acc = 0;
#pragma unroll
        for (int j = 0; j < R; ++j) acc ^= w[j];
        out[i] = (uint8_t)(acc & 1);
    }
}

struct GArgs { const uint64_t* table; uint64_t nwords; const uint4* keys; int key_mode; uint64_t n; uint8_t* out; int r; };
static void run_gather(void* p) {
    auto* a = (GArgs*)p;
    uint64_t g = (a->n + 255) / 256;
    if (g > 16384) g = 16384;
    if (a->r == 2)
        hipLaunchKernelGGL(k_gather<2>, dim3((uint32_t)g), dim3(256), 0, 0, a->table, a->nwords, a->keys, a->key_mode, a->n, a->out);
    else if (a->r == 6)
        hipLaunchKernelGGL(k_gather<6>, dim3((uint32_t)g), dim3(256), 0, 0, a->table, a->nwords, a->keys, a->key_mode, a->n, a->out);
    else
        hipLaunchKernelGGL(k_gather<10>, dim3((uint32_t)g), dim3(256), 0, 0, a->table, a->nwords, a->keys, a->key_mode, a->n, a->out);
}

// Returns ms for n threads x r gathers from a table of table_bytes.
extern "C" float micro_gather(uint64_t table_bytes, uint64_t n, int r, int key_mode) {
    uint64_t* table;
    uint4* keys = nullptr;
    uint8_t* out;
    if (hipMalloc(&table, table_bytes) != hipSuccess) return -2.f;
    if (hipMalloc(&out, n) != hipSuccess) return -2.f;
    if (key_mode && hipMalloc(&keys, 32 * n) != hipSuccess) return -2.f;
    hipMemset(table, 0x5a, table_bytes);
    if (keys) hipMemset(keys, 0x33, 32 * n);
    GArgs a{table, table_bytes / 8, keys, key_mode, n, out, r};
    float ms = time_launch(run_gather, &a);
    hipFree(table);
    hipFree(out);
    if (keys) hipFree(keys);
    return ms;
}

// ---------------------------------------------------------------------------
// Wave placement: which SIMD each wave of a workgroup lands on (HW_ID
// register, SIMD_ID = bits [5:4] on gfx9), and the CU id (bits [11:8]).
__global__ void k_hwid(uint32_t* out) {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = hw;
}

extern "C" int micro_hwid(uint32_t grid, uint32_t block, uint32_t* host_out) {
    uint32_t* d = nullptr;
    const size_t n = (size_t)grid * (block / 64);
    if (hipMalloc(&d, 4 * n) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_hwid, dim3(grid), dim3(block), 0, 0, d);
    hipMemcpy(host_out, d, 4 * n, hipMemcpyDeviceToHost);
    hipFree(d);
    return 0;
}

// ---------------------------------------------------------------------------
// Workgroup barrier cost: `iters` __syncthreads() in a loop, nothing else.
__global__ void k_barrier(uint32_t iters, uint32_t* sink) {
    uint32_t x = threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i) {
        x = x * 1664525u + 1013904223u;
        __syncthreads();
    }
    if (x == 0x12345678u) sink[0] = x;
}

// Same with a raw s_barrier (no fence).
__global__ void k_barrier_raw(uint32_t iters, uint32_t* sink) {
    uint32_t x = threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i) {
        x = x * 1664525u + 1013904223u;
        __builtin_amdgcn_s_barrier();
    }
    if (x == 0x12345678u) sink[0] = x;
}

extern "C" float micro_barrier(uint32_t grid, uint32_t block, uint32_t iters, int raw) {
    uint32_t* d = nullptr;
    hipMalloc(&d, 64);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    if (raw) hipLaunchKernelGGL(k_barrier_raw, dim3(grid), dim3(block), 0, 0, iters, d);
    else hipLaunchKernelGGL(k_barrier, dim3(grid), dim3(block), 0, 0, iters, d);
    hipEventRecord(a, 0);
    if (raw) hipLaunchKernelGGL(k_barrier_raw, dim3(grid), dim3(block), 0, 0, iters, d);
    else hipLaunchKernelGGL(k_barrier, dim3(grid), dim3(block), 0, 0, iters, d);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipFree(d);
    return ms;
}

// ---------------------------------------------------------------------------
// Same-address atomic contention (the level lists' append cursors): `waves`
// 64-lane workgroups, each spins `work` dependent VALU iterations (so the
// waves arrive together, as the mark kernel's do after their chains), then
// lane 0 issues one atomicAdd to counter (wave % n_addr), counters 256 B
// apart; n_addr = 0: no atomic (the baseline).
__global__ __launch_bounds__(64) void k_atomic(uint32_t work, uint32_t n_addr, uint32_t* ctr, uint32_t* sink) {
    uint32_t x = threadIdx.x + blockIdx.x;
    for (uint32_t i = 0; i < work; ++i) x = x * 1664525u + 1013904223u;
    if (n_addr && threadIdx.x == 0) x += atomicAdd(&ctr[64u * (blockIdx.x % n_addr)], 1u);
    if (x == 0x12345678u) sink[0] = x;
}

struct AArgs { uint32_t waves, work, n_addr; uint32_t *ctr, *sink; };
static void run_atomic(void* p) {
    auto* a = (AArgs*)p;
    hipLaunchKernelGGL(k_atomic, dim3(a->waves), dim3(64), 0, 0, a->work, a->n_addr, a->ctr, a->sink);
}

extern "C" float micro_atomic(uint32_t waves, uint32_t work, uint32_t n_addr) {
    uint32_t *ctr, *sink;
    if (hipMalloc(&ctr, 256 * 4096) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return -2.f;
    hipMemset(ctr, 0, 256 * 4096);
    AArgs a{waves, work, n_addr > 4096 ? 4096u : n_addr, ctr, sink};
    float ms = time_launch(run_atomic, &a);
    hipFree(ctr);
    hipFree(sink);
    return ms;
}
