// lag_chain.h -- the two-lane lagged SHA-256 round chain as inline-asm
// macros, shared by K1's duo/octo kernels (k1_sha.hip, where the scheme is
// described) and K2's two-lane chain waves (k2_graph.hip, k2_level_pl).
#pragma once

#define RF_LAG_STEP_P(x0, x1, x2, x3, z, zn, k, P1, P2, PART)                              \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[sq]\n\t"                                  \
    "v_xad_u32 %[" zn "], %[" x2 "], %[m], %[" k "]\n\t"                                     \
    "v_bitop3_b32 %[t3], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t"                         \
    "v_xor_b32_dpp %[t1], %[t0], %[t0] " P1 " row_mask:0xf bank_mask:0xf\n\t"                \
    "v_bitop3_b32 %[t3], %[t3], %[" x1 "], %[" x2 "] bitop3:0xca\n\t"                        \
    "v_add_u32_dpp %[" zn "], %[" x0 "], %[" zn "] " PART " row_mask:0xf bank_mask:0xf\n\t"  \
    "v_xor_b32_dpp %[t1], %[t0], %[t1] " P2 " row_mask:0xf bank_mask:0xf\n\t"                \
    "v_add3_u32 %[" x3 "], %[" z "], %[t1], %[t3]\n\t"
#define RF_LAG_STEP(x0, x1, x2, x3, z, zn, k) \
    RF_LAG_STEP_P(x0, x1, x2, x3, z, zn, k, "quad_perm:[1,2,0,3]", "quad_perm:[2,0,1,3]", "row_ror:8")

#define RF_LAG_GROUP                                        \
    RF_LAG_STEP("a", "b", "c", "d", "z", "y", "k1")         \
    RF_LAG_STEP("d", "a", "b", "c", "y", "z", "k2")         \
    RF_LAG_STEP("c", "d", "a", "b", "z", "y", "k3")         \
    RF_LAG_STEP("b", "c", "d", "a", "y", "z", "k4")

// X += H then H = X on the lanes of one half (bank mask 0x3 = e-lanes,
// 0xc = a-lanes); DPP identity only for the bank mask.
#define RF_LAG_FF(bm, x0, x1, x2, x3)                                                                 \
    "v_add_u32_dpp %[" x0 "], %[h0], %[" x0 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t" \
    "v_add_u32_dpp %[" x1 "], %[h1], %[" x1 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t" \
    "v_add_u32_dpp %[" x2 "], %[h2], %[" x2 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t" \
    "v_add_u32_dpp %[" x3 "], %[h3], %[" x3 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t" \
    "v_mov_b32_dpp %[h0], %[" x0 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t"            \
    "v_mov_b32_dpp %[h1], %[" x1 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t"            \
    "v_mov_b32_dpp %[h2], %[" x2 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t"            \
    "v_mov_b32_dpp %[h3], %[" x3 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t"

// H += X on one half (final feed-forward; X stays as it is)
#define RF_LAG_FIN(bm, x0, x1, x2, x3)                                                                \
    "v_add_u32_dpp %[h0], %[h0], %[" x0 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t"     \
    "v_add_u32_dpp %[h1], %[h1], %[" x1 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t"     \
    "v_add_u32_dpp %[h2], %[h2], %[" x2 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t"     \
    "v_add_u32_dpp %[h3], %[h3], %[" x3 "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" bm "\n\t"

#define RF_LAG_STATE [a] "+v"(Pa), [b] "+v"(Pb), [c] "+v"(Pc), [d] "+v"(Pd), [z] "+v"(Z), [y] "+v"(Y)
#define RF_LAG_TMP [t0] "=&v"(t0), [t1] "=&v"(t1), [t3] "=&v"(t3)
#define RF_LAG_H [h0] "+v"(Hr0), [h1] "+v"(Hr1), [h2] "+v"(Hr2), [h3] "+v"(Hr3)
#define RF_LAG_IN(k1v, k2v, k3v, k4v) \
    [sq] "v"(shq), [m] "v"(M), [k1] "v"(k1v), [k2] "v"(k2v), [k3] "v"(k3v), [k4] "v"(k4v)

namespace lag {
constexpr uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                            0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
}  // namespace lag

// Block-boundary corrections for the next boundary, from this block's
// chaining value H (both halves have applied it by the end of group 0):
//   c63: Z of the e-lanes' next round 0 = h + d + (K+W added at block start)
//        e: H7 + H3     a: 1
//   c64: e: + H2 (the partner's d is not fed forward yet)   a: - H4
//   c65: e: + H1                                            a: - H3
// (v_subrev_u32_dpp does not permute the operand one would expect; the
// negation goes through a temporary and a plain DPP move, t0 being free after
// the group's last step.)
#define RF_LAG_CORR_P(PART, BE, BA)                                                            \
    "v_sub_u32 %[t0], %[zero], %[h0]\n\t"                                                      \
    "v_add_u32_dpp %[c63], %[h3], %[h3] " PART " row_mask:0xf bank_mask:0xf\n\t"               \
    "v_mov_b32_dpp %[c63], %[one] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" BA "\n\t"       \
    "v_mov_b32_dpp %[c64], %[h2] " PART " row_mask:0xf bank_mask:" BE "\n\t"                   \
    "v_mov_b32_dpp %[c64], %[t0] " PART " row_mask:0xf bank_mask:" BA "\n\t"                   \
    "v_mov_b32_dpp %[c65], %[h1] " PART " row_mask:0xf bank_mask:" BE "\n\t"                   \
    "v_sub_u32_dpp %[c65], %[zero], %[h3] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:" BA "\n\t"
#define RF_LAG_CORR RF_LAG_CORR_P("row_ror:8", "0x3", "0xc")

// Two-lane form without the quad: every lane rotates X0 by all three Σ
// amounts of its half itself (per-lane shift registers s1..s3) and xors them
// (one v_bitop3), so a job needs only its e-lane and a-lane: 9 VALU per round
// and 32 jobs per wave.  The a-lane of the e-lane at half-row position i is
// position 7 - i (row_half_mirror), e-lanes sit in banks 0/2 (bank mask 0x5),
// a-lanes in banks 1/3 (0xa) -- the octo kernel's layout.
#define RF_L2_STEP(x0, x1, x2, x3, z, zn, k)                                                  \
    "v_alignbit_b32 %[t0], %[" x0 "], %[" x0 "], %[s1]\n\t"                                   \
    "v_alignbit_b32 %[t1], %[" x0 "], %[" x0 "], %[s2]\n\t"                                   \
    "v_xad_u32 %[" zn "], %[" x2 "], %[m], %[" k "]\n\t"                                      \
    "v_alignbit_b32 %[t2], %[" x0 "], %[" x0 "], %[s3]\n\t"                                   \
    "v_bitop3_b32 %[t3], %[" x0 "], %[" x2 "], %[m] bitop3:0x78\n\t"                          \
    "v_bitop3_b32 %[t1], %[t0], %[t1], %[t2] bitop3:0x96\n\t"                                 \
    "v_bitop3_b32 %[t3], %[t3], %[" x1 "], %[" x2 "] bitop3:0xca\n\t"                         \
    "v_add_u32_dpp %[" zn "], %[" x0 "], %[" zn "] row_half_mirror row_mask:0xf bank_mask:0xf\n\t" \
    "v_add3_u32 %[" x3 "], %[" z "], %[t1], %[t3]\n\t"

#define RF_L2_GROUP                                \
    RF_L2_STEP("a", "b", "c", "d", "z", "y", "k1") \
    RF_L2_STEP("d", "a", "b", "c", "y", "z", "k2") \
    RF_L2_STEP("c", "d", "a", "b", "z", "y", "k3") \
    RF_L2_STEP("b", "c", "d", "a", "y", "z", "k4")

#define RF_L2_GROUP0                                  \
    "s_nop 1\n\t" RF_LAG_FF("0x5", "a", "b", "c", "d") \
    "v_add_u32 %[z], %[z], %[kw0]\n\t"               \
    RF_L2_STEP("a", "b", "c", "d", "z", "y", "k1")    \
    RF_L2_STEP("d", "a", "b", "c", "y", "z", "k2")    \
    RF_LAG_FF("0xa", "c", "d", "a", "b")              \
    RF_L2_STEP("c", "d", "a", "b", "z", "y", "k3")    \
    RF_L2_STEP("b", "c", "d", "a", "y", "z", "k4")    \
    RF_LAG_CORR_P("row_half_mirror", "0x5", "0xa")

#define RF_L2_TMP [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
#define RF_L2_IN(k1v, k2v, k3v, k4v) \
    [s1] "v"(sh1), [s2] "v"(sh2), [s3] "v"(sh3), [m] "v"(M), [k1] "v"(k1v), [k2] "v"(k2v), [k3] "v"(k3v), [k4] "v"(k4v)

// The octo layout (k1_sha256_octo, k2_level_oct): eight jobs per wave, lanes
// 8f..8f+3 the e-half of job f, 8f+4..8f+7 its a-half; every lane of a quad
// ends a round with the full sigma (positions 0..2 rotate by the half's three
// amounts, position 3 repeats position 0's), the partner's X0 from the
// mirrored lane of the half-row, the halves' feed-forwards by banks 0x5 / 0xa.
#define RF_OCT_STEP(x0, x1, x2, x3, z, zn, k) \
    RF_LAG_STEP_P(x0, x1, x2, x3, z, zn, k, "quad_perm:[1,2,0,1]", "quad_perm:[2,0,1,2]", "row_half_mirror")
#define RF_OCT_GROUP                                        \
    RF_OCT_STEP("a", "b", "c", "d", "z", "y", "k1")         \
    RF_OCT_STEP("d", "a", "b", "c", "y", "z", "k2")         \
    RF_OCT_STEP("c", "d", "a", "b", "z", "y", "k3")         \
    RF_OCT_STEP("b", "c", "d", "a", "y", "z", "k4")
#define RF_OCT_GROUP0                                        \
    "s_nop 1\n\t" RF_LAG_FF("0x5", "a", "b", "c", "d")       \
    "v_add_u32 %[z], %[z], %[kw0]\n\t"                       \
    RF_OCT_STEP("a", "b", "c", "d", "z", "y", "k1")          \
    RF_OCT_STEP("d", "a", "b", "c", "y", "z", "k2")          \
    RF_LAG_FF("0xa", "c", "d", "a", "b")                     \
    RF_OCT_STEP("c", "d", "a", "b", "z", "y", "k3")          \
    RF_OCT_STEP("b", "c", "d", "a", "y", "z", "k4")          \
    RF_LAG_CORR_P("row_half_mirror", "0x5", "0xa")
