// host_sha.h -- the planner's host leg: SHA-256 on the host cores with the
// x86 SHA extensions (SHA-NI), internal to libreflow_hip.so.
//
// Why a host leg exists at all (DESIGN.md §5 "K1 hybrid"): SHA-256 is
// Merkle-Damgard, so one file is one strictly serial chain of compressions
// (bit-exactness forbids tree hashing).  A GPU wave runs one chain at
// ~1.1 us/block (issue-bound, ~56 MB/s); a host core with SHA-NI runs it at
// ~40 ns/block (~2.4 GB/s).  The planner (capi.cpp plan_split) therefore gives
// the longest chains of a skewed set to host threads -- the reference's own
// <=60-goroutine digest pool (local/executor.go:41,522-538) -- and keeps the
// many short chains on the GPU kernels, whichever makespan is smaller.
//
// FIPS 180-4 SHA-256, bit-exact with Go crypto/sha256 (reflow.Digester,
// flow.go:36); parity is tested against oracle/ through the C-ABI.
#pragma once
#include <stdint.h>

namespace rf {

// CPUID.(EAX=7,ECX=0):EBX[29] (SHA) and SSE4.1: the host leg needs both.
bool host_sha_available();
void host_sha_init(uint32_t st[8]);
// nblocks whole 64-byte blocks from st (a midstate), no padding.
void host_sha_blocks(uint32_t st[8], const uint8_t* p, uint64_t nblocks);
// n (1..4) independent messages at once: nblocks whole blocks of each, p[i]
// into midstate st[i].  One SHA-NI chain is bound by sha256rnds2's latency
// (32 dependent per block); interleaving n chains fills the pipeline
// (measured on the MI355X box's EPYC 9575F, one core: 2.44 / 3.53 / 4.19 /
// 4.31 GB/s for n = 1..4, tools/shani_ilp.cpp).
void host_sha_blocks_multi(int n, uint32_t* const* st, const uint8_t* const* p, uint64_t nblocks);
// Pads and finishes a message: `tail` holds its last (total_len % 64) bytes
// (tail_len < 64), everything before has gone through host_sha_blocks.
void host_sha_final(uint32_t st[8], const uint8_t* tail, uint64_t tail_len, uint64_t total_len,
                    uint8_t out32[32]);
// One whole message.
void host_sha256(const uint8_t* p, uint64_t len, uint8_t out32[32]);
// Measured bytes/s of one core on this machine with `ways` interleaved
// messages (8 MiB in total, best of 3; cached per ways in 1..4).
double host_sha_rate(int ways = 1);

}  // namespace rf
