// k3_reach.hip -- K3 family: reachability closure over reverse edges.
//
// Eval.dirty (eval.go:874-887): under NoCacheExtern a node is dirty iff it is
// an OpExtern or one of its Deps (transitively) is.  The reference recurses
// per node from Eval.todo (eval.go:910) without a memo -- exponential on a
// DAG with sharing; here every node's answer comes from one closure: seed =
// the OpExtern nodes, then level by level every consumer (reverse dep) of a
// frontier node is marked and appended to the next frontier.  A level is one
// launch; the host loops until a level adds nothing (DAG depth levels).
#include "engine.h"

namespace rf {

// Lane per frontier node; its consumers are visited in wave lockstep so each
// newly marked node is appended with one atomicAdd per wave (ballot + prefix).
__global__ __launch_bounds__(256) void k3_reach_step(const uint32_t* __restrict__ front, uint32_t n_front,
                                                     const uint64_t* __restrict__ cons_ptr,
                                                     const uint32_t* __restrict__ cons, uint32_t* bits,
                                                     uint32_t* __restrict__ next, uint32_t* n_next) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    uint64_t c = 0, ce = 0;
    if (t < n_front) {
        const uint32_t v = front[t];
        c = cons_ptr[v];
        ce = cons_ptr[v + 1];
    }
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    while (__any(c < ce)) {
        bool fresh = false;
        uint32_t k = 0;
        if (c < ce) {
            k = cons[c++];
            const uint32_t m = 1u << (k & 31);
            fresh = !(atomicOr(&bits[k >> 5], m) & m);
        }
        const uint64_t b = __ballot(fresh);
        if (b) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)b) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(n_next, (uint32_t)__popcll(b));
            base = __shfl(base, leader, 64);
            if (fresh) next[base + (uint32_t)__popcll(b & lt)] = k;
        }
    }
}

hipError_t launch_reach_step(const uint32_t* front, uint32_t n_front, const uint64_t* cons_ptr, const uint32_t* cons,
                             uint32_t* bits, uint32_t* next, uint32_t* n_next, hipStream_t s) {
    if (!n_front) return hipSuccess;
    hipLaunchKernelGGL(k3_reach_step, dim3((n_front + 255) / 256), dim3(256), 0, s, front, n_front, cons_ptr, cons,
                       bits, next, n_next);
    return hipGetLastError();
}

}  // namespace rf
