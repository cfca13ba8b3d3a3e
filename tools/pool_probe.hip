// Does hipMemsetAsync clear memory that hipMallocAsync hands out again after
// a hipFreeAsync on the same stream?  (diagnostic for the dedup stall)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void check(const unsigned* p, size_t n, unsigned want, unsigned long long* bad) {
    unsigned long long b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != want;
    if (b) atomicAdd(bad, b);
}
__global__ void scribble(unsigned* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (unsigned)i;
}

int main() {
    hipMemPool_t pool;
    hipDeviceGetDefaultMemPool(&pool, 0);
    unsigned long long thr = ~0ull;
    hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    unsigned long long* bad;
    hipMalloc(&bad, 8);
    const size_t n1 = 1u << 25, n2 = 10000000;
    for (int it = 0; it < 4; ++it) {
        void *a = nullptr, *b = nullptr;
        hipMallocAsync(&a, 4 * n1, s);
        hipMallocAsync(&b, 4 * n2, s);
        hipError_t e = hipMemsetAsync(a, 0xff, 4 * n1, s);
        hipMemsetAsync(bad, 0, 8, s);
        hipLaunchKernelGGL(check, dim3(1024), dim3(256), 0, s, (const unsigned*)a, n1, 0xffffffffu, bad);
        hipLaunchKernelGGL(scribble, dim3(1024), dim3(256), 0, s, (unsigned*)a, n1);
        hipLaunchKernelGGL(scribble, dim3(1024), dim3(256), 0, s, (unsigned*)b, n2);
        unsigned long long h = 0;
        hipMemcpyAsync(&h, bad, 8, hipMemcpyDeviceToHost, s);
        hipFreeAsync(b, s);
        hipFreeAsync(a, s);
        hipError_t e2 = hipStreamSynchronize(s);
        printf("iter %d: a=%p b=%p memset=%s sync=%s words not cleared: %llu\n", it, a, b, hipGetErrorString(e),
               hipGetErrorString(e2), h);
    }
    return 0;
}
