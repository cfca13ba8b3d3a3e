// d2h_probe.hip -- diagnostic: do D2H copies on one stream wait for a long
// kernel on another?  A spin kernel (1 workgroup, ~1 s, optional s_setprio 3)
// runs on stream A; meanwhile this thread times 8 MiB D2H copies on stream B
// into pinned memory.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void spin(unsigned long long cycles, int prio, int* out) {
    if (prio) __builtin_amdgcn_s_setprio(3);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int x = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < cycles) x += threadIdx.x;
    if (x == 12345) out[0] = x;
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int prio = argc > 1 ? atoi(argv[1]) : 0;
    const int flags = argc > 2 ? atoi(argv[2]) : 0;  // hipHostMalloc flags
    const int wgs = argc > 3 ? atoi(argv[3]) : 1;
    const size_t C = 8u << 20;
    void *dsrc, *h;
    int* dout;
    hipMalloc(&dsrc, 64 * C);
    hipMalloc(&dout, 4);
    hipMemset(dsrc, 1, 64 * C);
    hipHostMalloc(&h, C, flags);
    hipStream_t a, b;
    hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    // baseline copy rate
    double t0 = now();
    for (int i = 0; i < 16; ++i) hipMemcpyAsync(h, (char*)dsrc + i * C, C, hipMemcpyDeviceToHost, b);
    hipStreamSynchronize(b);
    printf("idle: 16 x 8 MiB D2H %.2f GB/s\n", 16.0 * C / (now() - t0) / 1e9);
    // spin ~1 s of the 100 MHz realtime clock on stream a
    hipLaunchKernelGGL(spin, dim3(wgs), dim3(128), 0, a, 100000000ull, prio, dout);
    t0 = now();
    for (int i = 0; i < 8; ++i) {
        const double c0 = now();
        hipMemcpyAsync(h, (char*)dsrc + i * C, C, hipMemcpyDeviceToHost, b);
        hipStreamSynchronize(b);
        printf("  copy %d during spin: %.2f ms (t=%.1f ms)\n", i, (now() - c0) * 1e3, (now() - t0) * 1e3);
    }
    hipStreamSynchronize(a);
    printf("spin done at %.1f ms (prio %d, host flags %d, %d WGs)\n", (now() - t0) * 1e3, prio, flags, wgs);
    return 0;
}
