// d2h_probe2.hip -- diagnostic: the K1 plan's launch sequence around the host
// leg, step by step.  Stream S records e0; stream SIDE waits on e0 (variant
// bit 1) and runs a ~1 s spin; 16 threads copy 8 MiB chunks D2H on their own
// streams with event record + hipEventSynchronize, their streams waiting on
// e0 first (variant bit 2); variant bit 4 launches a second short kernel on S.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

__global__ void spin(unsigned long long ticks, int* out) {
    __builtin_amdgcn_s_setprio(3);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int x = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x += threadIdx.x;
    if (x == 12345) out[0] = x;
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int var = argc > 1 ? atoi(argv[1]) : 0;
    const size_t C = 8u << 20;
    const int T = 16, CH = 8;
    void* dsrc;
    int* dout;
    (void)hipMalloc(&dsrc, (size_t)T * CH * C);
    (void)hipMalloc(&dout, 4);
    (void)hipMemset(dsrc, 1, (size_t)T * CH * C);
    hipStream_t S, SIDE;
    (void)hipStreamCreateWithFlags(&S, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&SIDE, hipStreamNonBlocking);
    hipEvent_t e0;
    (void)hipEventCreate(&e0);
    std::vector<hipStream_t> ws(T);
    std::vector<hipEvent_t> we(T);
    std::vector<void*> hb(T);
    for (int t = 0; t < T; ++t) {
        (void)hipStreamCreateWithFlags(&ws[t], hipStreamNonBlocking);
        (void)hipEventCreateWithFlags(&we[t], hipEventDisableTiming);
        (void)hipHostMalloc(&hb[t], C, 0);
    }
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, S);
    if (var & 1) (void)hipStreamWaitEvent(SIDE, e0, 0);
    hipLaunchKernelGGL(spin, dim3(15), dim3(128), 0, SIDE, 100000000ull, dout);
    if (var & 4) hipLaunchKernelGGL(spin, dim3(64), dim3(128), 0, S, 3000000ull, dout);
    const double t0 = now();
    std::vector<double> waited(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            (void)hipSetDevice(0);
            if (var & 2) (void)hipStreamWaitEvent(ws[t], e0, 0);
            for (int c = 0; c < CH; ++c) {
                (void)hipMemcpyAsync(hb[t], (char*)dsrc + ((size_t)t * CH + c) * C, C, hipMemcpyDeviceToHost, ws[t]);
                (void)hipEventRecord(we[t], ws[t]);
                const double a = now();
                (void)hipEventSynchronize(we[t]);
                waited[t] += now() - a;
            }
        });
    for (auto& x : th) x.join();
    const double tc = now() - t0;
    (void)hipStreamSynchronize(SIDE);
    double mx = 0;
    for (double w : waited) mx = mx > w ? mx : w;
    printf("variant %d: copies of %d threads done at %.1f ms (max thread wait %.1f ms), spin done at %.1f ms\n", var, T,
           tc * 1e3, mx * 1e3, (now() - t0) * 1e3);
    return 0;
}
