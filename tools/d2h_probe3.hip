// d2h_probe3.hip -- diagnostic: 16 threads copy 8 MiB chunks D2H while a ~1 s
// kernel runs on another stream.  mode 0: own HIP stream + event + blocking
// hipEventSynchronize; 1: the same, polling hipEventQuery; 2: own stream +
// hipStreamSynchronize; 3: one shared HIP stream per 8 threads; 4: ROCr
// hsa_amd_memory_async_copy (SDMA, no HIP stream) + an HSA signal per thread.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sched.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
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

static hsa_agent_t g_gpu, g_cpu;
static hsa_status_t find(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const size_t C = 8u << 20;
    const int T = 16, CH = 8;
    void* dsrc;
    int* dout;
    (void)hipMalloc(&dsrc, (size_t)T * CH * C);
    (void)hipMalloc(&dout, 4);
    (void)hipMemset(dsrc, 1, (size_t)T * CH * C);
    hipStream_t SIDE;
    (void)hipStreamCreateWithFlags(&SIDE, hipStreamNonBlocking);
    std::vector<hipStream_t> ws(T);
    std::vector<hipEvent_t> we(T);
    std::vector<void*> hb(T);
    std::vector<hsa_signal_t> sig(T);
    if (mode == 4) {
        hsa_init();
        hsa_iterate_agents(find, nullptr);
    }
    for (int t = 0; t < T; ++t) {
        if (mode != 3 || t < 2) (void)hipStreamCreateWithFlags(&ws[t], hipStreamNonBlocking);
        (void)hipEventCreateWithFlags(&we[t], hipEventDisableTiming);
        (void)hipHostMalloc(&hb[t], C, 0);
        if (mode == 4) hsa_signal_create(1, 0, nullptr, &sig[t]);
    }
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(spin, dim3(15), dim3(128), 0, SIDE, 100000000ull, dout);
    const double t0 = now();
    std::vector<double> waited(T, 0);
    std::vector<std::thread> th;
    std::mutex m3[2];
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            (void)hipSetDevice(0);
            for (int c = 0; c < CH; ++c) {
                char* src = (char*)dsrc + ((size_t)t * CH + c) * C;
                const double a = now();
                if (mode == 4) {
                    hsa_signal_store_relaxed(sig[t], 1);
                    hsa_amd_memory_async_copy(hb[t], g_cpu, src, g_gpu, C, 0, nullptr, sig[t]);
                    hsa_signal_wait_scacquire(sig[t], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
                } else if (mode == 3) {
                    std::lock_guard<std::mutex> lk(m3[t & 1]);
                    (void)hipMemcpyAsync(hb[t], src, C, hipMemcpyDeviceToHost, ws[t & 1]);
                    (void)hipStreamSynchronize(ws[t & 1]);
                } else {
                    (void)hipMemcpyAsync(hb[t], src, C, hipMemcpyDeviceToHost, ws[t]);
                    if (mode == 2) {
                        (void)hipStreamSynchronize(ws[t]);
                    } else {
                        (void)hipEventRecord(we[t], ws[t]);
                        if (mode == 1)
                            while (hipEventQuery(we[t]) == hipErrorNotReady) sched_yield();
                        else
                            (void)hipEventSynchronize(we[t]);
                    }
                }
                waited[t] += now() - a;
            }
        });
    for (auto& x : th) x.join();
    const double tc = now() - t0;
    (void)hipStreamSynchronize(SIDE);
    double mx = 0, mn = 1e9;
    for (double w : waited) {
        mx = mx > w ? mx : w;
        mn = mn < w ? mn : w;
    }
    printf("mode %d: %d threads x %d copies done at %.1f ms (thread wait min %.1f max %.1f ms), spin done at %.1f ms\n",
           mode, T, CH, tc * 1e3, mn * 1e3, mx * 1e3, (now() - t0) * 1e3);
    return 0;
}
