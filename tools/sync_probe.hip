// sync_probe.hip -- development microbenchmark (not part of the product): how
// long the host takes to see a stream's work finish, per device scheduling flag.
// usage: sync_probe FLAGS WHEN   FLAGS: -1 = leave the default, else the
// hipSetDeviceFlags value (1 spin, 2 yield, 4 blocking sync); WHEN: pre (before
// any other HIP call) or post (after the runtime is up, as under torch).
// Prints one JSON line: median / mean host microseconds of
//   empty       launch of an empty kernel + hipStreamSynchronize
//   busy50      a 50 us single-wave spin kernel + hipStreamSynchronize, minus 50
//   chain6      six dependent empty kernels + hipStreamSynchronize
//   devsync     empty kernel + hipDeviceSynchronize
// build: hipcc --offload-arch=gfx950 -O3 tools/sync_probe.hip -o tools/sync_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

__global__ void k_empty() {}

__global__ void k_busy(long long cycles) {  // s_memtime runs at 100 MHz on gfx9
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < cycles) {
    }
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));      \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
static void measure(const char* name, F f, double minus, bool last) {
    std::vector<double> t;
    for (int i = 0; i < 50; ++i) f();
    for (int i = 0; i < 1000; ++i) {
        const double a = now_us();
        f();
        t.push_back(now_us() - a - minus);
    }
    std::sort(t.begin(), t.end());
    double m = 0;
    for (double x : t) m += x;
    printf("\"%s\": {\"median_us\": %.2f, \"mean_us\": %.2f, \"p10_us\": %.2f}%s", name, t[t.size() / 2], m / t.size(),
           t[t.size() / 10], last ? "" : ", ");
}

int main(int argc, char** argv) {
    const int flags = argc > 1 ? atoi(argv[1]) : -1;
    const bool pre = argc > 2 ? strcmp(argv[2], "pre") == 0 : true;
    hipError_t fe = hipSuccess;
    if (flags >= 0 && pre) fe = hipSetDeviceFlags((unsigned)flags);
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    if (flags >= 0 && !pre) fe = hipSetDeviceFlags((unsigned)flags);
    unsigned got = 0;
    CK(hipGetDeviceFlags(&got));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    printf("{\"flags\": %d, \"when\": \"%s\", \"set_rc\": %d, \"device_flags\": %u, ", flags, pre ? "pre" : "post",
           (int)fe, got);
    measure("empty", [&] {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        CK(hipStreamSynchronize(st));
    }, 0.0, false);
    measure("busy50", [&] {
        hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, st, 5000LL);
        CK(hipStreamSynchronize(st));
    }, 50.0, false);
    measure("chain6", [&] {
        for (int i = 0; i < 6; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        CK(hipStreamSynchronize(st));
    }, 0.0, false);
    measure("devsync", [&] {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        CK(hipDeviceSynchronize());
    }, 0.0, true);
    printf("}\n");
    CK(hipStreamDestroy(st));
    return 0;
}
