// Launch cost of near-empty kernels by grid shape (HIP events around 200 launches
// each, after warmup): how much of a 1519-workgroup kernel's time is dispatch.
// Each workgroup's thread 0 stores one word so the kernel is not elided.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_touch(unsigned* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = blockIdx.x;
}

__global__ __launch_bounds__(256) void k_touch_lds(unsigned* out) {
    __shared__ unsigned s[2048 + 16];  // about k_stuffwrite's LDS
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s[5] + blockIdx.x;
}

int main() {
    unsigned* d;
    (void)hipMalloc(&d, 1 << 20);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int shapes[][2] = {{1519, 256}, {1519, 64}, {760, 256}, {380, 256}, {256, 256}, {1024, 256}, {3038, 128}, {1, 64}};
    for (int lds = 0; lds < 2; ++lds)
        for (auto& sh : shapes) {
            for (int i = 0; i < 20; ++i)
                if (lds) hipLaunchKernelGGL(k_touch_lds, dim3(sh[0]), dim3(sh[1]), 0, 0, d);
                else hipLaunchKernelGGL(k_touch, dim3(sh[0]), dim3(sh[1]), 0, 0, d);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(a, 0);
            const int n = 200;
            for (int i = 0; i < n; ++i)
                if (lds) hipLaunchKernelGGL(k_touch_lds, dim3(sh[0]), dim3(sh[1]), 0, 0, d);
                else hipLaunchKernelGGL(k_touch, dim3(sh[0]), dim3(sh[1]), 0, 0, d);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("%s grid %5d x %4d threads: %.2f us per launch (back to back)\n", lds ? "lds  " : "plain", sh[0], sh[1],
                   1e3f * ms / n);
        }
    return 0;
}
