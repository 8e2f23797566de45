// Microbenchmark: issue rate of packed f32 VALU ops (v_pk_add_f32 / v_pk_mul_f32)
// vs their scalar forms on gfx950.  Each thread runs 8 independent chains.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k_scalar(float* out, float a, int iters) {
    float x[16];
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
    }
    float s = 0; for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_packed(float* out, float a, int iters) {
    f2 x[8];
    f2 av = {a, a};
    for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(av));
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_packed_mul(float* out, float a, int iters) {
    f2 x[8];
    f2 av = {a, a};
    for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(av));
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
    float* d; hipMalloc(&d, 4096 * 256 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 4096, blocks = 4096, threads = 256;
    for (int rep = 0; rep < 2; ++rep) {
        float ms;
        hipEventRecord(e0); hipLaunchKernelGGL(k_scalar, dim3(blocks), dim3(threads), 0, 0, d, 1.0f, iters); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double adds = (double)blocks * threads * iters * 16;
        printf("scalar v_add_f32: %.3f ms, %.1f G lane-adds/s\n", ms, adds / ms / 1e6);
        hipEventRecord(e0); hipLaunchKernelGGL(k_packed, dim3(blocks), dim3(threads), 0, 0, d, 1.0f, iters); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("packed v_pk_add_f32: %.3f ms, %.1f G lane-adds/s\n", ms, adds / ms / 1e6);
        hipEventRecord(e0); hipLaunchKernelGGL(k_packed_mul, dim3(blocks), dim3(threads), 0, 0, d, 1.0f, iters); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("packed v_pk_mul_f32: %.3f ms, %.1f G lane-muls/s\n", ms, adds / ms / 1e6);
    }
    return 0;
}
