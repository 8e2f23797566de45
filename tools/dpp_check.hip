#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../dmmt-jpeg-encoder_amd/csrc/device_common.hpp"
__global__ void k(const unsigned* in, unsigned* a, unsigned* b, unsigned* c) {
    unsigned v = in[blockIdx.x * 256 + threadIdx.x];
    a[blockIdx.x * 256 + threadIdx.x] = dmmt::wave_incl_scan_full_u32(v);
    b[blockIdx.x * 256 + threadIdx.x] = dmmt::wave_incl_scan_u32(v);
    // 64-bit: values across the 2^32 carry
    const unsigned long long w = ((unsigned long long)v << 20) * 3ull + 0xFFFFF000ull;
    const unsigned prev = (unsigned)__shfl_up((int)v, 1, 64), next = (unsigned)__shfl_down((int)v, 1, 64);
    const int lane = threadIdx.x & 63;
    c[blockIdx.x * 256 + threadIdx.x] = (dmmt::wave_sum_full_u32(v) - dmmt::wave_sum_u32(v)) +
                                        (dmmt::wave_incl_scan_full_u64(w) != dmmt::wave_incl_scan_u64(w) ? 1u : 0u) +
                                        (dmmt::lane_prev_u32(v) != (lane ? prev : 0u) ? 1u : 0u) +
                                        (dmmt::lane_next_u32(v) != (lane < 63 ? next : 0u) ? 1u : 0u);
}
int main() {
    const int N = 256 * 64;
    unsigned *h = (unsigned*)malloc(N * 4), *ha = (unsigned*)malloc(N * 4), *hb = (unsigned*)malloc(N * 4), *hc = (unsigned*)malloc(N * 4);
    unsigned s = 12345; for (int i = 0; i < N; ++i) { s = s * 1103515245u + 12345u; h[i] = (s >> 16) & 0xFFFF; }
    unsigned *d, *a, *b, *c;
    (void)hipMalloc(&d, N * 4); (void)hipMalloc(&a, N * 4); (void)hipMalloc(&b, N * 4); (void)hipMalloc(&c, N * 4);
    (void)hipMemcpy(d, h, N * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(64), dim3(256), 0, 0, d, a, b, c);
    (void)hipMemcpy(ha, a, N * 4, hipMemcpyDeviceToHost); (void)hipMemcpy(hb, b, N * 4, hipMemcpyDeviceToHost); (void)hipMemcpy(hc, c, N * 4, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < N; ++i) bad += (ha[i] != hb[i]) + (hc[i] != 0);
    printf("dpp scan/sum mismatches: %d of %d\n", bad, 2 * N);
    return bad != 0;
}
