// latency_probe.hip -- development microbenchmark (not part of the product):
// single-workgroup latencies on the target GPU that the table kernel's design
// depends on.  Prints shader-clock cycles per step for
//   lds_chase   dependent ds_read_b32 pointer chase (1 wave)
//   valu_chain  dependent v_add_u32 chain (1 wave)
//   barrier     s_barrier round with 4 / 16 waves
//   lds_chase16 dependent chase while 15 other waves chase too
// build: hipcc --offload-arch=gfx950 -O3 tools/latency_probe.hip -o tools/latency_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_lds_chase(unsigned long long* out, int steps, int active_waves) {
    __shared__ int buf[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[i] = (i * 17 + 5) & 4095;
    __syncthreads();
    int p = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    if (wave >= active_waves) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; ++s) p = buf[p];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = (unsigned long long)p;
    }
}

__global__ void k_valu_chain(unsigned long long* out, int steps, int seed) {
    unsigned v = threadIdx.x + seed;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; ++s) {
        v = v * 3u + 1u;
        v ^= v >> 7;
        v += 0x9E37u;
        v = (v << 3) | (v >> 29);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = v;
    }
}

__global__ void k_barrier(unsigned long long* out, int steps) {
    __shared__ int x[1024];
    x[threadIdx.x] = threadIdx.x;
    __syncthreads();
    int acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; ++s) {
        x[threadIdx.x] = acc + s;
        __syncthreads();
        acc += x[(threadIdx.x + 1) % blockDim.x];
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = acc;
    }
}

__global__ void k_rt(unsigned long long* out, int steps) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned v = threadIdx.x;
    for (int s = 0; s < steps; ++s) v = v * 3u + 1u;
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = r1 - r0;
        out[2] = v;
    }
}

int main() {
    unsigned long long* d;
    unsigned long long h[4];
    hipMalloc(&d, 64);
    const int steps = 4096;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_rt, dim3(1), dim3(64), 0, 0, d, 1 << 20);
        hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
        printf("clock: %.0f MHz (memtime/realtime over a 1M-step loop)\n", (double)h[0] / (double)h[1] * 100.0);
        hipLaunchKernelGGL(k_lds_chase, dim3(1), dim3(64), 0, 0, d, steps, 1);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("lds_chase   1 wave : %.1f cycles/step\n", (double)h[0] / steps);
        hipLaunchKernelGGL(k_lds_chase, dim3(1), dim3(1024), 0, 0, d, steps, 16);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("lds_chase  16 waves: %.1f cycles/step\n", (double)h[0] / steps);
        hipLaunchKernelGGL(k_valu_chain, dim3(1), dim3(64), 0, 0, d, steps, 1);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("valu_chain  1 wave : %.1f cycles per 5-op step\n", (double)h[0] / steps);
        hipLaunchKernelGGL(k_barrier, dim3(1), dim3(256), 0, 0, d, steps);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("barrier     4 waves: %.1f cycles per (store, barrier, load, barrier)\n", (double)h[0] / steps);
        hipLaunchKernelGGL(k_barrier, dim3(1), dim3(1024), 0, 0, d, steps);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("barrier    16 waves: %.1f cycles per (store, barrier, load, barrier)\n", (double)h[0] / steps);
    }
    hipFree(d);
    return 0;
}
