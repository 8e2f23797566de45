// GPU check of csrc/wave_merge.hpp: the lane exchanges against __shfl, the wave's
// bitonic merger against std::merge on random runs -- the lower ascending, the
// upper descending (duplicates, padding, every run length) -- and the bitonic sort
// against std::sort (random keys among INF padding, duplicates).  Prints the mismatch counts; exit 0 when none.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../dmmt-jpeg-encoder_amd/csrc/wave_merge.hpp"

using namespace dmmt;

__global__ void k_exchange(const uint32_t* in, uint32_t* bad) {
    const uint32_t x = in[blockIdx.x * 64 + threadIdx.x];
    const int l = threadIdx.x;
    uint32_t b = 0;
    b += lane_xor<1>(x) != (uint32_t)__shfl((int)x, l ^ 1, 64);
    b += lane_xor<2>(x) != (uint32_t)__shfl((int)x, l ^ 2, 64);
    b += lane_xor<4>(x) != (uint32_t)__shfl((int)x, l ^ 4, 64);
    b += lane_xor<8>(x) != (uint32_t)__shfl((int)x, l ^ 8, 64);
    b += lane_xor<16>(x) != (uint32_t)__shfl((int)x, l ^ 16, 64);
    b += lane_xor<32>(x) != (uint32_t)__shfl((int)x, l ^ 32, 64);
    b += lane_reverse(x) != (uint32_t)__shfl((int)x, 63 - l, 64);
    bad[blockIdx.x * 64 + threadIdx.x] = b;
}

template <int EPL>
__global__ void k_merge(const uint32_t* in, uint32_t* out) {
    uint32_t x[EPL];
    const uint32_t* p = in + (size_t)blockIdx.x * 64 * EPL;
#pragma unroll
    for (int s = 0; s < EPL; ++s) x[s] = p[64 * s + threadIdx.x];
    merge_bitonic<EPL>(x);
    uint32_t* q = out + (size_t)blockIdx.x * 64 * EPL;
#pragma unroll
    for (int s = 0; s < EPL; ++s) q[64 * s + threadIdx.x] = x[s];
}

template <int E>
__global__ void k_sort(const uint32_t* in, uint32_t* out) {
    uint32_t x[E];
    const uint32_t* p = in + (size_t)blockIdx.x * 64 * E;
#pragma unroll
    for (int s = 0; s < E; ++s) x[s] = p[64 * s + threadIdx.x];
    sort_bitonic<E>(x);
    uint32_t* q = out + (size_t)blockIdx.x * 64 * E;
#pragma unroll
    for (int s = 0; s < E; ++s) q[64 * s + threadIdx.x] = x[s];
}

static uint64_t g = 88172645463325252ull;
static uint32_t rnd() {
    g ^= g << 13;
    g ^= g >> 7;
    g ^= g << 17;
    return (uint32_t)(g >> 20);
}

template <int EPL>
static long long check_merge(int trials) {
    const int S = 64 * EPL;
    std::vector<uint32_t> in((size_t)trials * S), want((size_t)trials * S), got((size_t)trials * S);
    for (int t = 0; t < trials; ++t) {
        uint32_t* a = &in[(size_t)t * S];
        const int na = (int)(rnd() % (S / 2 + 1)), nb = (int)(rnd() % (S / 2 + 1));
        const uint32_t range = (t % 3 == 0) ? 8u : (t % 3 == 1 ? 1000u : 0x7FFFFFFFu);
        for (int i = 0; i < S; ++i) a[i] = kMergeInf;
        for (int i = 0; i < na; ++i) a[i] = rnd() % range;
        for (int i = 0; i < nb; ++i) a[S / 2 + i] = rnd() % range;
        std::sort(a, a + na);
        std::sort(a + S / 2, a + S / 2 + nb);
        std::merge(a, a + S / 2, a + S / 2, a + S, &want[(size_t)t * S]);
        std::reverse(a + S / 2, a + S);  // the upper run descending (a bitonic sequence)
    }
    uint32_t *d_in, *d_out;
    (void)hipMalloc(&d_in, in.size() * 4);
    (void)hipMalloc(&d_out, in.size() * 4);
    (void)hipMemcpy(d_in, in.data(), in.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_merge<EPL>, dim3(trials), dim3(64), 0, 0, d_in, d_out);
    (void)hipMemcpy(got.data(), d_out, got.size() * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    long long bad = 0;
    for (size_t i = 0; i < got.size(); ++i) bad += got[i] != want[i];
    printf("merge EPL=%d (%d elements): %lld of %zu differ\n", EPL, S, bad, got.size());
    return bad;
}

template <int E>
static long long check_sort(int trials) {
    const int S = 64 * E;
    std::vector<uint32_t> in((size_t)trials * S), want, got((size_t)trials * S);
    for (int t = 0; t < trials; ++t) {
        const int n = (int)(rnd() % (S + 1));  // present keys; the rest INF (absent symbols)
        const uint32_t range = (t % 3 == 0) ? 8u : (t % 3 == 1 ? 1000u : 0x7FFFFFFFu);
        for (int i = 0; i < S; ++i) in[(size_t)t * S + i] = i < n ? rnd() % range : kMergeInf;
        for (int i = S - 1; i > 0; --i) std::swap(in[(size_t)t * S + i], in[(size_t)t * S + rnd() % (i + 1)]);
    }
    want = in;
    for (int t = 0; t < trials; ++t) std::sort(want.begin() + (size_t)t * S, want.begin() + (size_t)(t + 1) * S);
    uint32_t *d_in, *d_out;
    (void)hipMalloc(&d_in, in.size() * 4);
    (void)hipMalloc(&d_out, in.size() * 4);
    (void)hipMemcpy(d_in, in.data(), in.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_sort<E>, dim3(trials), dim3(64), 0, 0, d_in, d_out);
    (void)hipMemcpy(got.data(), d_out, got.size() * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    long long bad = 0;
    for (size_t i = 0; i < got.size(); ++i) bad += got[i] != want[i];
    printf("sort E=%d (%d keys): %lld of %zu differ\n", E, S, bad, got.size());
    return bad;
}

int main() {
    const int blocks = 64;
    std::vector<uint32_t> h(blocks * 64), hb(blocks * 64);
    for (auto& v : h) v = rnd();
    uint32_t *d, *b;
    (void)hipMalloc(&d, h.size() * 4);
    (void)hipMalloc(&b, h.size() * 4);
    (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_exchange, dim3(blocks), dim3(64), 0, 0, d, b);
    (void)hipMemcpy(hb.data(), b, hb.size() * 4, hipMemcpyDeviceToHost);
    long long bad = 0;
    for (uint32_t v : hb) bad += v;
    printf("lane exchanges: %lld mismatches\n", bad);
    bad += check_merge<1>(2000) + check_merge<2>(2000) + check_merge<4>(2000) + check_merge<8>(2000);
    bad += check_sort<1>(2000) + check_sort<2>(2000) + check_sort<4>(2000);
    printf(bad ? "FAIL\n" : "ok\n");
    return bad != 0;
}
