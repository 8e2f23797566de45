// wave_merge.hpp -- one wave64 merges two sorted sequences of u32 keys in registers
// (a bitonic merger: no LDS, no barrier), for k_hist's fused Huffman tables (the
// package-merge levels, length_limited.rs:37-134); and sorts up to 256 keys the
// same way (sort_bitonic: the tables' symbols by frequency, symbol_counting.rs:92-94).
//
// Layout: S = 64 * EPL elements, element e in lane e & 63, register slot e >> 6
// ("slot-major"); the first S/2 elements ascending, the last S/2 DESCENDING (a
// bitonic sequence), padding kMergeInf at the high end of each run.  merge_bitonic
// sorts the S elements ascending in place with half-cleaners of distance S/2 ... 1:
// slot pairs in registers for distances of 64 and more; lane pairs below that --
// distances 32 and 16 by a permlane swap of two slots that brings both partners
// into one lane, one min and one max, and the swap back (two slots at a time), 8,
// 2 and 1 over DPP, 4 over two DPP rotations.  Every lane of the wave must be
// active.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmmt {

constexpr uint32_t kMergeInf = 0xFFFFFFFFu;

// the value of lane (lane ^ D) for D = 1, 2, 4, 8 (DPP), 16, 32 (permlane swaps)
template <int D>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x) {
    const int lane = (int)(threadIdx.x & 63);
    if constexpr (D == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (D == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (D == 4) {
        // row_ror:12 reads lane + 4 of the row, row_ror:4 lane - 4
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x12C, 0xF, 0xF, false);
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xF, 0xF, false);
        return (lane & 4) ? dn : up;
    } else if constexpr (D == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (D == 16) {
        // rows 0 1 2 3 -> first: x0 x0 x2 x2, second: x1 x1 x3 x3
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else {
        static_assert(D == 32, "lane_xor: D in 1 .. 32");
        // halves -> first: lo lo, second: hi hi
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
}

// the value of lane 63 - lane (row_mirror, then the rows reversed)
__device__ __forceinline__ uint32_t lane_reverse(uint32_t x) {
    const uint32_t m = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);  // row_mirror
    return lane_xor<16>(lane_xor<32>(m));
}

// half-cleaner over lanes at distance D (1, 2, 4, 8): the lower lane keeps the min
template <int D, int EPL>
__device__ __forceinline__ void clean_lanes(uint32_t (&x)[EPL]) {
    const bool upper = (threadIdx.x & D) != 0;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const uint32_t y = lane_xor<D>(x[s]);
        x[s] = upper ? max(x[s], y) : min(x[s], y);
    }
}

template <int D>
__device__ __forceinline__ void clean_lanes_xor(uint32_t& x) {
    const bool upper = (threadIdx.x & D) != 0;
    const uint32_t y = lane_xor<D>(x);
    x = upper ? max(x, y) : min(x, y);
}

// half-cleaner at distance 32 or 16 over two slots at once: the swap puts a pair of
// partners of slot a in one lane (and one of slot b in another), one min and one
// max order it, the swap back restores the layout -- lower lane min, upper max
template <int D>
__device__ __forceinline__ void clean_swap2(uint32_t& a, uint32_t& b) {
    static_assert(D == 16 || D == 32, "permlane swap distances");
    const auto r = D == 32 ? __builtin_amdgcn_permlane32_swap(a, b, false, false)
                           : __builtin_amdgcn_permlane16_swap(a, b, false, false);
    const uint32_t lo = min((uint32_t)r[0], (uint32_t)r[1]), hi = max((uint32_t)r[0], (uint32_t)r[1]);
    const auto q = D == 32 ? __builtin_amdgcn_permlane32_swap(lo, hi, false, false)
                           : __builtin_amdgcn_permlane16_swap(lo, hi, false, false);
    a = q[0];
    b = q[1];
}

template <int D, int EPL>
__device__ __forceinline__ void clean_swap(uint32_t (&x)[EPL]) {
    if constexpr (EPL == 1) {
        clean_lanes_xor<D>(x[0]);
    } else {
#pragma unroll
        for (int s = 0; s < EPL; s += 2) clean_swap2<D>(x[s], x[s + 1]);
    }
}

template <int EPL>
__device__ __forceinline__ void merge_bitonic(uint32_t (&x)[EPL]) {
    static_assert(EPL == 1 || EPL == 2 || EPL == 4 || EPL == 8, "64, 128, 256 or 512 elements");
    // distances S/2 ... 64: slot s against s ^ (d / 64)
#pragma unroll
    for (int ds = EPL / 2; ds >= 1; ds >>= 1) {
#pragma unroll
        for (int s = 0; s < EPL; ++s)
            if (!(s & ds)) {
                const uint32_t a = x[s], b = x[s | ds];
                x[s] = min(a, b);
                x[s | ds] = max(a, b);
            }
    }
    // 32 ... 1 over lanes
    clean_swap<32, EPL>(x);
    clean_swap<16, EPL>(x);
    clean_lanes<8, EPL>(x);
    clean_lanes<4, EPL>(x);
    clean_lanes<2, EPL>(x);
    clean_lanes<1, EPL>(x);
}

// ---- full sort (k_hist's fused tail, phase 2): 64 * E keys, element e in lane
// e & 63 of slot e >> 6, sorted ascending in place.  Bitonic sort in the "flip"
// form: for each size k = 2 .. 64 E the pair (i, i ^ (k - 1)) -- the lower index
// keeps the min -- then half-cleaners k/4 .. 1 as in merge_bitonic.

// the value of lane (lane ^ M) for M = 2^j - 1
template <int M>
__device__ __forceinline__ uint32_t lane_flip(uint32_t x) {
    if constexpr (M == 1) {
        return lane_xor<1>(x);
    } else if constexpr (M == 3) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x1B, 0xF, 0xF, false);  // quad_perm [3,2,1,0]
    } else if constexpr (M == 7) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    } else if constexpr (M == 15) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);  // row_mirror
    } else if constexpr (M == 31) {
        return lane_xor<16>((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false));
    } else {
        static_assert(M == 63, "lane_flip: M in 1, 3, 7, 15, 31, 63");
        return lane_reverse(x);
    }
}

template <int M, int E>
__device__ __forceinline__ void flip_lanes(uint32_t (&x)[E]) {
    const bool upper = (threadIdx.x & ((M + 1) >> 1)) != 0;
#pragma unroll
    for (int s = 0; s < E; ++s) {
        const uint32_t y = lane_flip<M>(x[s]);
        x[s] = upper ? max(x[s], y) : min(x[s], y);
    }
}

// slots a < b at size 128 or 256: element (a, l) against (b, 63 - l)
__device__ __forceinline__ void flip_slots(uint32_t& a, uint32_t& b) {
    const uint32_t r = lane_reverse(b);
    const uint32_t lo = min(a, r), hi = max(a, r);
    a = lo;
    b = lane_reverse(hi);
}

template <int E>
__device__ __forceinline__ void sort_bitonic(uint32_t (&x)[E]) {
    static_assert(E == 1 || E == 2 || E == 4, "64, 128 or 256 keys");
    flip_lanes<1>(x);
    flip_lanes<3>(x);
    clean_lanes<1>(x);
    flip_lanes<7>(x);
    clean_lanes<2>(x);
    clean_lanes<1>(x);
    flip_lanes<15>(x);
    clean_lanes<4>(x);
    clean_lanes<2>(x);
    clean_lanes<1>(x);
    flip_lanes<31>(x);
    clean_lanes<8>(x);
    clean_lanes<4>(x);
    clean_lanes<2>(x);
    clean_lanes<1>(x);
    flip_lanes<63>(x);
    clean_swap<16>(x);
    clean_lanes<8>(x);
    clean_lanes<4>(x);
    clean_lanes<2>(x);
    clean_lanes<1>(x);
    if constexpr (E >= 2) {  // size 128
#pragma unroll
        for (int s = 0; s < E; s += 2) flip_slots(x[s], x[s + 1]);
        clean_swap<32>(x);
        clean_swap<16>(x);
        clean_lanes<8>(x);
        clean_lanes<4>(x);
        clean_lanes<2>(x);
        clean_lanes<1>(x);
    }
    if constexpr (E >= 4) {  // size 256
        flip_slots(x[0], x[3]);
        flip_slots(x[1], x[2]);
#pragma unroll
        for (int s = 0; s < 4; s += 2) {  // distance 64: slots (0, 1), (2, 3)
            const uint32_t a = x[s], b = x[s + 1];
            x[s] = min(a, b);
            x[s + 1] = max(a, b);
        }
        clean_swap<32>(x);
        clean_swap<16>(x);
        clean_lanes<8>(x);
        clean_lanes<4>(x);
        clean_lanes<2>(x);
        clean_lanes<1>(x);
    }
}

}  // namespace dmmt
