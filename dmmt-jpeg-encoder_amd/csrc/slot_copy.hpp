// slot_copy.hpp -- k_emit's copy of a block's private slot into its chunk's LDS
// window image (entropy.hip), kept in a header of its own so that the same code
// is compiled for the host by the CPU unit check tests/native/slot_copy_check.cpp
// (a bit-serial model of the chunk's stream, random stale slot contents).
// [binary_stream.rs:38-66 BitWriter::write_bits: the bits these words carry]
//
// A walker thread has written its block's nbits bits MSB-first from bit 0 of its
// slot (word i of column c at sSlot[i * STRIDE + c]); the words of the slot past
// the block's last one still hold whatever an earlier walk of that column, or an
// earlier workgroup on the CU, left there.  The copy, without a window clear:
//  read_slot   the block's thread reads all kSlotWords words of its walker's slot
//              at once and zeroes the ones past the block (`stale`, below);
//  copy_owned  (phase 1) stores, plainly, every window word whose first bit lies
//              in its block: word d0 + k = {slot[k-1], slot[k]} >> sh (slot[-1] =
//              0) for k >= 1, and k = 0 too when the block starts word-aligned --
//              each window word has exactly one such block, so no word needs
//              clearing and none is written twice;
//  copy_head   (phase 2, after a barrier) ORs the block's first 32 - sh bits into
//              word d0, which an earlier block owns (a word can collect the heads
//              of several short blocks).
// Why the stale words must be zeroed: the last word a block owns, d1, takes the
// low bits of {slot[k-1], slot[k]} >> sh from slot[k] with k = d1 - d0, which is
// past the block's words when sh > 0 and the block's tail is shorter than sh.
// Unmasked, those stale bits land right behind the block's last bit -- exactly
// where the next block's copy_head ORs its head -- as extra 1 bits.  That was the
// round-4 one-bit parity failure of the first clear-free build (profiles/STUDIES.md B).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define DMMT_SLOT_FN __device__ __forceinline__
#else
#define DMMT_SLOT_FN inline
#endif

namespace dmmt {

// words per private block slot (384 bits; a longer block sends its chunk down the
// re-walk path)
constexpr int kSlotWords = 12;

// {hi, lo} >> sh, low 32 bits (sh < 32): v_alignbit_b32 on the GPU
DMMT_SLOT_FN uint32_t slot_alignbit(uint32_t hi, uint32_t lo, uint32_t sh) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31u));
#endif
}

// OR into a window word another thread may be ORing into too (ds_or_b32)
DMMT_SLOT_FN void slot_window_or(uint32_t* p, uint32_t v) {
#ifdef __HIP_DEVICE_COMPILE__
    atomicOr(p, v);
#else
    *p |= v;
#endif
}

struct SlotWords {
    uint32_t w[kSlotWords];
};

template <int STRIDE>
DMMT_SLOT_FN void read_slot(const uint32_t* __restrict__ sSlot, int col, uint32_t nbits, SlotWords& W) {
    const int nsw = (int)((nbits + 31) >> 5);
#pragma unroll
    for (int k = 0; k < kSlotWords; ++k) W.w[k] = sSlot[k * STRIDE + col];
#pragma unroll
    for (int k = 0; k < kSlotWords; ++k) W.w[k] = k < nsw ? W.w[k] : 0u;  // words past the block: stale
}

// window words [w0, w0 + wn] (word w0 + wn: the next window's first word)
DMMT_SLOT_FN void copy_owned(const SlotWords& W, uint32_t s0, uint32_t nbits, uint32_t* sW, int w0, int wn) {
    if (!nbits) return;
    const uint32_t sh = s0 & 31u;
    const int d0 = (int)(s0 >> 5), d1 = (int)((s0 + nbits - 1) >> 5);
#pragma unroll
    for (int k = 0; k <= kSlotWords; ++k) {
        const int d = d0 + k;
        const uint32_t v = slot_alignbit(k ? W.w[k - 1] : 0u, k < kSlotWords ? W.w[k] : 0u, sh);
        if (d <= d1 && (k || !sh) && (unsigned)(d - w0) <= (unsigned)wn) sW[d - w0] = v;
    }
}

DMMT_SLOT_FN void copy_head(const SlotWords& W, uint32_t s0, uint32_t nbits, uint32_t* sW, int w0, int wn) {
    const uint32_t sh = s0 & 31u;
    const int d0 = (int)(s0 >> 5);
    if (nbits && sh && (unsigned)(d0 - w0) <= (unsigned)wn) slot_window_or(&sW[d0 - w0], W.w[0] >> sh);
}

}  // namespace dmmt
