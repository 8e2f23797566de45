// Host unit check of k_emit's clear-free window copy (csrc/slot_copy.hpp, the
// same source the kernel compiles) against a bit-serial model of the chunk's
// stream (binary_stream.rs:38-66: MSB-first concatenation of the blocks' bits).
//
// Each trial draws a chunk of 256 blocks -- bit counts from 0 to 384 (empty,
// word-aligned, one-bit, slot-filling and mixed), a random walker permutation
// (the kernel's sort by last non-zero position), slot words past every block
// filled with random stale data, and the window image pre-filled with garbage
// (the sort keys and earlier windows' words the kernel leaves there) -- and
// replays the kernel's phases: per window, phase 1 (read_slot + copy_owned and
// the zero word past the stream) for every thread, then phase 2 (copy_head).
// Small windows exercise the multi-window path too.
//
// usage: slot_copy_check [trials] [seed] [--unmasked]
//   --unmasked replays the copy with the stale slot words NOT zeroed (the first
//   clear-free build of round 4); the check must then find extra 1 bits.
// Exit 0 and "ok" when every stream matched; exit 1 with the first mismatch.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../dmmt-jpeg-encoder_amd/csrc/slot_copy.hpp"

using namespace dmmt;

constexpr int kThreads = 256;  // kEmitThreads (one thread per block)

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (uint32_t)(g_rng >> 11);
}

// the first clear-free form: every slot word as it lies in LDS
static void read_slot_unmasked(const uint32_t* sSlot, int col, SlotWords& W) {
    for (int k = 0; k < kSlotWords; ++k) W.w[k] = sSlot[k * kThreads + col];
}

static int block_bits(int mode) {
    switch (mode) {
        case 0: return (int)(rnd() % 385);                  // anything the slot holds
        case 1: return (int)(rnd() % 8);                    // tiny blocks (several heads per word)
        case 2: return 32 * (int)(rnd() % 13);              // word multiples
        case 3: return (rnd() & 1) ? 384 : (int)(rnd() % 40);
        default: return 6 + (int)(rnd() % 200);             // ~natural q90 blocks
    }
}

int main(int argc, char** argv) {
    int trials = argc > 1 ? atoi(argv[1]) : 2000;
    if (argc > 2) g_rng ^= strtoull(argv[2], nullptr, 10) * 0xD1B54A32D192ED03ull;
    const bool unmasked = argc > 3 && strcmp(argv[3], "--unmasked") == 0;
    std::vector<uint32_t> sSlot(kSlotWords * kThreads);
    long long words_checked = 0, mismatches = 0, missing_words = 0;
    for (int trial = 0; trial < trials; ++trial) {
        const int mode = trial % 5;
        const int nb = (trial % 7 == 0) ? 1 + (int)(rnd() % kThreads) : kThreads;  // a short last chunk
        uint32_t bits[kThreads] = {}, start[kThreads] = {};
        int walker[kThreads];  // the slot column (walking thread) of block t
        for (int t = 0; t < kThreads; ++t) walker[t] = t;
        for (int t = kThreads - 1; t > 0; --t) {
            const int j = (int)(rnd() % (uint32_t)(t + 1));
            const int x = walker[t];
            walker[t] = walker[j];
            walker[j] = x;
        }
        // stale slots, then each block's own words (bits after its end zero, as
        // SlotSink::finish leaves them)
        for (auto& x : sSlot) x = rnd() | (rnd() << 21);
        uint32_t total = 0;
        for (int t = 0; t < kThreads; ++t) {
            bits[t] = t < nb ? (uint32_t)block_bits(mode) : 0u;
            start[t] = total;
            total += bits[t];
            const int col = walker[t];
            const int nsw = (int)((bits[t] + 31) >> 5);
            for (int k = 0; k < nsw; ++k) {
                uint32_t v = rnd() ^ (rnd() << 16);
                const int used = (int)bits[t] - 32 * k;
                if (used < 32) v &= ~0u << (32 - used);
                sSlot[k * kThreads + col] = v;
            }
        }
        // the bit-serial model of the chunk's stream
        const int nw = (int)((total + 31) >> 5);
        std::vector<uint32_t> ref(nw + 1, 0u);
        for (int t = 0; t < kThreads; ++t)
            for (uint32_t i = 0; i < bits[t]; ++i) {
                const uint32_t bit = (sSlot[(i >> 5) * kThreads + walker[t]] >> (31 - (i & 31))) & 1u;
                const uint32_t p = start[t] + i;
                ref[p >> 5] |= bit << (31 - (p & 31));
            }
        // the kernel's window loop
        const int win = (trial % 3 == 0) ? 1024 : (trial % 3 == 1 ? 37 : 5);  // kEmitWords and small windows
        std::vector<uint32_t> sW(win + 2), got(nw, 0u);
        for (auto& x : sW) x = rnd();
        for (int w0 = 0; w0 < nw; w0 += win) {
            const int wn = nw - w0 < win ? nw - w0 : win;
            SlotWords sw[kThreads];
            for (int t = 0; t < kThreads; ++t) {  // phase 1
                if (unmasked)
                    read_slot_unmasked(sSlot.data(), walker[t], sw[t]);
                else
                    read_slot<kThreads>(sSlot.data(), walker[t], bits[t], sw[t]);
                if (t == 0 && w0 + wn >= nw) sW[wn] = 0u;
                copy_owned(sw[t], start[t], bits[t], sW.data(), w0, wn);
            }
            for (int t = 0; t < kThreads; ++t) copy_head(sw[t], start[t], bits[t], sW.data(), w0, wn);  // phase 2
            for (int i = 0; i < wn; ++i) got[w0 + i] = sW[i];
        }
        for (int i = 0; i < nw; ++i) {
            ++words_checked;
            if (got[i] != ref[i]) {
                missing_words += (ref[i] & ~got[i]) != 0;
                if (mismatches++ == 0)
                    printf("mismatch: trial %d mode %d window %d word %d of %d: got %08x want %08x (extra %08x, missing %08x)\n",
                           trial, mode, win, i, nw, got[i], ref[i], got[i] & ~ref[i], ref[i] & ~got[i]);
            }
        }
    }
    if (mismatches) {
        printf("FAIL: %lld of %lld words differ, %lld of them missing bits (%s copy)\n", mismatches, words_checked,
               missing_words, unmasked ? "unmasked" : "product");
        return 1;
    }
    printf("ok: %d chunks, %lld words identical to the bit-serial stream (%s copy)\n", trials, words_checked,
           unmasked ? "unmasked" : "product");
    return 0;
}
