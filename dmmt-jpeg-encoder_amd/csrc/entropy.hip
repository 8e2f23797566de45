// entropy.hip -- gfx950 entropy-coding back half: Huffman bit emission and byte
// stuffing.  [encoder.rs:264-404 write_image_data / write_{dc,ac}_from_block,
// binary_stream.rs:38-96 BitWriter, segment_marker_injector.rs:13-30]
//
// Three kernels, no inter-workgroup waiting anywhere (two launches for frames of
// at most kFusedOffsetsMaxChunks chunks, whose k_offsets work runs in k_emit's
// last workgroup: fused_offsets):
//  k_emit        one workgroup per chunk of kChunkBlocks blocks, one thread per
//                block: the bits of every block (a register walk), a workgroup
//                scan for the block offsets inside the chunk, every code placed
//                MSB-first into an LDS word image of the chunk's own bit stream,
//                which goes to the chunk's staging slot.  Per chunk it also
//                records its bit count, its first and last 16 bits and, for each
//                of the 8 residues the chunk's start can have modulo 8, the 0xFF
//                bytes lying wholly inside it (also packed one byte each for the
//                fused offsets) -- so no later pass re-reads the stream to count them.
//  k_offsets     one workgroup per frame: segmented scan of the chunk bit counts
//                (every chunk's bit offset in its restart segment); each chunk's
//                output bytes -- its bytes, a 0x00 per 0xFF (k_emit's count at its
//                actual alignment plus the byte it shares with the next chunk,
//                built from the recorded edge bits), the RST marker closing a
//                segment -- and their scan (every chunk's place in the file).
//  k_stuffwrite  one workgroup per chunk: the bytes whose first bit lies in the
//                chunk, shifted out of its staging slot (the last one built from
//                the edge bits, 1-padded at the end of the scan), a 0x00 after
//                every 0xFF, staged in LDS and stored coalesced after the header;
//                RSTm after a segment's last chunk, EOI and the file size by the
//                frame's last chunk.
//
// Restart intervals (extension, DRI/RSTn every N MCUs): each segment's scan
// starts byte-aligned, so the chunk grid restarts with every segment and the
// 1-padding closes each segment like the end of the scan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "jpeg_common.hpp"
#include "kernels.hpp"
#include "slot_copy.hpp"

namespace dmmt {

#ifdef DMMT_PHASE_TRACE
static __device__ unsigned long long g_trace[64];
#endif

static_assert(kChunkBlocks == 256 || kChunkBlocks == 512, "one thread per block, one workgroup per chunk");
constexpr int kEmitThreads = kChunkBlocks;
constexpr int kEmitWaves = kEmitThreads / 64;
#ifndef DMMT_EMIT_OCC
#define DMMT_EMIT_OCC 7  // k_emit workgroups per CU the launch bounds target (256-block chunks; study builds: others)
#endif
constexpr int kEmitOcc = kChunkBlocks == 256 ? DMMT_EMIT_OCC : 3;  // workgroups per CU

// LDS word window of k_emit: 32 Ki bits = 128 bits per block on average (the 4K
// q90 workload averages ~110).  A chunk with more is assembled in several
// windows, every block copying (or, on the re-walk path, re-emitting) only the
// words inside the window.
constexpr int kEmitWords = 4 * kChunkBlocks;
// Bytes per pass of k_stuffwrite (16 per thread).
constexpr int kStuffPass = 4096;
#ifndef DMMT_EMIT_BRANCHFREE
#define DMMT_EMIT_BRANCHFREE 1  // SlotSink stores a word per piece, no flush branch (0: study builds)
#endif
#ifndef DMMT_TAIL_DMA
#define DMMT_TAIL_DMA 1  // fused offsets: the packed 0xFF counts land in LDS with the first loads (0: study builds)
#endif
#ifndef DMMT_TAIL_NSEG1
#define DMMT_TAIL_NSEG1 1  // fused offsets: no chunk_span division per chunk without restart intervals (0: study builds)
#endif
#ifndef DMMT_EMIT_PRIO_ALWAYS
#define DMMT_EMIT_PRIO_ALWAYS 0  // study builds: the priorities with several lanes too (the round-5 behaviour)
#endif
#ifndef DMMT_EMIT_PRIO
#define DMMT_EMIT_PRIO 1  // k_emit's wave priorities by walk length (0: off, study builds)
#endif

// Chunk c of a frame: blocks [el0, el0 + nb) of restart segment seg (the chunk
// grid restarts with every segment; one segment without restart intervals).
struct ChunkSpan {
    long long el0;
    int nb;
    int seg;
    bool seg_first, seg_last;
};

__device__ __forceinline__ ChunkSpan chunk_span(const Geom& g, int c) {
    ChunkSpan r;
    r.seg = min(c / g.cps, g.nseg - 1);
    const int j = c - r.seg * g.cps;
    const long long sb = (long long)r.seg * g.seg_blocks;
    const long long se = min(sb + g.seg_blocks, g.bpf);
    r.el0 = sb + (long long)j * kChunkBlocks;
    r.nb = (int)min((long long)kChunkBlocks, se - r.el0);
    r.seg_first = j == 0;
    r.seg_last = r.el0 + r.nb == se;
    return r;
}

// The frame's last chunk of a joined stripe (no restart intervals, more stripes
// follow): its last byte runs on into the next stripe's first bits (g.next16).
__device__ __forceinline__ bool joined_tail(const Geom& g, int c) {
    return c == g.nch - 1 && g.more_after && g.restart_interval == 0;
}

// x mod d by a 16-bit reciprocal inv16 = ceil(2^16 / d): exact for x < 2^16 / d
// (here x < 256 + 6, d = blocks per MCU <= 6) -- three full-rate instructions
// instead of a division
__device__ __forceinline__ int mod_small(int x, int d, uint32_t inv16) {
    return x - (int)__umul24((uint32_t)d, __umul24((uint32_t)x, inv16) >> 16);
}

// One thread walks one block (64 zigzag coefficients held in 32 registers) in
// stream order (encoder.rs:356-404; categorize.rs:132-169): DC code + extra bits,
// then for each non-zero AC coefficient (run >> 4) ZRL codes and
// code((run & 15) << 4 | cat) + extra bits, EOB after trailing zeros.  The walk is
// fully unrolled so every coefficient access is a register.  Sink receives every
// piece (value right aligned, length in bits) in order.
struct BlockCoef {
    uint32_t w[32];  // coefficient 2i in the low half of w[i], 2i+1 in the high half
};

__device__ __forceinline__ void load_block(const int16_t* __restrict__ p, BlockCoef& b) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint4 v = q[i];
        b.w[4 * i] = v.x;
        b.w[4 * i + 1] = v.y;
        b.w[4 * i + 2] = v.z;
        b.w[4 * i + 3] = v.w;
    }
}

// the coefficient at zigzag position k, after zigzag_in_registers
__device__ __forceinline__ int coef_at(const BlockCoef& b, int k) {
    return (k & 1) ? ((int)b.w[k >> 1] >> 16) : (int)(int16_t)(b.w[k >> 1] & 0xFFFFu);
}

// Blocks arrive column-major (coef_pos); the walk wants zigzag order: one
// constant permutation of the 64 halves in registers, 32 word builds.  (Walking
// the column-major registers directly, coef_at(b, coef_pos(k)), is the same
// computation.  One round-2 build of that form computed wrong bits, differently
// from run to run: its register allocation put a v_lshlrev_b64's shift amount in
// the wave's last allocated VGPR, which MI355X got wrong (round 5,
// profiles/r03_kemit_fault_study.md; tools/last_vgpr_check.py, run on every linked
// library, refuses that pattern).  The study switch is
// profiles/r05_study_variants.patch; tests/test_gpu_regressions.py guards the shape.)
__device__ __forceinline__ void zigzag_in_registers(BlockCoef& b) {
    uint32_t z[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const int i0 = coef_pos(2 * j), i1 = coef_pos(2 * j + 1);
        const uint32_t lo = (b.w[i0 >> 1] >> (16 * (i0 & 1))) & 0xFFFFu;
        const uint32_t hi = (b.w[i1 >> 1] >> (16 * (i1 & 1))) & 0xFFFFu;
        z[j] = lo | (hi << 16);
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) b.w[j] = z[j];
}

// Code tables in LDS as (code, length) pairs: one ds_read_b64 per symbol gives
// both halves with no masking or shifting.  Every entry is pre-shifted by the
// category its symbol carries (its low 4 bits; a DC symbol is the category): the
// code shifted left by cat and the length plus cat, so a piece is the entry ORed
// with the cat extra bits (ZRL and EOB have category 0).
template <typename Sink>
__device__ __forceinline__ void walk_block(const BlockCoef& b, int dcd, const uint2* __restrict__ dctab,
                                           const uint2* __restrict__ actab, Sink& sink, int kmax = 63) {
    {
        const int cat = category_of(dcd);
        const uint2 e = dctab[cat];
        sink(e.x | extra_bits(dcd, cat), (int)e.y);
    }
    const uint2 z = actab[0xF0];
    // l16 = 16 * (position of the last non-zero + 1): the zero run before position
    // k is r16 / 16 with r16 = 16 * k - l16, (run & 15) << 4 = r16 & 0xF0
    int l16 = 16;
#pragma unroll
    for (int k = 1; k < 64; ++k) {
        if (k > kmax) continue;  // (wave-uniform) every later position is zero in every lane
        const int v = coef_at(b, k);
        if (v != 0) {
            const int r16 = 16 * k - l16;
            for (int r = r16 >> 8; r > 0; --r) sink(z.x, (int)z.y);
            const int cat = category_fast(v);
            const uint2 e = actab[(r16 & 0xF0) | cat];
            sink(e.x | extra_bits(v, cat), (int)e.y);
            l16 = 16 * k + 16;
        }
    }
    if (l16 < 16 * 64 || kmax < 63) {
        const uint2 e = actab[0];  // EOB
        sink(e.x, (int)e.y);
    }
}

struct CountSink {
    uint32_t n = 0;
    __device__ __forceinline__ void operator()(uint32_t, int len) { n += (uint32_t)len; }
};

// Appends pieces MSB-first into the LDS window image of words [lo, lo + n): the
// first and the last word of a block (shared with its neighbours) are ORed, the
// others stored plainly; words outside the window are dropped.
struct WindowSink {
    uint32_t* img;
    int lo, n;
    unsigned long long acc;
    int nacc;  // bits pending in acc (< 32 between pieces)
    int w;     // word index of the pending bits
    bool first;
    __device__ __forceinline__ void put(uint32_t word, bool shared) {
        const int i = w - lo;
        if ((unsigned)i < (unsigned)n) {
            if (shared)
                atomicOr(&img[i], word);
            else
                img[i] = word;
        }
    }
    __device__ __forceinline__ void operator()(uint32_t val, int len) {
        acc = (acc << len) | val;
        nacc += len;
        if (nacc >= 32) {
            nacc -= 32;
            put((uint32_t)(acc >> nacc), first);
            first = false;
            ++w;
        }
    }
    __device__ __forceinline__ void finish() {
        if (nacc > 0) put((uint32_t)(acc << (32 - nacc)), true);
    }
};

// The sinks never clear the bits they have flushed: with at most 32 bits per
// piece, bits above the pending ones are shifted past bit 31 of every word taken
// from acc, so the truncation to 32 bits drops them.

// Private block slots of k_emit: every thread writes its block's bits MSB-first
// from bit 0 of its own slot (no sharing, plain stores), word i of thread t at
// sSlot[i * kEmitThreads + t] (consecutive threads, consecutive banks).  A block
// that needs more than kSlotWords words (384 bits, slot_copy.hpp) sets `over`; the
// chunk then takes the re-walk path.  Small slots and window keep 7 workgroups
// resident per CU.
struct SlotSink {
    uint32_t* slot;  // &sSlot[tid]
    unsigned long long acc;
    int nacc;
    int wi;
#if DMMT_EMIT_BRANCHFREE
    // Branch-free: the word that holds the top pending bits is stored after every
    // piece -- complete (and final) when 32 bits are pending, else a partial word at
    // slot[wi] that a later store or finish() overwrites -- so a piece costs no
    // exec-mask branch (an s_and_saveexec / s_cbranch / s_or per piece otherwise).
    __device__ __forceinline__ void operator()(uint32_t val, int len) {
        acc = (acc << len) | val;
        nacc += len;               // < 64: at most 31 pending + a piece of at most 32
        const int full = nacc >> 5;  // 32 bits or more pending: a word is complete
        nacc &= 31;
        // past the slot the word lands in its last one: the chunk re-walks then
        slot[min(wi, kSlotWords - 1) * kEmitThreads] = (uint32_t)(acc >> nacc);
        wi += full;
    }
#else
    __device__ __forceinline__ void operator()(uint32_t val, int len) {
        acc = (acc << len) | val;
        nacc += len;
        if (nacc >= 32) {
            nacc -= 32;
            // past the slot the word lands in its last one: the chunk re-walks then
            slot[min(wi, kSlotWords - 1) * kEmitThreads] = (uint32_t)(acc >> nacc);
            ++wi;
        }
    }
#endif
    // (the bits after the block in its last word are zero; the slot's later words
    // are stale -- read_slot masks them)
    __device__ __forceinline__ uint32_t finish() {
        if (nacc > 0 && wi < kSlotWords) slot[wi * kEmitThreads] = (uint32_t)(acc << (32 - nacc));
        return (uint32_t)wi * 32u + (uint32_t)nacc;
    }
};

// The slot's copy into the window (read_slot, copy_owned, copy_head) is in
// slot_copy.hpp, shared with its host unit check.

// 16 bits of an MSB-first word stream starting at bit p (p & 31 taken; words a, b
// hold bits from (p & ~31))
__device__ __forceinline__ uint32_t bits16_at(uint32_t a, uint32_t b, int p) {
    const unsigned long long x = ((unsigned long long)a << 32) | b;
    return (uint32_t)(x >> (48 - (p & 31))) & 0xFFFFu;
}

struct NoMark {
    template <typename I>
    __device__ void operator()(I) const {}
};
template <typename Mark = NoMark>
__device__ __forceinline__ void fused_offsets(const uint32_t* __restrict__ cbits, const uint32_t* __restrict__ cff,
                              const unsigned long long* __restrict__ cff8, uint8_t* sFF8,
                              const uint32_t* __restrict__ cedge, const Geom& g, unsigned long long* __restrict__ bit0,
                              unsigned long long* __restrict__ outo, unsigned long long* __restrict__ total,
                              unsigned long long* sWaveV, int* sWaveF, Mark mark = Mark());
static_assert(kArriveWords == kArriveFrameWords, "the host sizes the counters");

// ---------------------------------------------------------------------- k_emit
// fuse: the frame's last workgroup to finish also computes every chunk's offsets
// (fused_offsets; `arrive` counts the finished workgroups per frame and is zero
// between launches), so no k_offsets launch follows
__global__ __launch_bounds__(kEmitThreads, kEmitOcc) void k_emit(const int16_t* coef, const int16_t* __restrict__ dcdiff,
                                              const uint8_t* __restrict__ lastnz,
                                              const uint32_t* __restrict__ code_tab, Geom g,
                                              uint32_t* __restrict__ stage, uint32_t* __restrict__ chunk_bits,
                                              uint32_t* __restrict__ chunk_ff, uint32_t* __restrict__ chunk_edge,
                                              uint32_t* __restrict__ ac_hist, uint32_t* __restrict__ dc_hist,
                                              int fuse, uint32_t* __restrict__ arrive,
                                              unsigned long long* __restrict__ chunk_bit0,
                                              unsigned long long* __restrict__ chunk_out,
                                              unsigned long long* __restrict__ total_out,
                                              unsigned long long* __restrict__ chunk_ff8, int prio) {
    // code tables: [luma AC 256][chroma AC 256][luma DC 16][chroma DC 16]
    __shared__ uint2 sTab[2 * 256 + 2 * 16];
    // the window image; during the sort and the walk its first words hold the
    // walk order, the keys and the blocks' bit counts (read before the window
    // loop, whose first clear follows two barriers)
    __shared__ uint32_t sW[kEmitWords + 2];
    __shared__ __attribute__((aligned(16))) uint32_t sSlot[kSlotWords * kEmitThreads];
    __shared__ uint32_t sWave[kEmitWaves];
    __shared__ uint32_t sFF[8];
    __shared__ uint32_t sEdge[3];  // word 0, the two words holding bits total-16 .. total-1
    __shared__ uint32_t sBin[65];  // walk order: blocks counted, then started, by last non-zero position
    __shared__ unsigned long long sOffV[kEmitWaves + 1];  // fused offsets: the scans' wave totals, the carry
    __shared__ int sOffF[kEmitWaves];
    __shared__ uint32_t sLast;
    using OrderT = std::conditional_t<(kEmitThreads > 256), uint16_t, uint8_t>;
    uint32_t* const sBits = sW;                                                      // bit count of block t
    OrderT* const sOrder = reinterpret_cast<OrderT*>(sW + kEmitThreads);               // block walked by thread u
    uint8_t* const sKey = reinterpret_cast<uint8_t*>(sW + kEmitThreads + kEmitThreads * (int)sizeof(OrderT) / 4);  // its last non-zero position
    DMMT_TRACE_START;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const unsigned chunk = blockIdx.x;
    const ChunkSpan span = chunk_span(g, (int)chunk);
    const long long el0 = span.el0;
    const int nb = span.nb;
    const long long e = (long long)frame * g.bpf + el0 + tid;
    const size_t cid = (size_t)frame * g.nch + chunk;
    // the chunk's first block's place in its MCU (bpf < 2^31: 32-bit, once per
    // wave) and a 16-bit reciprocal of the blocks per MCU for the per-lane mod
    const int r0 = (int)((uint32_t)el0 % (uint32_t)g.bpm);
    const uint32_t inv16 = (65536u + (uint32_t)g.bpm - 1u) / (uint32_t)g.bpm;
    // every global load of the prologue is issued before any is used (one latency,
    // not three): the code tables -- code_tab is [luma DC][luma AC][chroma DC]
    // [chroma AC] x 256; two AC words per thread, one DC word for threads below 32
    // -- and the block's last non-zero position (at a clamped index past nb)
    const bool valid = tid < nb;
    const uint32_t* ct = code_tab + (size_t)frame * 1024;
    const int tt = tid & 255;
    const uint32_t tac0 = ct[256 + tt], tac1 = ct[768 + tt];
    const uint32_t tdc = ct[((tt & 31) < 16 ? 0 : 512 - 16) + (tt & 31)];
    const uint32_t lz = lastnz[valid ? e : (long long)frame * g.bpf + el0];
    if (tid < 256) {  // (pre-shifted by the symbol's category, walk_block)
        const int c = tid & 15;
        sTab[tid] = make_uint2((tac0 & 0xFFFFu) << c, (tac0 >> 16) + c);
        sTab[256 + tid] = make_uint2((tac1 & 0xFFFFu) << c, (tac1 >> 16) + c);
    }
    if (tid < 32) sTab[512 + tid] = make_uint2((tdc & 0xFFFFu) << (tid & 15), (tdc >> 16) + (tid & 15));
    if (chunk == 0) {  // the histogram replicas k_tables read: zero for the next launch
        for (int i = tid; i < kHistReps * 512; i += kEmitThreads) ac_hist[(size_t)frame * kHistReps * 512 + i] = 0u;
        for (int i = tid; i < kHistReps * 32; i += kEmitThreads) dc_hist[(size_t)frame * kHistReps * 32 + i] = 0u;
    }
    if (tid < 8) sFF[tid] = 0u;
    if (tid < 3) sEdge[tid] = 0u;
    if (tid < 65) sBin[tid] = 0u;
    // Walk order: a wave pays for every zigzag position at which any of its 64
    // blocks still has a non-zero coefficient, so the chunk's blocks are handed to
    // the threads sorted by their last non-zero position (k_front's lastnz): at
    // 4K q90 the mean over waves of the last such position falls from 61 to 39.
    // Thread u walks block sOrder[u] into its own slot u; after the scan (in
    // stream order) it shifts that slot into the window at the block's offset.
    const int key = valid ? (int)lz : 64;
    __syncthreads();
    const uint32_t rank = atomicAdd(&sBin[key], 1u);
    __syncthreads();
    if (tid < 64) {
        const uint32_t c = sBin[tid];
        const uint32_t inc = wave_incl_scan_full_u32(c);  // (wave 0 whole)
        sBin[tid] = inc - c;  // first position of bin tid
    }
    __syncthreads();
    const int mine = valid ? (int)(sBin[key] + rank) : tid;
    if (valid) {
        sOrder[mine] = (OrderT)tid;
        sKey[mine] = (uint8_t)key;
    }
    __syncthreads();
    DMMT_TRACE(0);
    uint32_t wbits = 0;  // the bits of the block this thread walks
    bool slot_over = false;
    {
#if DMMT_EMIT_PRIO
        // The waves walk sorted blocks, the heaviest last, and every wave of the
        // workgroup waits for the slowest at the barrier after the walk: the longer a
        // wave's walk, the higher its issue priority on its SIMD (4K q90, one lane:
        // k_emit 27.0 -> 23.1 us).  Only when the context runs one lane (prio): with
        // several, the raised waves take issue slots from the other lanes' kernels,
        // -1.5 % on the settled 4-lane bench (profiles/r06_emit_prio_ab.txt)
        if (prio) {  // (uniform)
            if (wave == 3) __builtin_amdgcn_s_setprio(3);
            else if (wave == 2) __builtin_amdgcn_s_setprio(2);
            else if (wave == 1) __builtin_amdgcn_s_setprio(1);
        }
#endif
        // one walk: the block's bits into this thread's private slot, and its bit count
        if (valid) {
            const int p = sOrder[tid];
            const long long ep = (long long)frame * g.bpf + el0 + p;
            BlockCoef b;
            load_block(coef + ep * 64, b);
            zigzag_in_registers(b);
            const int dp = dcdiff[ep];
            DMMT_TRACE(4);
            const int kp = mod_small(r0 + p, g.bpm, inv16);
            const bool lum = kp < g.n_luma;
            // the wave's walk stops after the last position any of its blocks uses
            const int kmax = __builtin_amdgcn_readfirstlane((int)sKey[min(64 * wave + 63, nb - 1)]);
            SlotSink ss{sSlot + tid, 0ull, 0, 0};
            walk_block(b, dp, sTab + 512 + (lum ? 0 : 16), sTab + (lum ? 0 : 256), ss, kmax);
            wbits = ss.finish();
            slot_over = wbits > (uint32_t)kSlotWords * 32u;
            sBits[p] = wbits;
            DMMT_TRACE(5);
        }
    }
#if DMMT_EMIT_PRIO
    if (prio) __builtin_amdgcn_s_setprio(0);
#endif
    // a block too long for its slot sends the whole chunk down the re-walk path
    const bool over = __syncthreads_or(slot_over) != 0;
    const uint32_t bits = valid ? sBits[tid] : 0u;
    const int k = valid ? mod_small(r0 + tid, g.bpm, inv16) : 0;
    const bool lum_t = k < g.n_luma;
    // offsets inside the chunk by a workgroup scan
    const uint32_t incl = wave_incl_scan_full_u32(bits);
    if (lane == 63) sWave[wave] = incl;
    __syncthreads();
    uint32_t start = incl - bits;
    uint32_t total = 0;
#pragma unroll
    for (int q = 0; q < kEmitWaves; ++q) {
        start += q < wave ? sWave[q] : 0u;
        total += sWave[q];
    }
    DMMT_TRACE(1);

    uint32_t* slot = stage + cid * (size_t)kChunkWordsCap;
    const int nw = (int)((total + 31) >> 5);
    const int we1 = total >= 16 ? (int)((total - 16) >> 5) : 0;  // word holding bit total-16
    uint32_t ff[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int w0 = 0; w0 < nw; w0 += kEmitWords) {  // uniform; one window unless the chunk is huge
        const int wn = min(kEmitWords, nw - w0);
        if (!over) {  // (uniform) block tid's bits from its walker's slot (column `mine`)
            SlotWords sw;
            read_slot<kEmitThreads>(sSlot, mine, bits, sw);
            if (tid == 0 && w0 + wn >= nw) sW[wn] = 0u;  // past the stream: no block owns it
            copy_owned(sw, start, bits, sW, w0, wn);
            __syncthreads();
            copy_head(sw, start, bits, sW, w0, wn);
        } else {
            for (int i = tid; i <= wn; i += kEmitThreads) sW[i] = 0u;  // + the next window's first word
            __syncthreads();
        }
        if (over && bits && start < (uint32_t)(w0 + wn + 1) * 32u && start + bits > (uint32_t)w0 * 32u) {
            {
                // the block again (L2 / MALL) and a second walk straight into the
                // window: holding it in registers across the scan would halve the
                // occupancy of this kernel
                BlockCoef b;
                load_block(coef + e * 64, b);
                zigzag_in_registers(b);
                WindowSink ws{sW, w0, wn + 1, 0ull, (int)(start & 31), (int)(start >> 5), true};
                walk_block(b, dcdiff[e], sTab + 512 + (lum_t ? 0 : 16), sTab + (lum_t ? 0 : 256), ws);
                ws.finish();
            }
        }
        __syncthreads();
        for (int i = tid; i < wn; i += kEmitThreads) {
            const uint32_t a = sW[i], c = sW[i + 1];
            slot[w0 + i] = a;
            const int wi = w0 + i;
            if (wi == 0) sEdge[0] = a;
            if (wi == we1) {  // the pair holding the last 16 bits (c is zero past the end)
                sEdge[1] = a;
                sEdge[2] = c;
            }
            // runs of 8 ones starting at bit p of word a: bit 31-p of m
            const unsigned long long x = ((unsigned long long)a << 32) | c;
            unsigned long long z = x & (x << 1);
            z &= z << 2;
            z &= z << 4;
            const uint32_t m = (uint32_t)(z >> 32);
            if (m) {
#pragma unroll
                for (int r = 0; r < 8; ++r) ff[r] += __popc(m & (0x80808080u >> r));
            }
        }
        __syncthreads();
    }
    DMMT_TRACE(2);
    // the eight residue counts two to a word (16-bit fields: a wave's count stays
    // below 64 * 4 * 56 < 2^16), summed over the wave by DPP
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t v = wave_sum_full_u32(ff[2 * r] | (ff[2 * r + 1] << 16));
        if (lane == 0 && v) {
            atomicAdd(&sFF[2 * r], v & 0xFFFFu);
            atomicAdd(&sFF[2 * r + 1], v >> 16);
        }
    }
    __syncthreads();
    // The chunk's summary (its bits, edge bits and eight 0xFF counts), stored by
    // thread 0 as agent-scope atomics: the frame's last workgroup reads it when the
    // offsets are fused.
    if (tid == 0) {
        const uint32_t first16 = sEdge[0] >> 16;
        uint32_t last16;
        if (total >= 16)
            last16 = bits16_at(sEdge[1], sEdge[2], (int)(total - 16));
        else
            last16 = total ? sEdge[0] >> (32 - total) : 0u;
        unsigned long long f8 = 0;  // the same counts one byte each (fused_offsets reads them with its first loads)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            __hip_atomic_store(chunk_ff + cid * 8 + r, sFF[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            f8 |= (unsigned long long)min(sFF[r], 255u) << (8 * r);
        }
        __hip_atomic_store(chunk_ff8 + cid, f8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(chunk_bits + cid, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(chunk_edge + cid, (first16 << 16) | last16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (fuse) {  // (uniform) count this workgroup in once its summary is published (arrive_last)
        if (tid == 0) sLast = arrive_last(arrive + (size_t)frame * kArriveWords, chunk, (unsigned)g.nch);
        __syncthreads();
        DMMT_TRACE(6);
        if (sLast) {  // every other chunk of the frame is done: its offsets
            arrive_acquire();
            const size_t fb = (size_t)frame * g.nch;
#ifdef DMMT_PHASE_TRACE
            auto mark = [&](auto i) { DMMT_TRACE(decltype(i)::value); };
#else
            NoMark mark;
#endif
            // (the packed counts go to sSlot, which no wave reads any more)
            fused_offsets(chunk_bits + fb, chunk_ff + fb * 8, chunk_ff8 + fb, reinterpret_cast<uint8_t*>(sSlot),
                          chunk_edge + fb, g, chunk_bit0 + fb, chunk_out + fb, total_out + frame, sOffV, sOffF, mark);
        }
    }
    DMMT_TRACE(3);
    DMMT_TRACE_FLUSH(0, 0);
}

// The byte that starts m1 (1..7) bits before the end of a chunk: those last m1
// bits of the chunk, then the next chunk's first bits (same restart segment),
// then 1-bits where the segment or the scan ends (binary_stream.rs:89-96).
__device__ __forceinline__ uint32_t boundary_byte(int m1, uint32_t last16, bool has_next, uint32_t n_next,
                                                  uint32_t first16_next) {
    uint32_t v = last16 & ((1u << m1) - 1u);
    int m2 = 8 - m1;
    if (has_next) {
        const int t = (int)min((uint32_t)m2, n_next);
        v = (v << t) | (t ? first16_next >> (16 - t) : 0u);
        m2 -= t;
    }
    return ((v << m2) | ((1u << m2) - 1u)) & 0xFFu;
}

// Output bytes of chunk c, whose bits start at b0 inside its (byte-aligned)
// restart segment: the bytes whose first bit lies in the chunk, a 0x00 after each
// of them that is 0xFF (the interior ones counted by k_emit at the chunk's
// alignment, plus the byte it shares with the next chunk or the 1-padding), and
// the RST marker after the last chunk of every segment but the frame's last.
__device__ __forceinline__ unsigned long long chunk_out_bytes(const uint32_t* __restrict__ cff,
                                                              const uint32_t* __restrict__ cbits,
                                                              const uint32_t* __restrict__ cedge, const Geom& g,
                                                              int c, unsigned long long b0) {
    const ChunkSpan sp = chunk_span(g, c);
    const uint32_t n = cbits[c];
    const unsigned long long e = b0 + n;
    unsigned long long out = ((e + 7) >> 3) - ((b0 + 7) >> 3);
    out += cff[(size_t)c * 8 + ((8 - (b0 & 7)) & 7)];
    if ((e & 7) && (e & ~7ull) >= b0) {
        const bool jt = joined_tail(g, c);
        const bool has_next = !sp.seg_last || jt;
        const uint32_t nn = jt ? (uint32_t)g.next_bits : (has_next ? cbits[c + 1] : 0u);
        const uint32_t fn = jt ? g.next16 : (has_next ? cedge[c + 1] >> 16 : 0u);
        const uint32_t byte = boundary_byte((int)(e & 7), cedge[c] & 0xFFFFu, has_next, nn, fn);
        out += byte == 0xFFu ? 1u : 0u;
    }
    if (sp.seg_last && (c != g.nch - 1 || (g.more_after && g.restart_interval > 0))) out += 2;  // RSTm (extension)
    return out;
}

// workgroup (NW waves) exclusive scan; *tot receives the total
template <int NW>
__device__ __forceinline__ unsigned long long block_scan_nw(unsigned long long v, unsigned long long* sWave,
                                                            unsigned long long* tot) {
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const unsigned long long incl = wave_incl_scan_full_u64(v);  // (every thread takes part)
    if (lane == 63) sWave[wave] = incl;
    __syncthreads();
    unsigned long long pre = incl - v, all = 0;
    for (int q = 0; q < NW; ++q) {
        if (q < wave) pre += sWave[q];
        all += sWave[q];
    }
    __syncthreads();
    *tot = all;
    return pre;
}

// Segmented (flag, value) pair: value accumulated since the last segment start.
// (f1, v1) + (f2, v2) = (f1 | f2, f2 ? v2 : v1 + v2), associative.
__device__ __forceinline__ void seg_combine(bool& f, unsigned long long& v, bool f2, unsigned long long v2) {
    v = f2 ? v2 : v + v2;
    f = f || f2;
}

// workgroup (NW waves) exclusive segmented scan of (flag, value)
template <int NW>
__device__ __forceinline__ unsigned long long block_segscan_nw(bool f, unsigned long long v,
                                                               unsigned long long* sWaveV, int* sWaveF,
                                                               bool* flag_out = nullptr) {
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    bool fi = f;
    unsigned long long vi = v;
    // inclusive within the wave over DPP: row shifts 1, 2, 4, 8 (a lane without a
    // source gets (0, false), the identity), then the row broadcasts 15 and 31;
    // the earlier element is always the left operand
    auto step = [&](unsigned long long pv, int pf) {
        bool ff = pf != 0;
        seg_combine(ff, pv, fi, vi);
        fi = ff;
        vi = pv;
    };
    step(dpp_u64<0x111, 0xF, 0xF, true>(vi), __builtin_amdgcn_update_dpp(0, (int)fi, 0x111, 0xF, 0xF, true));
    step(dpp_u64<0x112, 0xF, 0xF, true>(vi), __builtin_amdgcn_update_dpp(0, (int)fi, 0x112, 0xF, 0xF, true));
    step(dpp_u64<0x114, 0xF, 0xF, true>(vi), __builtin_amdgcn_update_dpp(0, (int)fi, 0x114, 0xF, 0xF, true));
    step(dpp_u64<0x118, 0xF, 0xF, true>(vi), __builtin_amdgcn_update_dpp(0, (int)fi, 0x118, 0xF, 0xF, true));
    step(dpp_u64<0x142, 0xA, 0xF, false>(vi), __builtin_amdgcn_update_dpp(0, (int)fi, 0x142, 0xA, 0xF, false));
    step(dpp_u64<0x143, 0xC, 0xF, false>(vi), __builtin_amdgcn_update_dpp(0, (int)fi, 0x143, 0xC, 0xF, false));
    if (lane == 63) {
        sWaveV[wave] = vi;
        sWaveF[wave] = fi;
    }
    // exclusive within the wave: the previous lane's inclusive value (lane 0: identity)
    const unsigned long long ve = dpp_u64<0x138, 0xF, 0xF, true>(vi);
    const int fe = __builtin_amdgcn_update_dpp(0, (int)fi, 0x138, 0xF, 0xF, true);
    __syncthreads();
    bool cf = false;
    unsigned long long cv = 0;
    for (int q = 0; q < wave; ++q) seg_combine(cf, cv, sWaveF[q] != 0, sWaveV[q]);
    bool rf = cf;
    unsigned long long rv = cv;
    seg_combine(rf, rv, fe != 0, ve);
    __syncthreads();
    if (flag_out) *flag_out = rf;
    return rv;
}

__device__ __forceinline__ unsigned long long block_scan_1024(unsigned long long v, unsigned long long* sWave,
                                                              unsigned long long* tot) {
    return block_scan_nw<16>(v, sWave, tot);
}
__device__ __forceinline__ unsigned long long block_segscan_1024(bool f, unsigned long long v,
                                                                 unsigned long long* sWaveV, int* sWaveF) {
    return block_segscan_nw<16>(f, v, sWaveV, sWaveF);
}

// The chunk offsets of one frame computed by k_emit's last workgroup to finish
// (frames of at most kFusedOffsetsMaxChunks chunks; k_offsets otherwise): what
// k_offsets computes, with 256 threads, in rounds of kFusedRoundChunks chunks (6
// per thread in registers; 8 spill at k_emit's 72 VGPRs), each round carrying the
// bit position and the byte count of the ones before it.  The other workgroups'
// summaries (bits, 0xFF counts, edges) were stored write-through (agent scope)
// before they counted themselves in, so they are read with agent-scope loads; the
// bit scan comes first, then only the 0xFF count at each chunk's own alignment
// residue is loaded.  sWaveV holds kEmitWaves + 1 words (the last: the carry).
static_assert(kFusedRoundChunks % kEmitThreads == 0, "whole chunks per thread of the fused offsets");
static_assert(kFusedRoundChunks % (2 * kEmitThreads) == 0 && kFusedRoundChunks * 8 <= kSlotWords * kEmitThreads * 4,
              "a round's packed 0xFF counts: whole 16-byte pieces per thread, inside k_emit's slot area");
static_assert((unsigned long long)kFusedOffsetsMaxChunks * kChunkBlocks * kMaxBlockBits < (1ull << 32),
              "a fused frame's bit offsets fit 32 bits");
// (mark: phase marks of the tracer build, DMMT_PHASE_TRACE; a no-op otherwise)
template <typename Mark>
__device__ __forceinline__ void fused_offsets(const uint32_t* __restrict__ cbits, const uint32_t* __restrict__ cff,
                              const unsigned long long* __restrict__ cff8, uint8_t* sFF8,
                              const uint32_t* __restrict__ cedge, const Geom& g, unsigned long long* __restrict__ bit0,
                              unsigned long long* __restrict__ outo, unsigned long long* __restrict__ total,
                              unsigned long long* sWaveV, int* sWaveF, Mark mark) {
    // (32-bit offsets: the static_assert above; they keep the chunks' state in few registers)
    constexpr int KP = kFusedRoundChunks / kEmitThreads, NT = kEmitThreads;
    const int tid = threadIdx.x;
    const int nch = g.nch;
    uint32_t carry_run = 0, carry_out = 0;  // the bit position after, and the bytes of, the rounds before
    for (int r0 = 0; r0 < nch; r0 += kFusedRoundChunks) {  // uniform
        const int rn = min(kFusedRoundChunks, nch - r0);
        const int per = (rn + NT - 1) / NT;  // <= KP
        const int c0 = r0 + min(tid * per, rn), c1 = r0 + min(tid * per + per, rn);
#if DMMT_TAIL_DMA
        // The round's packed 0xFF counts straight into LDS (global_load_lds, 16 bytes =
        // two chunks per lane, sc1: agent scope like ld_agent), issued with the loads
        // below: the count at each chunk's residue is then an LDS read, not a second
        // round trip.  The first barrier of the bit scan waits for them.
        {
            const int npairs = (rn + 1) >> 1;
#pragma unroll
            for (int i = 0; i < kFusedRoundChunks / 2 / NT; ++i) {
                const int pc = min(i * NT + tid, npairs - 1);  // (a chunk past an odd round's end: the padding)
                __builtin_amdgcn_global_load_lds((const void*)(cff8 + r0 + 2 * pc),
                                                 (void*)(sFF8 + 16 * (i * NT + (tid & ~63))), 16, 0, 16);
            }
        }
#endif
        uint32_t nbits[KP], edge[KP];
#pragma unroll
        for (int i = 0; i < KP; ++i) {  // every load issued before any is used (clamped indices)
            const int c = min(c0 + i, nch - 1);
            nbits[i] = ld_agent(cbits + c);
            edge[i] = ld_agent(cedge + c);
        }
        const int cl = min(c1, nch - 1);  // the chunk after this thread's last
        const uint32_t nlast = ld_agent(cbits + cl), elast = ld_agent(cedge + cl);
        uint32_t firstm = 0, seglm = 0;  // per chunk i: bit i
#pragma unroll
        for (int i = 0; i < KP; ++i) nbits[i] = c0 + i < c1 ? nbits[i] : 0u;
        if (DMMT_TAIL_NSEG1 && g.nseg == 1) {  // (uniform) one segment: only chunk 0 starts it, only the frame's last ends it
            firstm = c0 == 0 && c0 < c1 ? 1u : 0u;
            seglm = c1 == nch && c0 < c1 ? 1u << (c1 - 1 - c0) : 0u;
        } else {
#pragma unroll
            for (int i = 0; i < KP; ++i) {
                const int c = c0 + i;
                if (c < c1) {
                    const ChunkSpan sp = chunk_span(g, c);
                    firstm |= (uint32_t)sp.seg_first << i;
                    seglm |= (uint32_t)sp.seg_last << i;
                }
            }
        }
        bool f = false;
        unsigned long long v = 0;
#pragma unroll
        for (int i = 0; i < KP; ++i)
            if (c0 + i < c1) seg_combine(f, v, (firstm >> i) & 1u, nbits[i] + (c0 + i == 0 ? (uint32_t)g.bit_phase : 0u));
        bool fx;
        const uint32_t ex = (uint32_t)block_segscan_nw<kEmitWaves>(f, v, sWaveV, sWaveF, &fx);
        mark(std::integral_constant<int, 7>{});  // the bits and edges loaded, the bit scan
        uint32_t run = fx ? ex : carry_run + ex;  // (a segment start before it in this round resets the carry)
        uint32_t b0[KP];
#pragma unroll
        for (int i = 0; i < KP; ++i) {
            b0[i] = 0;
            if (c0 + i < c1) {
                if ((firstm >> i) & 1u) run = c0 + i == 0 ? (uint32_t)g.bit_phase : 0u;
                b0[i] = run;
                run += nbits[i];
            }
        }
        if (c0 < c1 && c1 == r0 + rn) sWaveV[kEmitWaves] = run;  // the round's last chunk: the next carry
        uint32_t ob[KP];
#if DMMT_TAIL_DMA
#pragma unroll
        for (int i = 0; i < KP; ++i) {  // the 0xFF bytes inside the chunk at its actual alignment
            const int cc = min(c0 + i, nch - 1);
            const uint32_t slot = (8u - (b0[i] & 7u)) & 7u;
            ob[i] = sFF8[8 * (cc - r0) + slot];
            if (ob[i] == 255u) ob[i] = ld_agent(cff + (size_t)cc * 8 + slot);  // a count the byte cannot hold
        }
#else
#pragma unroll
        for (int i = 0; i < KP; ++i)  // the 0xFF bytes inside the chunk at its actual alignment
            ob[i] = ld_agent(cff + (size_t)min(c0 + i, nch - 1) * 8 + ((8 - (b0[i] & 7)) & 7));
#endif
        uint32_t mine = 0;
#pragma unroll
        for (int i = 0; i < KP; ++i) {
            const int c = c0 + i;
            if (c >= c1) {
                ob[i] = 0;
                continue;
            }
            const uint32_t e = b0[i] + nbits[i];
            uint32_t o = ((e + 7) >> 3) - ((b0[i] + 7) >> 3) + ob[i];
            if ((e & 7) && (e & ~7u) >= b0[i]) {
                // the byte shared with the next chunk of the segment (or the padding)
                const bool segl = (seglm >> i) & 1u;
                const bool jt = segl && joined_tail(g, c);
                const bool hasn = !segl || jt;
                const uint32_t nn = jt ? (uint32_t)g.next_bits : i + 1 < KP && c + 1 < c1 ? nbits[min(i + 1, KP - 1)] : nlast;
                const uint32_t en = jt ? g.next16 << 16 : i + 1 < KP && c + 1 < c1 ? edge[min(i + 1, KP - 1)] : elast;
                const uint32_t byte = boundary_byte((int)(e & 7), edge[i] & 0xFFFFu, hasn, nn, en >> 16);
                o += byte == 0xFFu ? 1u : 0u;
            }
            if (((seglm >> i) & 1u) && (c != nch - 1 || (g.more_after && g.restart_interval > 0))) o += 2;  // RSTm
            ob[i] = o;
            mine += o;
        }
        mark(std::integral_constant<int, 8>{});  // the 0xFF counts at each chunk's residue loaded, the bytes
        unsigned long long tot = 0;
        uint32_t orun = carry_out + (uint32_t)block_scan_nw<kEmitWaves>(mine, sWaveV, &tot);  // (its barriers publish the carry)
        mark(std::integral_constant<int, 9>{});  // the byte scan
#pragma unroll
        for (int i = 0; i < KP; ++i) {
            const int c = c0 + i;
            if (c >= c1) continue;
            bit0[c] = b0[i];
            outo[c] = orun;
            orun += ob[i];
        }
        carry_out += (uint32_t)tot;
        carry_run = (uint32_t)sWaveV[kEmitWaves];
        __syncthreads();  // (the carry word is rewritten by the next round)
        mark(std::integral_constant<int, 10>{});  // the offsets stored
    }
    if (tid == 0) *total = carry_out;
}

// -------------------------------------------------------------------- k_offsets
__global__ __launch_bounds__(1024) void k_offsets(const uint32_t* __restrict__ chunk_bits,
                                                  const uint32_t* __restrict__ chunk_ff,
                                                  const uint32_t* __restrict__ chunk_edge, Geom g,
                                                  unsigned long long* __restrict__ chunk_bit0,
                                                  unsigned long long* __restrict__ chunk_out,
                                                  unsigned long long* __restrict__ total_out) {
    __shared__ unsigned long long sWave[16];
    __shared__ int sWaveF[16];
    const int tid = threadIdx.x;
    const int frame = blockIdx.x;
    const int nch = g.nch;
    const uint32_t* cbits = chunk_bits + (size_t)frame * nch;
    const uint32_t* cff = chunk_ff + (size_t)frame * nch * 8;
    const uint32_t* cedge = chunk_edge + (size_t)frame * nch;
    unsigned long long* bit0 = chunk_bit0 + (size_t)frame * nch;
    unsigned long long* outo = chunk_out + (size_t)frame * nch;
    const int per = (nch + 1023) / 1024;
    const int c0 = min(tid * per, nch), c1 = min(c0 + per, nch);

    constexpr int KP = 2;
    if (per <= KP) {  // uniform: every input of the chunk in registers before the scans
        uint32_t nbits[KP], ffr[KP][8], edge[KP], nnext[KP], enext[KP];
        bool first[KP], segl[KP], hasn[KP];
#pragma unroll
        for (int i = 0; i < KP; ++i) {
            const int c = c0 + i;
            nbits[i] = edge[i] = nnext[i] = enext[i] = 0u;
            first[i] = segl[i] = hasn[i] = false;
#pragma unroll
            for (int r = 0; r < 8; ++r) ffr[i][r] = 0u;
            if (c < c1) {
                const ChunkSpan sp = chunk_span(g, c);
                first[i] = sp.seg_first;
                segl[i] = sp.seg_last;
                hasn[i] = !sp.seg_last;
                nbits[i] = cbits[c];
                edge[i] = cedge[c];
                const uint4 a = reinterpret_cast<const uint4*>(cff + (size_t)c * 8)[0];
                const uint4 b = reinterpret_cast<const uint4*>(cff + (size_t)c * 8)[1];
                ffr[i][0] = a.x, ffr[i][1] = a.y, ffr[i][2] = a.z, ffr[i][3] = a.w;
                ffr[i][4] = b.x, ffr[i][5] = b.y, ffr[i][6] = b.z, ffr[i][7] = b.w;
                if (!sp.seg_last) {
                    nnext[i] = cbits[c + 1];
                    enext[i] = cedge[c + 1];
                } else if (joined_tail(g, c)) {
                    hasn[i] = true;
                    nnext[i] = (uint32_t)g.next_bits;
                    enext[i] = g.next16 << 16;
                }
            }
        }
        bool f = false;
        unsigned long long v = 0;
#pragma unroll
        for (int i = 0; i < KP; ++i)
            if (c0 + i < c1) seg_combine(f, v, first[i], nbits[i] + (c0 + i == 0 ? (uint32_t)g.bit_phase : 0u));
        unsigned long long run = block_segscan_1024(f, v, sWave, sWaveF);
        unsigned long long b0[KP], ob[KP], mine = 0;
#pragma unroll
        for (int i = 0; i < KP; ++i) {
            const int c = c0 + i;
            b0[i] = ob[i] = 0;
            if (c >= c1) continue;
            if (first[i]) run = c == 0 ? (unsigned long long)g.bit_phase : 0ull;
            b0[i] = run;
            const unsigned long long e = run + nbits[i];
            unsigned long long o = ((e + 7) >> 3) - ((run + 7) >> 3);
            const int rsd = (8 - (int)(run & 7)) & 7;
            uint32_t ffc = 0;
#pragma unroll
            for (int r = 0; r < 8; ++r) ffc = r == rsd ? ffr[i][r] : ffc;
            o += ffc;
            if ((e & 7) && (e & ~7ull) >= run) {
                const uint32_t byte = boundary_byte((int)(e & 7), edge[i] & 0xFFFFu, hasn[i], nnext[i], enext[i] >> 16);
                o += byte == 0xFFu ? 1u : 0u;
            }
            if (segl[i] && (c != nch - 1 || (g.more_after && g.restart_interval > 0))) o += 2;  // RSTm (extension)
            ob[i] = o;
            mine += o;
            run = e;
        }
        unsigned long long tot = 0;
        unsigned long long orun = block_scan_1024(mine, sWave, &tot);
#pragma unroll
        for (int i = 0; i < KP; ++i) {
            const int c = c0 + i;
            if (c >= c1) continue;
            bit0[c] = b0[i];
            outo[c] = orun;
            orun += ob[i];
        }
        if (tid == 0) total_out[frame] = tot;
        return;
    }

    // bit offsets inside the restart segments: segmented scan of the chunk bits
    bool f = false;
    unsigned long long v = 0;
    for (int c = c0; c < c1; ++c)
        seg_combine(f, v, chunk_span(g, c).seg_first, cbits[c] + (c == 0 ? (unsigned long long)g.bit_phase : 0ull));
    unsigned long long run = block_segscan_1024(f, v, sWave, sWaveF);
    unsigned long long mine = 0;
    for (int c = c0; c < c1; ++c) {
        if (chunk_span(g, c).seg_first) run = c == 0 ? (unsigned long long)g.bit_phase : 0ull;
        bit0[c] = run;
        mine += chunk_out_bytes(cff, cbits, cedge, g, c, run);
        run += cbits[c];
    }
    // output offsets: plain scan of the chunk output bytes
    unsigned long long tot = 0;
    unsigned long long orun = block_scan_1024(mine, sWave, &tot);
    for (int c = c0; c < c1; ++c) {
        outo[c] = orun;
        orun += chunk_out_bytes(cff, cbits, cedge, g, c, bit0[c]);
    }
    if (tid == 0) total_out[frame] = tot;
}

// ----------------------------------------------------------------- k_stuffwrite
__global__ __launch_bounds__(256, 8) void k_stuffwrite(const uint32_t* __restrict__ stage,
                                                    const uint32_t* __restrict__ chunk_bits,
                                                    const uint32_t* __restrict__ chunk_edge,
                                                    const unsigned long long* __restrict__ chunk_bit0,
                                                    const unsigned long long* __restrict__ chunk_out,
                                                    const unsigned long long* __restrict__ total_out,
                                                    const uint32_t* __restrict__ hdr_len, Geom g,
                                                    uint8_t* __restrict__ out, size_t out_stride,
                                                    uint32_t* __restrict__ out_len, int* __restrict__ status) {
    __shared__ uint32_t sWave[4];
    __shared__ __attribute__((aligned(16))) uint8_t sOut[2 * kStuffPass + 16];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const int c = blockIdx.x;
    const size_t cid = (size_t)frame * g.nch + c;
    const bool last = c == g.nch - 1;
    const size_t cidn = last ? cid : cid + 1;
    // every global load of the prologue is issued before any is used: the frame's
    // and the chunk's words, the next chunk's (its bits and edge for the shared last
    // byte, its output offset for a closing RSTm), and this thread's slot words of
    // the first pass -- word 4 tid on, whatever the chunk's first bit (which lies in
    // the slot's first byte) -- so one latency, not four
    const uint32_t hdr = hdr_len[frame];
    const unsigned long long tot = total_out[frame];
    const unsigned long long b0 = chunk_bit0[cid];
    const uint32_t n = chunk_bits[cid], edge = chunk_edge[cid];
    const uint32_t n_next = chunk_bits[cidn], edge_next = chunk_edge[cidn];
    const unsigned long long cout = chunk_out[cid], cout_next = chunk_out[cidn];
    const uint32_t* slot = stage + cid * (size_t)kChunkWordsCap;
    uint32_t wv0[5];
    {
        const uint4 q = *reinterpret_cast<const uint4*>(slot + 4 * tid);
        wv0[0] = q.x, wv0[1] = q.y, wv0[2] = q.z, wv0[3] = q.w;
        wv0[4] = slot[4 * tid + 4];
    }
    // (the compiler would sink each load to its first use, past the branches below)
    asm volatile("" ::"s"(hdr), "s"(tot), "s"(b0), "s"(n), "s"(edge), "s"(n_next), "s"(edge_next), "s"(cout),
                 "s"(cout_next), "v"(wv0[0]), "v"(wv0[1]), "v"(wv0[2]), "v"(wv0[3]), "v"(wv0[4]));
    const unsigned long long end = (unsigned long long)hdr + tot;
    if (end + 2 > out_stride) {  // uniform over the frame
        if (c == 0 && tid == 0) {
            out_len[frame] = 0;  // reported as DMMT_E_CAPACITY by the host
            raise_status(status, 16);
        }
        return;
    }
    // This chunk's own summary, checked before any store (uniform over the
    // workgroup, a few scalar compares): its bits fit its staging slot, and its
    // stuffed bytes -- at most two per scan byte, the closing RST marker included
    // -- lie between its offset and the next chunk's (the frame total for the last)
    // inside the frame's output slot.  The summaries come from k_emit and the offsets
    // scan, so this only fires on a broken producer (the round-5 grouped-offsets
    // timing ablation, which left the per-chunk offsets unset, stored through them
    // and faulted: profiles/r05_grouped_offsets_ab.txt); it then raises the capacity
    // error instead of writing out of bounds.
    {
        const unsigned long long cend = last ? tot : cout_next;
        const unsigned long long sbytes = ((unsigned long long)n + 7) / 8 + 1;
        if (n > (uint32_t)kChunkWordsCap * 32u || cout > cend || cend > tot ||
            (unsigned long long)hdr + cout + 2 * sbytes > out_stride) {
            if (tid == 0) {
                out_len[frame] = 0;
                raise_status(status, 16);
            }
            return;
        }
    }
    const ChunkSpan sp = chunk_span(g, c);
    uint8_t* const base = out + (size_t)frame * out_stride + hdr;
    if (tid == 0) {
        if (last && !g.more_after) {  // EOI (encoder.rs:131) and the file size
            base[tot] = 0xFF;
            base[tot + 1] = 0xD9;
            out_len[frame] = (uint32_t)(end + 2);
        } else if (sp.seg_last && g.restart_interval > 0) {  // RSTm closing restart segment m (extension; not stuffed)
            const unsigned long long at = (last ? tot : cout_next) - 2;
            base[at] = 0xFF;
            base[at + 1] = (uint8_t)(0xD0 + ((g.seg_base + sp.seg) & 7));
            if (last) out_len[frame] = (uint32_t)end;  // a stripe that more stripes follow
        } else if (last) {
            out_len[frame] = (uint32_t)end;  // a joined stripe that more stripes follow
        }
    }
    const unsigned long long e = b0 + n;
    const unsigned long long kbeg = (b0 + 7) >> 3, kend = (e + 7) >> 3;
    if (kend <= kbeg) return;  // a tail chunk inside the previous chunk's last byte
    const unsigned long long nbytes = kend - kbeg;
    // the chunk's last byte, when shared with the next chunk or the padding
    const bool shared_tail = (e & 7) != 0;
    uint32_t tail = 0;
    if (shared_tail) {
        const bool jt = joined_tail(g, c);
        const bool has_next = !sp.seg_last || jt;
        tail = boundary_byte((int)(e & 7), edge & 0xFFFFu, has_next,
                             jt ? (uint32_t)g.next_bits : (has_next ? n_next : 0u),
                             jt ? g.next16 : (has_next ? edge_next >> 16 : 0u));
    }
    const unsigned off = (unsigned)(8 * kbeg - b0);  // the first owned byte starts this many bits into the chunk
    uint8_t* o = base + cout;
    for (unsigned long long pos = 0; pos < nbytes; pos += kStuffPass) {  // uniform
        // the pass is staged at o's alignment (sOut[delta + i] = output byte i), so
        // it leaves LDS in aligned 16-byte stores
        const uint32_t delta = (uint32_t)(reinterpret_cast<uintptr_t>(o) & 15u);
        const unsigned long long kb = pos + 16u * (unsigned)tid;          // first of my 16 bytes (chunk-relative)
        const int nvalid = kb < nbytes ? (int)min(16ull, nbytes - kb) : 0;
        uint32_t x[4] = {0u, 0u, 0u, 0u};  // my 16 bytes, MSB first
        uint32_t cnt = 0;
        if (nvalid) {
            const unsigned long long p = off + 8 * kb;  // bit position in the chunk stream (off < 8)
            const size_t wi = (size_t)(p >> 5);
            const int sh = (int)(p & 31);
            uint32_t wv[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) wv[i] = pos ? slot[wi + i] : wv0[i];  // (pass 0: wi = 4 tid)
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = sh ? (wv[i] << sh) | (wv[i + 1] >> (32 - sh)) : wv[i];
            if (shared_tail && nbytes - 1 - kb < 16) {  // the shared / padded last byte
                const int j = (int)(nbytes - 1 - kb), sft = 24 - 8 * (j & 3);
                x[j >> 2] = (x[j >> 2] & ~(0xFFu << sft)) | (tail << sft);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {  // 0xFF bytes among the valid ones
                const int nv = min(max(nvalid - 4 * i, 0), 4);
                const uint32_t vmask = nv ? 0x80808080u & (0xFFFFFFFFu << (32 - 8 * nv)) : 0u;
                const uint32_t t = ~x[i];
                const uint32_t nonzero = (((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
                cnt += (uint32_t)__popc(~nonzero & vmask);
            }
        }
        const uint32_t incl = wave_incl_scan_full_u32(cnt);
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        uint32_t pre = incl - cnt;
        for (int q = 0; q < wave; ++q) pre += sWave[q];
        const uint32_t ffs = sWave[0] + sWave[1] + sWave[2] + sWave[3];
        // stage the stuffed pass in LDS, then store it with consecutive lanes on
        // consecutive bytes (coalesced)
        if (nvalid) {
            uint32_t dst = delta + (uint32_t)tid * 16u + pre;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (j < nvalid) {
                    const uint32_t b = (x[j >> 2] >> (24 - 8 * (j & 3))) & 0xFFu;
                    sOut[dst++] = (uint8_t)b;
                    if (b == 0xFFu) sOut[dst++] = 0x00;
                }
            }
        }
        __syncthreads();
        const unsigned long long in_pass = nbytes - pos < (unsigned long long)kStuffPass ? nbytes - pos : kStuffPass;
        const uint32_t len = (uint32_t)in_pass + ffs;
        const uint32_t send = delta + len;  // staged bytes [delta, send)
        uint8_t* const oa = o - delta;      // 16-byte aligned
        for (uint32_t sb = 16u * (uint32_t)tid; sb < send; sb += 16u * 256u) {
            if (sb >= delta && sb + 16u <= send) {
                *reinterpret_cast<uint4*>(oa + sb) = *reinterpret_cast<const uint4*>(sOut + sb);
            } else {  // the pass's first and last 16-byte pieces: only its own bytes
                for (uint32_t i = max(sb, delta); i < min(sb + 16u, send); ++i) oa[i] = sOut[i];
            }
        }
        o += len;
        __syncthreads();  // sWave / sOut reuse
    }
}

// --------------------------------------------------------------------- launchers
bool offsets_fusable(const Geom& g) { return g.nch <= kFusedOffsetsMaxChunks; }

hipError_t launch_emit(int n_frames, const Geom& g, const Work& w, bool fuse_offsets, hipStream_t st, bool prio) {
    const int fuse = fuse_offsets && offsets_fusable(g) ? 1 : 0;
    hipLaunchKernelGGL(k_emit, dim3(g.nch, n_frames), dim3(kEmitThreads), 0, st, (const int16_t*)w.coef,
                       (const int16_t*)w.dcdiff, (const uint8_t*)w.lastnz, (const uint32_t*)w.code_tab, g, w.stage, w.chunk_bits, w.chunk_ff,
                       w.chunk_edge, w.ac_hist, w.dc_hist, fuse, w.arrive, w.chunk_bit0, w.chunk_out, w.total_out,
                       w.chunk_ff8, prio || DMMT_EMIT_PRIO_ALWAYS ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_offsets(int n_frames, const Geom& g, const Work& w, hipStream_t st) {
    hipLaunchKernelGGL(k_offsets, dim3(n_frames), dim3(1024), 0, st, (const uint32_t*)w.chunk_bits,
                       (const uint32_t*)w.chunk_ff, (const uint32_t*)w.chunk_edge, g, w.chunk_bit0, w.chunk_out,
                       w.total_out);
    return hipGetLastError();
}

hipError_t launch_stuffwrite(int n_frames, const Geom& g, const Work& w, uint8_t* out, size_t out_stride,
                             uint32_t* out_len, hipStream_t st) {
    hipLaunchKernelGGL(k_stuffwrite, dim3(g.nch, n_frames), dim3(256), 0, st, (const uint32_t*)w.stage,
                       (const uint32_t*)w.chunk_bits, (const uint32_t*)w.chunk_edge,
                       (const unsigned long long*)w.chunk_bit0, (const unsigned long long*)w.chunk_out,
                       (const unsigned long long*)w.total_out, (const uint32_t*)w.hdr_len, g, out, out_stride,
                       out_len, w.status);
    return hipGetLastError();
}

}  // namespace dmmt

#ifdef DMMT_PHASE_TRACE
extern "C" int dmmt_debug_trace_entropy(unsigned long long* out64) {
    if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(dmmt::g_trace), 64 * 8) != hipSuccess) return -1;
    unsigned long long z[64] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(dmmt::g_trace), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
