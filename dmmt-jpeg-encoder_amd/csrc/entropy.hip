// entropy.hip -- gfx950 entropy-coding back half: bit packing and byte stuffing.
//
// Four launches, no inter-workgroup waiting anywhere:
//  k_bits        one workgroup per chunk of kChunkBlocks blocks: bits of every
//                block (kept for k_place) and the chunk total; the total is also
//                added into its "super" counter (kSuper chunks per super).
//  k_place       one workgroup per chunk: its bit offset in the frame's scan is
//                the sum of the supers before it plus the chunk totals before it
//                in its own super (a few dozen L2 reads), block offsets by a
//                wave scan, every code placed MSB-first into an LDS word image
//                which goes out byte-swapped (memory order = stream order).
//                [encoder.rs:264-404 write_image_data / write_{dc,ac}_from_block,
//                binary_stream.rs:38-66 BitWriter]
//  k_ffcount     0xFF bytes per kStuffSeg-byte segment of the packed scan (+ super
//                counters), the last byte padded with 1-bits (binary_stream.rs:89-96)
//  k_stuffwrite  segment offset from the same two-level sums; the bytes after the
//                header with a 0x00 after every 0xFF (segment_marker_injector.rs:13-30),
//                EOI (encoder.rs:131), file size; zeroes the packed words it read so
//                the next launch's k_place can OR into a clean buffer.
//
// The bit passes run one thread per block (256 blocks per workgroup): the walk
// over a block's 64 coefficients is serial by nature and cheapest as a fully
// unrolled register loop; the workgroup scan of the block bit counts gives
// every thread its exact bit position.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "jpeg_common.hpp"
#include "kernels.hpp"

namespace dmmt {

#ifdef DMMT_PHASE_TRACE
static __device__ unsigned long long g_trace[64];
#endif

// Sum of the counters before index `i` of a two-level (super, item) counter set,
// by one wave: supers [0, i/kSuper) + items [kSuper*(i/kSuper), i).
template <typename T>
__device__ __forceinline__ unsigned long long prefix_two_level(const unsigned long long* __restrict__ supers,
                                                               const T* __restrict__ items, unsigned i) {
    const int lane = lane_id();
    const unsigned s = i / kSuper;
    unsigned long long acc = 0;
    for (unsigned j = (unsigned)lane; j < s; j += 64) acc += supers[j];
    for (unsigned j = s * kSuper + (unsigned)lane; j < i; j += 64) acc += (unsigned long long)items[j];
    return wave_sum_u64(acc);
}

static_assert(kChunkBlocks == 256, "one thread per block, one workgroup per chunk");

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

__device__ __forceinline__ int coef_at(const BlockCoef& b, int k) {
    return (k & 1) ? ((int)b.w[k >> 1] >> 16) : (int)(int16_t)(b.w[k >> 1] & 0xFFFFu);
}

template <typename Sink>
__device__ __forceinline__ void walk_block(const BlockCoef& b, int dcd, const uint32_t* __restrict__ dctab,
                                           const uint32_t* __restrict__ actab, Sink& sink) {
    {
        const int cat = category_of(dcd);
        const uint32_t e = dctab[cat];
        sink(((e & 0xFFFFu) << cat) | extra_bits(dcd, cat), (int)(e >> 16) + cat);
    }
    const uint32_t z = actab[0xF0];
    int run = 0;
#pragma unroll
    for (int k = 1; k < 64; ++k) {
        const int v = coef_at(b, k);
        if (v != 0) {
            for (int r = run >> 4; r > 0; --r) sink(z & 0xFFFFu, (int)(z >> 16));
            const int cat = category_of(v);
            const uint32_t e = actab[((run & 15) << 4) | cat];
            sink(((e & 0xFFFFu) << cat) | extra_bits(v, cat), (int)(e >> 16) + cat);
            run = 0;
        } else {
            ++run;
        }
    }
    if (run) {
        const uint32_t e = actab[0];  // EOB
        sink(e & 0xFFFFu, (int)(e >> 16));
    }
}

struct CountSink {
    uint32_t n = 0;
    __device__ __forceinline__ void operator()(uint32_t, int len) { n += (uint32_t)len; }
};

// Appends pieces MSB-first into a word image: words wholly inside the block are
// stored plainly, the first and last (shared with the neighbouring blocks) are
// ORed atomically.  LDS image = MSB-first words; global image (slow path) =
// byte-swapped words (memory order = stream order).
struct EmitSink {
    uint32_t* img;
    bool lds;
    unsigned long long acc;
    int nacc;     // bits pending in acc
    size_t w;     // next word index
    bool first;
    __device__ __forceinline__ void put(uint32_t word, bool shared) {
        const uint32_t v = lds ? word : __builtin_bswap32(word);
        if (shared)
            atomicOr(&img[w], v);
        else
            img[w] = v;
    }
    __device__ __forceinline__ void operator()(uint32_t val, int len) {
        acc = (acc << len) | val;
        nacc += len;
        if (nacc >= 32) {
            nacc -= 32;
            put((uint32_t)(acc >> nacc), first);
            first = false;
            ++w;
            acc &= (1ull << nacc) - 1ull;
        }
    }
    __device__ __forceinline__ void finish() {
        if (nacc > 0) put((uint32_t)(acc << (32 - nacc)), true);
    }
};

// ---------------------------------------------------------------------- k_bits
__global__ __launch_bounds__(256) void k_bits(const int16_t* __restrict__ coef, const int16_t* __restrict__ dcdiff,
                                              const uint32_t* __restrict__ code_tab, Geom g,
                                              uint16_t* __restrict__ block_bits, uint32_t* __restrict__ chunk_bits,
                                              unsigned long long* __restrict__ super_bits,
                                              uint32_t* __restrict__ ac_hist, uint32_t* __restrict__ dc_hist) {
    __shared__ uint32_t sTab[4 * 256];
    __shared__ uint32_t sWave[4];
    DMMT_TRACE_START;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const unsigned chunk = blockIdx.x;
    const long long el0 = (long long)chunk * kChunkBlocks;
    const int nb = (int)min((long long)kChunkBlocks, g.bpf - el0);
    const long long e = (long long)frame * g.bpf + el0 + tid;
    for (int i = tid; i < 1024; i += 256) sTab[i] = code_tab[(size_t)frame * 1024 + i];
    if (chunk == 0) {  // the histogram replicas k_tables read: zero for the next launch
        for (int i = tid; i < kHistReps * 512; i += 256) ac_hist[(size_t)frame * kHistReps * 512 + i] = 0u;
        for (int i = tid; i < kHistReps * 32; i += 256) dc_hist[(size_t)frame * kHistReps * 32 + i] = 0u;
    }
    const bool valid = tid < nb;
    BlockCoef b;
    int dcd = 0;
    if (valid) {
        load_block(coef + e * 64, b);
        dcd = dcdiff[e];
    }
    __syncthreads();
    DMMT_TRACE(0);
    uint32_t bits = 0;
    if (valid) {
        const int k = ((int)(el0 % g.bpm) + tid) % g.bpm;
        const uint32_t* tb = sTab + (k < g.n_luma ? 0 : 512);
        CountSink cs;
        walk_block(b, dcd, tb, tb + 256, cs);
        bits = cs.n;
        block_bits[e] = (uint16_t)bits;
    }
    const uint32_t ws = wave_sum_u32(bits);
    if (lane == 0) sWave[wave] = ws;
    __syncthreads();
    if (tid == 0) {
        const uint32_t total = sWave[0] + sWave[1] + sWave[2] + sWave[3];
        chunk_bits[(size_t)frame * g.nch + chunk] = total;
        atomicAdd(&super_bits[(size_t)frame * g.nsuper + chunk / kSuper], (unsigned long long)total);
    }
    DMMT_TRACE(1);
    DMMT_TRACE_FLUSH(0);
}

// --------------------------------------------------------------------- k_place
// LDS word image capacity of one chunk: 128 Ki bits = 512 bits per block on
// average (the 4K q90 workload averages ~110).  A chunk that needs more (worst
// case kMaxBlockBits per block) writes straight into the zeroed global buffer
// instead: slower, same bytes.
constexpr int kPackWords = 4096;

__global__ __launch_bounds__(256) void k_place(const int16_t* __restrict__ coef, const int16_t* __restrict__ dcdiff,
                                               const uint32_t* __restrict__ code_tab, Geom g,
                                               const uint16_t* __restrict__ block_bits,
                                               const uint32_t* __restrict__ chunk_bits,
                                               const unsigned long long* __restrict__ super_bits,
                                               unsigned long long* __restrict__ total_bits,
                                               uint32_t* __restrict__ packed, int* __restrict__ status) {
    __shared__ uint32_t sW[kPackWords + 2];
    __shared__ uint32_t sTab[4 * 256];
    __shared__ uint32_t sWave[4];
    __shared__ unsigned long long sBase;
    DMMT_TRACE_START;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const unsigned chunk = blockIdx.x;
    const long long el0 = (long long)chunk * kChunkBlocks;
    const int nb = (int)min((long long)kChunkBlocks, g.bpf - el0);
    const long long e = (long long)frame * g.bpf + el0 + tid;
    for (int i = tid; i < 1024; i += 256) sTab[i] = code_tab[(size_t)frame * 1024 + i];
    const bool valid = tid < nb;
    BlockCoef b;
    int dcd = 0;
    uint32_t mine = 0;
    if (valid) {
        load_block(coef + e * 64, b);
        dcd = dcdiff[e];
        mine = block_bits[e];
    }
    // block offsets within the chunk: workgroup scan of the block bit counts
    const uint32_t incl = wave_incl_scan_u32(mine);
    if (lane == 63) sWave[wave] = incl;
    if (wave == 0) {
        const unsigned long long pre =
            prefix_two_level(super_bits + (size_t)frame * g.nsuper, chunk_bits + (size_t)frame * g.nch, chunk);
        if (lane == 0) sBase = pre;
    }
    __syncthreads();
    DMMT_TRACE(4);
    uint32_t wpre = 0;
    for (int w = 0; w < wave; ++w) wpre += sWave[w];
    const uint32_t total = sWave[0] + sWave[1] + sWave[2] + sWave[3];
    const unsigned long long bit0 = sBase;
    if (tid == 0 && chunk == (unsigned)g.nch - 1) total_bits[frame] = bit0 + total;
    const int shift = (int)(bit0 & 31);
    const int nw = (int)((shift + (unsigned long long)total + 31) >> 5);
    if (((bit0 + total + 31) >> 5) + 1 > (unsigned long long)g.packed_words) {
        if (tid == 0) atomicOr(status, 8);
        return;  // uniform; the host reports DMMT_E_CAPACITY
    }
    uint32_t* const pk = packed + (size_t)frame * g.packed_words + (bit0 >> 5);
    const bool in_lds = nw + 1 <= kPackWords + 2;
    if (in_lds)
        for (int i = tid; i < nw + 1; i += 256) sW[i] = 0u;
    __syncthreads();
    DMMT_TRACE(5);
    if (valid) {
        const int k = ((int)(el0 % g.bpm) + tid) % g.bpm;
        const uint32_t* tb = sTab + (k < g.n_luma ? 0 : 512);
        const uint32_t start = (uint32_t)shift + wpre + incl - mine;  // bit position in the image
        EmitSink es{in_lds ? sW : pk, in_lds, 0ull, (int)(start & 31), (size_t)(start >> 5), true};
        walk_block(b, dcd, tb, tb + 256, es);
        es.finish();
    }
    __syncthreads();
    DMMT_TRACE(6);
    if (in_lds) {  // interior words plain, the two edge words ORed (shared with neighbouring chunks)
        for (int i = tid; i < nw; i += 256) {
            const uint32_t v = __builtin_bswap32(sW[i]);
            if (i == 0 || i == nw - 1)
                atomicOr(&pk[i], v);
            else
                pk[i] = v;
        }
    }
    DMMT_TRACE(7);
    DMMT_TRACE_FLUSH(0);
}

// ------------------------------------------------------------------- stuffing
struct ScanBytes {
    unsigned long long nbytes;
    unsigned pad;  // 1-bits padding the last byte
    unsigned nseg;
};

__device__ __forceinline__ ScanBytes scan_bytes(unsigned long long tb) {
    ScanBytes s;
    s.nbytes = (tb + 7) >> 3;
    s.pad = (unsigned)((8 - (tb & 7)) & 7);
    s.nseg = (unsigned)((s.nbytes + kStuffSeg - 1) / kStuffSeg);
    return s;
}

// The 16 scan bytes of thread `tid` in segment `seg` (the last byte 1-padded) and
// their 0xFF count; with `clear` also zeroes the packed words read (k_stuffwrite:
// restores the all-zero invariant for the next launch's k_place).
__device__ __forceinline__ uint32_t load16(uint8_t* __restrict__ pb, const ScanBytes& s, unsigned seg, int tid,
                                           uint8_t (&v)[16], bool clear) {
    const unsigned long long b0 = (unsigned long long)seg * kStuffSeg + (unsigned)tid * 16u;
    if (b0 + 16 <= s.nbytes) {
        const uint4 q = *reinterpret_cast<const uint4*>(pb + b0);
        const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = (uint8_t)(wv[j >> 2] >> (8 * (j & 3)));
        if (clear) *reinterpret_cast<uint4*>(pb + b0) = make_uint4(0, 0, 0, 0);
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = b0 + j < s.nbytes ? pb[b0 + j] : 0;
        if (clear) {
            const unsigned long long wend = (s.nbytes + 3) >> 2;
            for (int j = 0; j < 4; ++j) {
                const unsigned long long wi = (b0 >> 2) + j;
                if (wi < wend) reinterpret_cast<uint32_t*>(pb)[wi] = 0u;
            }
        }
    }
    const unsigned long long last = s.nbytes - 1;
    if (s.pad && b0 <= last && last < b0 + 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (b0 + j == last) v[j] |= (uint8_t)((1u << s.pad) - 1u);
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) cnt += (b0 + j < s.nbytes && v[j] == 0xFF) ? 1u : 0u;
    return cnt;
}

__global__ __launch_bounds__(256) void k_ffcount(uint32_t* __restrict__ packed,
                                                 const unsigned long long* __restrict__ total_bits, Geom g,
                                                 uint32_t* __restrict__ seg_ff, unsigned long long* __restrict__ super_ff) {
    __shared__ uint32_t sWave[4];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const ScanBytes s = scan_bytes(total_bits[frame]);
    if (s.nbytes > (unsigned long long)g.packed_words * 4) return;
    uint8_t* pb = reinterpret_cast<uint8_t*>(packed + (size_t)frame * g.packed_words);
    for (unsigned seg = blockIdx.x; seg < s.nseg; seg += gridDim.x) {
        uint8_t v[16];
        const uint32_t cnt = wave_sum_u32(load16(pb, s, seg, tid, v, false));
        if (lane == 0) sWave[wave] = cnt;
        __syncthreads();
        if (tid == 0) {
            const uint32_t tot = sWave[0] + sWave[1] + sWave[2] + sWave[3];
            seg_ff[(size_t)frame * g.nseg_cap + seg] = tot;
            if (tot) atomicAdd(&super_ff[(size_t)frame * g.nsuper_seg + seg / kSuper], (unsigned long long)tot);
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_stuffwrite(uint32_t* __restrict__ packed,
                                                    const unsigned long long* __restrict__ total_bits,
                                                    const uint32_t* __restrict__ hdr_len, Geom g,
                                                    const uint32_t* __restrict__ seg_ff,
                                                    const unsigned long long* __restrict__ super_ff,
                                                    uint8_t* __restrict__ out, size_t out_stride,
                                                    uint32_t* __restrict__ out_len, int* __restrict__ status) {
    __shared__ uint32_t sWave[4];
    __shared__ unsigned long long sBase;
    __shared__ uint8_t sOut[2 * kStuffSeg];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const ScanBytes s = scan_bytes(total_bits[frame]);
    const uint32_t hdr = hdr_len[frame];
    const bool fits = s.nbytes <= (unsigned long long)g.packed_words * 4 && hdr + 2 * s.nbytes + 2 <= out_stride;
    if (!fits) {
        if (blockIdx.x == 0 && tid == 0) {
            out_len[frame] = 0;  // reported as DMMT_E_CAPACITY by the host
            atomicOr(status, 16);
        }
        return;
    }
    uint8_t* pb = reinterpret_cast<uint8_t*>(packed + (size_t)frame * g.packed_words);
    uint8_t* o = out + (size_t)frame * out_stride + hdr;
    for (unsigned seg = blockIdx.x; seg < s.nseg; seg += gridDim.x) {
        uint8_t v[16];
        const uint32_t cnt = load16(pb, s, seg, tid, v, true);
        const uint32_t incl = wave_incl_scan_u32(cnt);
        if (lane == 63) sWave[wave] = incl;
        if (wave == 0) {
            const unsigned long long pre = prefix_two_level(super_ff + (size_t)frame * g.nsuper_seg,
                                                            seg_ff + (size_t)frame * g.nseg_cap, seg);
            if (lane == 0) sBase = pre;
        }
        __syncthreads();
        // stage the stuffed segment in LDS, then store it with consecutive lanes on
        // consecutive bytes (coalesced)
        uint32_t pre = 0;
        for (int w = 0; w < wave; ++w) pre += sWave[w];
        uint32_t dst = (uint32_t)tid * 16u + pre + (incl - cnt);
        const unsigned long long b0 = (unsigned long long)seg * kStuffSeg + (unsigned)tid * 16u;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (b0 + j < s.nbytes) {
                sOut[dst++] = v[j];
                if (v[j] == 0xFF) sOut[dst++] = 0x00;
            }
        }
        __syncthreads();
        const unsigned long long seg0 = (unsigned long long)seg * kStuffSeg;
        const unsigned long long in_seg = s.nbytes - seg0 < (unsigned long long)kStuffSeg ? s.nbytes - seg0 : kStuffSeg;
        const uint32_t ffs = sWave[0] + sWave[1] + sWave[2] + sWave[3];
        const uint32_t seg_len = (uint32_t)in_seg + ffs;
        uint8_t* od = o + seg0 + sBase;
        for (uint32_t i = (uint32_t)tid; i < seg_len; i += 256) od[i] = sOut[i];
        if (tid == 0 && seg == s.nseg - 1) {  // EOI (encoder.rs:131) and the file size
            const unsigned long long total = (unsigned long long)hdr + s.nbytes + sBase + ffs;
            uint8_t* of = out + (size_t)frame * out_stride;
            of[total] = 0xFF;
            of[total + 1] = 0xD9;
            out_len[frame] = (uint32_t)(total + 2);
        }
        __syncthreads();  // sWave / sBase / sOut reuse
    }
}

// --------------------------------------------------------------------- launchers
hipError_t launch_bits(int n_frames, const Geom& g, const Work& w, hipStream_t st) {
    hipLaunchKernelGGL(k_bits, dim3(g.nch, n_frames), dim3(256), 0, st, (const int16_t*)w.coef,
                       (const int16_t*)w.dcdiff, (const uint32_t*)w.code_tab, g, w.block_bits, w.chunk_bits,
                       w.super_bits, w.ac_hist, w.dc_hist);
    return hipGetLastError();
}

hipError_t launch_place(int n_frames, const Geom& g, const Work& w, hipStream_t st) {
    hipLaunchKernelGGL(k_place, dim3(g.nch, n_frames), dim3(256), 0, st, (const int16_t*)w.coef,
                       (const int16_t*)w.dcdiff, (const uint32_t*)w.code_tab, g, (const uint16_t*)w.block_bits,
                       (const uint32_t*)w.chunk_bits, (const unsigned long long*)w.super_bits, w.total_bits, w.packed,
                       w.status);
    return hipGetLastError();
}

static int seg_grid(const Geom& g, int n_frames) {
    int per_frame = 2048 / n_frames;
    if (per_frame < 1) per_frame = 1;
    const int cap = g.nseg_cap < 1 ? 1 : g.nseg_cap;
    return cap < per_frame ? cap : per_frame;
}

hipError_t launch_ffcount(int n_frames, const Geom& g, const Work& w, hipStream_t st) {
    hipLaunchKernelGGL(k_ffcount, dim3(seg_grid(g, n_frames), n_frames), dim3(256), 0, st, w.packed,
                       (const unsigned long long*)w.total_bits, g, w.seg_ff, w.super_ff);
    return hipGetLastError();
}

hipError_t launch_stuffwrite(int n_frames, const Geom& g, const Work& w, uint8_t* out, size_t out_stride,
                             uint32_t* out_len, hipStream_t st) {
    hipLaunchKernelGGL(k_stuffwrite, dim3(seg_grid(g, n_frames), n_frames), dim3(256), 0, st, w.packed,
                       (const unsigned long long*)w.total_bits, (const uint32_t*)w.hdr_len, g,
                       (const uint32_t*)w.seg_ff, (const unsigned long long*)w.super_ff, out, out_stride, out_len,
                       w.status);
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
