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
// Lane layout of the bit passes: 16 lanes per block, 4 blocks per wave; lane l
// of a block owns zigzag positions 4l..4l+3 (one 8-byte load).  The previous
// non-zero coefficient before a lane's first position comes from a ballot of
// "lane has a non-zero" and one shuffle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "jpeg_common.hpp"
#include "kernels.hpp"

namespace dmmt {

static_assert(kChunkBlocks == 64, "one wave scans the block offsets of a chunk");

// Token walk of one lane's 4 zigzag positions in stream order (encoder.rs:356-404),
// without data-dependent branches so the 16 lanes of a block run in lockstep.
// Position 0 = DC: code(cat(diff)) + extra bits.  A non-zero AC coefficient:
// (run >> 4) ZRL codes, then code((run & 15) << 4 | cat) + extra bits
// (categorize.rs:132-151).  Position 63 zero = EOB.  Per position k the lane gets
// (nz[k] ZRLs, main piece val[k] of len[k] bits); len 0 = nothing.
__device__ __forceinline__ void lane_walk(const int (&c)[4], int gl, int prev, int dcd, const uint32_t* __restrict__ dctab,
                                          const uint32_t* __restrict__ actab, uint32_t (&val)[4], int (&len)[4],
                                          int (&nz)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int p = 4 * gl + k;
        const bool dc = p == 0;
        const int v = dc ? dcd : c[k];
        const bool nzv = !dc && v != 0;
        const bool eob = p == 63 && v == 0;
        const int run = p - prev - 1;
        const int cat = category_of(v);
        const uint32_t e = dc ? dctab[cat] : actab[nzv ? (((run & 15) << 4) | cat) : 0];
        const bool has = dc || nzv || eob;
        val[k] = ((e & 0xFFFFu) << cat) | extra_bits(v, cat);
        len[k] = has ? (int)(e >> 16) + cat : 0;
        nz[k] = nzv ? (run >> 4) : 0;
        prev = nzv ? p : prev;
    }
}

__device__ __forceinline__ void unpack4(uint2 raw, int (&c)[4]) {
    c[0] = (int16_t)(raw.x & 0xFFFFu);
    c[1] = (int16_t)(raw.x >> 16);
    c[2] = (int16_t)(raw.y & 0xFFFFu);
    c[3] = (int16_t)(raw.y >> 16);
}

// position of the previous non-zero AC coefficient before this lane's 4 (0 = none)
__device__ __forceinline__ int prev_nonzero(const int (&c)[4], int gl, int group) {
    uint32_t m = (c[0] != 0 ? 1u : 0u) | (c[1] != 0 ? 2u : 0u) | (c[2] != 0 ? 4u : 0u) | (c[3] != 0 ? 8u : 0u);
    if (gl == 0) m &= ~1u;  // position 0 is the DC, never a "previous non-zero"
    const unsigned long long any = __ballot(m != 0);
    const uint32_t gm = (uint32_t)(any >> (group * 16)) & 0xFFFFu;
    const uint32_t below = gm & ((1u << gl) - 1u);
    const int last = m ? 4 * gl + (31 - __clz((int)m)) : 0;
    const int src = below ? (31 - __clz((int)below)) : 0;
    const int from = __shfl(last, group * 16 + src, 64);
    return below ? from : 0;
}

// OR `len` bits of `val` (right aligned) at bit `p` of a word image: the LDS image
// holds MSB-first words; the global buffer holds the same words byte-swapped
// (memory order = stream order), so the slow path swaps before its atomic OR.
__device__ __forceinline__ void put_bits(uint32_t* __restrict__ words, unsigned long long p, uint32_t val, int len,
                                         bool lds) {
    const int off = (int)(p & 31);
    const unsigned long long v = (unsigned long long)val << (64 - off - len);
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    const size_t wi = (size_t)(p >> 5);
    if (hi) atomicOr(&words[wi], lds ? hi : __builtin_bswap32(hi));
    if (lo) atomicOr(&words[wi + 1], lds ? lo : __builtin_bswap32(lo));
}

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

// ---------------------------------------------------------------------- k_bits
__global__ __launch_bounds__(256) void k_bits(const int16_t* __restrict__ coef, const int16_t* __restrict__ dcdiff,
                                              const uint32_t* __restrict__ code_tab, Geom g,
                                              uint16_t* __restrict__ block_bits, uint32_t* __restrict__ chunk_bits,
                                              unsigned long long* __restrict__ super_bits) {
    __shared__ uint32_t sTab[4 * 256];
    __shared__ uint32_t sWave[4];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int group = lane >> 4, gl = lane & 15;
    const int frame = blockIdx.y;
    const unsigned chunk = blockIdx.x;
    const long long el0 = (long long)chunk * kChunkBlocks;
    const int nb = (int)min((long long)kChunkBlocks, g.bpf - el0);
    const long long base = (long long)frame * g.bpf + el0;
    for (int i = tid; i < 1024; i += 256) sTab[i] = code_tab[(size_t)frame * 1024 + i];

    // this wave's 16 blocks: all loads in flight before the tables are needed
    uint2 raw[4];
    int dcd[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int b = wave * 16 + it * 4 + group;
        const bool valid = b < nb;
        raw[it] = valid ? *reinterpret_cast<const uint2*>(coef + (base + b) * 64 + 4 * gl) : make_uint2(0, 0);
        dcd[it] = (valid && gl == 0) ? (int)dcdiff[base + b] : 0;
    }
    __syncthreads();
    uint32_t acc = 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int b = wave * 16 + it * 4 + group;
        const bool valid = b < nb;
        int c[4];
        unpack4(raw[it], c);
        const int prev = prev_nonzero(c, gl, group);
        const int k = (int)((el0 + b) % g.bpm);
        const uint32_t* tb = sTab + (k < g.n_luma ? 0 : 512);
        const uint32_t zl = tb[256 + 0xF0] >> 16;
        uint32_t val[4];
        int len[4], nz[4];
        lane_walk(c, gl, prev, dcd[it], tb, tb + 256, val, len, nz);
        uint32_t nbits = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) nbits += (uint32_t)nz[j] * zl + (uint32_t)len[j];
        nbits = valid ? nbits : 0u;
        nbits += __shfl_xor(nbits, 8, 16);
        nbits += __shfl_xor(nbits, 4, 16);
        nbits += __shfl_xor(nbits, 2, 16);
        nbits += __shfl_xor(nbits, 1, 16);
        if (gl == 0 && valid) block_bits[base + b] = (uint16_t)nbits;
        acc += nbits;
    }
    // every lane of a group holds its group's block sum: count it once per group
    acc = (gl == 0) ? acc : 0u;
    acc = wave_sum_u32(acc);
    if (lane == 0) sWave[wave] = acc;
    __syncthreads();
    if (tid == 0) {
        const uint32_t total = sWave[0] + sWave[1] + sWave[2] + sWave[3];
        chunk_bits[(size_t)frame * g.nch + chunk] = total;
        atomicAdd(&super_bits[(size_t)frame * g.nsuper + chunk / kSuper], (unsigned long long)total);
    }
}

// --------------------------------------------------------------------- k_place
// LDS word image capacity of one chunk: 32 Ki bits = 512 bits per block on
// average (the 4K q90 workload averages ~110).  A chunk that needs more (worst
// case kMaxBlockBits per block) is placed straight into the zeroed global buffer
// with atomic ORs instead: slower, same bytes.
constexpr int kPackWords = 1024;

__global__ __launch_bounds__(256) void k_place(const int16_t* __restrict__ coef, const int16_t* __restrict__ dcdiff,
                                               const uint32_t* __restrict__ code_tab, Geom g,
                                               const uint16_t* __restrict__ block_bits,
                                               const uint32_t* __restrict__ chunk_bits,
                                               const unsigned long long* __restrict__ super_bits,
                                               unsigned long long* __restrict__ total_bits,
                                               uint32_t* __restrict__ packed, int* __restrict__ status) {
    __shared__ uint32_t sW[kPackWords + 2];
    __shared__ uint32_t sTab[4 * 256];
    __shared__ uint32_t sOff[kChunkBlocks];
    __shared__ uint32_t sTotal;
    __shared__ unsigned long long sBase;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int group = lane >> 4, gl = lane & 15;
    const int frame = blockIdx.y;
    const unsigned chunk = blockIdx.x;
    const long long el0 = (long long)chunk * kChunkBlocks;
    const int nb = (int)min((long long)kChunkBlocks, g.bpf - el0);
    const long long base = (long long)frame * g.bpf + el0;
    for (int i = tid; i < 1024; i += 256) sTab[i] = code_tab[(size_t)frame * 1024 + i];

    uint2 raw[4];
    int dcd[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int b = wave * 16 + it * 4 + group;
        const bool valid = b < nb;
        raw[it] = valid ? *reinterpret_cast<const uint2*>(coef + (base + b) * 64 + 4 * gl) : make_uint2(0, 0);
        dcd[it] = (valid && gl == 0) ? (int)dcdiff[base + b] : 0;
    }
    if (wave == 0) {  // chunk offset (two-level sums) and block offsets within the chunk
        const unsigned long long pre =
            prefix_two_level(super_bits + (size_t)frame * g.nsuper, chunk_bits + (size_t)frame * g.nch, chunk);
        const uint32_t v = lane < nb ? (uint32_t)block_bits[base + lane] : 0u;
        const uint32_t incl = wave_incl_scan_u32(v);
        const uint32_t total = __shfl(incl, 63, 64);
        sOff[lane] = incl - v;
        if (lane == 0) {
            sBase = pre;
            sTotal = total;
            if (chunk == (unsigned)g.nch - 1) total_bits[frame] = pre + total;
        }
    }
    __syncthreads();
    const unsigned long long bit0 = sBase;
    const uint32_t total = sTotal;
    const int shift = (int)(bit0 & 31);
    const int nw = (int)((shift + (unsigned long long)total + 31) >> 5);
    if (((bit0 + total + 31) >> 5) + 1 > (unsigned long long)g.packed_words) {
        if (tid == 0) atomicOr(status, 8);
        return;  // uniform; the host reports DMMT_E_CAPACITY
    }
    uint32_t* const pk = packed + (size_t)frame * g.packed_words + (bit0 >> 5);
    const bool in_lds = nw + 1 <= kPackWords + 2;
    uint32_t* const img = in_lds ? sW : pk;  // slow path: OR into the zeroed global buffer
    if (in_lds)
        for (int i = tid; i < nw + 1; i += 256) sW[i] = 0u;
    __syncthreads();

#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int b = wave * 16 + it * 4 + group;
        const bool valid = b < nb;
        int c[4];
        unpack4(raw[it], c);
        const int prev = prev_nonzero(c, gl, group);
        const int k = (int)((el0 + b) % g.bpm);
        const uint32_t* tb = sTab + (k < g.n_luma ? 0 : 512);
        const uint32_t z = tb[256 + 0xF0];
        const uint32_t zc = z & 0xFFFFu;
        const int zl = (int)(z >> 16);
        uint32_t val[4];
        int len[4], nz[4];
        lane_walk(c, gl, prev, dcd[it], tb, tb + 256, val, len, nz);
        uint32_t mine = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) mine += (uint32_t)nz[j] * (uint32_t)zl + (uint32_t)len[j];
        mine = valid ? mine : 0u;
        uint32_t incl = mine;  // inclusive scan over the 16 lanes of the block
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t t = __shfl_up(incl, d, 16);
            if (gl >= d) incl += t;
        }
        if (valid) {
            unsigned long long pos = (unsigned long long)sOff[b] + (unsigned)shift + (incl - mine);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                for (int r = 0; r < nz[j]; ++r) {
                    put_bits(img, pos, zc, zl, in_lds);
                    pos += (unsigned)zl;
                }
                if (len[j]) {
                    put_bits(img, pos, val[j], len[j], in_lds);
                    pos += (unsigned)len[j];
                }
            }
        }
    }
    __syncthreads();
    if (in_lds) {  // interior words plain, the two edge words ORed (shared with neighbours)
        for (int i = tid; i < nw; i += 256) {
            const uint32_t v = __builtin_bswap32(sW[i]);
            if (i == 0 || i == nw - 1)
                atomicOr(&pk[i], v);
            else
                pk[i] = v;
        }
    }
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
                       w.super_bits);
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
