// entropy.hip -- gfx950 entropy-coding back half: bit packing and byte stuffing.
//
//  k_pack   one workgroup per chunk of kChunkBlocks blocks (chunk = atomic ticket):
//           pass 1 counts every block's bits, a workgroup scan gives block
//           offsets, a decoupled look-back over the chunk totals gives the
//           chunk's bit offset in the frame's scan, pass 2 places every code
//           MSB-first into an LDS word image which goes out byte-swapped
//           (memory order = stream order).  [encoder.rs:264-404 write_image_data
//           / write_{dc,ac}_from_block, binary_stream.rs:38-66 BitWriter]
//  k_stuff  one workgroup per 4 KiB segment of the packed scan (ticket):
//           counts 0xFF bytes, decoupled look-back over the counts, writes the
//           bytes after the header with a 0x00 after every 0xFF; pads the last
//           byte with 1-bits and appends EOI; zeroes the packed words it read so
//           the next launch's k_pack can OR into a clean buffer.
//           [segment_marker_injector.rs:13-30, binary_stream.rs:89-96,
//           encoder.rs:131]
//
// Lane layout of both entropy passes: 16 lanes per block, 4 blocks per wave;
// lane l of a block owns zigzag positions 4l..4l+3 (one 8-byte load).  The
// previous non-zero coefficient before a lane's first position comes from a
// ballot of "lane has a non-zero" and one shuffle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "jpeg_common.hpp"
#include "kernels.hpp"

namespace dmmt {

// Walk the 4 coefficients of one lane in stream order (encoder.rs:356-404):
// position 0 = DC code + extra bits; a non-zero AC coefficient = (run>>4) ZRL
// codes then code(run&15, cat) + extra bits (categorize.rs:132-151); position 63
// zero = EOB.  EMIT=false returns the lane's bit count; EMIT=true ORs the pieces
// into the LDS word image starting at bit `pos`.
template <bool EMIT>
__device__ __forceinline__ uint32_t lane4(const int (&c)[4], int gl, int prev, int dcd, const uint32_t* __restrict__ dctab,
                                          const uint32_t* __restrict__ actab, uint32_t* __restrict__ words,
                                          unsigned long long pos) {
    uint32_t nbits = 0;
    auto put = [&](uint32_t val, int len) {
        if (EMIT && len > 0) {
            const unsigned long long p = pos + nbits;
            const int off = (int)(p & 31);
            const unsigned long long v = (unsigned long long)val << (64 - off - len);
            const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
            const size_t wi = (size_t)(p >> 5);
            if (hi) atomicOr(&words[wi], hi);
            if (lo) atomicOr(&words[wi + 1], lo);
        }
        nbits += (uint32_t)len;
    };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int p = 4 * gl + k;
        const int v = c[k];
        if (p == 0) {
            const int cat = category_of(dcd);
            const uint32_t e = dctab[cat];
            put(((e & 0xFFFFu) << cat) | extra_bits(dcd, cat), (int)(e >> 16) + cat);
        } else if (v != 0) {
            const int run = p - prev - 1;
            if (run >= 16) {
                const uint32_t z = actab[0xF0];
                for (int r = run >> 4; r > 0; --r) put(z & 0xFFFFu, (int)(z >> 16));
            }
            const int cat = category_of(v);
            const uint32_t e = actab[((run & 15) << 4) | cat];
            put(((e & 0xFFFFu) << cat) | extra_bits(v, cat), (int)(e >> 16) + cat);
            prev = p;
        } else if (p == 63) {
            const uint32_t e = actab[0];  // EOB: trailing zeros
            put(e & 0xFFFFu, (int)(e >> 16));
        }
    }
    return nbits;
}

// load this lane's 4 coefficients and find the previous non-zero position
__device__ __forceinline__ void lane_setup(const int16_t* __restrict__ blk, bool valid, int gl, int group, int (&c)[4],
                                           int& prev) {
    c[0] = c[1] = c[2] = c[3] = 0;
    if (valid) {
        const uint2 raw = *reinterpret_cast<const uint2*>(blk + 4 * gl);
        c[0] = (int16_t)(raw.x & 0xFFFFu);
        c[1] = (int16_t)(raw.x >> 16);
        c[2] = (int16_t)(raw.y & 0xFFFFu);
        c[3] = (int16_t)(raw.y >> 16);
    }
    uint32_t m = (c[0] != 0 ? 1u : 0u) | (c[1] != 0 ? 2u : 0u) | (c[2] != 0 ? 4u : 0u) | (c[3] != 0 ? 8u : 0u);
    if (gl == 0) m &= ~1u;  // position 0 is the DC, never a "previous non-zero"
    const unsigned long long any = __ballot(m != 0);
    const uint32_t gm = (uint32_t)(any >> (group * 16)) & 0xFFFFu;
    const uint32_t below = gm & ((1u << gl) - 1u);
    const int last = m ? 4 * gl + (31 - __clz((int)m)) : 0;
    const int src = below ? (31 - __clz((int)below)) : 0;
    const int from = __shfl(last, group * 16 + src, 64);
    prev = below ? from : 0;
}

__global__ __launch_bounds__(256) void k_pack(const int16_t* __restrict__ coef, const int16_t* __restrict__ dcdiff,
                                              const uint32_t* __restrict__ code_tab, Geom g,
                                              unsigned* __restrict__ tickets,           // [frames], zeroed by k_dcdiff
                                              unsigned long long* __restrict__ lb,      // [frames][nch], zeroed by k_dcdiff
                                              unsigned long long* __restrict__ total_bits,
                                              uint32_t* __restrict__ packed, int* __restrict__ status) {
    constexpr int MAXW = (31 + kChunkBlocks * kMaxBlockBits + 63) / 32 + 1;
    __shared__ uint32_t sW[MAXW];
    __shared__ uint32_t sTab[4 * 256];
    __shared__ uint32_t sBits[kChunkBlocks];
    __shared__ uint32_t sOff[kChunkBlocks];
    __shared__ uint32_t sWave[4];
    __shared__ unsigned sChunk;
    __shared__ unsigned long long sBase;

    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int group = lane >> 4, gl = lane & 15;
    const int frame = blockIdx.y;
    if (tid == 0) sChunk = atomicAdd(&tickets[frame], 1u);
    for (int i = tid; i < 1024; i += 256) sTab[i] = code_tab[(size_t)frame * 1024 + i];
    __syncthreads();
    const unsigned chunk = sChunk;
    if (chunk >= (unsigned)g.nch) return;  // uniform
    const long long el0 = (long long)chunk * kChunkBlocks;
    const int nb = (int)min((long long)kChunkBlocks, g.bpf - el0);
    const long long base = (long long)frame * g.bpf + el0;

    // ---- pass 1: bits per block
    for (int it = 0; it < kChunkBlocks / 16; ++it) {
        const int b = it * 16 + wave * 4 + group;
        const bool valid = b < nb;
        const long long e = base + (valid ? b : 0);
        int c[4], prev;
        lane_setup(coef + e * 64, valid, gl, group, c, prev);
        const int k = (int)((el0 + b) % g.bpm);
        const uint32_t* tb = sTab + (k < g.n_luma ? 0 : 512);
        const int dcd = (valid && gl == 0) ? (int)dcdiff[e] : 0;
        uint32_t nbits = valid ? lane4<false>(c, gl, prev, dcd, tb, tb + 256, nullptr, 0) : 0u;
        nbits += __shfl_xor(nbits, 8, 16);
        nbits += __shfl_xor(nbits, 4, 16);
        nbits += __shfl_xor(nbits, 2, 16);
        nbits += __shfl_xor(nbits, 1, 16);
        if (gl == 0 && valid) sBits[b] = nbits;
    }
    __syncthreads();

    // ---- block offsets within the chunk, chunk total (kChunkBlocks == 128: waves 0-1)
    uint32_t total = 0;
    {
        const uint32_t v = (tid < nb) ? sBits[tid] : 0u;
        const uint32_t incl = wave_incl_scan_u32(v);
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        uint32_t pre = 0;
        for (int w = 0; w < wave; ++w) pre += sWave[w];
        if (tid < kChunkBlocks) sOff[tid] = pre + incl - v;
        total = sWave[0] + sWave[1];
    }

    // ---- chunk offset in the frame's scan: decoupled look-back
    if (wave == 0) {
        const unsigned long long excl = lookback(lb + (size_t)frame * g.nch, chunk, total, status);
        if (lane == 0) {
            sBase = excl;
            if (chunk == (unsigned)g.nch - 1) total_bits[frame] = excl + total;
        }
    }
    __syncthreads();
    const unsigned long long bit0 = sBase;
    const int shift = (int)(bit0 & 31);
    const int nw = (int)((shift + (unsigned long long)total + 31) >> 5);
    if (total > (uint32_t)kChunkBlocks * kMaxBlockBits || ((bit0 + total + 31) >> 5) + 1 > (unsigned long long)g.packed_words) {
        if (tid == 0) atomicOr(status, 8);
        return;  // uniform
    }
    for (int i = tid; i < nw + 1; i += 256) sW[i] = 0u;
    __syncthreads();

    // ---- pass 2: place the bits
    for (int it = 0; it < kChunkBlocks / 16; ++it) {
        const int b = it * 16 + wave * 4 + group;
        const bool valid = b < nb;
        const long long e = base + (valid ? b : 0);
        int c[4], prev;
        lane_setup(coef + e * 64, valid, gl, group, c, prev);
        const int k = (int)((el0 + b) % g.bpm);
        const uint32_t* tb = sTab + (k < g.n_luma ? 0 : 512);
        const int dcd = (valid && gl == 0) ? (int)dcdiff[e] : 0;
        const uint32_t mine = valid ? lane4<false>(c, gl, prev, dcd, tb, tb + 256, nullptr, 0) : 0u;
        uint32_t incl = mine;  // inclusive scan over the 16 lanes of the block
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t t = __shfl_up(incl, d, 16);
            if (gl >= d) incl += t;
        }
        if (valid) {
            const unsigned long long pos = (unsigned long long)sOff[b] + (unsigned)shift + (incl - mine);
            lane4<true>(c, gl, prev, dcd, tb, tb + 256, sW, pos);
        }
    }
    __syncthreads();

    // ---- out: interior words plain, the two edge words ORed (shared with neighbours)
    uint32_t* pk = packed + (size_t)frame * g.packed_words + (bit0 >> 5);
    for (int i = tid; i < nw; i += 256) {
        const uint32_t v = __builtin_bswap32(sW[i]);
        if (i == 0 || i == nw - 1)
            atomicOr(&pk[i], v);
        else
            pk[i] = v;
    }
}

// --------------------------------------------------------------------- k_stuff
__global__ __launch_bounds__(256) void k_stuff(uint32_t* __restrict__ packed,
                                               const unsigned long long* __restrict__ total_bits,
                                               const uint32_t* __restrict__ hdr_len, Geom g,
                                               unsigned* __restrict__ tickets,        // [frames], zeroed by k_dcdiff
                                               unsigned long long* __restrict__ lb,   // [frames][nseg_cap], zeroed by k_dcdiff
                                               uint8_t* __restrict__ out, size_t out_stride,
                                               uint32_t* __restrict__ out_len, int* __restrict__ status) {
    __shared__ uint32_t sWave[4];
    __shared__ unsigned sSeg;
    __shared__ unsigned long long sBase;
    __shared__ uint8_t sOut[2 * kStuffSeg];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const unsigned long long tb = total_bits[frame];
    const unsigned long long nbytes = (tb + 7) >> 3;
    const unsigned pad = (unsigned)((8 - (tb & 7)) & 7);
    const unsigned nseg = (unsigned)((nbytes + kStuffSeg - 1) / kStuffSeg);
    const uint32_t hdr = hdr_len[frame];
    const bool fits = nbytes <= (unsigned long long)g.packed_words * 4 && hdr + 2 * nbytes + 2 <= out_stride;
    uint8_t* pb = reinterpret_cast<uint8_t*>(packed + (size_t)frame * g.packed_words);
    uint8_t* o = out + (size_t)frame * out_stride + hdr;
    unsigned long long* lbf = lb + (size_t)frame * g.nseg_cap;

    for (;;) {
        if (tid == 0) sSeg = atomicAdd(&tickets[frame], 1u);
        __syncthreads();
        const unsigned seg = sSeg;
        if (seg >= nseg || !fits) break;  // uniform
        const unsigned long long b0 = (unsigned long long)seg * kStuffSeg + (unsigned)tid * 16u;
        uint8_t v[16];
        uint32_t cnt = 0;
        if (b0 + 16 <= nbytes && b0 + 16 <= ((nbytes + 3) & ~3ull)) {
            const uint4 q = *reinterpret_cast<const uint4*>(pb + b0);
            const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = (uint8_t)(wv[j >> 2] >> (8 * (j & 3)));
            if (b0 + 16 == nbytes && pad) v[15] |= (uint8_t)((1u << pad) - 1u);
            *reinterpret_cast<uint4*>(pb + b0) = make_uint4(0, 0, 0, 0);  // clean for the next launch
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const unsigned long long i = b0 + j;
                uint8_t x = 0;
                if (i < nbytes) {
                    x = pb[i];
                    if (i == nbytes - 1 && pad) x |= (uint8_t)((1u << pad) - 1u);
                }
                v[j] = x;
            }
            // zero every word this thread covered that lies inside the written range
            const unsigned long long wend = (nbytes + 3) >> 2;
            for (int j = 0; j < 4; ++j) {
                const unsigned long long wi = (b0 >> 2) + j;
                if (wi < wend) reinterpret_cast<uint32_t*>(pb)[wi] = 0u;
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) cnt += (b0 + j < nbytes && v[j] == 0xFF) ? 1u : 0u;
        const uint32_t incl = wave_incl_scan_u32(cnt);
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        if (wave == 0) {
            const unsigned long long agg = sWave[0] + sWave[1] + sWave[2] + sWave[3];
            const unsigned long long excl = lookback(lbf, seg, agg, status);
            if (lane == 0) sBase = excl;
            if (lane == 0 && seg == nseg - 1) {  // EOI (encoder.rs:131) and the file size
                const unsigned long long total = (unsigned long long)hdr + nbytes + excl + agg;
                uint8_t* of = out + (size_t)frame * out_stride;
                of[total] = 0xFF;
                of[total + 1] = 0xD9;
                out_len[frame] = (uint32_t)(total + 2);
            }
        }
        // stage the stuffed segment in LDS, then store it with consecutive lanes on
        // consecutive bytes (coalesced) at its look-back offset
        uint32_t pre = 0;
        for (int w = 0; w < wave; ++w) pre += sWave[w];
        uint32_t dst = (uint32_t)tid * 16u + pre + (incl - cnt);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (b0 + j < nbytes) {
                sOut[dst++] = v[j];
                if (v[j] == 0xFF) sOut[dst++] = 0x00;
            }
        }
        __syncthreads();
        const unsigned long long seg0 = (unsigned long long)seg * kStuffSeg;
        const unsigned long long in_seg = nbytes - seg0 < (unsigned long long)kStuffSeg ? nbytes - seg0 : kStuffSeg;
        const uint32_t seg_len = (uint32_t)in_seg + sWave[0] + sWave[1] + sWave[2] + sWave[3];
        uint8_t* od = o + seg0 + sBase;
        for (uint32_t i = (uint32_t)tid; i < seg_len; i += 256) od[i] = sOut[i];
        __syncthreads();  // sSeg / sWave / sOut reuse
    }
    if (!fits && blockIdx.x == 0 && tid == 0) {
        out_len[frame] = 0;  // reported as DMMT_E_CAPACITY by the host
        atomicOr(status, 16);
    }
}

hipError_t launch_pack(int n_frames, const Geom& g, const Work& w, hipStream_t st) {
    hipLaunchKernelGGL(k_pack, dim3(g.nch, n_frames), dim3(256), 0, st, (const int16_t*)w.coef,
                       (const int16_t*)w.dcdiff, (const uint32_t*)w.code_tab, g, w.tickets, w.lb_pack, w.total_bits,
                       w.packed, w.status);
    return hipGetLastError();
}

hipError_t launch_stuff(int n_frames, const Geom& g, const Work& w, uint8_t* out, size_t out_stride, uint32_t* out_len,
                        hipStream_t st) {
    int per_frame = 1024 / n_frames;
    if (per_frame < 1) per_frame = 1;
    int gx = g.nseg_cap < per_frame ? g.nseg_cap : per_frame;
    if (gx < 1) gx = 1;
    hipLaunchKernelGGL(k_stuff, dim3(gx, n_frames), dim3(256), 0, st, w.packed, (const unsigned long long*)w.total_bits,
                       (const uint32_t*)w.hdr_len, g, w.tickets + n_frames, w.lb_stuff, out, out_stride, out_len,
                       w.status);
    return hipGetLastError();
}

}  // namespace dmmt
