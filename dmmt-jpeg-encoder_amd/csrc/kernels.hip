// kernels.hip -- gfx950 kernels of the baseline-JPEG encode path.
//
// Pipeline per launch batch (all frames share one geometry; frame = blockIdx.y
// or blockIdx.x as noted).  Reference stages in brackets (paths relative to the
// reference repository):
//
//  k_front      pixels -> quantised zigzag blocks in MCU emission order + AC
//               symbol histograms.  [color.rs:45-100, padder.rs:12-42,
//               subsampling.rs:102-310, arai.rs:29-104, quantizer.rs:53-62,
//               block_entangler.rs:5-77, block_fold_iterator.rs:53-148,
//               categorize.rs:132-151, symbol_counting.rs:55-74]
//  k_dcdiff     DC prediction in emission order + DC histograms
//               [categorize.rs:153-169]
//  k_tables     one workgroup per frame: package-merge code lengths, canonical
//               codes, JFIF header bytes [symbol_counting.rs:85-94,
//               length_limited.rs:37-134, huffman/encoder.rs:45-157,
//               encoder.rs:125-262]
//  k_bits       bits per block and per chunk of kChunkBlocks blocks
//  k_scan       per frame: exclusive scan of chunk bit counts
//  k_pack       MSB-first bit packing at exact bit offsets [encoder.rs:264-404,
//               binary_stream.rs:38-96]
//  k_stuff_*    0xFF -> 0xFF 0x00 stuffing, 1-padding, EOI
//               [segment_marker_injector.rs:13-30, binary_stream.rs:89-96]
//
// Floating point: this file is compiled with -ffp-contract=off and without
// fast-math, f32 '/' is the correctly rounded IEEE division (hipcc default),
// roundf rounds half away from zero -- the reference's Rust f32 semantics.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jpeg_common.hpp"
#include "kernels.hpp"

namespace dmmt {

__constant__ uint8_t c_zigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                     12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                     35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                     58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
// zigzag position of natural index n
__constant__ uint8_t c_inv_zigzag[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                         3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                         10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                         21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// ------------------------------------------------------------------ helpers

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ unsigned long long wave_incl_scan_u64(unsigned long long v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned long long t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ int bit_length(uint32_t v) { return v ? 32 - __clz((int)v) : 0; }

// categorize.rs:22-32 category of a value (|v| <= 32767 here)
__device__ __forceinline__ int category_of(int v) { return bit_length((uint32_t)(v < 0 ? -v : v)); }

// categorize.rs:34-46: the `cat` low bits of the extra-bits pattern
__device__ __forceinline__ uint32_t extra_bits(int v, int cat) {
    uint32_t p = v > 0 ? (uint32_t)v : (uint32_t)(v - 1);
    return cat ? (p & ((1u << cat) - 1u)) : 0u;
}

// quantizer.rs:60: round(d / q) half away from zero, Rust's saturating `as i16`
__device__ __forceinline__ int16_t quantize(float d, float q) {
    float x = roundf(d / q);
    if (x != x) return 0;
    x = fminf(fmaxf(x, -32768.0f), 32767.0f);
    return (int16_t)(int)x;
}

// arai.rs:7-26 constants, f32 literals as written in the reference
#define DMMT_A1 0.70710678118654752440f
#define DMMT_A2 0.5411961f
#define DMMT_A3 DMMT_A1
#define DMMT_A4 1.3065629f
#define DMMT_A5 0.3826834f

// arai.rs:29-92: 8-point AAN butterfly with the output scaling folded in
__device__ __forceinline__ void arai8(float (&v)[8]) {
    const float v10 = v[0] + v[7], v11 = v[1] + v[6], v12 = v[2] + v[5], v13 = v[3] + v[4];
    const float v14 = v[3] - v[4], v15 = v[2] - v[5], v16 = v[1] - v[6], v17 = v[0] - v[7];
    const float v20 = v10 + v13, v21 = v11 + v12, v22 = v11 - v12, v23 = v10 - v13;
    const float v24 = (-v14) - v15, v25 = v15 + v16, v26 = v16 + v17;
    const float v30 = v20 + v21, v31 = v20 - v21, v32 = v22 + v23;
    const float v42 = v32 * DMMT_A1;
    const float v44 = ((-v24) * DMMT_A2) - ((v24 + v26) * DMMT_A5);
    const float v45 = v25 * DMMT_A3;
    const float v46 = (v26 * DMMT_A4) - ((v26 + v24) * DMMT_A5);
    const float v52 = v42 + v23, v53 = v23 - v42, v55 = v45 + v17, v57 = v17 - v45;
    const float v64 = v44 + v57, v65 = v55 + v46, v66 = v55 - v46, v67 = v57 - v44;
    v[0] = v30 * 0.3535533f;
    v[4] = v31 * 0.35355338f;
    v[2] = v52 * 0.27059805f;
    v[6] = v53 * 0.6532815f;
    v[5] = v64 * 0.4499881f;
    v[1] = v65 * 0.2548978f;
    v[7] = v66 * 1.2814577f;
    v[3] = v67 * 0.30067244f;
}

// color.rs:75-100
__device__ __forceinline__ void rgb_to_ycbcr(float r, float g, float b, float& y, float& cb, float& cr) {
    const float k128 = 128.0f / 255.0f;
    y = (((r * 0.299f + g * 0.587f) + b * 0.114f) - k128) * 255.0f;
    cb = ((r * -0.1687f + g * -0.3312f) + b * 0.5f) * 255.0f;
    cr = ((r * 0.5f + g * -0.4186f) + b * -0.0813f) * 255.0f;
}

// ============================================================== k_front
//
// One workgroup (256 threads) per tile = TM horizontally adjacent MCUs of one
// MCU row (256 padded pixel columns, 8*VR rows), grid-strided over the frame's
// tiles; blockIdx.y = frame.
//  A  pixels -> YCbCr in LDS; chroma box-averaged in the reference's sum order
//  B  row DCT: one lane per (block, row), in place in LDS
//  C  column DCT + quantise: one lane per (block, column) -> zigzag int16 in LDS,
//     laid out in local MCU emission order
//  D  coalesced 16-byte stores of the tile's blocks + DC values
//  E  AC symbols: one wave per block, lane = zigzag position, ballot finds the
//     previous non-zero coefficient; LDS histogram, flushed once per workgroup.

template <int HR, int VR, typename Sample>
__global__ __launch_bounds__(256) void k_front(const Sample* __restrict__ rgb, size_t frame_stride, Geom g,
                                               const float* __restrict__ norm_lut,
                                               const float* __restrict__ qtab,  // [2][64] natural, as f32
                                               int16_t* __restrict__ coef, int16_t* __restrict__ dc,
                                               uint32_t* __restrict__ ac_hist,  // [frames][reps][2][256]
                                               int* __restrict__ status) {
    constexpr int TM = 32 / HR;
    constexpr int ROWS = 8 * VR;
    constexpr int NLUMA = HR * VR;
    constexpr int BPM = NLUMA + 2;
    constexpr int NB = TM * BPM;
    constexpr int NYB = 32 * VR;   // Y blocks in the tile
    constexpr int CW = 256 / HR;   // chroma samples per tile row
    constexpr int CB = CW / 8;     // chroma blocks per component
    constexpr int YS = 256 + 4;    // padded LDS row strides (floats)
    constexpr int CS = CW + 4;
    constexpr int NGROUP = (ROWS / VR) * CW;  // subsampling groups per tile

    __shared__ float sY[ROWS * YS];
    __shared__ float sCb[8 * CS];
    __shared__ float sCr[8 * CS];
    __shared__ __attribute__((aligned(16))) int16_t sCoef[NB * 64];
    __shared__ uint32_t sHist[2 * 256];
    __shared__ float sLut[256];
    __shared__ float sQ[128];

    const int tid = threadIdx.x;
    const int frame = blockIdx.y;
    const Sample* img = rgb + (size_t)frame * frame_stride;
    for (int i = tid; i < 512; i += 256) sHist[i] = 0;
    if (tid < 128) sQ[tid] = qtab[tid];
    if (sizeof(Sample) == 1) sLut[tid] = norm_lut[tid];
    __syncthreads();

    const int tiles_per_row = (g.mcux + TM - 1) / TM;
    const int ntiles = tiles_per_row * g.mcuy;
    int bad = 0;

    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int my = tile / tiles_per_row;
        const int mx0 = (tile - my * tiles_per_row) * TM;
        const int x0 = mx0 * 8 * HR;
        const int y0 = my * ROWS;

        // ---- A: color conversion + subsampling (padder.rs: outside = black)
        for (int grp = tid; grp < NGROUP; grp += 256) {
            const int gc = grp % CW;
            const int gr = grp / CW;
            float cbs = 0.0f, crs = 0.0f;
#pragma unroll
            for (int dx = 0; dx < HR; ++dx) {  // Subsampler::rect: x outer, y inner
#pragma unroll
                for (int dy = 0; dy < VR; ++dy) {
                    const int px = x0 + gc * HR + dx;
                    const int py = y0 + gr * VR + dy;
                    float r = 0.0f, gg = 0.0f, b = 0.0f;
                    if (px < g.width && py < g.height) {
                        const Sample* p = img + ((size_t)py * g.width + px) * 3;
                        const uint32_t ir = p[0], ig = p[1], ib = p[2];
                        bad |= (int)(ir > (uint32_t)g.maxval) | (int)(ig > (uint32_t)g.maxval) |
                               (int)(ib > (uint32_t)g.maxval);
                        if (sizeof(Sample) == 1) {
                            r = sLut[ir];
                            gg = sLut[ig];
                            b = sLut[ib];
                        } else {
                            r = norm_lut[ir];
                            gg = norm_lut[ig];
                            b = norm_lut[ib];
                        }
                    }
                    float y, cb, cr;
                    rgb_to_ycbcr(r, gg, b, y, cb, cr);
                    sY[(gr * VR + dy) * YS + gc * HR + dx] = y;
                    if (dx == 0 && dy == 0) {
                        cbs = cb;
                        crs = cr;
                    } else {
                        cbs = cbs + cb;
                        crs = crs + cr;
                    }
                }
            }
            if (HR * VR > 1) {  // average() divides by the sample count
                cbs = cbs / (float)(HR * VR);
                crs = crs / (float)(HR * VR);
            }
            sCb[gr * CS + gc] = cbs;
            sCr[gr * CS + gc] = crs;
        }
        __syncthreads();

        // ---- B: row pass (stride 1), arai.rs:97-99
        for (int job = tid; job < NB * 8; job += 256) {
            const int row = job & 7;
            const int blk = job >> 3;
            float* p;
            if (blk < NYB)
                p = sY + ((blk / 32) * 8 + row) * YS + (blk % 32) * 8;
            else if (blk < NYB + CB)
                p = sCb + row * CS + (blk - NYB) * 8;
            else
                p = sCr + row * CS + (blk - NYB - CB) * 8;
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = p[i];
            arai8(v);
#pragma unroll
            for (int i = 0; i < 8; ++i) p[i] = v[i];
        }
        __syncthreads();

        // ---- C: column pass (stride 8), arai.rs:100-102, then quantise
        for (int job = tid; job < NB * 8; job += 256) {
            const int col = job & 7;
            const int blk = job >> 3;
            const float* p;
            int stride, comp, el;
            if (blk < NYB) {
                const int by = blk / 32, bx = blk % 32;
                p = sY + (by * 8) * YS + bx * 8 + col;
                stride = YS;
                comp = 0;
                el = (bx / HR) * BPM + by * HR + (bx % HR);  // TL,TR,BL,BR (block_entangler.rs:69-77)
            } else if (blk < NYB + CB) {
                const int cx = blk - NYB;
                p = sCb + cx * 8 + col;
                stride = CS;
                comp = 1;
                el = cx * BPM + NLUMA;
            } else {
                const int cx = blk - NYB - CB;
                p = sCr + cx * 8 + col;
                stride = CS;
                comp = 1;
                el = cx * BPM + NLUMA + 1;
            }
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = p[i * stride];
            arai8(v);
            int16_t* o = sCoef + el * 64;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int nat = r * 8 + col;
                o[c_inv_zigzag[nat]] = quantize(v[r], sQ[comp * 64 + nat]);
            }
        }
        __syncthreads();

        // ---- D: write the tile's blocks (contiguous in emission order) and DCs
        const int nmcu_valid = min(TM, g.mcux - mx0);
        const int nblk = nmcu_valid * BPM;
        const long long e0 = (long long)frame * g.bpf + ((long long)my * g.mcux + mx0) * BPM;
        {
            const uint4* src = reinterpret_cast<const uint4*>(sCoef);
            uint4* dst = reinterpret_cast<uint4*>(coef + e0 * 64);
            for (int i = tid; i < nblk * 8; i += 256) dst[i] = src[i];
            for (int b = tid; b < nblk; b += 256) dc[e0 + b] = sCoef[b * 64];
        }

        // ---- E: AC run/size symbols (categorize.rs:132-151)
        {
            const int wave = tid >> 6, lane = lane_id();
            for (int b = wave; b < nblk; b += 4) {
                const int c = sCoef[b * 64 + lane];
                const unsigned long long nz = __ballot(c != 0) & ~1ull;
                const int t = (b % BPM) < NLUMA ? 0 : 1;
                if (lane > 0 && c != 0) {
                    const unsigned long long below = nz & ((1ull << lane) - 1ull);
                    const int p = below ? 63 - __clzll(below) : 0;
                    const int run = lane - p - 1;
                    atomicAdd(&sHist[t * 256 + (((run & 15) << 4) | category_of(c))], 1u);
                    if (run >= 16) atomicAdd(&sHist[t * 256 + 0xF0], (uint32_t)(run >> 4));
                }
                if (lane == 63 && c == 0) atomicAdd(&sHist[t * 256], 1u);  // EOB
            }
        }
        __syncthreads();
    }

    if (bad) atomicOr(status, 1);
    uint32_t* gh = ac_hist + ((size_t)frame * kHistReps + (blockIdx.x % kHistReps)) * 512;
    for (int i = tid; i < 512; i += 256) {
        const uint32_t v = sHist[i];
        if (v) atomicAdd(&gh[i], v);
    }
}

// ============================================================== k_dcdiff
// DC difference per component in emission order (categorize.rs:153-169), with
// the predictor reset at restart-interval starts (extension), + DC histograms.
__global__ __launch_bounds__(256) void k_dcdiff(const int16_t* __restrict__ dc, int16_t* __restrict__ dcdiff, Geom g,
                                                uint32_t* __restrict__ dc_hist /*[frames][reps][2][16]*/) {
    __shared__ uint32_t sH[32];
    const int tid = threadIdx.x;
    const int frame = blockIdx.y;
    if (tid < 32) sH[tid] = 0;
    __syncthreads();
    const long long base = (long long)frame * g.bpf;
    for (long long el = (long long)blockIdx.x * 256 + tid; el < g.bpf; el += (long long)gridDim.x * 256) {
        const int m = (int)(el / g.bpm);
        const int k = (int)(el - (long long)m * g.bpm);
        const bool restart = g.restart_interval > 0 && (m % g.restart_interval) == 0;
        long long prev = -1;
        if (k > 0 && k < g.n_luma)
            prev = el - 1;
        else if (m > 0 && !restart)
            prev = (k == 0) ? el - g.bpm + g.n_luma - 1 : el - g.bpm;
        const int cur = dc[base + el];
        const int pv = prev >= 0 ? (int)dc[base + prev] : 0;
        const int16_t d = (int16_t)(cur - pv);  // i16 subtraction
        dcdiff[base + el] = d;
        atomicAdd(&sH[(k < g.n_luma ? 0 : 16) + category_of(d)], 1u);
    }
    __syncthreads();
    if (tid < 32 && sH[tid]) atomicAdd(&dc_hist[((size_t)frame * kHistReps + blockIdx.x % kHistReps) * 32 + tid], sH[tid]);
}

// ============================================================== k_tables
// One 1024-thread workgroup per frame; thread group tab = tid/256 builds table
// tab (0 luma DC, 1 luma AC, 2 chroma DC, 3 chroma AC), thread s = symbol.
//  1 sum the histogram replicas (and zero them for the next launch)
//  2 rank symbols by (frequency, symbol): the stable ascending sort of
//    symbol_counting.rs:92-94 over the f>0 filter of 25-32
//  3 package-merge, limit 15 (length_limited.rs:37-134): level k = merge of
//    the pairwise packages of level k-1 with the leaves, ties leaf-first
//  4 solution from the deepest level (n-1 packages), lengths, +1 on the least
//    frequent symbol (symbol_counting.rs:85-90)
//  5 canonical codes over the reversed list (huffman/encoder.rs:45-67,116-119)
//  6 header bytes SOI .. SOS (encoder.rs:125-262)

#define PM_LEVELS 15

__device__ __forceinline__ void put_be16(uint8_t* p, int v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

__global__ __launch_bounds__(1024) void k_tables(uint32_t* __restrict__ ac_hist, uint32_t* __restrict__ dc_hist,
                                                 uint32_t* __restrict__ code_tab,  // [frames][4][256]
                                                 uint8_t* __restrict__ out, size_t out_stride,
                                                 uint32_t* __restrict__ hdr_len, Geom g,
                                                 const uint8_t* __restrict__ qtab_u8,  // [2][64] natural
                                                 int bits_per_channel, int* __restrict__ status) {
    __shared__ unsigned long long sFreq[4][256];
    __shared__ unsigned long long sSortF[4][256];
    __shared__ uint8_t sSortS[4][256];
    __shared__ unsigned long long sLev[2][4][512];
    __shared__ uint8_t sKind[4][PM_LEVELS][512];
    __shared__ int sN[4];
    __shared__ int sLeaf[4][PM_LEVELS];
    __shared__ int sCnt[4][PM_LEVELS];
    __shared__ int sLen[4][256];
    __shared__ uint32_t sScan[4][256];
    __shared__ int sBits[4][16];

    const int tid = threadIdx.x;
    const int tab = tid >> 8;
    const int s = tid & 255;
    const int frame = blockIdx.x;

    // ---- 1
    unsigned long long f = 0;
    if (tab & 1) {
        for (int r = 0; r < kHistReps; ++r) {
            uint32_t* p = &ac_hist[(((size_t)frame * kHistReps + r) * 2 + (tab >> 1)) * 256 + s];
            f += *p;
            *p = 0;
        }
    } else if (s < 16) {
        for (int r = 0; r < kHistReps; ++r) {
            uint32_t* p = &dc_hist[((size_t)frame * kHistReps + r) * 32 + (tab >> 1) * 16 + s];
            f += *p;
            *p = 0;
        }
    }
    sFreq[tab][s] = f;
    if (s < 16) sBits[tab][s] = 0;
    if (s < PM_LEVELS) sCnt[tab][s] = 0;
    if (s == 0) sN[tab] = 0;
    __syncthreads();

    // ---- 2
    int rank = -1;
    if (f > 0) {
        rank = 0;
        for (int t = 0; t < 256; ++t) {
            const unsigned long long ft = sFreq[tab][t];
            rank += (ft > 0 && (ft < f || (ft == f && t < s))) ? 1 : 0;
        }
        atomicAdd(&sN[tab], 1);
    }
    __syncthreads();
    const int n = sN[tab];
    if (rank >= 0) {
        sSortF[tab][rank] = f;
        sSortS[tab][rank] = (uint8_t)s;
        sLev[0][tab][rank] = f;
        sKind[tab][0][rank] = 0;
    }
    if (s == 0 && (n == 0 || ((tab & 1) && sFreq[tab][0xFF] > 0))) atomicOr(status, 2);
    __syncthreads();

    // ---- 3
    int size_prev = n;
    for (int k = 1; k < PM_LEVELS; ++k) {
        const unsigned long long* prev = sLev[(k - 1) & 1][tab];
        unsigned long long* cur = sLev[k & 1][tab];
        const int np = size_prev >> 1;
        if (s < n) {  // leaf s: after every package strictly lighter
            const unsigned long long fl = sSortF[tab][s];
            int lo = 0, hi = np;  // first package j with P_j >= fl
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (prev[2 * mid] + prev[2 * mid + 1] < fl)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            cur[s + lo] = fl;
            sKind[tab][k][s + lo] = 0;
        }
        if (s < np) {  // package s: after every leaf not heavier
            const unsigned long long P = prev[2 * s] + prev[2 * s + 1];
            int lo = 0, hi = n;  // first leaf with f > P
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (sSortF[tab][mid] <= P)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            cur[s + lo] = P;
            sKind[tab][k][s + lo] = 1;
        }
        size_prev = n + np;
        __syncthreads();
    }

    // ---- 4
    int packages = n - 1;
    for (int k = PM_LEVELS - 1; k >= 0; --k) {
        const int c = 2 * packages;
        const bool l0 = s < c && sKind[tab][k][s] == 0;
        const bool l1 = s + 256 < c && sKind[tab][k][s + 256] == 0;
        const unsigned long long b0 = __ballot(l0), b1 = __ballot(l1);
        if ((tid & 63) == 0) atomicAdd(&sCnt[tab][k], __popcll(b0) + __popcll(b1));
        __syncthreads();
        const int leafs = sCnt[tab][k];
        sLeaf[tab][k] = leafs;  // same value from every thread of the table
        packages = c - leafs;
    }
    __syncthreads();
    int len = 0;
    if (s < n) {
        for (int k = 0; k < PM_LEVELS; ++k) len += s < sLeaf[tab][k] ? 1 : 0;
        if (s == 0) len += 1;
        sLen[tab][s] = len;
        atomicAdd(&sBits[tab][len - 1], 1);
    }
    // ---- 5: code(i) = sum_{t>i} 2^(16 - len_t), exclusive over the reversed list
    __syncthreads();  // sLen complete
    {
        uint32_t w = 0;
        if (s < n) w = 1u << (16 - sLen[tab][n - 1 - s]);  // weight at reversed position s
        sScan[tab][s] = w;
        __syncthreads();
        for (int d = 1; d < 256; d <<= 1) {
            const uint32_t add = s >= d ? sScan[tab][s - d] : 0u;
            __syncthreads();
            sScan[tab][s] += add;
            __syncthreads();
        }
    }
    uint32_t* ct = code_tab + ((size_t)frame * 4 + tab) * 256;
    if (rank >= 0) {
        const int rpos = n - 1 - rank;  // position in the reversed (most frequent first) list
        const uint32_t excl = rpos > 0 ? sScan[tab][rpos - 1] : 0u;
        const int L = sLen[tab][rank];
        const uint32_t pat = excl & 0xFFFFu;  // left aligned u16 (wrapping as in the reference)
        ct[s] = ((uint32_t)L << 16) | (pat >> (16 - L));
    } else {
        ct[s] = 0;
    }
    __syncthreads();

    // ---- 6: header
    uint8_t* o = out + (size_t)frame * out_stride;
    const int nLAC = sN[1], nLDC = sN[0], nCAC = sN[3], nCDC = sN[2];
    const int pos_dht0 = 2 + 18 + 69 + 69 + 19;
    const int dht_off[4] = {pos_dht0 + (4 + 17 + nLAC),                                       // luma DC
                            pos_dht0,                                                         // luma AC
                            pos_dht0 + (4 + 17 + nLAC) + (4 + 17 + nLDC) + (4 + 17 + nCAC),   // chroma DC
                            pos_dht0 + (4 + 17 + nLAC) + (4 + 17 + nLDC)};                    // chroma AC
    const int pos_after_dht = pos_dht0 + 4 * (4 + 17) + nLAC + nLDC + nCAC + nCDC;
    const int pos_sos = pos_after_dht + (g.restart_interval > 0 ? 6 : 0);
    // DHT symbols in reversed order (encoder.rs:180)
    if (rank >= 0) o[dht_off[tab] + 4 + 17 + (n - 1 - rank)] = (uint8_t)s;
    if (s < 16) o[dht_off[tab] + 5 + s] = (uint8_t)sBits[tab][s];
    if (s == 0) {
        uint8_t* d = o + dht_off[tab];
        d[0] = 0xFF;
        d[1] = 0xC4;
        put_be16(d + 2, 2 + 17 + n);
        const uint8_t kind[4] = {0x00, 0x11, 0x02, 0x13};  // encoder.rs:92-98 TableKind
        d[4] = kind[tab];
    }
    if (tid == 0) {
        o[0] = 0xFF;
        o[1] = 0xD8;  // SOI
        const uint8_t app0[18] = {0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0, 0x01, 0x02, 0x00, 0x00, 0x48, 0x00, 0x48, 0, 0};
        for (int i = 0; i < 18; ++i) o[2 + i] = app0[i];
        for (int t = 0; t < 2; ++t) {  // DQT, table in zigzag order (encoder.rs:193-212)
            uint8_t* d = o + 20 + 69 * t;
            d[0] = 0xFF;
            d[1] = 0xDB;
            put_be16(d + 2, 67);
            d[4] = (uint8_t)t;
        }
        uint8_t* sof = o + 158;  // encoder.rs:227-245
        sof[0] = 0xFF;
        sof[1] = 0xC0;
        put_be16(sof + 2, 17);
        sof[4] = (uint8_t)bits_per_channel;
        put_be16(sof + 5, g.height);
        put_be16(sof + 7, g.width);
        sof[9] = 3;
        sof[10] = 1;
        sof[11] = (uint8_t)((g.hr << 4) | g.vr);
        sof[12] = 0;
        sof[13] = 2;
        sof[14] = 0x11;
        sof[15] = 1;
        sof[16] = 3;
        sof[17] = 0x11;
        sof[18] = 1;
        if (g.restart_interval > 0) {  // extension: DRI
            uint8_t* d = o + pos_after_dht;
            d[0] = 0xFF;
            d[1] = 0xDD;
            put_be16(d + 2, 4);
            put_be16(d + 4, g.restart_interval);
        }
        const uint8_t sos[14] = {0xFF, 0xDA, 0x00, 0x0C, 0x03, 0x01, 0x01, 0x02, 0x23, 0x03, 0x23, 0x00, 0x3F, 0x00};
        for (int i = 0; i < 14; ++i) o[pos_sos + i] = sos[i];
        hdr_len[frame] = (uint32_t)(pos_sos + 14);
    }
    if (tid < 128) {
        const int t = tid >> 6, i = tid & 63;
        o[20 + 69 * t + 5 + i] = qtab_u8[t * 64 + c_zigzag[i]];
    }
}

// ============================================================== entropy tokens
// Lane i of a wave holds zigzag coefficient i of one block.  Pieces emitted by
// the lane, in stream order (encoder.rs:356-404):
//   lane 0        DC code + DC extra bits
//   lane i>=1, c!=0  (run>>4) x ZRL code, then code(run&15, cat) + extra bits
//   lane 63, c==0  EOB (trailing zeros, categorize.rs:147-149)
struct LaneTok {
    uint32_t main_val;  // code << cat | extra (right aligned)
    int main_len;
    int nzrl;
    uint32_t zrl_code;
    int zrl_len;
    int eob;  // lane 63 only: main is the EOB code
};

__device__ __forceinline__ LaneTok lane_tokens(int lane, int c, unsigned long long nz, int dcd,
                                               const uint32_t* __restrict__ dctab, const uint32_t* __restrict__ actab) {
    LaneTok t{0u, 0, 0, 0u, 0, 0};
    if (lane == 0) {
        const int cat = category_of(dcd);
        const uint32_t e = dctab[cat];
        const int L = (int)(e >> 16);
        t.main_val = ((e & 0xFFFFu) << cat) | extra_bits(dcd, cat);
        t.main_len = L + cat;
    } else if (c != 0) {
        const unsigned long long below = nz & ((1ull << lane) - 1ull);
        const int p = below ? 63 - __clzll(below) : 0;
        const int run = lane - p - 1;
        const int cat = category_of(c);
        const uint32_t e = actab[((run & 15) << 4) | cat];
        t.main_val = ((e & 0xFFFFu) << cat) | extra_bits(c, cat);
        t.main_len = (int)(e >> 16) + cat;
        t.nzrl = run >> 4;
        if (t.nzrl) {
            const uint32_t z = actab[0xF0];
            t.zrl_code = z & 0xFFFFu;
            t.zrl_len = (int)(z >> 16);
        }
    } else if (lane == 63) {
        const uint32_t e = actab[0];
        t.main_val = e & 0xFFFFu;
        t.main_len = (int)(e >> 16);
        t.eob = 1;
    }
    return t;
}

__device__ __forceinline__ int lane_bits(const LaneTok& t) { return t.nzrl * t.zrl_len + t.main_len; }

// ============================================================== k_bits
__global__ __launch_bounds__(256) void k_bits(const int16_t* __restrict__ coef, const int16_t* __restrict__ dcdiff,
                                              const uint32_t* __restrict__ code_tab, Geom g,
                                              uint32_t* __restrict__ block_bits, unsigned long long* __restrict__ chunk_bits) {
    __shared__ uint32_t sTab[4 * 256];
    __shared__ unsigned long long sPart[4];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y, chunk = blockIdx.x;
    for (int i = tid; i < 1024; i += 256) sTab[i] = code_tab[(size_t)frame * 1024 + i];
    __syncthreads();
    const long long el0 = (long long)chunk * kChunkBlocks;
    const int nb = (int)min((long long)kChunkBlocks, g.bpf - el0);
    const long long base = (long long)frame * g.bpf + el0;
    unsigned long long acc = 0;
    for (int b = wave; b < nb; b += 4) {
        const long long e = base + b;
        const int c = coef[e * 64 + lane];
        const unsigned long long nz = __ballot(c != 0) & ~1ull;
        const int k = (int)((el0 + b) % g.bpm);
        const uint32_t* tb = sTab + (k < g.n_luma ? 0 : 512);
        const int dcd = lane == 0 ? (int)dcdiff[e] : 0;
        const LaneTok t = lane_tokens(lane, c, nz, dcd, tb, tb + 256);
        const uint32_t sum = wave_sum_u32((uint32_t)lane_bits(t));
        if (lane == 0) block_bits[e] = sum;
        acc += sum;
    }
    if (lane == 0) sPart[wave] = acc;
    __syncthreads();
    if (tid == 0) chunk_bits[(size_t)frame * g.nch + chunk] = sPart[0] + sPart[1] + sPart[2] + sPart[3];
}

// ============================================================== k_scan
// Per frame: exclusive scan of chunk bit counts -> chunk bit offsets; zero the
// first and last word of every chunk (the only words two chunks can share; the
// pack kernel ORs into them atomically and stores every other word plainly).
__global__ __launch_bounds__(1024) void k_scan(const unsigned long long* __restrict__ chunk_bits,
                                               unsigned long long* __restrict__ chunk_off,
                                               unsigned long long* __restrict__ total_bits, Geom g,
                                               uint32_t* __restrict__ packed) {
    __shared__ unsigned long long sWave[16];
    __shared__ unsigned long long sCarry;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.x;
    const unsigned long long* cb = chunk_bits + (size_t)frame * g.nch;
    unsigned long long* co = chunk_off + (size_t)frame * g.nch;
    uint32_t* pk = packed + (size_t)frame * g.packed_words;
    if (tid == 0) sCarry = 0;
    __syncthreads();
    for (int base = 0; base < g.nch; base += 1024) {
        const int i = base + tid;
        const unsigned long long v = i < g.nch ? cb[i] : 0ull;
        const unsigned long long incl = wave_incl_scan_u64(v);
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        unsigned long long wpre = 0;
        for (int w = 0; w < wave; ++w) wpre += sWave[w];
        const unsigned long long excl = sCarry + wpre + incl - v;
        if (i < g.nch) {
            co[i] = excl;
            if (v > 0 && ((excl + v - 1) >> 5) < (unsigned long long)g.packed_words) {
                pk[excl >> 5] = 0u;
                pk[(excl + v - 1) >> 5] = 0u;
            }
        }
        __syncthreads();
        if (tid == 1023) sCarry = excl + v;
        __syncthreads();
    }
    if (tid == 0) total_bits[frame] = sCarry;
}

// ============================================================== k_pack
// One workgroup per chunk of kChunkBlocks blocks: block offsets by an in-group
// scan of block_bits, one wave per block places each lane's pieces with LDS
// atomicOr into an MSB-first word image of the chunk's bit range, then the
// words go out byte-swapped (memory order = stream order).
__device__ __forceinline__ void put_piece(uint32_t* w, unsigned long long pos, uint32_t val, int len) {
    if (len <= 0) return;
    const int off = (int)(pos & 31);
    const unsigned long long v = (unsigned long long)val << (64 - off - len);
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    const size_t wi = (size_t)(pos >> 5);
    if (hi) atomicOr(&w[wi], hi);
    if (lo) atomicOr(&w[wi + 1], lo);
}

__global__ __launch_bounds__(256) void k_pack(const int16_t* __restrict__ coef, const int16_t* __restrict__ dcdiff,
                                              const uint32_t* __restrict__ code_tab, Geom g,
                                              const uint32_t* __restrict__ block_bits,
                                              const unsigned long long* __restrict__ chunk_off,
                                              const unsigned long long* __restrict__ chunk_bits,
                                              uint32_t* __restrict__ packed) {
    constexpr int MAXW = (31 + kChunkBlocks * kMaxBlockBits + 63) / 32 + 1;
    __shared__ uint32_t sW[MAXW];
    __shared__ uint32_t sTab[4 * 256];
    __shared__ uint32_t sOff[kChunkBlocks];
    __shared__ uint32_t sWave[4];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y, chunk = blockIdx.x;
    const long long el0 = (long long)chunk * kChunkBlocks;
    const int nb = (int)min((long long)kChunkBlocks, g.bpf - el0);
    const long long base = (long long)frame * g.bpf + el0;
    const unsigned long long bit0 = chunk_off[(size_t)frame * g.nch + chunk];
    const unsigned long long nbits = chunk_bits[(size_t)frame * g.nch + chunk];
    const int shift = (int)(bit0 & 31);
    // bounds guard: a chunk can never exceed kChunkBlocks * kMaxBlockBits bits
    if (nbits > (unsigned long long)kChunkBlocks * kMaxBlockBits ||
        ((bit0 + nbits + 31) >> 5) + 1 > (unsigned long long)g.packed_words)
        return;
    const int nw = (int)((shift + nbits + 31) >> 5);
    for (int i = tid; i < 1024; i += 256) sTab[i] = code_tab[(size_t)frame * 1024 + i];
    for (int i = tid; i < nw + 1; i += 256) sW[i] = 0u;
    // block offsets within the chunk (kChunkBlocks <= 256: one value per thread)
    {
        const uint32_t v = tid < nb ? block_bits[base + tid] : 0u;
        const uint32_t incl = wave_incl_scan_u32(v);
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        uint32_t pre = 0;
        for (int w = 0; w < wave; ++w) pre += sWave[w];
        if (tid < kChunkBlocks) sOff[tid] = pre + incl - v + (uint32_t)shift;
    }
    __syncthreads();
    for (int b = wave; b < nb; b += 4) {
        const long long e = base + b;
        const int c = coef[e * 64 + lane];
        const unsigned long long nz = __ballot(c != 0) & ~1ull;
        const int k = (int)((el0 + b) % g.bpm);
        const uint32_t* tb = sTab + (k < g.n_luma ? 0 : 512);
        const int dcd = lane == 0 ? (int)dcdiff[e] : 0;
        const LaneTok t = lane_tokens(lane, c, nz, dcd, tb, tb + 256);
        const uint32_t nbl = (uint32_t)lane_bits(t);
        const uint32_t incl = wave_incl_scan_u32(nbl);
        unsigned long long pos = (unsigned long long)sOff[b] + (incl - nbl);
        for (int z = 0; z < t.nzrl; ++z) {
            put_piece(sW, pos, t.zrl_code, t.zrl_len);
            pos += (unsigned long long)t.zrl_len;
        }
        put_piece(sW, pos, t.main_val, t.main_len);
    }
    __syncthreads();
    uint32_t* pk = packed + (size_t)frame * g.packed_words + (bit0 >> 5);
    for (int i = tid; i < nw; i += 256) {
        const uint32_t v = __builtin_bswap32(sW[i]);
        if (i == 0 || i == nw - 1)
            atomicOr(&pk[i], v);
        else
            pk[i] = v;
    }
}

// ============================================================== stuffing
// Packed scan bytes -> output bytes after the header, 0x00 after every 0xFF,
// last partial byte padded with 1-bits (binary_stream.rs:89-96), EOI.
__device__ __forceinline__ uint8_t scan_byte(const uint8_t* pb, unsigned long long i, unsigned long long nbytes,
                                             int pad_bits) {
    uint8_t v = pb[i];
    if (i == nbytes - 1 && pad_bits) v |= (uint8_t)((1u << pad_bits) - 1u);
    return v;
}

__global__ __launch_bounds__(256) void k_stuff_count(const uint32_t* __restrict__ packed,
                                                     const unsigned long long* __restrict__ total_bits, Geom g,
                                                     uint32_t* __restrict__ seg_ff) {
    __shared__ uint32_t sWave[4];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const unsigned long long tb = total_bits[frame];
    const unsigned long long nbytes = (tb + 7) >> 3;
    const int pad = (int)((8 - (tb & 7)) & 7);
    const int nseg = (int)((nbytes + kStuffSeg - 1) / kStuffSeg);
    const uint8_t* pb = reinterpret_cast<const uint8_t*>(packed + (size_t)frame * g.packed_words);
    if (nbytes > (unsigned long long)g.packed_words * 4) return;
    for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
        uint32_t cnt = 0;
        const unsigned long long b0 = (unsigned long long)seg * kStuffSeg + tid * 16;
        for (int j = 0; j < 16; ++j) {
            const unsigned long long i = b0 + j;
            if (i < nbytes) cnt += scan_byte(pb, i, nbytes, pad) == 0xFF;
        }
        cnt = wave_sum_u32(cnt);
        if (lane == 0) sWave[wave] = cnt;
        __syncthreads();
        if (tid == 0) seg_ff[(size_t)frame * g.nseg_cap + seg] = sWave[0] + sWave[1] + sWave[2] + sWave[3];
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void k_stuff_scan(uint32_t* __restrict__ seg_ff,  // in: counts, out: offsets
                                                     const unsigned long long* __restrict__ total_bits,
                                                     const uint32_t* __restrict__ hdr_len, Geom g,
                                                     uint8_t* __restrict__ out, size_t out_stride,
                                                     uint32_t* __restrict__ out_len) {
    __shared__ uint32_t sWave[16];
    __shared__ uint32_t sCarry;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.x;
    const unsigned long long tb = total_bits[frame];
    const unsigned long long nbytes = (tb + 7) >> 3;
    const int nseg = (int)((nbytes + kStuffSeg - 1) / kStuffSeg);
    uint32_t* sf = seg_ff + (size_t)frame * g.nseg_cap;
    if (tid == 0) sCarry = 0;
    __syncthreads();
    for (int base = 0; base < nseg; base += 1024) {
        const int i = base + tid;
        const uint32_t v = i < nseg ? sf[i] : 0u;
        const uint32_t incl = wave_incl_scan_u32(v);
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        uint32_t wpre = 0;
        for (int w = 0; w < wave; ++w) wpre += sWave[w];
        const uint32_t excl = sCarry + wpre + incl - v;
        if (i < nseg) sf[i] = excl;
        __syncthreads();
        if (tid == 1023) sCarry = excl + v;
        __syncthreads();
    }
    if (tid == 0) {
        const unsigned long long total = (unsigned long long)hdr_len[frame] + nbytes + sCarry;
        uint8_t* o = out + (size_t)frame * out_stride;
        if (total + 2 <= out_stride && nbytes <= (unsigned long long)g.packed_words * 4) {
            o[total] = 0xFF;  // EOI (encoder.rs:131)
            o[total + 1] = 0xD9;
            out_len[frame] = (uint32_t)(total + 2);
        } else {
            out_len[frame] = 0;  // reported as DMMT_E_CAPACITY by the host
        }
    }
}

__global__ __launch_bounds__(256) void k_stuff_write(const uint32_t* __restrict__ packed,
                                                     const unsigned long long* __restrict__ total_bits,
                                                     const uint32_t* __restrict__ seg_off,
                                                     const uint32_t* __restrict__ hdr_len, Geom g,
                                                     uint8_t* __restrict__ out, size_t out_stride) {
    __shared__ uint32_t sWave[4];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    const unsigned long long tb = total_bits[frame];
    const unsigned long long nbytes = (tb + 7) >> 3;
    const int pad = (int)((8 - (tb & 7)) & 7);
    const int nseg = (int)((nbytes + kStuffSeg - 1) / kStuffSeg);
    const uint8_t* pb = reinterpret_cast<const uint8_t*>(packed + (size_t)frame * g.packed_words);
    uint8_t* o = out + (size_t)frame * out_stride + hdr_len[frame];
    if (nbytes > (unsigned long long)g.packed_words * 4 || hdr_len[frame] + 2 * nbytes + 2 > out_stride) return;
    for (int seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
        const unsigned long long b0 = (unsigned long long)seg * kStuffSeg + tid * 16;
        uint8_t v[16];
        uint32_t cnt = 0;
        for (int j = 0; j < 16; ++j) {
            const unsigned long long i = b0 + j;
            v[j] = i < nbytes ? scan_byte(pb, i, nbytes, pad) : 0;
            cnt += (i < nbytes && v[j] == 0xFF);
        }
        const uint32_t incl = wave_incl_scan_u32(cnt);
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        uint32_t pre = seg_off[(size_t)frame * g.nseg_cap + seg];
        for (int w = 0; w < wave; ++w) pre += sWave[w];
        unsigned long long dst = b0 + pre + (incl - cnt);
        for (int j = 0; j < 16; ++j) {
            if (b0 + j >= nbytes) break;
            o[dst++] = v[j];
            if (v[j] == 0xFF) o[dst++] = 0x00;
        }
        __syncthreads();
    }
}

// ============================================================== operator: DCT only
// Discrete8x8CosineTransformer::transform over a block-contiguous f32 array
// (cosine_transform.rs:55-73, arai.rs:95-104); one lane per row, then column.
__global__ __launch_bounds__(256) void k_dct_blocks(float* __restrict__ data, long long nblocks) {
    __shared__ float s[32 * 65];
    const int tid = threadIdx.x;
    for (long long b0 = (long long)blockIdx.x * 32; b0 < nblocks; b0 += (long long)gridDim.x * 32) {
        const int nbk = (int)min(32LL, nblocks - b0);
        for (int i = tid; i < nbk * 64; i += 256) s[(i >> 6) * 65 + (i & 63)] = data[b0 * 64 + i];
        __syncthreads();
        {
            const int blk = tid >> 3, row = tid & 7;
            if (blk < nbk) {
                float v[8];
                for (int i = 0; i < 8; ++i) v[i] = s[blk * 65 + row * 8 + i];
                arai8(v);
                for (int i = 0; i < 8; ++i) s[blk * 65 + row * 8 + i] = v[i];
            }
        }
        __syncthreads();
        {
            const int blk = tid >> 3, col = tid & 7;
            if (blk < nbk) {
                float v[8];
                for (int i = 0; i < 8; ++i) v[i] = s[blk * 65 + i * 8 + col];
                arai8(v);
                for (int i = 0; i < 8; ++i) s[blk * 65 + i * 8 + col] = v[i];
            }
        }
        __syncthreads();
        for (int i = tid; i < nbk * 64; i += 256) data[b0 * 64 + i] = s[(i >> 6) * 65 + (i & 63)];
        __syncthreads();
    }
}

// ============================================================== synthetic input
// SURVEY.md 8(d) generator: base = (x + 8y) % 256 (dct_timing.rs:150-160),
// R = base, G = (base + 85 f + (y >> 3)) % 256, B = (255 - base + (x >> 4)) % 256,
// plus 4-bit xorshift32 noise per channel, clamped to 255.
__device__ __forceinline__ uint32_t xorshift32(uint32_t x) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return x;
}

__global__ __launch_bounds__(256) void k_synthetic(uint8_t* __restrict__ rgb, int w, int h, int n_frames,
                                                   int first_frame, uint32_t seed) {
    const long long npx = (long long)w * h;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < npx * n_frames;
         i += (long long)gridDim.x * 256) {
        const int fl = (int)(i / npx);
        const long long pi = i - (long long)fl * npx;
        const int y = (int)(pi / w), x = (int)(pi - (long long)y * w);
        const uint32_t f = (uint32_t)(first_frame + fl);
        const uint32_t base = (uint32_t)(x + 8 * y) & 255u;
        const uint32_t n = xorshift32(seed ^ (uint32_t)(f * (uint32_t)npx + (uint32_t)pi));
        const uint32_t r = base + (n & 15u);
        const uint32_t g = ((base + 85u * f + ((uint32_t)y >> 3)) & 255u) + ((n >> 4) & 15u);
        const uint32_t b = ((255u - base + ((uint32_t)x >> 4)) & 255u) + ((n >> 8) & 15u);
        uint8_t* p = rgb + i * 3;
        p[0] = (uint8_t)min(r, 255u);
        p[1] = (uint8_t)min(g, 255u);
        p[2] = (uint8_t)min(b, 255u);
    }
}

// explicit instantiations of the front kernel
template __global__ void k_front<1, 1, uint8_t>(const uint8_t*, size_t, Geom, const float*, const float*, int16_t*, int16_t*, uint32_t*, int*);
template __global__ void k_front<2, 1, uint8_t>(const uint8_t*, size_t, Geom, const float*, const float*, int16_t*, int16_t*, uint32_t*, int*);
template __global__ void k_front<2, 2, uint8_t>(const uint8_t*, size_t, Geom, const float*, const float*, int16_t*, int16_t*, uint32_t*, int*);
template __global__ void k_front<1, 1, uint16_t>(const uint16_t*, size_t, Geom, const float*, const float*, int16_t*, int16_t*, uint32_t*, int*);
template __global__ void k_front<2, 1, uint16_t>(const uint16_t*, size_t, Geom, const float*, const float*, int16_t*, int16_t*, uint32_t*, int*);
template __global__ void k_front<2, 2, uint16_t>(const uint16_t*, size_t, Geom, const float*, const float*, int16_t*, int16_t*, uint32_t*, int*);

}  // namespace dmmt

// ============================================================== standalone AC symbol pass
// Back-half entry (dmmt_encode_coefficients): blocks come from the host, so the
// DC values and AC histograms k_front would have produced are rebuilt here.
namespace dmmt {
__global__ __launch_bounds__(256) void k_ac_hist(const int16_t* __restrict__ coef, Geom g, int16_t* __restrict__ dc,
                                                 uint32_t* __restrict__ ac_hist) {
    __shared__ uint32_t sHist[512];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int frame = blockIdx.y;
    for (int i = tid; i < 512; i += 256) sHist[i] = 0;
    __syncthreads();
    const long long base = (long long)frame * g.bpf;
    for (long long el = (long long)blockIdx.x * 4 + wave; el < g.bpf; el += (long long)gridDim.x * 4) {
        const int c = coef[(base + el) * 64 + lane];
        if (lane == 0) dc[base + el] = (int16_t)c;
        const unsigned long long nz = __ballot(c != 0) & ~1ull;
        const int t = (int)(el % g.bpm) < g.n_luma ? 0 : 1;
        if (lane > 0 && c != 0) {
            const unsigned long long below = nz & ((1ull << lane) - 1ull);
            const int p = below ? 63 - __clzll(below) : 0;
            const int run = lane - p - 1;
            atomicAdd(&sHist[t * 256 + (((run & 15) << 4) | category_of(c))], 1u);
            if (run >= 16) atomicAdd(&sHist[t * 256 + 0xF0], (uint32_t)(run >> 4));
        }
        if (lane == 63 && c == 0) atomicAdd(&sHist[t * 256], 1u);
    }
    __syncthreads();
    uint32_t* gh = ac_hist + ((size_t)frame * kHistReps + (blockIdx.x % kHistReps)) * 512;
    for (int i = tid; i < 512; i += 256)
        if (sHist[i]) atomicAdd(&gh[i], sHist[i]);
}
}  // namespace dmmt

// ============================================================== launchers
namespace dmmt {

static inline int clampi(long long v, int lo, int hi) { return (int)(v < lo ? lo : (v > hi ? hi : v)); }

template <int HR, int VR, typename S>
static void front_impl(const void* rgb, size_t stride_elems, int n_frames, const Geom& g, const Work& w,
                       hipStream_t st) {
    constexpr int TM = 32 / HR;
    const long long ntiles = (long long)((g.mcux + TM - 1) / TM) * g.mcuy;
    dim3 grid(clampi(ntiles, 1, (int)(1536 / n_frames > 0 ? 1536 / n_frames : 1)), n_frames);
    hipLaunchKernelGGL((k_front<HR, VR, S>), grid, dim3(256), 0, st, (const S*)rgb, stride_elems, g, w.norm_lut,
                       w.qtab, w.coef, w.dc, w.ac_hist, w.status);
}

hipError_t launch_front(const void* rgb, size_t frame_stride_bytes, int sample_bytes, int n_frames, const Geom& g,
                        const Work& w, hipStream_t st) {
    const size_t se = frame_stride_bytes / (size_t)sample_bytes;
    if (sample_bytes == 1) {
        if (g.hr == 1)
            front_impl<1, 1, uint8_t>(rgb, se, n_frames, g, w, st);
        else if (g.vr == 1)
            front_impl<2, 1, uint8_t>(rgb, se, n_frames, g, w, st);
        else
            front_impl<2, 2, uint8_t>(rgb, se, n_frames, g, w, st);
    } else {
        if (g.hr == 1)
            front_impl<1, 1, uint16_t>(rgb, se, n_frames, g, w, st);
        else if (g.vr == 1)
            front_impl<2, 1, uint16_t>(rgb, se, n_frames, g, w, st);
        else
            front_impl<2, 2, uint16_t>(rgb, se, n_frames, g, w, st);
    }
    return hipGetLastError();
}

hipError_t launch_ac_hist(int n_frames, const Geom& g, const Work& w, hipStream_t st) {
    dim3 grid(clampi((g.bpf + 3) / 4, 1, 1024 / n_frames > 0 ? 1024 / n_frames : 1), n_frames);
    hipLaunchKernelGGL(k_ac_hist, grid, dim3(256), 0, st, (const int16_t*)w.coef, g, w.dc, w.ac_hist);
    return hipGetLastError();
}

hipError_t launch_stage(Stage s, int n_frames, const Geom& g, const Work& w, int bits_per_channel, uint8_t* out,
                        size_t out_stride, uint32_t* out_len, hipStream_t st) {
    const int per_frame = 2048 / n_frames > 0 ? 2048 / n_frames : 1;
    switch (s) {
    case ST_DCDIFF: {
        dim3 grid(clampi((g.bpf + 255) / 256, 1, per_frame / 2 > 0 ? per_frame / 2 : 1), n_frames);
        hipLaunchKernelGGL(k_dcdiff, grid, dim3(256), 0, st, (const int16_t*)w.dc, w.dcdiff, g, w.dc_hist);
        break;
    }
    case ST_TABLES:
        hipLaunchKernelGGL(k_tables, dim3(n_frames), dim3(1024), 0, st, w.ac_hist, w.dc_hist, w.code_tab, out, out_stride,
                           w.hdr_len, g, w.qtab_u8, bits_per_channel, w.status);
        break;
    case ST_BITS:
        hipLaunchKernelGGL(k_bits, dim3(g.nch, n_frames), dim3(256), 0, st, (const int16_t*)w.coef,
                           (const int16_t*)w.dcdiff, (const uint32_t*)w.code_tab, g, w.block_bits, w.chunk_bits);
        break;
    case ST_SCAN:
        hipLaunchKernelGGL(k_scan, dim3(n_frames), dim3(1024), 0, st, (const unsigned long long*)w.chunk_bits,
                           w.chunk_off, w.total_bits, g, w.packed);
        break;
    case ST_PACK:
        hipLaunchKernelGGL(k_pack, dim3(g.nch, n_frames), dim3(256), 0, st, (const int16_t*)w.coef,
                           (const int16_t*)w.dcdiff, (const uint32_t*)w.code_tab, g, (const uint32_t*)w.block_bits,
                           (const unsigned long long*)w.chunk_off, (const unsigned long long*)w.chunk_bits, w.packed);
        break;
    case ST_STUFF_COUNT:
        hipLaunchKernelGGL(k_stuff_count, dim3(clampi(g.nseg_cap, 1, per_frame), n_frames), dim3(256), 0, st,
                           (const uint32_t*)w.packed, (const unsigned long long*)w.total_bits, g, w.seg_ff);
        break;
    case ST_STUFF_SCAN:
        hipLaunchKernelGGL(k_stuff_scan, dim3(n_frames), dim3(1024), 0, st, w.seg_ff,
                           (const unsigned long long*)w.total_bits, (const uint32_t*)w.hdr_len, g, out, out_stride,
                           out_len);
        break;
    case ST_STUFF_WRITE:
        hipLaunchKernelGGL(k_stuff_write, dim3(clampi(g.nseg_cap, 1, per_frame), n_frames), dim3(256), 0, st,
                           (const uint32_t*)w.packed, (const unsigned long long*)w.total_bits,
                           (const uint32_t*)w.seg_ff, (const uint32_t*)w.hdr_len, g, out, out_stride);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_dct_blocks(float* data, long long nblocks, hipStream_t st) {
    hipLaunchKernelGGL(k_dct_blocks, dim3(clampi((nblocks + 31) / 32, 1, 2048)), dim3(256), 0, st, data, nblocks);
    return hipGetLastError();
}

hipError_t launch_synthetic(uint8_t* rgb, int w, int h, int n_frames, int first_frame, uint32_t seed,
                            hipStream_t st) {
    const long long n = (long long)w * h * n_frames;
    hipLaunchKernelGGL(k_synthetic, dim3(clampi((n + 255) / 256, 1, 8192)), dim3(256), 0, st, rgb, w, h, n_frames,
                       first_frame, seed);
    return hipGetLastError();
}

}  // namespace dmmt
