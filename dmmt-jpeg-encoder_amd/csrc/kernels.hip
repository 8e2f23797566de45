// kernels.hip -- gfx950 kernels of the baseline-JPEG encode path.
//
// Pipeline per launch batch (all frames share one geometry; frame = blockIdx.y
// or blockIdx.x as noted).  Reference stages in brackets (paths relative to the
// reference repository):
//
//  k_front      pixels -> quantised blocks in MCU emission order.  [color.rs:45-100,
//               padder.rs:12-42, subsampling.rs:102-310, arai.rs:29-104,
//               quantizer.rs:53-62, block_entangler.rs:5-77,
//               block_fold_iterator.rs:53-148]
//  k_hist       per block: DC prediction in emission order, AC run/size symbols;
//               DC and AC histograms [categorize.rs:132-169, symbol_counting.rs:55-74]
//  k_tables     one workgroup per (table, frame): package-merge code lengths, canonical
//               codes, JFIF header bytes [symbol_counting.rs:85-94,
//               length_limited.rs:37-134, huffman/encoder.rs:45-157,
//               encoder.rs:125-262]
//  k_emit, k_offsets, k_stuffwrite (entropy.hip): Huffman bit emission per
//               chunk, chunk offsets, byte stuffing, EOI [encoder.rs:264-404,
//               binary_stream.rs:38-96, segment_marker_injector.rs:13-30]
//
// Floating point: this file is compiled with -ffp-contract=off and without
// fast-math, f32 '/' is the correctly rounded IEEE division (hipcc default),
// roundf rounds half away from zero -- the reference's Rust f32 semantics.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "device_common.hpp"
#include "jpeg_common.hpp"
#include "kernels.hpp"
#include "wave_merge.hpp"

namespace dmmt {

#ifdef DMMT_PHASE_TRACE
static __device__ unsigned long long g_trace[64];
#endif

__constant__ uint8_t c_zigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                     12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                     35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                     58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
// zigzag position of natural index n
__constant__ uint8_t c_inv_zigzag[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                         3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                         10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                         21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// quantizer.rs:60: round(d / q) half away from zero, Rust's saturating `as i16`
__device__ __forceinline__ int16_t quantize(float d, float q) {
    float x = roundf(d / q);
    if (x != x) return 0;
    x = fminf(fmaxf(x, -32768.0f), 32767.0f);
    return (int16_t)(int)x;
}

// Image<f32> dots: quantize(d, q) over the 8 rows of one column (row r scaled by
// q[8r], rq[8r] = 1/q) without the division in the common case, branch-free on
// the fast path.  t = d * (1/q) is within 1.5 * 2^-23 * |t| of the correctly
// rounded quotient, so both round alike unless t lies within a * 2^-20 of a
// half-integer.  Round half away from zero of a = |t| is
// trunc(a + 0.5) there, exactly: a < 2^22 and a's fraction is farther than
// a * 2^-20 > ulp(a + 0.5) / 2 from 1/2, so the addition cannot round across an
// integer -- and the rare lanes outside it redone with the division afterwards.
__device__ __forceinline__ void quantize_col8(const float (&v)[8], const float* q, const float* rq, int (&x)[8]) {
    bool slow = false;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const float t = v[r] * rq[8 * r];
        const float a = fabsf(t);
        slow |= !(a < 4194304.0f && fabsf(__builtin_amdgcn_fractf(a) - 0.5f) > a * 0x1p-20f);
        const float n = copysignf(fminf(truncf(a + 0.5f), 32768.0f), t);  // saturating `as i16` below
        x[r] = (int)fminf(n, 32767.0f);
    }
    if (slow) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float a = fabsf(v[r] * rq[8 * r]);
            if (!(a < 4194304.0f && fabsf(__builtin_amdgcn_fractf(a) - 0.5f) > a * 0x1p-20f))
                x[r] = quantize(v[r], q[8 * r]);
        }
    }
}

// arai.rs:7-26 constants, f32 literals as written in the reference
#define DMMT_A1 0.70710678118654752440f
#define DMMT_A2 0.5411961f
#define DMMT_A3 DMMT_A1
#define DMMT_A4 1.3065629f
#define DMMT_A5 0.3826834f

// arai.rs:85-92 output scaling, by output index
#define DMMT_S0 0.3535533f
#define DMMT_S1 0.2548978f
#define DMMT_S2 0.27059805f
#define DMMT_S3 0.30067244f
#define DMMT_S4 0.35355338f
#define DMMT_S5 0.4499881f
#define DMMT_S6 0.6532815f
#define DMMT_S7 1.2814577f
__constant__ float c_arai_scale[8] = {DMMT_S0, DMMT_S1, DMMT_S2, DMMT_S3, DMMT_S4, DMMT_S5, DMMT_S6, DMMT_S7};

// arai.rs:29-84: 8-point AAN butterfly, output k before its scaling factor
__device__ __forceinline__ void arai8_unscaled(float (&v)[8]) {
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
    v[0] = v30;
    v[4] = v31;
    v[2] = v52;
    v[6] = v53;
    v[5] = v64;
    v[1] = v65;
    v[7] = v66;
    v[3] = v67;
}

// arai.rs:29-92: the butterfly with its output scaling
__device__ __forceinline__ void arai8(float (&v)[8]) {
    arai8_unscaled(v);
    v[0] = v[0] * DMMT_S0;
    v[1] = v[1] * DMMT_S1;
    v[2] = v[2] * DMMT_S2;
    v[3] = v[3] * DMMT_S3;
    v[4] = v[4] * DMMT_S4;
    v[5] = v[5] * DMMT_S5;
    v[6] = v[6] * DMMT_S6;
    v[7] = v[7] * DMMT_S7;
}

// Quantisation for integer samples, whose coefficients are bounded: the samples
// normalise into [0, 1] (a larger one is an error, color.rs:63-65), so Y, Cb, Cr
// lie in [-128, 128] and every FDCT output in [-2048, 2048] (DC = sum / 8, AC at
// most (1/4) * 64 * 128), to within a few ulps; with q >= 1, |d/q| <= 2049 and
// the saturation of `as i16` cannot trigger.
// The column pass's output scaling is folded into the reciprocal: u = the
// unscaled column outputs (arai8_unscaled, the reference's butterfly values),
// crq[8r] = fl(scale_r * fl(1/q)).  t = fl(u * crq) and the reference's
// fl(fl(u * scale_r) / q) are both the exact quotient u * scale_r / q times at
// most three, resp. two, factors (1 + d), |d| <= 2^-24, so they lie within
// 5.0001 * 2^-24 * |t| < 2^-21 * |t| of each other.  Where
// |t - rint(t)| + 2^-21 * |t| < 1/2 the reference's quotient therefore lies in the
// same open interval (n - 1/2, n + 1/2) around n = rint(t): no tie, and round half
// away from zero gives n.  Both terms are exact in f32 (Sterbenz; a power-of-two
// scaling; one fma) and their sum rounds by at most 2^-25, covered by testing against
// 1/2 - 2^-20.  The margin scales with |t|: small coefficients -- nearly all of
// them -- take the exact path only within ~|t| * 2^-20 of a half-integer, so a wave
// almost never has a lane there.  The other lanes (and NaN: maxval 0, q 0) redo d
// and the division afterwards.
// The eight distances are folded with max before one compare; a NaN (only from
// 0/0, maxval 0: `nan_possible`) would vanish in the max, so that case always
// takes the exact path.
__device__ __forceinline__ float quant_margin(float t, float n) {
    return __builtin_fmaf(fabsf(t), 0x1p-21f, fabsf(t - n));  // (the product is exact: one rounding)
}
__device__ __forceinline__ void quantize_col8_scaled(const float (&u)[8], const float* q, const float* crq,
                                                     bool nan_possible, int (&x)[8]) {
    float dist = 0.0f;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const float t = u[r] * crq[8 * r];
        const float n = __builtin_rintf(t);
        dist = fmaxf(dist, quant_margin(t, n));
        x[r] = (int)n;
    }
    if (nan_possible || !(dist < 0.49999905f)) {  // 1/2 - 2^-20
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float t = u[r] * crq[8 * r];
            if (!(quant_margin(t, __builtin_rintf(t)) < 0.49999905f)) x[r] = quantize(u[r] * c_arai_scale[r], q[8 * r]);
        }
    }
}

// color.rs:75-100
__device__ __forceinline__ void rgb_to_ycbcr(float r, float g, float b, float& y, float& cb, float& cr) {
    const float k128 = 128.0f / 255.0f;
    y = (((r * 0.299f + g * 0.587f) + b * 0.114f) - k128) * 255.0f;
    cb = ((r * -0.1687f + g * -0.3312f) + b * 0.5f) * 255.0f;
    cr = ((r * 0.5f + g * -0.4186f) + b * -0.0813f) * 255.0f;
}

// ============================================================== k_front

// Raw pixel staging: a tile row is 256 pixels = RB bytes, fetched as the RC
// aligned 16-byte chunks that cover it at any alignment (byte loads only for a
// chunk that crosses the frame's first or last byte).  Chunk q of a tile is
// chunk q % RC of tile row q / RC; thread t owns chunks t, t+256, ...  In LDS a
// tile row starts at row * RS, its first pixel `misalign` bytes further.  Every
// byte of a tile row past the image's right edge, and every row past its bottom,
// stages as 0: sample 0 normalises to 0.0, the reference's black padding
// (padder.rs:12-42), so phase A needs no bounds checks.
template <typename Sample, int ROWS>
struct RawTile {
    static constexpr int RB = 256 * 3 * (int)sizeof(Sample);
    static constexpr int RC = RB / 16 + 1;
    static constexpr int RS = RC * 16;
    static constexpr int NCHUNK = ROWS * RC;
    static constexpr int NQ = (NCHUNK + 255) / 256;
    static constexpr int BYTES = NCHUNK * 16;

    __device__ static __forceinline__ long long row_start(const Geom& g, int x0, int py) {
        return ((long long)py * g.width + x0) * 3 * (long long)sizeof(Sample);
    }
    __device__ static __forceinline__ int misalign(const uint8_t* fbase, long long start) {
        return (int)(((uintptr_t)fbase + (uintptr_t)start) & 15u);
    }

    // misalign() from 32-bit arithmetic: only the address's low 4 bits matter
    __device__ static __forceinline__ int misalign32(const uint8_t* fbase, const Geom& g, int x0, int py) {
        return (int)(((uint32_t)(uintptr_t)fbase + (uint32_t)(py * g.width + x0) * (uint32_t)(3 * sizeof(Sample))) & 15u);
    }

    __device__ static __forceinline__ void load(const uint8_t* __restrict__ fbase, long long fbytes, const Geom& g,
                                                int x0, int y0, int tid, uint4 (&v)[NQ]) {
        // Interior tile (wave-uniform): every row inside the image, no pixel past its
        // right edge, every chunk inside the frame's bytes -- plain aligned loads, no
        // masking.  The bytes a chunk holds beyond the tile row are never read.
        const long long last = row_start(g, x0, y0 + ROWS - 1);
        if (x0 + 256 <= g.width && y0 + ROWS <= g.height && row_start(g, x0, y0) >= 16 && last + RB + 16 <= fbytes) {
            const uint8_t* tb = fbase + row_start(g, x0, y0);
            const uint32_t rowpitch = (uint32_t)g.width * (uint32_t)(3 * sizeof(Sample));
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
                const int q = tid + 256 * i;
                const int row = q / RC, j = q - (q / RC) * RC;
                const uint8_t* r = tb + (size_t)((uint32_t)row * rowpitch);  // pointer arithmetic: stays global
                const uint8_t* a = r - ((uint32_t)(uintptr_t)r & 15u) + 16u * (uint32_t)j;
                v[i] = q < NCHUNK ? ld16_nt(a) : make_uint4(0u, 0u, 0u, 0u);
            }
            return;
        }
        const long long rowbytes = (long long)min(256, g.width - x0) * 3 * (long long)sizeof(Sample);
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
            v[i] = make_uint4(0u, 0u, 0u, 0u);
            const int q = tid + 256 * i;
            const int row = q / RC, j = q - (q / RC) * RC;
            const int py = y0 + row;
            if (q >= NCHUNK || py >= g.height) continue;
            const long long start = row_start(g, x0, py);
            const long long c = start - misalign(fbase, start) + 16LL * j;  // frame-relative
            if (c >= start + rowbytes) continue;
            if (c >= 0 && c + 16 <= fbytes) {
                v[i] = ld16_nt(fbase + c);
            } else {
                uint32_t w[4] = {0u, 0u, 0u, 0u};
                for (int k = 0; k < 16; ++k)
                    if (c + k >= 0 && c + k < fbytes) w[k >> 2] |= (uint32_t)fbase[c + k] << (8 * (k & 3));
                v[i] = make_uint4(w[0], w[1], w[2], w[3]);
            }
            const long long keep = start + rowbytes - c;  // bytes of the chunk inside the tile row
            if (keep < 16) {  // zero the rest: past the image's right edge the tile reads black
                uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const long long n = keep - 4 * k;
                    w[k] &= n >= 4 ? 0xFFFFFFFFu : (n <= 0 ? 0u : (1u << (8 * n)) - 1u);
                }
                v[i] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
    }

    __device__ static __forceinline__ void stage(uint8_t* sRaw, int tid, const uint4 (&v)[NQ]) {
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
            const int q = tid + 256 * i;
            if (q < NCHUNK) reinterpret_cast<uint4*>(sRaw)[q] = v[i];
        }
    }
};

// One workgroup (256 threads) per tile = TM horizontally adjacent MCUs of one
// MCU row (256 padded pixel columns, 8*VR rows), looping over the frame's tiles
// (grid = resident workgroups; blockIdx.y = frame) with the next tile's pixels
// prefetched into registers while the current one computes.
//  A  colour + subsampling + row DCT, fused: one thread per (chroma row, luma
//     block column) converts its 8 x VR pixels (raw bytes from LDS), box-averages
//     the chroma in the reference's sum order and runs the row pass of its VR
//     luma rows and of the chroma rows in registers -> block-major LDS (stride
//     BS); with 4:2:x the two threads of a chroma block swap four chroma samples
//     over DPP and take one chroma row pass each
//  C  column DCT + quantise (quantize_col8_scaled): one lane per (block, column),
//     the column's 8 coefficients kept in registers for
//  D  their store: 16 B per lane, 8 lanes per block (blocks are column-major in
//     HBM, coef_pos).  The symbols are counted by k_hist, one thread per block:
//     a walk over the block costs a third of the instructions the same counts
//     cost here, spread over the block's 8 lanes.
// Two barriers per tile: the next tile's staging barrier also keeps its phase A
// from overwriting sT before every wave has read its columns.
template <int HR, int VR, typename Sample, int WPE>
__global__ __launch_bounds__(256, WPE) void k_front(const Sample* __restrict__ rgb, size_t frame_stride, Geom g,
                                               const float* __restrict__ norm_lut,
                                               const float* __restrict__ qtab,  // [2][64] natural, as f32
                                               int16_t* __restrict__ coef, int* __restrict__ status) {
    constexpr int TM = 32 / HR;      // MCUs per tile
    constexpr int ROWS = 8 * VR;     // pixel rows per tile
    constexpr int NLUMA = HR * VR;
    constexpr int BPM = NLUMA + 2;
    constexpr int NB = TM * BPM;     // blocks per tile
    constexpr int NYB = 32 * VR;     // Y blocks: 32 columns x VR rows
    constexpr int CB = TM;           // chroma blocks per component
    constexpr int BS = 72;           // LDS floats per block: 64 + pad (conflict-free column reads)
    // Block b starts at b * BS + 4 * f(b), f(b) = bit 2 of b, flipped for Cr: the
    // 16-byte row stores of phase A (ds_write_b128, lanes in groups of 8 on 8
    // consecutive blocks -- and Cb next to Cr with 4:2:x) start on 8 distinct
    // 4-bank offsets mod 32, and the column reads of phase C (32 lanes = 4
    // consecutive blocks x 8 columns) still hit 32 distinct banks.  With the plain
    // stride the stores were 2-way conflicted.
    auto blk_base = [](int b) { return b * BS + 4 * (((b >> 2) ^ (b >= NYB + CB ? 1 : 0)) & 1); };
    constexpr int SP = HR;           // threads per (chroma row, chroma block): one per luma block column
    constexpr int NJ = 8 * CB * SP;  // fused jobs (chroma row, chroma block, luma block column): 256
    constexpr int NCS = 8 / SP;      // chroma samples of a job
    constexpr int SB = (int)sizeof(Sample);
    constexpr int PXB = 8 * 3 * SB;  // raw bytes of one job row (8 pixels)
    constexpr int PXW = PXB / 4;
    constexpr int NCJ = NB * 8;      // column jobs
    constexpr int JPT = (NCJ + 255) / 256;
    using Raw = RawTile<Sample, ROWS>;

    // row-transformed blocks (A -> C)
    __shared__ __attribute__((aligned(16))) float sT[NB * BS + 4];
    __shared__ __attribute__((aligned(16))) uint8_t sRaw[Raw::BYTES];
    __shared__ float sLut[256];
    __shared__ float sQ[128];
    __shared__ float sRQ[128];  // 1/q, correctly rounded; integer samples: fl(scale_row * fl(1/q))

    DMMT_TRACE_START;
    const int tid = threadIdx.x;
    const int frame = blockIdx.y;
    const uint8_t* fbase = reinterpret_cast<const uint8_t*>(rgb + (size_t)frame * frame_stride);
    const long long fbytes = (long long)g.width * g.height * 3 * SB;
    if (tid < 128) sQ[tid] = qtab[tid];
    if (tid < 128) sRQ[tid] = SB == 4 ? 1.0f / qtab[tid] : c_arai_scale[(tid >> 3) & 7] * (1.0f / qtab[tid]);
    if (SB == 1) sLut[tid] = norm_lut[tid];
    const int col = tid & 7;  // the column pass always handles column tid & 7

    const int tiles_per_row = (g.mcux + TM - 1) / TM;
    const int ntiles = tiles_per_row * g.mcuy;
    int bad = 0;
    const bool check_range = SB != 4 && g.maxval < (SB == 1 ? 255 : 65535);

    uint4 raw[Raw::NQ];
    if ((int)blockIdx.x < ntiles) {
        const int my = blockIdx.x / tiles_per_row;
        Raw::load(fbase, fbytes, g, (blockIdx.x - my * tiles_per_row) * TM * 8 * HR, my * ROWS, tid, raw);
    }
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int my = tile / tiles_per_row;
        const int mx0 = (tile - my * tiles_per_row) * TM;
        const int x0 = mx0 * 8 * HR;
        const int y0 = my * ROWS;

        Raw::stage(sRaw, tid, raw);
        __syncthreads();
        {  // prefetch the next tile's pixels; they land while this tile computes
            const int nt = tile + gridDim.x;
            if (nt < ntiles) {
                const int ny = nt / tiles_per_row;
                Raw::load(fbase, fbytes, g, (nt - ny * tiles_per_row) * TM * 8 * HR, ny * ROWS, tid, raw);
            }
        }

        // ---- A: colour + subsampling + row pass (color.rs:75-100, padder.rs: outside
        //      = black, subsampling.rs Subsampler::rect x outer / y inner, arai.rs:97-99)
        // the range check (color.rs:63-65) only where a sample can exceed maxval:
        // not for u8 samples with maxval 255 or u16 with 65535 (the PPM norm)
        auto phase_a = [&](auto range_check) {
            constexpr bool CHECK = decltype(range_check)::value;
            const int h = tid % SP, job = tid / SP;
            const int c = job % CB, r = job / CB;  // chroma block, chroma row
            const int lx0 = c * 8 * HR + 8 * h;    // first pixel column of the job
            uint32_t pw[VR][SB == 4 ? 1 : PXW];    // raw bytes of the job's VR pixel rows (integer samples)
            const float* fsrc[VR];                 // the rows themselves (float samples)
#pragma unroll
            for (int dy = 0; dy < VR; ++dy) {
                const int ly = r * VR + dy;
                const int mis = Raw::misalign32(fbase, g, x0, y0 + ly);
                const uint8_t* src = sRaw + ly * Raw::RS + mis + lx0 * 3 * SB;
                fsrc[dy] = reinterpret_cast<const float*>(src);
                if constexpr (SB == 4) {
                    pw[dy][0] = 0u;
                } else if ((mis & 7) == 0) {
#pragma unroll
                    for (int k = 0; k < PXW / 2; ++k) {
                        const uint2 u = reinterpret_cast<const uint2*>(src)[k];
                        pw[dy][2 * k] = u.x;
                        pw[dy][2 * k + 1] = u.y;
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < PXW; ++k)
                        pw[dy][k] = (uint32_t)src[4 * k] | ((uint32_t)src[4 * k + 1] << 8) |
                                    ((uint32_t)src[4 * k + 2] << 16) | ((uint32_t)src[4 * k + 3] << 24);
                }
            }
            float yv[VR][8];
            float cbv[8], crv[8];  // (4:2:x: the job's NCS = 4 samples first)
            uint32_t smax = 0;  // largest sample of the job (a sample above maxval panics in color.rs:63-65)
#pragma unroll
            for (int k = 0; k < NCS; ++k) {  // chroma sample k of the job
                float cbs = 0.0f, crs = 0.0f;
#pragma unroll
                for (int dx = 0; dx < HR; ++dx) {
#pragma unroll
                    for (int dy = 0; dy < VR; ++dy) {
                        const int jx = k * HR + dx;  // pixel within the job row
                        float rr, gg, bb;
                        if constexpr (SB == 4) {  // Image<f32> dots as given (0.0 past the edges)
                            rr = fsrc[dy][jx * 3];
                            gg = fsrc[dy][jx * 3 + 1];
                            bb = fsrc[dy][jx * 3 + 2];
                        } else {
                            uint32_t sv[3];
#pragma unroll
                            for (int ch = 0; ch < 3; ++ch) {
                                const int si = jx * 3 + ch;  // sample index in the row
                                sv[ch] = SB == 1 ? (pw[dy][si >> 2] >> (8 * (si & 3))) & 0xFFu
                                                 : (pw[dy][si >> 1] >> (16 * (si & 1))) & 0xFFFFu;
                            }
                            if constexpr (CHECK) smax = max(smax, max(sv[0], max(sv[1], sv[2])));
                            if (SB == 1) {
                                rr = sLut[sv[0]];
                                gg = sLut[sv[1]];
                                bb = sLut[sv[2]];
                            } else {
                                rr = norm_lut[sv[0]];
                                gg = norm_lut[sv[1]];
                                bb = norm_lut[sv[2]];
                            }
                        }
                        float y, cb, cr;
                        rgb_to_ycbcr(rr, gg, bb, y, cb, cr);
                        yv[dy][jx] = y;
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
                cbv[k] = cbs;
                crv[k] = crs;
            }
            if constexpr (CHECK) bad |= (int)(smax > (uint32_t)g.maxval);  // status bit 1
#pragma unroll
            for (int dy = 0; dy < VR; ++dy) {
                const int ly = r * VR + dy;
                arai8(yv[dy]);
                float4* o = reinterpret_cast<float4*>(sT + blk_base((ly >> 3) * 32 + c * HR + h) + (ly & 7) * 8);
                o[0] = make_float4(yv[dy][0], yv[dy][1], yv[dy][2], yv[dy][3]);
                o[1] = make_float4(yv[dy][4], yv[dy][5], yv[dy][6], yv[dy][7]);
            }
            if constexpr (SP == 1) {
                arai8(cbv);
                arai8(crv);
                float4* ob = reinterpret_cast<float4*>(sT + blk_base(NYB + c) + r * 8);
                ob[0] = make_float4(cbv[0], cbv[1], cbv[2], cbv[3]);
                ob[1] = make_float4(cbv[4], cbv[5], cbv[6], cbv[7]);
                float4* orr = reinterpret_cast<float4*>(sT + blk_base(NYB + CB + c) + r * 8);
                orr[0] = make_float4(crv[0], crv[1], crv[2], crv[3]);
                orr[1] = make_float4(crv[4], crv[5], crv[6], crv[7]);
            } else {
                // the pair (h = 0, 1) holds chroma samples 0..3 and 4..7 of the row:
                // h = 0 takes the row pass of Cb, h = 1 that of Cr, each swapping
                // the four samples the other needs (DPP quad_perm [1,0,3,2]: lane ^ 1)
                float fr[8];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float send = h ? cbv[k] : crv[k];
                    const float recv = __int_as_float(
                        __builtin_amdgcn_update_dpp(0, __float_as_int(send), 0xB1, 0xF, 0xF, false));
                    fr[k] = h ? recv : cbv[k];
                    fr[4 + k] = h ? crv[k] : recv;
                }
                arai8(fr);
                float4* oc = reinterpret_cast<float4*>(sT + blk_base(NYB + (h ? CB : 0) + c) + r * 8);
                oc[0] = make_float4(fr[0], fr[1], fr[2], fr[3]);
                oc[1] = make_float4(fr[4], fr[5], fr[6], fr[7]);
            }
        };
        if (tid < NJ) {
            if (check_range)
                phase_a(std::integral_constant<bool, true>{});
            else
                phase_a(std::integral_constant<bool, false>{});
        }
        __syncthreads();
        DMMT_TRACE(0);

        // ---- C: column pass (stride 8, arai.rs:100-102), quantise (quantizer.rs:53-62)
        // ---- D: the tile's blocks in MCU emission order (block_entangler.rs:69-77,
        //      block_fold_iterator.rs:53-148), only those of MCUs inside the image
        const int nvalid = min(TM, g.mcux - mx0) * BPM;
        const long long e0 = (long long)frame * g.bpf + ((long long)my * g.mcux + mx0) * BPM;
        int16_t* const cbase = coef + e0 * 64;  // (uniform: the stores take a 32-bit lane offset)
        static_assert(NCJ % 256 == 0, "JPT column jobs for every thread");
#pragma unroll
        for (int jj = 0; jj < JPT; ++jj) {
            const int blk = (tid + 256 * jj) >> 3;
            int x[8];
            {
                const float* q = sQ + (blk < NYB ? 0 : 64) + col;
                const float* rq = sRQ + (blk < NYB ? 0 : 64) + col;
                float v[8];
                const float* tb = sT + blk_base(blk) + col;
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = tb[i * 8];
                if constexpr (SB == 4) {  // Image<f32> dots: unbounded coefficients
                    arai8(v);
                    quantize_col8(v, q, rq, x);
                } else {
                    arai8_unscaled(v);
                    quantize_col8_scaled(v, q, rq, g.maxval == 0, x);
                }
            }
            int el;
            if (blk < NYB) {
                const int by = blk / 32, bx = blk % 32;
                el = (bx / HR) * BPM + by * HR + (bx % HR);  // TL,TR,BL,BR (block_entangler.rs:69-77)
            } else if (blk < NYB + CB) {
                el = (blk - NYB) * BPM + NLUMA;
            } else {
                el = (blk - NYB - CB) * BPM + NLUMA + 1;
            }
            const bool valid = el < nvalid;  // (uniform over the block's 8 lanes)
            if (valid) {
                uint32_t pk[4];  // the low halves of two coefficients per word (one v_perm_b32)
#pragma unroll
                for (int i = 0; i < 4; ++i) pk[i] = __builtin_amdgcn_perm((uint32_t)x[2 * i + 1], (uint32_t)x[2 * i], 0x05040100u);
                *reinterpret_cast<uint4*>(cbase + (el * 64 + 8 * col)) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            }
        }
        DMMT_TRACE(2);
    }

    if (bad) raise_status(status, bad);  // 1: sample above maxval
    DMMT_TRACE(5);
    DMMT_TRACE_FLUSH(0, 0);
}

// ============================================================== k_hist
// One thread per block, emission order (grid-stride over the frame's blocks):
//  * the DC difference to the previous block of the component (categorize.rs:
//    153-169; the predictor reset at restart-interval starts, an extension) and
//    the DC histograms;
//  * the block's AC symbols (categorize.rs:132-151): a register walk over its 63
//    AC coefficients in zigzag order -- a ZRL per 16 zeros before a non-zero,
//    (run & 15) << 4 | category, EOB after trailing zeros -- counted into the AC
//    histograms (symbol_counting.rs:55-74), and its last non-zero position
//    (k_emit's walk order).
// The DC is read from the block itself (index 0 of the column-major block).
// CHECK: an AC -32768 can occur (Image<f32> dots or host blocks); it has no
// category (categorize.rs:25-30).  Integer samples bound |v| by 2049 and skip the
// test (four instructions per position of the walk).
struct HistCoef {
    uint32_t w[32];  // zigzag position 2i in the low half of w[i], 2i+1 in the high half
};

// (the fused tables, defined below)
constexpr int kTailSmallWords = 4 + 4 * 16;
__device__ __forceinline__ void tables_tail(uint8_t* lds, const uint32_t* ac_hist, const uint32_t* dc_hist, int frame,
                                            const Geom& g, uint32_t* __restrict__ code_tab, uint8_t* __restrict__ out,
                                            size_t out_stride, uint32_t* __restrict__ hdr_len,
                                            const uint8_t* __restrict__ qtab_u8, int bits_per_channel,
                                            int* __restrict__ status, int* sCnt, int* sBits);
constexpr int kHistCopies = 4, kHistCopyWords = 545;
constexpr int kTailLdsBytes = 7072;  // tables_tail's per-table regions (static_assert below)

// FUSE (tables_fusable): the frame's last workgroup to finish also builds the four
// Huffman tables and the header (tables_tail), so no k_tables launch follows.
// Eight waves per SIMD (at most 64 VGPRs): the tail alone would take more, and the
// histogram loop wants the occupancy.
template <bool CHECK, bool FUSE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_hist(const int16_t* __restrict__ coef, int16_t* __restrict__ dcdiff,
                                              uint8_t* __restrict__ lastnz, Geom g,
                                              uint32_t* __restrict__ ac_hist /*[frames][reps][2][256]*/,
                                              uint32_t* __restrict__ dc_hist /*[frames][reps][2][16]*/,
                                              int* __restrict__ status, uint32_t* __restrict__ arrive,
                                              uint32_t* __restrict__ code_tab, uint8_t* __restrict__ out,
                                              size_t out_stride, uint32_t* __restrict__ hdr_len,
                                              const uint8_t* __restrict__ qtab_u8, int bits_per_channel) {
    // four copies of the histograms (lane & 3): the lanes of a wave often count
    // the same symbol at the same position; 545 words apart (different banks).
    // FUSE: the same LDS then holds the tables' work (tables_tail).
    constexpr int NC = kHistCopies, HS = kHistCopyWords;
    constexpr int kWords = FUSE && kTailLdsBytes / 4 > NC * HS ? kTailLdsBytes / 4 : NC * HS;
    __shared__ __attribute__((aligned(16))) uint32_t sH[kWords];  // per copy: [AC luma 256][AC chroma 256][DC luma 16][DC chroma 16]
    __shared__ int sSmall[FUSE ? kTailSmallWords : 1];
    __shared__ uint32_t sLastWg;
    const int tid = threadIdx.x;
    const int frame = blockIdx.y;
    for (int i = tid; i < NC * HS; i += 256) sH[i] = 0;
    __syncthreads();
    uint32_t* const H = sH + HS * (tid & 3);
    const long long base = (long long)frame * g.bpf;
    const int lane = lane_id();
    int bad = 0;
    // block el = MCU m, block k of it (bpf < 2^31: every index fits 32 bits); the
    // loop steps (m, k) and m mod the restart interval instead of dividing again
    const uint32_t bpf = (uint32_t)g.bpf, bpm = (uint32_t)g.bpm, ri = (uint32_t)max(g.restart_interval, 1);
    const uint32_t stride = gridDim.x * 256u, sm = stride / bpm, sk = stride - sm * bpm;
    uint32_t el = blockIdx.x * 256u + (uint32_t)tid;
    uint32_t m = el / bpm, k = el - m * bpm, mr = m % ri;
    const uint32_t smr = sm % ri;
    for (; el < bpf; el += stride) {
        const long long e = base + el;
        const uint4* q = reinterpret_cast<const uint4*>(coef + e * 64);
        uint32_t cw[32];  // column-major (coef_pos)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint4 v = q[i];
            cw[4 * i] = v.x, cw[4 * i + 1] = v.y, cw[4 * i + 2] = v.z, cw[4 * i + 3] = v.w;
        }
        const int t = k < (uint32_t)g.n_luma ? 0 : 1;
        // DC: the predictor is the previous block of the component, usually a few
        // lanes back in this wave (its DC over a lane shuffle), else a load -- issued
        // here, used after the AC walk, so that the walk hides its latency
        const bool restart = g.restart_interval > 0 && mr == 0;
        int back = 0;  // blocks back to the predictor; 0: none (predictor 0)
        if (k > 0 && k < (uint32_t)g.n_luma)
            back = 1;
        else if (m > 0 && !restart)
            back = (k == 0) ? (int)bpm - g.n_luma + 1 : (int)bpm;
        const int cur = (int)(int16_t)(cw[0] & 0xFFFFu);
        const int nb = __shfl_up(cur, (unsigned)back, 64);  // (lanes below `back` get their own)
        int pv = 0;
        if (back) pv = lane >= back ? nb : (int)coef[(e - back) * 64];
        // AC: zigzag order in registers (a constant permutation of the 64 halves)
        HistCoef b;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int i0 = coef_pos(2 * j), i1 = coef_pos(2 * j + 1);
            const uint32_t lo = (cw[i0 >> 1] >> (16 * (i0 & 1))) & 0xFFFFu;
            const uint32_t hi = (cw[i1 >> 1] >> (16 * (i1 & 1))) & 0xFFFFu;
            b.w[j] = lo | (hi << 16);
        }
        uint32_t* h = H + 256 * t;
        // l16 = 16 * (position of the last non-zero + 1): the zero run before position
        // kk is r16 / 16 with r16 = 16 * kk - l16, (run & 15) << 4 = r16 & 0xF0
        int l16 = 16;
        uint32_t zrl = 0;
#pragma unroll
        for (int kk = 1; kk < 64; ++kk) {
            const int v = (kk & 1) ? ((int)b.w[kk >> 1] >> 16) : (int)(int16_t)(b.w[kk >> 1] & 0xFFFFu);
            if (v != 0) {
                if (CHECK && v == -32768) bad |= 4;
                const int r16 = 16 * kk - l16;
                zrl += (uint32_t)(r16 >> 8);
                atomicAdd(&h[(r16 & 0xF0) | category_fast(v)], 1u);
                l16 = 16 * kk + 16;
            }
        }
        if (zrl) atomicAdd(&h[0xF0], zrl);
        if (l16 < 16 * 64) atomicAdd(&h[0], 1u);  // EOB
        lastnz[e] = (uint8_t)((l16 >> 4) - 1);      // 0: no non-zero AC coefficient
        {
            const int16_t d = (int16_t)(cur - pv);  // i16 subtraction
            bad |= d == -32768 ? 4 : 0;               // no category (categorize.rs:25-30)
            dcdiff[e] = d;
            atomicAdd(&H[512 + 16 * t + category_of(d)], 1u);
        }
        m += sm, k += sk, mr += smr;
        if (k >= bpm) k -= bpm, ++m, ++mr;
        if (mr >= ri) mr -= ri;
    }
    if (bad) raise_status(status, bad);
    __syncthreads();
    const size_t rep = (size_t)frame * kHistReps + blockIdx.x % kHistReps;
    for (int i = tid; i < 544; i += 256) {
        uint32_t v = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) v += sH[HS * c + i];
        if (!v) continue;
        if (i < 512)
            atomicAdd(&ac_hist[rep * 512 + i], v);
        else
            atomicAdd(&dc_hist[rep * 32 + (i - 512)], v);
    }
    if (FUSE) {  // count this workgroup in (arrive_last); the frame's last one builds the tables
#if !DMMT_ARRIVE_FORMAL
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's flush atomics have completed
#endif
        __syncthreads();  // (also: every wave's sH reads are done before the tail reuses the LDS)
        if (tid == 0) sLastWg = arrive_last(arrive + (size_t)frame * kArriveWords, blockIdx.x, gridDim.x);
        __syncthreads();
        if (sLastWg) {
            arrive_acquire();
            tables_tail(reinterpret_cast<uint8_t*>(sH), ac_hist, dc_hist, frame, g, code_tab, out, out_stride, hdr_len,
                        qtab_u8, bits_per_channel, status, sSmall, sSmall + 4);
        }
    }
}

// ============================================================== k_tables
// One 512-thread workgroup per (table, frame): blockIdx.x = table (0 luma DC,
// 1 luma AC, 2 chroma DC, 3 chroma AC); thread s < 256 = symbol / leaf s,
// thread 256 + j = package j.
//  1 histograms summed over the replicas (k_emit zeroes them after this launch);
//    every workgroup counts the present symbols of all four tables, which place
//    the DHT segments
//  2 compact the present symbols and rank them by (frequency, symbol): the stable
//    ascending sort of symbol_counting.rs:92-94 over the f>0 filter of 25-32
//  3 package-merge, limit 15 (length_limited.rs:37-134): level k = merge of the
//    pairwise packages of level k-1 with the leaves, ties leaf-first.  A leaf's
//    count of lighter packages never falls from one level to the next and a
//    package's count of leaves not heavier never rises (every level's items are
//    no heavier than the previous level's at the same index), so each search
//    gallops from its previous answer: usually one or two LDS reads per level
//  4 solution from the deepest level (n-1 packages): a scalar chain over
//    per-level package bitmasks with word prefix counts; lengths, +1 on the least
//    frequent symbol (symbol_counting.rs:85-90)
//  5 canonical codes over the reversed list (huffman/encoder.rs:45-67,116-119)
//  6 this table's DHT segment; table 0's workgroup also writes SOI, APP0, DQT,
//    SOF0, [DRI], SOS (encoder.rs:125-262)

#define PM_LEVELS 15

__device__ __forceinline__ void put_be16(uint8_t* p, int v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

// The table's DHT segment (encoder.rs:169-181: BITS, then the symbols most frequent
// first, i.e. symrank -- symbols by ascending frequency -- reversed) and, for table
// 0, SOI, APP0, DQT x2, SOF0, [DRI], SOS (encoder.rs:125-262) and the header length;
// a later stripe of an image (dmmt_stripe_*) writes no header.  Written by threads
// t0, t0 + step, ... of the table (k_tables: 256 per table; k_hist's fused tail: 64,
// whose table-0 wave passes the DQT bytes of zigzag position t0 already loaded:
// dq = luma | chroma << 8, else -1).
__device__ void write_table_header(uint8_t* o, int tab, int t0, int step, int n, const int nt[4],
                                   const uint8_t* symrank, const int* bits16, const Geom& g,
                                   const uint8_t* __restrict__ qtab_u8, int bits_per_channel, uint32_t* hdr_len,
                                   int dq = -1) {
    if (!g.stripe_first) {  // a later stripe of an image: tables only, no header
        if (tab == 0 && t0 == 0) *hdr_len = 0;
        return;
    }
    const int pos_dht0 = 2 + 18 + 69 + 69 + 19;
    const int off_lac = pos_dht0;
    const int off_ldc = off_lac + 21 + nt[1];
    const int off_cac = off_ldc + 21 + nt[0];
    const int off_cdc = off_cac + 21 + nt[3];
    const int dht = tab == 0 ? off_ldc : tab == 1 ? off_lac : tab == 2 ? off_cdc : off_cac;
    for (int s = t0; s < n; s += step) o[dht + 21 + s] = symrank[n - 1 - s];  // DHT symbols in reversed order (encoder.rs:180)
    for (int s = t0; s < 16; s += step) o[dht + 5 + s] = (uint8_t)bits16[s];
    if (t0 == 0) {
        uint8_t* d = o + dht;
        d[0] = 0xFF;
        d[1] = 0xC4;
        put_be16(d + 2, 2 + 17 + n);
        const uint8_t kind[4] = {0x00, 0x11, 0x02, 0x13};  // encoder.rs:92-98 TableKind
        d[4] = kind[tab];
    }
    if (tab != 0) return;
    const int pos_after_dht = pos_dht0 + 4 * 21 + nt[0] + nt[1] + nt[2] + nt[3];
    const int pos_sos = pos_after_dht + (g.restart_interval > 0 ? 6 : 0);
    if (t0 == 0) {
        o[0] = 0xFF;
        o[1] = 0xD8;  // SOI
        const uint8_t app0[18] = {0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0, 0x01, 0x02, 0x00, 0x00, 0x48, 0x00, 0x48, 0, 0};
        for (int i = 0; i < 18; ++i) o[2 + i] = app0[i];
        for (int q = 0; q < 2; ++q) {  // DQT, table in zigzag order (encoder.rs:193-212)
            uint8_t* d = o + 20 + 69 * q;
            d[0] = 0xFF;
            d[1] = 0xDB;
            put_be16(d + 2, 67);
            d[4] = (uint8_t)q;
        }
        uint8_t* sof = o + 158;  // encoder.rs:227-245
        sof[0] = 0xFF;
        sof[1] = 0xC0;
        put_be16(sof + 2, 17);
        sof[4] = (uint8_t)bits_per_channel;
        put_be16(sof + 5, g.sof_height);
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
        *hdr_len = (uint32_t)(pos_sos + 14);
    }
    if (dq >= 0) {
        o[25 + t0] = (uint8_t)dq;
        o[94 + t0] = (uint8_t)(dq >> 8);
        return;
    }
    for (int s = t0; s < 128; s += step) {
        const int q = s >> 6, i = s & 63;
        o[20 + 69 * q + 5 + i] = qtab_u8[q * 64 + c_zigzag[i]];
    }
}

// #{j < m : pair sum prev[2j] + prev[2j+1] < x}, known to be >= lb (sums ascending)
__device__ __forceinline__ int packages_below(const unsigned long long* prev, int m, unsigned long long x, int lb) {
    const ulonglong2* pr = reinterpret_cast<const ulonglong2*>(prev);
    int lo = lb, hi = m, step = 1;  // every j < lo is below x; the answer is in [lo, hi]
    while (lo < hi) {               // gallop up
        const int probe = min(lo + step - 1, hi - 1);
        const ulonglong2 p = pr[probe];
        if (p.x + p.y < x) {
            lo = probe + 1;
            step <<= 1;
        } else {
            hi = probe;
            break;
        }
    }
    while (lo < hi) {  // bisect [lo, hi]
        const int mid = (lo + hi) >> 1;
        const ulonglong2 p = pr[mid];
        if (p.x + p.y < x)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// #{i < m : f[i] <= x}, known to be <= ub (f ascending)
__device__ __forceinline__ int leaves_not_above(const unsigned long long* f, int m, unsigned long long x, int ub) {
    int lo = 0, hi = min(ub, m), step = 1;  // every i < lo is <= x, every i >= hi is > x
    while (lo < hi) {                       // gallop down
        const int probe = max(hi - step, lo);
        if (f[probe] <= x) {
            lo = probe + 1;
            break;
        }
        hi = probe;
        step <<= 1;
    }
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (f[mid] <= x)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(512) void k_tables(const uint32_t* __restrict__ ac_hist,
                                                const uint32_t* __restrict__ dc_hist,
                                                uint32_t* __restrict__ code_tab,  // [frames][4][256]
                                                uint8_t* __restrict__ out, size_t out_stride,
                                                uint32_t* __restrict__ hdr_len, Geom g,
                                                const uint8_t* __restrict__ qtab_u8,  // [2][64] natural
                                                int bits_per_channel, int* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) unsigned long long sKey[256];  // present symbols, symbol order
    __shared__ __attribute__((aligned(16))) unsigned long long sF[256];    // frequencies, ascending
    __shared__ __attribute__((aligned(16))) unsigned long long sLev[2][512];
    __shared__ unsigned long long sPk[PM_LEVELS][8];  // package positions per level (bitmask)
    __shared__ int sPkCum[PM_LEVELS][8];              // packages in the words before
    __shared__ uint8_t sSym[256];  // symbols by rank
    __shared__ int sLen[256];      // code length by rank
    __shared__ int sCnt[4][4];     // [wave][table] present symbols
    __shared__ int sLeaf[PM_LEVELS];
    __shared__ uint32_t sWave[4];
    __shared__ int sBits[16];

    DMMT_TRACE_START;
    const int tab = blockIdx.x, frame = blockIdx.y;
    const int t = threadIdx.x, lane = lane_id();
    const int s = t & 255, wave = s >> 6;
    const bool sym_thread = t < 256;

    // ---- 1
    unsigned long long fr[4] = {0, 0, 0, 0};
    if (sym_thread) {
        uint32_t va[2][kHistReps], vd[2][kHistReps];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int r = 0; r < kHistReps; ++r) {
                va[c][r] = ac_hist[(((size_t)frame * kHistReps + r) * 2 + c) * 256 + s];
                vd[c][r] = s < 16 ? dc_hist[((size_t)frame * kHistReps + r) * 32 + c * 16 + s] : 0u;
            }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            unsigned long long a = 0, d = 0;
#pragma unroll
            for (int r = 0; r < kHistReps; ++r) {
                a += va[c][r];
                d += vd[c][r];
            }
            fr[2 * c] = d;
            fr[2 * c + 1] = a;
        }
    }
    const unsigned long long f = fr[tab];
    const unsigned long long own = __ballot(f > 0);
    if (sym_thread) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned long long b = __ballot(fr[q] > 0);
            if (lane == 0) sCnt[wave][q] = __popcll(b);
        }
        if (s < 16) sBits[s] = 0;
    } else if (s < PM_LEVELS * 8) {
        sPk[s >> 3][s & 7] = 0ull;
    }
    __syncthreads();
    int nt[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) nt[q] = sCnt[0][q] + sCnt[1][q] + sCnt[2][q] + sCnt[3][q];
    const int n = nt[tab];
    if (sym_thread && f > 0) {
        int idx = __popcll(own & ((1ull << lane) - 1ull));
        for (int w = 0; w < wave; ++w) idx += sCnt[w][tab];
        sKey[idx] = (f << 8) | (unsigned)s;
    }
    if (sym_thread && ((s == 0 && n == 0) || ((tab & 1) && s == 0xFF && f > 0))) raise_status(status, 2);
    __syncthreads();
    DMMT_TRACE(10);

    // ---- 2: rank = present keys below mine
    if (sym_thread && f > 0) {
        const unsigned long long mykey = (f << 8) | (unsigned)s;
        const ulonglong2* k2 = reinterpret_cast<const ulonglong2*>(sKey);
        int r = 0;
        for (int j = 0; j < (n >> 1); ++j) {
            const ulonglong2 kk = k2[j];
            r += (kk.x < mykey ? 1 : 0) + (kk.y < mykey ? 1 : 0);
        }
        if (n & 1) r += sKey[n - 1] < mykey ? 1 : 0;
        sF[r] = f;
        sSym[r] = (uint8_t)s;
        sLev[0][r] = f;
    }
    __syncthreads();
    DMMT_TRACE(11);

    // ---- 3
    {
        int size_prev = n, np_prev = 0;
        int cnt = sym_thread ? 0 : n;  // previous answer: lower bound (leaf) / upper bound (package)
        const unsigned long long fl = sym_thread && s < n ? sF[s] : 0ull;
        for (int k = 1; k < PM_LEVELS; ++k) {
            const unsigned long long* prev = sLev[(k - 1) & 1];
            unsigned long long* cur = sLev[k & 1];
            const int np = size_prev >> 1;
            if (sym_thread) {
                if (s < n) {  // leaf s: after every package strictly lighter
                    cnt = packages_below(prev, np, fl, cnt);
                    cur[s + cnt] = fl;
                }
            } else if (s < np) {  // package s: after every leaf not heavier
                const ulonglong2 pp = reinterpret_cast<const ulonglong2*>(prev)[s];
                const unsigned long long P = pp.x + pp.y;
                cnt = leaves_not_above(sF, n, P, s < np_prev ? cnt : n);
                const int pos = s + cnt;
                cur[pos] = P;
                atomicOr(&sPk[k][pos >> 6], 1ull << (pos & 63));
            }
            np_prev = np;
            size_prev = n + np;
            __syncthreads();
        }
    }
    DMMT_TRACE(12);

    // ---- 4: leaves in the solution prefix of every level, deepest first: the
    // prefix of level k holds 2 * (packages taken at level k+1) items; the packages
    // among them are the ones taken at level k-1
    if (!sym_thread && s < PM_LEVELS * 8) {
        const int k = s >> 3, w = s & 7;
        int c = 0;
        for (int q = 0; q < w; ++q) c += __popcll(sPk[k][q]);
        sPkCum[k][w] = c;
    }
    __syncthreads();
    if (t == 0) {
        int packages = n - 1;
        for (int k = PM_LEVELS - 1; k >= 0; --k) {
            const int c = max(2 * packages, 0);  // <= 2n - 2 < 512
            const int w = c >> 6, b = c & 63;
            const int pk = sPkCum[k][w] + __popcll(sPk[k][w] & ((1ull << b) - 1ull));
            sLeaf[k] = c - pk;
            packages = pk;
        }
    }
    __syncthreads();
    if (sym_thread && s < n) {
        int len = s == 0 ? 1 : 0;
#pragma unroll
        for (int k = 0; k < PM_LEVELS; ++k) len += s < sLeaf[k] ? 1 : 0;
        sLen[s] = len;
        atomicAdd(&sBits[len - 1], 1);
    }
    __syncthreads();
    DMMT_TRACE(13);

    // ---- 5: code(p) = sum over reversed positions before p of 2^(16 - len)
    uint32_t* ct = code_tab + ((size_t)frame * 4 + tab) * 256;
    {
        const int rk = n - 1 - s;  // rank at reversed position s
        const uint32_t wgt = sym_thread && s < n ? 1u << (16 - sLen[rk]) : 0u;
        const uint32_t incl = wave_incl_scan_full_u32(wgt);
        if (sym_thread && lane == 63) sWave[wave] = incl;
        __syncthreads();
        uint32_t excl = incl - wgt;
        for (int q = 0; q < wave; ++q) excl += sWave[q];
        if (sym_thread && f == 0) ct[s] = 0;
        __syncthreads();  // the zeroes before the codes (a present symbol's entry is written by another thread)
        if (sym_thread && s < n) {
            const int L = sLen[rk];
            const uint32_t pat = excl & 0xFFFFu;  // left aligned u16 (wrapping as in the reference)
            ct[sSym[rk]] = ((uint32_t)L << 16) | (pat >> (16 - L));
        }
    }
    DMMT_TRACE(14);

    // ---- 6: header
    if (!sym_thread) return;
    write_table_header(out + (size_t)frame * out_stride, tab, s, 256, n, nt, sSym, sBits, g, qtab_u8, bits_per_channel,
                       hdr_len + frame);
    DMMT_TRACE(15);
    DMMT_TRACE_FLUSH(0, 1);
}

// ============================================================== fused tables
// k_tables' work done by k_hist's last workgroup of a frame (tables_fusable): wave
// t builds table t (0 luma DC, 1 luma AC, 2 chroma DC, 3 chroma AC).  Frequencies in
// 32 bits: the host fuses only frames whose symbol counts, and thus every package
// weight (at most 15 times their sum), stay below 2^30.  The phases of k_tables:
//  1 the 8 replicas summed (agent-scope loads after the arrival); symbol s = lane
//    + 64 q; the present symbols counted
//  2 symbol_counting.rs:92-94's stable ascending sort over the f > 0 filter of
//    25-32: keys (frequency << 8 | s) sorted in registers (sort_bitonic,
//    wave_merge.hpp; absent symbols are kMergeInf and sort last) when every
//    frequency is below 2^24; else the 64-bit keys compacted and ranked
//    (tail_rank)
//  3 package-merge, limit 15 (length_limited.rs:37-134), in registers: level k is
//    the merge of the leaves (ascending) with the pair sums of level k-1
//    (ascending), ties leaf first -- keys (weight << 1 | is_package), one
//    bitonic merger of the wave (wave_merge.hpp) per level, the package
//    positions of every level kept as 64-bit masks (a ballot per register slot,
//    parked in a lane of a VGPR)
//  4 the solution from the deepest level (n-1 packages), every lane alike, lengths,
//    +1 on the least frequent (symbol_counting.rs:85-90)
//  5 canonical codes over the reversed list (huffman/encoder.rs:45-67,116-119)
//  6 the DHT segment, and for table 0 the rest of the header (write_table_header)
// One barrier: before 6 (every table's symbol count).  LDS per table (bytes):
// F u32[cap] | the keys u64[cap] | Sym u8[cap]; cap = 256 for the AC tables, 16 DC.
#ifndef DMMT_TAIL_SORT2
#define DMMT_TAIL_SORT2 1  // an AC table of at most 128 symbols sorted in two register slots (0: study builds)
#endif
constexpr int kTailLevels = 15;
constexpr int kTailBase[4] = {0, 208, 3536, 3744};
static_assert(kTailBase[3] + 3328 == kTailLdsBytes, "tables_tail's LDS regions");

// The tail's phases pass data between the lanes of ONE wave through LDS: a wave's
// LDS operations complete in order, so no s_barrier -- only no code motion across.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Levels 1-14 of the package-merge over n leaves F (ascending) in 64 * EPL element
// merges (n <= 32 * EPL): slot-major, the leaves ascending in the lower half
// (static), the packages DESCENDING in the upper (element S/2 + m holds package
// S/2 - 1 - m), so each level is one bitonic merge.  Level k's package positions
// (a ballot per slot) and the packages before each slot are kept in lane k EPL + s
// of two VGPR pairs, and the solution chain reads them back
// (readlane): leaf[k] = the leaves in the solution prefix of level k.
template <int EPL>
__device__ __forceinline__ void tail_levels(const uint32_t* F, int n, int (&leaf)[kTailLevels]) {
    const int lane = lane_id();
    constexpr int H = EPL == 1 ? 1 : EPL / 2;  // register slots per half (EPL 1: lanes 0-31 / 32-63)
    // leaf index of lower-half slot t / package index of upper-half slot t in this lane
    auto leaf_index = [&](int t) { return EPL == 1 ? lane : 64 * t + lane; };
    auto pkg_index = [&](int t) { return EPL == 1 ? 63 - lane : 32 * EPL - 1 - 64 * t - lane; };
    uint32_t lk[H], pk[H];
    int np = n >> 1;
#pragma unroll
    for (int t = 0; t < H; ++t) {
        const int i = leaf_index(t), j = pkg_index(t);
        lk[t] = i < n ? F[min(i, 255)] << 1 : kMergeInf;
        pk[t] = j >= 0 && j < np ? ((F[2 * j] + F[2 * j + 1]) << 1) | 1u : kMergeInf;  // level 1: pairs of the leaves
    }
    // entry e = k EPL + s (level 0: no packages) in lane e & 63 of register e >> 6
    uint32_t mlo[2] = {0u, 0u}, mhi[2] = {0u, 0u}, mcum[2] = {0u, 0u};
    // the gather's source (see below): lane 2 (31 - (lane & 31)), upper-half slot t's
    // packages from slot EPL - 1 - 2t - (lane >> 5)
    const int src = 8 * (31 - (lane & 31));
    for (int k = 1; k < kTailLevels; ++k) {
        uint32_t x[EPL];
        if constexpr (EPL == 1) {
            x[0] = lane < 32 ? lk[0] : pk[0];
        } else {
#pragma unroll
            for (int t = 0; t < H; ++t) {
                x[t] = lk[t];
                x[H + t] = pk[t];
            }
        }
        merge_bitonic<EPL>(x);
        int before = 0;
#pragma unroll
        for (int s = 0; s < EPL; ++s) {
            const unsigned long long m = __ballot((x[s] & 1u) != 0u);
            const int e = k * EPL + s;
            const bool here = lane == (e & 63);
            if (EPL < 8 || e < 64) {  // (uniform)
                mlo[0] = here ? (uint32_t)m : mlo[0];
                mhi[0] = here ? (uint32_t)(m >> 32) : mhi[0];
                mcum[0] = here ? (uint32_t)before : mcum[0];
            } else {
                mlo[1] = here ? (uint32_t)m : mlo[1];
                mhi[1] = here ? (uint32_t)(m >> 32) : mhi[1];
                mcum[1] = here ? (uint32_t)before : mcum[1];
            }
            before += __popcll(m);
        }
        // the next level's packages: pairs (2j, 2j + 1) -- neighbouring lanes of a
        // slot -- summed in the even lane, then gathered to their descending places
        const int npn = (n + np) >> 1;
        uint32_t q[EPL];
#pragma unroll
        for (int s = 0; s < EPL; ++s) q[s] = (x[s] >> 1) + (lane_xor<1>(x[s]) >> 1);
#pragma unroll
        for (int t = 0; t < H; ++t) {
            uint32_t v;
            if constexpr (EPL == 1) {
                v = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)q[0]);
            } else {
                const uint32_t vh = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)q[EPL - 1 - 2 * t]);
                const uint32_t vl = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)q[EPL - 2 - 2 * t]);
                v = (lane & 32) ? vl : vh;
            }
            const int j = pkg_index(t);
            pk[t] = j >= 0 && j < npn ? (v << 1) | 1u : kMergeInf;
        }
        np = npn;
    }
    // the solution, deepest level first: the prefix of level k holds 2 * (packages
    // taken at level k+1) items, the packages among them are the ones taken at level
    // k-1 (every lane computes it: uniform values)
    int packages = n - 1;
#pragma unroll
    for (int k = kTailLevels - 1; k >= 0; --k) {
        const int cc = max(2 * packages, 0);  // <= 2n - 2 < 64 EPL
        const int e = k * EPL + (cc >> 6), b = cc & 63;
        uint32_t lo, hi, cm;
        if (EPL < 8 || e < 64) {
            lo = (uint32_t)__builtin_amdgcn_readlane((int)mlo[0], e);
            hi = (uint32_t)__builtin_amdgcn_readlane((int)mhi[0], e);
            cm = (uint32_t)__builtin_amdgcn_readlane((int)mcum[0], e);
        } else {
            lo = (uint32_t)__builtin_amdgcn_readlane((int)mlo[1], e - 64);
            hi = (uint32_t)__builtin_amdgcn_readlane((int)mhi[1], e - 64);
            cm = (uint32_t)__builtin_amdgcn_readlane((int)mcum[1], e - 64);
        }
        const unsigned long long m = (((unsigned long long)hi << 32) | lo) & ((1ull << b) - 1ull);
        const int pkc = (int)cm + __popcll(m);
        leaf[k] = cc - pkc;
        packages = pkc;
    }
}

// rank of every present key among the n keys (the stable ascending sort by
// frequency, symbol_counting.rs:92-94: ties by symbol, which the key's low byte
// carries); leaf rank -> F (frequency), Sym.  NS key slots per lane (key i at lane
// i % 64, slot i / 64); the keys read eight at a time, loads together; K: u32 keys
// (frequency << 8 | s) when every frequency is below 2^24, else u64.
template <int NS, typename K>
__device__ __forceinline__ void tail_rank(const K* Key, int n, uint32_t* F, uint8_t* Sym) {
    const int lane = lane_id();
    K mk[NS];
    uint32_t rk[NS];
#pragma unroll
    for (int r = 0; r < NS; ++r) {
        mk[r] = lane + 64 * r < n ? Key[lane + 64 * r] : (K)~(K)0;
        rk[r] = 0u;
    }
    constexpr int V = 16 / sizeof(K);  // keys per 16-byte read
    int j = 0;
    for (; j + 4 * V <= n; j += 4 * V) {
        K kk[4 * V];
#pragma unroll
        for (int u = 0; u < 4 * V; ++u) kk[u] = Key[j + u];
#pragma unroll
        for (int u = 0; u < 4 * V; ++u)
#pragma unroll
            for (int r = 0; r < NS; ++r) rk[r] += kk[u] < mk[r] ? 1u : 0u;
    }
    for (; j < n; ++j) {
        const K kk = Key[j];
#pragma unroll
        for (int r = 0; r < NS; ++r) rk[r] += kk < mk[r] ? 1u : 0u;
    }
#pragma unroll
    for (int r = 0; r < NS; ++r)
        if (lane + 64 * r < n) {
            F[rk[r]] = (uint32_t)(mk[r] >> 8);
            Sym[rk[r]] = (uint8_t)mk[r];
        }
}

template <typename K>
__device__ __forceinline__ void tail_rank_any(const K* Key, int n, uint32_t* F, uint8_t* Sym) {
    const int ns = (n + 63) >> 6;  // (uniform in the wave)
    if (ns <= 1)
        tail_rank<1>(Key, n, F, Sym);
    else if (ns == 2)
        tail_rank<2>(Key, n, F, Sym);
    else
        tail_rank<4>(Key, n, F, Sym);
}

__device__ __forceinline__ void tables_tail(uint8_t* lds, const uint32_t* ac_hist, const uint32_t* dc_hist, int frame,
                                            const Geom& g, uint32_t* __restrict__ code_tab, uint8_t* __restrict__ out,
                                            size_t out_stride, uint32_t* __restrict__ hdr_len,
                                            const uint8_t* __restrict__ qtab_u8, int bits_per_channel,
                                            int* __restrict__ status, int* sCnt, int* sBits) {
    const int lane = lane_id(), tab = threadIdx.x >> 6;
    const bool ac = tab & 1;
    const int c = tab >> 1;
    const int cap = ac ? 256 : 16;
    uint8_t* const base = lds + kTailBase[tab];
    uint32_t* const F = reinterpret_cast<uint32_t*>(base);
    unsigned long long* const Key = reinterpret_cast<unsigned long long*>(F + cap);
    uint8_t* const Sym = reinterpret_cast<uint8_t*>(F + 3 * cap);
    int* const bits16 = sBits + 16 * tab;

    // ---- 1 (AC: symbols lane + 64 q; DC: symbol lane < 16 -- coalesced loads)
    uint32_t f[4] = {0u, 0u, 0u, 0u};
    if (ac) {
        const uint32_t* h = ac_hist + ((size_t)frame * kHistReps * 2 + c) * 256 + lane;
#pragma unroll
        for (int r = 0; r < kHistReps; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) f[q] += ld_agent(h + (size_t)r * 512 + 64 * q);
    } else if (lane < 16) {
        const uint32_t* h = dc_hist + (size_t)frame * kHistReps * 32 + c * 16 + lane;
#pragma unroll
        for (int r = 0; r < kHistReps; ++r) f[0] += ld_agent(h + (size_t)r * 32);
    }
    // table 0's wave: its lane's DQT bytes (zigzag position lane of both tables, kept
    // in zigzag order by the host), loaded with the histograms rather than after
    // the tables
    int dq = -1;
    if (tab == 0 && g.stripe_first) dq = (int)qtab_u8[128 + lane] | ((int)qtab_u8[192 + lane] << 8);
    // keys (frequency << 8 | symbol): u32 while every frequency is below 2^24
    const bool k32 = __ballot(((f[0] | f[1] | f[2] | f[3]) >> 24) != 0u) == 0ull;
    uint32_t* const ct = code_tab + ((size_t)frame * 4 + tab) * 256;
    int n = 0;
    unsigned long long pres[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        pres[q] = __ballot(f[q] > 0u);
        if (f[q] == 0u) ct[lane + 64 * q] = 0;  // (a present symbol's entry: phase 5)
        n += __popcll(pres[q]);
    }
    // k_tables' checks: a table without symbols; symbol 0xFF in an AC table (the
    // reference's lookup table has 255 entries)
    raise_status(status, ((lane == 0 && n == 0) || (ac && lane == 63 && f[3] > 0u)) ? 2 : 0);  // (s 255: lane 63, q 3)
    if (lane == 0) sCnt[tab] = n;  // (read by every wave in phase 6, after the barrier)
    if (lane < 16) bits16[lane] = 0;

    // ---- 2: the present keys in ascending order (absent symbols: kMergeInf, last)
    // -> F (frequency), Sym by leaf rank
    if (k32) {
        if (ac && (!DMMT_TAIL_SORT2 || n > 128)) {
            uint32_t x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) x[q] = f[q] ? (f[q] << 8) | (uint32_t)(lane + 64 * q) : kMergeInf;
            sort_bitonic<4>(x);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (lane + 64 * q < n) {
                    F[lane + 64 * q] = x[q] >> 8;
                    Sym[lane + 64 * q] = (uint8_t)x[q];
                }
        } else if (ac) {  // (uniform) at most 128 present symbols: compacted into two slots, half the network
            uint32_t* const K32 = reinterpret_cast<uint32_t*>(Key);
            int at = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (f[q]) K32[at + __popcll(pres[q] & ((1ull << lane) - 1ull))] = (f[q] << 8) | (uint32_t)(lane + 64 * q);
                at += __popcll(pres[q]);
            }
            wave_lds_sync();
            uint32_t x[2] = {lane < n ? K32[lane] : kMergeInf, lane + 64 < n ? K32[lane + 64] : kMergeInf};
            sort_bitonic<2>(x);
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (lane + 64 * q < n) {
                    F[lane + 64 * q] = x[q] >> 8;
                    Sym[lane + 64 * q] = (uint8_t)x[q];
                }
        } else {
            uint32_t x[1] = {f[0] ? (f[0] << 8) | (uint32_t)lane : kMergeInf};
            sort_bitonic<1>(x);
            if (lane < n) {
                F[lane] = x[0] >> 8;
                Sym[lane] = (uint8_t)x[0];
            }
        }
    } else {  // rank among 64-bit keys, compacted slot by slot (order immaterial: the keys carry their symbols)
        int at = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (f[q]) Key[at + __popcll(pres[q] & ((1ull << lane) - 1ull))] = ((unsigned long long)f[q] << 8) | (unsigned)(lane + 64 * q);
            at += __popcll(pres[q]);
        }
        wave_lds_sync();
        tail_rank_any(Key, n, F, Sym);
    }
    wave_lds_sync();

    // ---- 3, 4 (wave-uniform choice of the merge width)
    int leaf[kTailLevels];
    if (n <= 32)
        tail_levels<1>(F, n, leaf);
    else if (n <= 64)
        tail_levels<2>(F, n, leaf);
    else if (n <= 128)
        tail_levels<4>(F, n, leaf);
    else
        tail_levels<8>(F, n, leaf);

    uint32_t len[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = lane + 64 * r;
        len[r] = 0;
        if (i < n) {
            uint32_t L = i == 0 ? 1u : 0u;
#pragma unroll
            for (int k = 0; k < kTailLevels; ++k) L += i < leaf[k] ? 1u : 0u;
            len[r] = L;
            atomicAdd(&bits16[L - 1], 1);
        }
    }

    // ---- 5: code(rank i) = sum over the ranks above i of 2^(16 - len), mod 2^16
    {
        uint32_t carry = 0;
        uint32_t inc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t wgt = len[r] ? 1u << (16 - len[r]) : 0u;
            inc[r] = carry + wave_incl_scan_full_u32(wgt);
            carry = (uint32_t)__builtin_amdgcn_readlane((int)inc[r], 63);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = lane + 64 * r;
            if (i < n) {
                const uint32_t pat = (carry - inc[r]) & 0xFFFFu;  // left aligned u16 (wrapping as in the reference)
                ct[Sym[i]] = (len[r] << 16) | (pat >> (16 - len[r]));
            }
        }
    }
    __syncthreads();  // every table's count (sCnt); this wave's BITS

    // ---- 6
    const int nt[4] = {sCnt[0], sCnt[1], sCnt[2], sCnt[3]};
    write_table_header(out + (size_t)frame * out_stride, tab, lane, 64, n, nt, Sym, bits16, g, qtab_u8,
                       bits_per_channel, hdr_len + frame, dq);
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
                                                   int first_frame, uint32_t seed, int row0, int rows) {
    const long long npx = (long long)w * h;       // the whole frame (the noise index)
    const long long nout = (long long)w * rows;   // rows [row0, row0 + rows) are generated
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nout * n_frames;
         i += (long long)gridDim.x * 256) {
        const int fl = (int)(i / nout);
        const long long pi = i - (long long)fl * nout + (long long)row0 * w;
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

}  // namespace dmmt

// ============================================================== launchers
namespace dmmt {

#ifndef FRONT_WPE_420
#define FRONT_WPE_420 3
#endif

static inline int clampi(long long v, int lo, int hi) { return (int)(v < lo ? lo : (v > hi ? hi : v)); }

// Waves per SIMD k_front is compiled for (register budget 512 / WPE): u8 4:4:4
// and 4:2:2 fit 128 registers, four resident workgroups per CU; the rest keep the
// allocation the compiler picks.
template <int HR, int VR, typename S>
constexpr int front_wpe() {
    return sizeof(S) == 1 ? (HR * VR == 4 ? FRONT_WPE_420 : 4) : 1;
}

template <int HR, int VR, typename S>
static void front_impl(const void* rgb, size_t stride_elems, int n_frames, const Geom& g, const Work& w,
                       hipStream_t st, int per_cu_cap) {
    constexpr int TM = 32 / HR;
    const long long ntiles = (long long)((g.mcux + TM - 1) / TM) * g.mcuy;
    // one workgroup per resident slot: each loops over tiles, prefetching the next
    static int resident = 0, n_cus = 0;
    static bool per_cu_env = false;
    if (!resident) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_front<HR, VR, S, front_wpe<HR, VR, S>()>, 256, 0) != hipSuccess ||
            per_cu < 1)
            per_cu = 2;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        if (const char* e = getenv("DMMT_FRONT_PER_CU")) {  // tuning knob (both lane modes)
            per_cu = atoi(e) > 0 ? atoi(e) : per_cu;
            per_cu_env = true;
        }
        resident = per_cu * cus;
        n_cus = cus;
    }
    // per_cu_cap: fewer resident workgroups per CU (a context of several lanes)
    const int res = per_cu_cap > 0 && !per_cu_env ? std::min(resident, per_cu_cap * n_cus) : resident;
    dim3 grid(clampi(ntiles, 1, res / n_frames > 0 ? res / n_frames : 1), n_frames);
    hipLaunchKernelGGL((k_front<HR, VR, S, front_wpe<HR, VR, S>()>), grid, dim3(256), 0, st, (const S*)rgb, stride_elems, g, w.norm_lut,
                       w.qtab, w.coef, w.status);
}

hipError_t launch_front(const void* rgb, size_t frame_stride_bytes, int sample_bytes, int n_frames, const Geom& g,
                        const Work& w, hipStream_t st, int per_cu_cap) {
    const size_t se = frame_stride_bytes / (size_t)sample_bytes;
    if (sample_bytes == 4) {
        if (g.hr == 1)
            front_impl<1, 1, float>(rgb, se, n_frames, g, w, st, per_cu_cap);
        else if (g.vr == 1)
            front_impl<2, 1, float>(rgb, se, n_frames, g, w, st, per_cu_cap);
        else
            front_impl<2, 2, float>(rgb, se, n_frames, g, w, st, per_cu_cap);
    } else if (sample_bytes == 1) {
        if (g.hr == 1)
            front_impl<1, 1, uint8_t>(rgb, se, n_frames, g, w, st, per_cu_cap);
        else if (g.vr == 1)
            front_impl<2, 1, uint8_t>(rgb, se, n_frames, g, w, st, per_cu_cap);
        else
            front_impl<2, 2, uint8_t>(rgb, se, n_frames, g, w, st, per_cu_cap);
    } else {
        if (g.hr == 1)
            front_impl<1, 1, uint16_t>(rgb, se, n_frames, g, w, st, per_cu_cap);
        else if (g.vr == 1)
            front_impl<2, 1, uint16_t>(rgb, se, n_frames, g, w, st, per_cu_cap);
        else
            front_impl<2, 2, uint16_t>(rgb, se, n_frames, g, w, st, per_cu_cap);
    }
    return hipGetLastError();
}

// The fused tail counts in 32 bits: a frame's symbols (at most 64 per block) times
// the 15 levels a package can sum over stay below 2^30 (a key weight << 1 | tag
// stays below its merge's padding); stripes keep k_tables
// (their histograms are summed on the host first)
#ifndef DMMT_HIST_WG_CAP
#define DMMT_HIST_WG_CAP 1024  // k_hist workgroups per launch (study builds: other caps)
#endif
bool tables_fusable(const Geom& g) { return g.stripe_first && !g.more_after && g.bpf * 64 * 16 < (1ll << 30); }

hipError_t launch_hist(int n_frames, const Geom& g, const Work& w, int check_cat, hipStream_t st, bool fuse_tables,
                       int bits_per_channel, uint8_t* out, size_t out_stride, int wg_cap) {
    // at most 1024 workgroups (4K: 1.5 blocks per thread): fewer histogram
    // flushes; 4K q90 bench 157.5 -> 159.6 Gpx/s, 8K 4:2:0 296.6 -> 299.0 against
    // one block per thread.  512 is faster pipelined still but k_hist alone +4 us,
    // so a context of several lanes passes wg_cap = DMMT_HIST_WG_CAP_LANES (512:
    // settled 4-lane bench +2.4 %, profiles/r06_hist_cap_lanes_ab.txt) and one lane
    // keeps the default
    const int cap = wg_cap > 0 ? wg_cap : DMMT_HIST_WG_CAP;
    const int per_frame = cap / n_frames > 0 ? cap / n_frames : 1;
    dim3 grid(clampi((g.bpf + 255) / 256, 1, per_frame), n_frames);
    const bool fuse = fuse_tables && tables_fusable(g);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, (const int16_t*)w.coef, w.dcdiff, w.lastnz, g, w.ac_hist,
                           w.dc_hist, w.status, w.arrive, w.code_tab, out, out_stride, w.hdr_len, w.qtab_u8,
                           bits_per_channel);
    };
    if (check_cat)
        fuse ? go(k_hist<true, true>) : go(k_hist<true, false>);
    else
        fuse ? go(k_hist<false, true>) : go(k_hist<false, false>);
    return hipGetLastError();
}

hipError_t launch_tables(int n_frames, const Geom& g, const Work& w, int bits_per_channel, uint8_t* out,
                         size_t out_stride, hipStream_t st) {
    hipLaunchKernelGGL(k_tables, dim3(4, n_frames), dim3(512), 0, st, (const uint32_t*)w.ac_hist,
                       (const uint32_t*)w.dc_hist, w.code_tab, out, out_stride,
                       w.hdr_len, g, w.qtab_u8, bits_per_channel, w.status);
    return hipGetLastError();
}

hipError_t launch_dct_blocks(float* data, long long nblocks, hipStream_t st) {
    hipLaunchKernelGGL(k_dct_blocks, dim3(clampi((nblocks + 31) / 32, 1, 2048)), dim3(256), 0, st, data, nblocks);
    return hipGetLastError();
}

hipError_t launch_synthetic(uint8_t* rgb, int w, int h, int n_frames, int first_frame, uint32_t seed, int row0,
                            int rows, hipStream_t st) {
    const long long n = (long long)w * rows * n_frames;
    hipLaunchKernelGGL(k_synthetic, dim3(clampi((n + 255) / 256, 1, 8192)), dim3(256), 0, st, rgb, w, h, n_frames,
                       first_frame, seed, row0, rows);
    return hipGetLastError();
}

}  // namespace dmmt

#ifdef DMMT_PHASE_TRACE
// development builds only: copy out and clear this file's phase counters
extern "C" int dmmt_debug_trace_kernels(unsigned long long* out64) {
    if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(dmmt::g_trace), 64 * 8) != hipSuccess) return -1;
    unsigned long long z[64] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(dmmt::g_trace), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
