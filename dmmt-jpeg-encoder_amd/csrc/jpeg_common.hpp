// jpeg_common.hpp -- constants and geometry shared by host and device code.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace dmmt {

// frequency_block.rs:1-5: natural index of zigzag position i
static constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Coefficient blocks in HBM are column-major in natural order (k_front stores one
// 8-coefficient column per lane, 16 bytes): zigzag position k of a block sits at
// index coef_pos(k) of its 64 int16.  The C ABI's blocks stay in zigzag order
// (frequency_block.rs), converted on the host.
constexpr int coef_pos(int k) { return (kZigzag[k] & 7) * 8 + (kZigzag[k] >> 3); }

// Histogram replicas per frame: the front/DC kernels add their per-workgroup
// histograms into replica (blockIdx.x % kHistReps) to spread atomic traffic.
static constexpr int kHistReps = 8;  // (measured: 16 and 4 replicas pipeline 1-2 % slower)
// Blocks per entropy chunk (k_emit / k_stuffwrite): one workgroup each.
#ifndef DMMT_CHUNK_BLOCKS
#define DMMT_CHUNK_BLOCKS 256
#endif
static constexpr int kChunkBlocks = DMMT_CHUNK_BLOCKS;
// Worst-case entropy-coded bits of one block: 64 tokens (the DC, then at most 63
// AC tokens -- a ZRL or the EOB stands for at least one zero) of code <= 16 +
// extra bits <= 15.  Integer samples keep |coef| <= 2049 (category <= 12), but
// Image<f32> dots and host blocks reach category 15 (categorize.rs:22-32).
static constexpr int kMaxBlockBits = 31 * 64;
// Staging words of one chunk's bit stream (worst case).
static constexpr long long kChunkWordsCap = (long long)kChunkBlocks * kMaxBlockBits / 32;
// Upper bound of the header the table kernel writes (SOI..SOS incl. DRI).
static constexpr int kMaxHeaderBytes = 2 + 18 + 2 * 69 + 19 + 4 * (4 + 17 + 256) + 6 + 14;

// Geometry of one frame (all frames of a launch share it).
struct Geom {
    int width, height;      // unpadded (SOF carries these, encoder.rs:231-240)
    int wp, hp;             // padded to (8*hr, 8*vr) multiples (transformer.rs:48-51)
    int hr, vr;             // chroma subsampling rates
    int n_luma, bpm;        // Y blocks per MCU, blocks per MCU
    int mcux, mcuy, nmcu;   // MCU grid
    int maxval;             // PPM max value
    int restart_interval;   // 0 = reference behaviour
    long long bpf;          // blocks per frame
    int nch;                // entropy chunks per frame (chunks never straddle a restart segment)
    int nseg;               // restart segments per frame (1 without restart intervals)
    int cps;                // chunks per full segment
    long long seg_blocks;   // blocks per full segment
    long long max_scan_bytes;  // worst-case entropy-coded bytes per frame (before stuffing)
    // MCU-row stripe of a larger image (dmmt_stripe_*; a whole frame otherwise)
    int sof_height;         // image height written into SOF
    int seg_base;           // global index of the first restart segment (RSTm numbering)
    int stripe_first;       // the stripe starts the image: write the header
    int more_after;         // more stripes follow: close with RSTm (restart mode) instead of EOI
    // joined stripes (no restart intervals, reference-exact): the stripe's scan
    // continues the previous stripe's mid-byte and runs on into the next one
    int bit_phase;          // global scan bit offset of the stripe's first bit, mod 8
    int next_bits;          // bits of the scan after the stripe known here (0..16)
    uint32_t next16;        // those bits, MSB-aligned in 16
};

inline Geom make_geom(int width, int height, int subsampling, int maxval, int restart_interval) {
    Geom g{};
    g.width = width;
    g.height = height;
    g.hr = subsampling == 0 ? 1 : 2;
    g.vr = subsampling == 2 ? 2 : 1;
    g.wp = (width + 8 * g.hr - 1) / (8 * g.hr) * (8 * g.hr);
    g.hp = (height + 8 * g.vr - 1) / (8 * g.vr) * (8 * g.vr);
    g.n_luma = g.hr * g.vr;
    g.bpm = g.n_luma + 2;
    g.mcux = g.wp / (8 * g.hr);
    g.mcuy = g.hp / (8 * g.vr);
    g.nmcu = g.mcux * g.mcuy;
    g.maxval = maxval;
    g.restart_interval = restart_interval;
    g.bpf = (long long)g.nmcu * g.bpm;
    // restart segments (extension): every restart_interval MCUs the scan restarts
    // byte-aligned; the chunk grid restarts with it
    g.nseg = restart_interval > 0 ? (g.nmcu + restart_interval - 1) / restart_interval : 1;
    g.seg_blocks = restart_interval > 0 ? (long long)restart_interval * g.bpm : g.bpf;
    g.cps = (int)((g.seg_blocks + kChunkBlocks - 1) / kChunkBlocks);
    const long long last_seg_blocks = g.bpf - (long long)(g.nseg - 1) * g.seg_blocks;
    g.nch = (g.nseg - 1) * g.cps + (int)((last_seg_blocks + kChunkBlocks - 1) / kChunkBlocks);
    g.max_scan_bytes = (g.bpf * kMaxBlockBits + 7) / 8;
    g.sof_height = height;
    g.seg_base = 0;
    g.stripe_first = 1;
    g.more_after = 0;
    g.bit_phase = 0;
    g.next_bits = 0;
    g.next16 = 0;
    return g;
}

// Worst-case JPEG size: header + every scan byte stuffed + per restart segment a
// stuffed pad byte and the RST marker + EOI.
inline size_t max_jpeg_bytes(const Geom& g) {
    return (size_t)kMaxHeaderBytes + (size_t)g.max_scan_bytes * 2 + 4 * (size_t)g.nmcu + 2 + 64;
}

// host: record the payload of a reference error variant for dmmt_last_error_detail /
// dmmt_last_error_message (ppm.cpp); returns code
int error_detail(int code, int detail);

}  // namespace dmmt
