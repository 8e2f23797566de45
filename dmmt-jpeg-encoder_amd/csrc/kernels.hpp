// kernels.hpp -- host-side launchers of the gfx950 kernels (kernels.hip, entropy.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jpeg_common.hpp"

namespace dmmt {

// Device workspace of one launch batch (see the kernels for each buffer's role).
struct Work {
    int16_t* coef;                  // [frames][bpf][64] zigzag, emission order
    int16_t* dcdiff;                // [frames][bpf]
    uint8_t* lastnz;                // [frames][bpf] zigzag position of the last non-zero AC (0: none)
    uint32_t* ac_hist;              // [frames][reps][2][256], zero between launches
    uint32_t* dc_hist;              // [frames][reps][2][16], zero between launches
    uint32_t* code_tab;             // [frames][4][256]  (len << 16) | code
    uint32_t* hdr_len;              // [frames]
    uint32_t* stage;                // [frames][nch][kChunkWordsCap] each chunk's own bit stream, MSB first
    uint32_t* chunk_bits;           // [frames][nch] bits of the chunk
    uint32_t* chunk_ff;             // [frames][nch][8] 0xFF bytes inside the chunk per alignment residue
    unsigned long long* chunk_ff8;  // [frames * nch + 2] the same eight counts one byte each (255: take chunk_ff's)
    uint32_t* chunk_edge;           // [frames][nch] first 16 bits << 16 | last 16 bits
    unsigned long long* chunk_bit0; // [frames][nch] bit offset of the chunk in its restart segment
    unsigned long long* chunk_out;  // [frames][nch] offset of the chunk's output bytes after the header
    unsigned long long* total_out;  // [frames] stuffed scan bytes incl. RST markers
    uint32_t* arrive;               // [frames][kArriveFrameWords] k_emit's finished workgroups (fused offsets), zero between launches
    int* status;                    // error words (raise_status): bit k of the error kinds -> word k; 1 value>max, 2 table, 4 category range, 16 output capacity
    const float* norm_lut;          // maxval-normalisation table
    const float* qtab;              // [2][64] f32
    const uint8_t* qtab_u8;         // [2][64] natural order, then [2][64] zigzag (the DQT bytes)
};

enum Stage { ST_FRONT = 0, ST_HIST, ST_TABLES, ST_EMIT, ST_OFFSETS, ST_STUFFWRITE, ST_COUNT };

// per_cu_cap: at most this many resident k_front workgroups per CU (0: as many as
// fit, 4); a context of several lanes passes DMMT_FRONT_PER_CU_LANES
hipError_t launch_front(const void* rgb, size_t frame_stride_bytes, int sample_bytes, int n_frames, const Geom& g,
                        const Work& w, hipStream_t st, int per_cu_cap = 0);
#ifndef DMMT_FRONT_PER_CU_LANES
#define DMMT_FRONT_PER_CU_LANES 2  // k_front workgroups per CU with several lanes (profiles/r06_front_per_cu_lanes_ab.txt)
#endif
// DC differences, AC and DC histograms, last non-zero positions of the blocks in
// w.coef (check_cat: an AC -32768, which has no category, can occur)
// fuse_tables: when tables_fusable(g), the frame's last k_hist workgroup also does
// launch_tables' work (code tables, header into out), and no launch_tables follows
bool tables_fusable(const Geom& g);
// wg_cap: at most this many workgroups per launch (0: the default, DMMT_HIST_WG_CAP)
hipError_t launch_hist(int n_frames, const Geom& g, const Work& w, int check_cat, hipStream_t st,
                       bool fuse_tables = false, int bits_per_channel = 8, uint8_t* out = nullptr,
                       size_t out_stride = 0, int wg_cap = 0);
#ifndef DMMT_HIST_WG_CAP_LANES
#define DMMT_HIST_WG_CAP_LANES 512  // k_hist's cap when the context runs several lanes (profiles/r06_hist_cap_lanes_ab.txt)
#endif
hipError_t launch_tables(int n_frames, const Geom& g, const Work& w, int bits_per_channel, uint8_t* out,
                         size_t out_stride, hipStream_t st);
// fuse_offsets: when offsets_fusable(g), k_emit's last workgroup per frame also
// computes the chunk offsets (chunk_bit0, chunk_out, total_out), and no
// launch_offsets is needed; otherwise launch_offsets follows as before
constexpr int kFusedRoundChunks = 1536;       // per round of the fused scan (4K 4:4:4: 1519 chunks, one round)
constexpr int kFusedOffsetsMaxChunks = 4 * kFusedRoundChunks;  // (8K 4:2:0: 3038 chunks, two rounds)
constexpr int kArriveFrameWords = 65 * 32;  // k_emit's arrival counters per frame (Work::arrive)
bool offsets_fusable(const Geom& g);
// prio: k_emit's heavier waves raise their issue priority (a context of one lane:
// shorter frames; with several lanes it costs the others' kernels issue slots)
hipError_t launch_emit(int n_frames, const Geom& g, const Work& w, bool fuse_offsets, hipStream_t st, bool prio);
hipError_t launch_offsets(int n_frames, const Geom& g, const Work& w, hipStream_t st);
hipError_t launch_stuffwrite(int n_frames, const Geom& g, const Work& w, uint8_t* out, size_t out_stride,
                             uint32_t* out_len, hipStream_t st);
// P3 body decoding (ppm_device.hip): text [body_offset, len) -> nsamples samples of
// sample_bytes each.  The comment-free path (when ppm_fast_path) runs first and
// writes its report into host-mapped memory (24 bytes, zeroed by the caller before
// the launch: u32 '#' seen, u32 parse error, u32 sample above maxval, u32, u64 tokens
// found); counts: 4 ppm_counts_capacity(n) bytes, row_base 8 * 1024 bytes.  If it
// saw a '#', the general path redoes the body: misc (device, 24 bytes: u32 status
// (1 parse error, 2 sample above maxval), u32, u64 tokens found), maps and chunk_in
// 8 max(n, 1024) bytes each (n = ppm_chunk_count(...)).
size_t ppm_chunk_count(const uint8_t* text, size_t body_offset, size_t len);
size_t ppm_counts_capacity(long long nch);
constexpr size_t kPpmReportBytes = 32;  // one comment-free report (24 bytes used)
bool ppm_fast_path(const uint8_t* text, size_t body_offset, size_t len);
hipError_t launch_ppm_p3_fast(const uint8_t* text, size_t body_offset, size_t len, uint32_t* counts,
                              unsigned long long* row_base, void* report, void* out, int sample_bytes,
                              unsigned long long nsamples, uint32_t maxval, hipStream_t st);
hipError_t launch_ppm_p3_general(const uint8_t* text, size_t body_offset, size_t len, unsigned long long* maps,
                                 unsigned long long* chunk_in, void* misc, void* out, int sample_bytes,
                                 unsigned long long nsamples, uint32_t maxval, hipStream_t st);
// P6 samples (big-endian u16 or u8) already in device memory -> host-endian samples
// (maxval and status unused: the encoder checks the range, as for dmmt_parse_ppm)
hipError_t launch_ppm_p6(const uint8_t* samples, void* out, int sample_bytes, unsigned long long nsamples,
                         uint32_t maxval, uint32_t* status, hipStream_t st);
hipError_t launch_dct_blocks(float* data, long long nblocks, hipStream_t st);
hipError_t launch_synthetic(uint8_t* rgb, int w, int h, int n_frames, int first_frame, uint32_t seed, int row0,
                            int rows, hipStream_t st);

}  // namespace dmmt
