/*
 * cpu_ref -- CPU restatement of the SilverlightningY/dmmt-jpeg-encoder encode path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/, the smoke
 * check in __graft_entry__.py and bench.py's cpu_baseline leg may load it.  The
 * product (dmmt-jpeg-encoder_amd/) never links, loads or calls it.
 *
 * The reference is Rust and cannot be built in this image (no cargo/rustc), so
 * this is a stage-by-stage restatement in plain C, compiled with
 * -ffp-contract=off and no fast-math so every f32 operation rounds exactly as
 * the Rust code does.  It is pinned by the reference's own known-answer tests
 * and by the two reference-produced files in /root/reference/tests
 * (output_image_2.jpg: back half, output_image.jpg: front half of a flat
 * block); see tests/test_oracle_*.py and DESIGN.md "Oracle".
 */
#ifndef DMMT_CPU_REF_H
#define DMMT_CPU_REF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { REF_P444 = 0, REF_P422 = 1, REF_P420 = 2 };

enum {
    REF_OK = 0,
    REF_E_VALUE_EXCEEDS_MAX = -100, /* color.rs:63-65 panics */
    REF_E_CATEGORY_RANGE = -101,    /* categorize.rs:25-30 panics */
    REF_E_INVALID_ARGUMENT = -102,  /* empty image / padded size overflows u16 */
    REF_E_SYMBOL_MISSING = -103,    /* huffman/encoder.rs:33 table has 255 slots */
    REF_E_OOM = -104,
};

/* JpegTransformationOptions (jpeg.rs:31-39) with the table pair resolved
 * (quantization_tables.rs:286-327); tables are in natural (row-major) order. */
typedef struct {
    int preset;           /* REF_P444 / REF_P422 / REF_P420 */
    int bits_per_channel; /* written into SOF only (encoder.rs:235) */
    uint8_t luma_q[64];
    uint8_t chroma_q[64];
    int restart_interval; /* extension (not in the reference): DRI + RSTn every N MCUs, 0 = reference */
} ref_options;

/* ---- stage entry points (each cites the reference function it restates) ---- */
float ref_normalize(uint16_t value, uint16_t max);                    /* color.rs:45-53 */
void ref_rgb_to_ycbcr(float r, float g, float b, float out[3]);       /* color.rs:75-100 (Y, Cb, Cr) */
void ref_fast_arai(float* p, int stride);                             /* arai.rs:29-92 */
void ref_dct_block(float* block);                                     /* arai.rs:95-104 */
int16_t ref_quantize_value(float d, uint8_t q);                       /* quantizer.rs:60 */
int ref_category(int value);                                          /* categorize.rs:22-32 (-1 = panic) */
uint16_t ref_category_pattern(int value, int category);               /* categorize.rs:34-46, left aligned */
/* package-merge code lengths for ascending sorted frequencies (length_limited.rs:37-134);
 * returns 0 or -1 when the reference would panic (too many symbols) */
int ref_package_merge(const uint64_t* sorted_freq, int n, int limit, int* lengths);
/* Sorted (stable by frequency) symbol list + code lengths incl. the "+1" of
 * symbol_counting.rs:85-90.  hist[256] in, returns number of symbols. */
int ref_code_lengths(const uint64_t* hist, int nsym_max, uint8_t* symbols, int* lengths);
/* canonical codes of huffman/encoder.rs:45-67,116-119: codes[] right aligned */
void ref_assign_codes(const uint8_t* symbols, const int* lengths, int n, uint16_t* code, uint8_t* len);

/* Subsample + resort one padded plane into 8x8 block-contiguous order
 * (subsampling.rs:102-310 with the presets of 33-54).  out holds
 * (w/hr)*(h/vr) floats. */
void ref_subsample_resort(const float* plane, int w, int h, int hr, int vr, int average, int square, float* out);

/* ---- whole-path entry points ---- */
/* Front half: padded image -> quantized blocks, zigzag order, MCU emission order. */
int ref_forward(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt,
                int16_t** coef_zz, size_t* nblocks);
/* Back half: emission-order zigzag blocks -> complete JPEG file. */
int ref_encode_coefficients(const int16_t* coef_zz, size_t nblocks, int width, int height,
                            const ref_options* opt, uint8_t** out, size_t* out_len);
/* Whole encode: JpegImageWriter::write_image (jpeg.rs:64-75). */
int ref_encode(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt,
               uint8_t** out, size_t* out_len);
/* Same, with the Arai DCT stage fanned out over n_threads pthreads in 700-block
 * jobs, the reference's only parallel stage (transformer.rs:126-148). */
int ref_encode_mt(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt,
                  int n_threads, uint8_t** out, size_t* out_len);
/* the same results with every front-half stage split over n_threads (test speed only) */
int ref_forward_par(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt, int n_threads,
                    int16_t** coef_zz, size_t* nblocks);
int ref_encode_par(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt, int n_threads,
                   uint8_t** out, size_t* out_len);
void ref_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
