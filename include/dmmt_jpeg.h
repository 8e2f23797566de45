/*
 * dmmt_jpeg.h -- C ABI of the MI355X (gfx950) baseline-JPEG encode path.
 *
 * Drop-in boundary for SilverlightningY/dmmt-jpeg-encoder's encoder seam.  Every
 * entry point names the reference interface it replaces (paths relative to the
 * reference repository).  Plain C types only: no HIP, no torch types.  The
 * reference's Rust host would bind these through an `extern "C"` block; see
 * INTEGRATION.md for that binding.
 *
 * Return convention: 0 = OK, negative = error (dmmt_strerror).  Where the
 * reference panics (value above maxval, category > 15, empty image) these
 * functions return an error code instead; they never abort.
 *
 * Output bytes are identical to the reference CPU encoder's for the same image
 * and options (restart_interval == 0).
 */
#ifndef DMMT_JPEG_H
#define DMMT_JPEG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMMT_ABI_VERSION 1

/* ---- error codes: the reference's error::Error variants (error.rs:3-22), in order,
 *      then codes for states where the reference panics or that only a GPU has. */
enum dmmt_status {
    DMMT_OK = 0,
    DMMT_E_PPM_MISSING_TOKEN = -1,          /* PPMFileDoesNotContainRequiredToken */
    DMMT_E_PPM_PARSE_TOKEN = -2,            /* ParsingOfTokenFailed */
    DMMT_E_PPM_INCOMPLETE_PIXEL = -3,       /* IncompletePixelParsed */
    DMMT_E_PPM_SIZE_MISMATCH = -4,          /* MismatchOfSizeBetweenHeaderAndValues */
    DMMT_E_INPUT_NOT_FOUND = -5,            /* InputFileNotFound */
    DMMT_E_NO_READ_PERMISSION = -6,         /* NoReadPermissionForInputFile */
    DMMT_E_OPEN_INPUT = -7,                 /* UnableToOpenInputFileForReading */
    DMMT_E_OPEN_OUTPUT = -8,                /* UnableToOpenOutputFileForWriting */
    DMMT_E_WRITE_START_OF_FILE = -9,        /* FailedToWriteStartOfFile */
    DMMT_E_WRITE_HUFFMAN_TABLES = -10,      /* FailedToWriteHuffmanTables */
    DMMT_E_WRITE_END_OF_FILE = -11,         /* FailedToWriteEndOfFile */
    DMMT_E_WRITE_JFIF = -12,                /* FailedToWriteJfifApplicationHeader */
    DMMT_E_WRITE_QUANTIZATION_TABLE = -13,  /* FailedToWriteQuantizationTable */
    DMMT_E_WRITE_START_OF_FRAME = -14,      /* FailedToWriteStartOfFrame */
    DMMT_E_WRITE_START_OF_SCAN = -15,       /* FailedToWriteStartOfScan */
    DMMT_E_WRITE_IMAGE_DATA = -16,          /* FailedToWriteImageData */
    DMMT_E_HUFFMAN_SYMBOL_MISSING = -17,    /* HuffmanSymbolNotPresentInTranslator */
    DMMT_E_WRITE_BLOCK = -18,               /* FailedToWriteBlock */
    /* reference panics */
    DMMT_E_VALUE_EXCEEDS_MAX = -100,        /* color.rs:63-65 */
    DMMT_E_CATEGORY_RANGE = -101,           /* categorize.rs:25-30 */
    DMMT_E_INVALID_ARGUMENT = -102,         /* empty image, padded size > u16, bad option */
    /* device */
    DMMT_E_HIP = -200,                      /* a HIP runtime call failed */
    DMMT_E_OUT_OF_MEMORY = -201,
    DMMT_E_NO_DEVICE = -202,                /* no gfx950 device visible: there is no CPU fallback */
    DMMT_E_CAPACITY = -203,                 /* caller-provided device output buffer too small */
    DMMT_E_DEVICE_MISMATCH = -204           /* a context's pooled buffer is not on its GPU */
};

/* ChromaSubsamplingPreset (subsampling.rs:11-55) */
enum dmmt_subsampling { DMMT_P444 = 0, DMMT_P422 = 1, DMMT_P420 = 2 };

/* QuantizationTablePreset (quantization_tables.rs:232-327), in the reference's order */
enum dmmt_quant_preset {
    DMMT_Q_SPECIFICATION = 0,
    DMMT_Q_FLAT = 1,
    DMMT_Q_MSSIM_KODAK_TUNED = 2,
    DMMT_Q_PSNR_HVS_N_KODAK_TUNED = 3,
    DMMT_Q_DCTUNE_PERCEPTUAL_OPTIMIZATION = 4,
    DMMT_Q_A_VISUAL_DETECTION_MODEL = 5,
    DMMT_Q_AN_IMPROVED_DETECTION_MODEL = 6
};

/* Image<f32> (image.rs:7-11).  Either before normalisation -- the raw PPM samples
 * and maxval (ppm.rs:145-163), sample_bytes 1 (uint8) or 2 (uint16, host endian);
 * the library reproduces `v as f32 / max as f32` (color.rs:45-53) on the device and
 * reports a sample above maxval (color.rs:63-65) -- or exactly the reference's
 * Image<f32> dots: sample_bytes 4, float R,G,B already normalised (maxval unused),
 * the form JpegImageWriter (jpeg.rs:48-75) receives.  rgb is interleaved R,G,B,
 * row-major. */
typedef struct dmmt_image {
    uint16_t width;
    uint16_t height;
    uint16_t maxval;
    uint16_t sample_bytes;
    const void* rgb;
} dmmt_image;

/* JpegTransformationOptions (jpeg.rs:31-39) with the table pair resolved. */
typedef struct dmmt_options {
    int32_t subsampling;      /* dmmt_subsampling; cli.rs default P420 */
    int32_t bits_per_channel; /* 8/16/32, written into SOF only (encoder.rs:235) */
    uint8_t luma_q[64];       /* natural (row-major) order, 1..255 */
    uint8_t chroma_q[64];
    int32_t n_threads;        /* the reference's CPU thread count (cli.rs:104-109); unused on GPU */
    int32_t restart_interval; /* 0 = reference behaviour; >0 = DRI/RSTn every N MCUs (extension) */
} dmmt_options;

/* A batch of equally sized frames already resident in device memory (HBM). */
typedef struct dmmt_device_frames {
    const void* d_rgb;          /* n_frames frames, frame f at d_rgb + f * frame_stride */
    size_t frame_stride;        /* bytes between frames */
    int32_t n_frames;
    uint16_t width, height, maxval, sample_bytes; /* as dmmt_image */
    uint8_t* d_out;             /* JPEG f written at d_out + f * out_stride */
    size_t out_stride;          /* >= dmmt_max_jpeg_bytes(width, height, subsampling) */
    uint32_t* d_out_len;        /* device array [n_frames] of JPEG sizes */
} dmmt_device_frames;

typedef struct dmmt_ctx dmmt_ctx;

/* ---- context ---------------------------------------------------------------------- */
/* Replaces the ThreadPool the reference threads through convert_ppm_to_jpeg
 * (lib.rs:62) and JpegImageWriter::new (jpeg.rs:48-62): owns one GPU, its stream and
 * pooled device workspace.  Fails with DMMT_E_NO_DEVICE when no gfx950 GPU is visible. */
int dmmt_ctx_create(int device, dmmt_ctx** out);
void dmmt_ctx_destroy(dmmt_ctx* ctx);
int dmmt_device_count(int* count);
/* Waits for all work of the context (every lane, and caller streams the context's
 * device runs) and returns the first error of the asynchronous dmmt_encode_device
 * calls made since the last synchronize (then clears it).  The synchronous calls
 * report their own errors and never those of asynchronous ones. */
int dmmt_ctx_synchronize(dmmt_ctx* ctx);

/* ---- the encoder seam --------------------------------------------------------------- */
/* JpegImageWriter::write_image (jpeg.rs:64-75) = Transformer::transform
 * (transformer.rs:188-221) + Encoder::encode (encoder.rs:125-135), whole path on the
 * GPU.  *out is allocated by the library, free it with dmmt_free. */
int dmmt_jpeg_encode(dmmt_ctx* ctx, const dmmt_image* img, const dmmt_options* opt, uint8_t** out,
                     size_t* out_len);
/* Many independent images in as few launches as possible (images of equal size share
 * launches).  outs[i]/lens[i] as dmmt_jpeg_encode. */
int dmmt_jpeg_encode_batch(dmmt_ctx* ctx, const dmmt_image* imgs, int n, const dmmt_options* opt,
                           uint8_t** outs, size_t* lens);
/* Device-resident form: frames in HBM -> JPEG files in HBM, enqueued on `stream`
 * (a hipStream_t, NULL = the context's stream), no host synchronisation.  Errors the
 * kernels find (a sample above maxval, ...) are reported by dmmt_ctx_synchronize. */
int dmmt_encode_device(dmmt_ctx* ctx, const dmmt_device_frames* frames, const dmmt_options* opt, void* stream);
/* Pipelined device encodes (extension of the above; the reference encodes one image at a
 * time on the host): with n lanes (1..DMMT_MAX_LANES, default 1) a context keeps n
 * workspaces and streams, and consecutive dmmt_encode_device calls with stream NULL go
 * round-robin to them, so one call's latency-bound kernels (Huffman tables, offsets)
 * overlap the next calls' kernels.  Calls with stream NULL then run concurrently: their
 * inputs must be complete when the call is made, their outputs are complete after
 * dmmt_ctx_synchronize.  A non-NULL stream always uses lane 0's workspace: the call waits
 * (on the device) for the work already queued on lane 0, and later lane-0 work waits
 * for it. */
#define DMMT_MAX_LANES 8
int dmmt_ctx_set_lanes(dmmt_ctx* ctx, int n);
size_t dmmt_max_jpeg_bytes(uint16_t width, uint16_t height, int32_t subsampling);

/* ---- one image across several GPUs (extension) ---------------------------------------- */
/* A run of whole MCU rows of one image (BASELINE config 4): with a restart
 * interval (dmmt_options.restart_interval > 0) every stripe that starts and ends on an
 * interval boundary encodes independently once the Huffman tables -- global per image --
 * are known.  Protocol, one context per GPU:
 *   dmmt_stripe_analyze  front half + the stripe's symbol histograms (host, uint64)
 *   (exchange)           element-wise sum of every stripe's histograms
 *   dmmt_stripe_encode   tables from the sum, the stripe's bytes: the JFIF header if it is
 *                        the first stripe, its restart segments, then RSTm (more stripes
 *                        follow) or EOI (the image ends)
 * The stripes' outputs concatenated in row order are byte-identical to dmmt_jpeg_encode of
 * the whole image with the same restart interval.  Without restart intervals see
 * "joined stripes" below. */
typedef struct dmmt_stripe {
    const void* d_rgb;          /* device: the stripe's pixel rows only, interleaved R,G,B */
    uint16_t width, height;     /* the whole image */
    uint16_t maxval, sample_bytes;
    int32_t mcu_row0, mcu_rows; /* MCU rows [mcu_row0, mcu_row0 + mcu_rows) */
} dmmt_stripe;
#define DMMT_STRIPE_HIST_WORDS (2 * (16 + 256)) /* [luma DC][luma AC][chroma DC][chroma AC] */
int dmmt_stripe_analyze(dmmt_ctx* ctx, const dmmt_stripe* stripe, const dmmt_options* opt,
                        uint64_t hist[DMMT_STRIPE_HIST_WORDS]);
/* d_out: device buffer of out_cap >= dmmt_stripe_max_bytes bytes; *out_len (host) = bytes written */
int dmmt_stripe_encode(dmmt_ctx* ctx, const uint64_t hist_sum[DMMT_STRIPE_HIST_WORDS], uint8_t* d_out,
                       size_t out_cap, uint64_t* out_len);
size_t dmmt_stripe_max_bytes(const dmmt_stripe* stripe, const dmmt_options* opt);

/* Joined stripes: restart_interval 0, the reference's own stream (SURVEY.md 8(e)
 * "reference-exact mode").  Any MCU-row split works; stripe k's scan starts at
 * global bit B_k = bits of stripes 0..k-1, usually mid-byte.  Protocol:
 *   dmmt_stripe_analyze      as above; the stripe's first block per component is
 *                            counted with predictor 0
 *   dmmt_stripe_dc_edges     its first and last DC per component (Y, Cb, Cr)
 *   (exchange 1)             all-gather of the edges; rank k > 0 applies
 *   dmmt_stripe_fix_dc_hist  with stripe k-1's last DCs (categorize.rs:153-169
 *                            across the seam), then the histogram sum
 *   dmmt_stripe_measure      tables, the stripe's bits: its length and first 16 bits;
 *                            the first stripe's JFIF header goes into d_out
 *   (exchange 2)             all-gather of (bits, first16): B_k and the 16 bits of
 *                            the scan after stripe k (fewer where the scan ends)
 *   dmmt_stripe_write        the bytes whose first bit lies in the stripe (the byte
 *                            it shares with the next stripe included), stuffed; EOI
 *                            after the last stripe
 * The outputs concatenated in row order are byte-identical to dmmt_jpeg_encode of the
 * whole image (encoder.rs:125-135, 264-282). */
int dmmt_stripe_dc_edges(dmmt_ctx* ctx, int16_t first_dc[3], int16_t last_dc[3]);
void dmmt_stripe_fix_dc_hist(uint64_t hist[DMMT_STRIPE_HIST_WORDS], const int16_t first_dc[3],
                             const int16_t prev_last_dc[3]);
/* prev_last_dc: stripe k-1's last DCs (zeros for the first stripe); d_out as dmmt_stripe_encode */
int dmmt_stripe_measure(dmmt_ctx* ctx, const uint64_t hist_sum[DMMT_STRIPE_HIST_WORDS], const int16_t prev_last_dc[3],
                        uint8_t* d_out, size_t out_cap, uint64_t* bits, uint32_t* first16);
/* bit_offset: B_k; next16: the next_bits (<= 16) scan bits after the stripe, MSB-aligned */
int dmmt_stripe_write(dmmt_ctx* ctx, uint64_t bit_offset, uint32_t next_bits, uint32_t next16, uint64_t* out_len);

/* ---- several GPUs from one process (extension) ---------------------------------------------
 * The reference's only fan-out is a CPU thread pool: ThreadPool::new(n) (lib.rs:62) handed to
 * transform_on_threadpool (cosine_transform.rs:55-73) for the DCT.  A multi-GPU context is the
 * GPU counterpart: one member context per device id (ids may repeat: several contexts on one
 * GPU) and one host thread per member.  Every entry point accepts it:
 *   dmmt_jpeg_encode / dmmt_convert_ppm_to_jpeg   the image as MCU-row stripes, one per member,
 *                       the exchange of SURVEY.md 8(e) done on the host (no RCCL); the bytes
 *                       are identical to a single-GPU encode (restart_interval 0: the
 *                       reference's own stream, stripes joined mid-byte; > 0: stripes of whole
 *                       restart intervals)
 *   dmmt_jpeg_encode_batch   frames round-robin over the members, outputs in input order
 *   dmmt_ctx_synchronize / _set_lanes / _set_profiling / _profile   every member
 *   any other call (device memory, stage-level, stripe_* steps)      member 0
 * Device-resident work names the member explicitly (dmmt_encode_device_multi,
 * dmmt_encode_striped_device) or goes to a member context (dmmt_ctx_member).
 * Each call locks the contexts it uses for its own duration, but a stripe_* sequence
 * (analyze, measure, write) spans several calls: a group context -- and its members -- must not
 * run a stripe_* sequence on one thread while another thread runs a group encode on it (the
 * group's striped encodes use the members' stripe state).  Give concurrent work its own context.
 * Operation across distinct physical GPUs is built the same way but has only been tested with
 * repeated device ids on one GPU (no multi-GPU host was available). */
#define DMMT_MAX_GROUP 64
int dmmt_ctx_create_multi(const int* device_ids, int n, dmmt_ctx** out);
int dmmt_ctx_num_devices(const dmmt_ctx* ctx);       /* members (1 for dmmt_ctx_create contexts) */
dmmt_ctx* dmmt_ctx_member(dmmt_ctx* ctx, int i);     /* borrowed; a single-device context is its own member 0 */
/* one host image as MCU-row stripes over the members (n_stripes <= 0: all of them; at most one
 * per member; fewer where the image has fewer MCU rows or restart intervals) */
int dmmt_jpeg_encode_striped(dmmt_ctx* ctx, const dmmt_image* img, const dmmt_options* opt, int n_stripes,
                             uint8_t** out, size_t* out_len);
/* frames[i] in member i's HBM (n_frames 0: none), enqueued as dmmt_encode_device with a NULL stream */
int dmmt_encode_device_multi(dmmt_ctx* ctx, const dmmt_device_frames* frames, int n, const dmmt_options* opt);
/* stripes[i] in member i's HBM, in row order from MCU row 0; stripe i's bytes to d_outs[i]
 * (caps[i] >= dmmt_stripe_max_bytes), lens[i] = their count: concatenated, the JPEG file */
int dmmt_encode_striped_device(dmmt_ctx* ctx, const dmmt_stripe* stripes, int n, const dmmt_options* opt,
                               uint8_t* const* d_outs, const size_t* caps, uint64_t* lens);

/* ---- stage-level entry points (parity tests) ---------------------------------------- */
/* Front half only (transformer.rs:188-199): quantised zigzag blocks, MCU emission order
 * (block_fold_iterator.rs:53-148), 64 int16 per block, into coef (host). */
int dmmt_forward_blocks(dmmt_ctx* ctx, const dmmt_image* img, const dmmt_options* opt, int16_t* coef,
                        size_t cap_blocks, size_t* nblocks);
/* Back half only (transformer.rs:199-220 + encoder.rs:125-282): emission-order zigzag
 * blocks (host) -> JPEG file. */
int dmmt_encode_coefficients(dmmt_ctx* ctx, const int16_t* coef, size_t nblocks, uint16_t width,
                             uint16_t height, const dmmt_options* opt, uint8_t** out, size_t* out_len);
/* Discrete8x8CosineTransformer::transform_on_threadpool (cosine_transform.rs:55-73) with
 * the Arai transformer (arai.rs:95-104): in-place 2-D DCT of every 64-float block of a
 * host array, computed on the GPU.  len is the number of floats (multiple of 64). */
int dmmt_dct_transform(dmmt_ctx* ctx, float* blocks, size_t len);

/* ---- host helpers --------------------------------------------------------------------- */
/* QuantizationTablePreset::to_pair (quantization_tables.rs:286-327), natural order */
int dmmt_quantization_preset(int32_t preset, uint8_t luma[64], uint8_t chroma[64]);
/* Extension: IJG quality scaling of the Annex K tables (quality 1..100; 50 = Specification) */
int dmmt_quality_tables(int32_t quality, uint8_t luma[64], uint8_t chroma[64]);
void dmmt_default_options(dmmt_options* opt); /* cli.rs defaults: P420, 8 bit, Specification */
/* PPMImageReader::read_image (ppm.rs:19-25; P3 as the reference, plus binary P6).
 * Samples are returned raw (uint16) with their maxval; free img->rgb with dmmt_free. */
int dmmt_read_ppm(const char* path, dmmt_image* img);
int dmmt_parse_ppm(const uint8_t* data, size_t len, dmmt_image* img);
/* PPM ingest on the GPU.  The header (ppm.rs:145-222
 * parse_header .. parse_max_value) is read on the host from the file's first bytes;
 * body_offset is the first byte after the whitespace that ended the max value. */
typedef struct {
    uint16_t width, height, maxval;
    int32_t binary;       /* 0: P3, the reference's format; 1: P6 (extension) */
    uint64_t body_offset;
} dmmt_ppm_header;
int dmmt_parse_ppm_header(const uint8_t* data, size_t len, dmmt_ppm_header* hdr);
/* PPMParser::parse_all_dots + the checks after it (ppm.rs:165-175, 224-252; the
 * RangeColorFormat panic of color.rs:63-65 for P3) on the GPU: d_text holds the whole
 * file (len bytes, header included) in device memory; d_rgb receives width*height*3
 * samples, uint8 when maxval <= 255 else uint16 -- the same image dmmt_parse_ppm
 * returns, and the same error codes.  Enqueued on stream (NULL: the context's stream)
 * and synchronised before returning. */
int dmmt_decode_ppm_device(dmmt_ctx* ctx, const uint8_t* d_text, size_t len, const dmmt_ppm_header* hdr,
                           void* d_rgb, void* stream);
/* convert_ppm_to_jpeg (lib.rs:59-77): read the PPM file, decode its samples and encode
 * them on the GPU (dmmt_decode_ppm_device, then the encode path), write the file. */
int dmmt_convert_ppm_to_jpeg(dmmt_ctx* ctx, const char* input_path, const char* output_path,
                             const dmmt_options* opt);
/* Extension: convert_ppm_to_jpeg (lib.rs:59-77) for a stream of files already in device
 * memory.  File i: its whole text (header included, parsed beforehand with
 * dmmt_parse_ppm_header) -> its JPEG at d_out (out_capacity >= dmmt_max_jpeg_bytes(width,
 * height, opt->subsampling)), the JPEG's size in *d_out_len (device memory).  The files are
 * decoded and encoded back to back over the context's lanes (dmmt_ctx_set_lanes), with no
 * synchronisation between files: a P3 body is decoded on the comment-free path on the
 * assumption that it has no '#' and no error, and encoded at once; its report is checked
 * after the batch, and a file whose body needs the general path (a comment, a '+' sign,
 * an 8-bit sample written with leading zeros),
 * or that fails (its own decode report or its own encode's error words), is redone on its
 * own.  codes[i] receives file i's result: the code dmmt_decode_ppm_device and then the
 * encode would return for it (a failed file's size is 0).  Returns the first non-zero code,
 * DMMT_OK when every file succeeded; synchronised before returning.
 * dmmt_last_error_detail / dmmt_last_error_message: the payload of the file whose code is
 * returned (the first that failed). */
typedef struct {
    const uint8_t* d_text;   /* the whole file in device memory */
    size_t len;
    dmmt_ppm_header header;
    uint8_t* d_out;
    size_t out_capacity;
    uint32_t* d_out_len;     /* device */
} dmmt_ppm_file;
int dmmt_convert_ppm_device_batch(dmmt_ctx* ctx, const dmmt_ppm_file* files, int32_t n, const dmmt_options* opt,
                                  int32_t* codes);
/* Diagnostic: how many files the context's last dmmt_convert_ppm_device_batch redid on their
 * own (a '#' or '+' in the text, or a failure); -1 before the first batch. */
int dmmt_ctx_batch_redone(dmmt_ctx* ctx);
/* The payload the reference's Error variant carries (error.rs:3-22), for the last error a PPM
 * entry point (dmmt_parse_ppm, dmmt_read_ppm, dmmt_parse_ppm_header, dmmt_decode_ppm_device,
 * dmmt_convert_ppm_to_jpeg) returned on the calling thread: IncompletePixelParsed(n) -> n
 * (ppm.rs:239-245); PPMFileDoesNotContainRequiredToken / ParsingOfTokenFailed -> the token
 * (0 "P3 Header", 1 "Width Header", 2 "Height Header", 3 "Max Value Header", 4 "Color
 * Component Value", ppm.rs:80-84).  dmmt_last_error_message: the variant's Display text with
 * that payload (error.rs:25-60), "" when the last PPM call on this thread succeeded. */
int dmmt_last_error_detail(void);
const char* dmmt_last_error_message(void);
void dmmt_free(void* p);
const char* dmmt_strerror(int code);
/* name of the error variant as in error.rs ("MismatchOfSizeBetweenHeaderAndValues", ...) */
const char* dmmt_error_name(int code);

/* ---- measurement ---------------------------------------------------------------------- */
/* enable = 0 off, 1 every stage, otherwise a bitmask of stages (bit s = stage s).  While
 * on, every launch of a selected stage is bracketed by HIP events on the stream it is
 * launched on; dmmt_ctx_profile returns the summed milliseconds per stage (stage names
 * via dmmt_stage_name) and the number of recorded launches, and resets nothing. */
int dmmt_ctx_set_profiling(dmmt_ctx* ctx, int enable);
int dmmt_ctx_profile(dmmt_ctx* ctx, double* ms, int32_t* launches, int n_stages);
int dmmt_num_stages(void);
const char* dmmt_stage_name(int stage);
/* Multi-GPU readiness: every pooled device buffer of the context lies on the context's GPU
 * (hipPointerGetAttributes); for a multi-GPU context every member is checked on its own
 * host thread, with the group's pooled staging buffers.  Every allocation the library makes
 * (pooled buffers, dmmt_device_malloc) is checked once, when it is made, against the
 * device the context bound the thread to; the calls do not repeat the check.  *device (may
 * be NULL): the context's (first) device.  DMMT_E_DEVICE_MISMATCH on a mismatch. */
int dmmt_ctx_check_device(dmmt_ctx* ctx, int32_t* device);
/* device memory for callers without their own allocator (bench, tests) */
int dmmt_device_malloc(dmmt_ctx* ctx, size_t bytes, void** ptr);
int dmmt_device_free(dmmt_ctx* ctx, void* ptr);
int dmmt_memcpy_h2d(dmmt_ctx* ctx, void* dst, const void* src, size_t bytes);
int dmmt_memcpy_d2h(dmmt_ctx* ctx, void* dst, const void* src, size_t bytes);
/* synthetic frames (SURVEY.md 8(d) generator) written straight into device memory */
int dmmt_fill_synthetic(dmmt_ctx* ctx, void* d_rgb, uint16_t width, uint16_t height, int32_t n_frames,
                        int32_t first_frame, uint32_t seed);
/* rows [row0, row0 + rows) of synthetic frame `frame` of a width x height image (a stripe) */
int dmmt_fill_synthetic_rows(dmmt_ctx* ctx, void* d_rgb, uint16_t width, uint16_t height, int32_t row0,
                             int32_t rows, int32_t frame, uint32_t seed);
const char* dmmt_build_info(void);

#ifdef __cplusplus
}
#endif
#endif
