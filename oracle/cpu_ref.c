/*
 * cpu_ref.c -- CPU restatement of the reference encode path (TEST INFRASTRUCTURE).
 *
 * Header comment of cpu_ref.h applies.  Build: oracle/Makefile, always with
 * -ffp-contract=off and without fast-math (Rust never contracts a*b+c).
 * Every function names the reference file:line it restates; paths are relative
 * to the reference repository root.
 */
#include "cpu_ref.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ color */

/* color.rs:45-53: `value.red as f32 / value.max as f32` */
float ref_normalize(uint16_t value, uint16_t max) { return (float)value / (float)max; }

/* color.rs:75-100.  Evaluation order is the Rust expression order:
 * ((wr + wg) + wb) - 128/255, then * 255.  No clamping. */
void ref_rgb_to_ycbcr(float r, float g, float b, float out[3]) {
    const float k128 = 128.0f / 255.0f; /* `128_f32 / 255_f32`, f32 division */
    float wr = r * 0.299f, wg = g * 0.587f, wb = b * 0.114f;
    out[0] = (((wr + wg) + wb) - k128) * 255.0f;
    wr = r * -0.1687f;
    wg = g * -0.3312f;
    wb = b * 0.5f;
    out[1] = ((wr + wg) + wb) * 255.0f;
    wr = r * 0.5f;
    wg = g * -0.4186f;
    wb = b * -0.0813f;
    out[2] = ((wr + wg) + wb) * 255.0f;
}

/* ------------------------------------------------------------- subsampling */

/* subsampling.rs:102-310.  ChannelRowView/ChannelColumnView walk the plane in
 * steps of (hr, vr); Skip takes the top-left sample (subsampling.rs:214),
 * Average sums Subsampler::rect (x outer, y inner, subsampling.rs:108-122) and
 * divides by the sample count (average(), 231-236).  The f32 `Sum` starts from
 * -0.0 (Rust >= 1.83) which is the identity, so the first sample starts the
 * chain.  ChannelSquareResorter (238-310) scatters into 8x8 block-contiguous
 * order: idx = (row/8)*(rowlen*8) + (col/8)*64 + (row%8)*8 + col%8. */
void ref_subsample_resort(const float* plane, int w, int h, int hr, int vr, int average, int square, float* out) {
    int sw = w / hr, sh = h / vr;
    for (int sy = 0; sy < sh; ++sy) {
        int row = sy * vr;
        for (int sx = 0; sx < sw; ++sx) {
            int col = sx * hr;
            float v;
            if (!average) {
                v = plane[(size_t)row * w + col];
            } else {
                int first = 1;
                float acc = 0.0f;
                for (int x = 0; x < hr; ++x) {
                    int cx = col + x;
                    if (cx > w - 1) cx = w - 1; /* cmp::min(last_column_index, ..) */
                    for (int y = 0; y < vr; ++y) {
                        int cy = row + y;
                        if (cy > h - 1) cy = h - 1;
                        float s = plane[(size_t)cy * w + cx];
                        if (first) {
                            acc = s;
                            first = 0;
                        } else {
                            acc = acc + s;
                        }
                    }
                }
                v = acc / (float)(hr * vr);
            }
            size_t sq = (size_t)square;
            size_t idx = (size_t)(sy / square) * ((size_t)sw * sq) + (size_t)(sx / square) * sq * sq +
                         (size_t)(sy % square) * sq + (size_t)(sx % square);
            out[idx] = v;
        }
    }
}

/* ---------------------------------------------------------------- DCT */

/* arai.rs:7-26, the f32 literals exactly as written there */
#define A1 0.70710678118654752440f /* FRAC_1_SQRT_2 */
#define A2 0.5411961f
#define A3 A1
#define A4 1.3065629f
#define A5 0.3826834f
#define S0 0.3535533f
#define S1 0.2548978f
#define S2 0.27059805f
#define S3 0.30067244f
#define S4 0.35355338f
#define S5 0.4499881f
#define S6 0.6532815f
#define S7 1.2814577f

/* arai.rs:29-92, one 8-point AAN butterfly in place with output scaling */
void ref_fast_arai(float* p, int stride) {
    float v00 = p[0], v01 = p[stride], v02 = p[2 * stride], v03 = p[3 * stride];
    float v04 = p[4 * stride], v05 = p[5 * stride], v06 = p[6 * stride], v07 = p[7 * stride];

    float v10 = v00 + v07, v11 = v01 + v06, v12 = v02 + v05, v13 = v03 + v04;
    float v14 = v03 - v04, v15 = v02 - v05, v16 = v01 - v06, v17 = v00 - v07;

    float v20 = v10 + v13, v21 = v11 + v12, v22 = v11 - v12, v23 = v10 - v13;
    float v24 = (-v14) - v15, v25 = v15 + v16, v26 = v16 + v17;

    float v30 = v20 + v21, v31 = v20 - v21, v32 = v22 + v23;

    float v42 = v32 * A1;
    float v44 = ((-v24) * A2) - ((v24 + v26) * A5);
    float v45 = v25 * A3;
    float v46 = (v26 * A4) - ((v26 + v24) * A5);

    float v52 = v42 + v23, v53 = v23 - v42, v55 = v45 + v17, v57 = v17 - v45;

    float v64 = v44 + v57, v65 = v55 + v46, v66 = v55 - v46, v67 = v57 - v44;

    p[0] = v30 * S0;
    p[4 * stride] = v31 * S4;
    p[2 * stride] = v52 * S2;
    p[6 * stride] = v53 * S6;
    p[5 * stride] = v64 * S5;
    p[1 * stride] = v65 * S1;
    p[7 * stride] = v66 * S7;
    p[3 * stride] = v67 * S3;
}

/* arai.rs:95-104: 8 row passes (stride 1) then 8 column passes (stride 8) */
void ref_dct_block(float* block) {
    for (int i = 0; i < 8; ++i) ref_fast_arai(block + 8 * i, 1);
    for (int i = 0; i < 8; ++i) ref_fast_arai(block + i, 8);
}

/* --------------------------------------------------------------- quantizer */

/* quantizer.rs:60: `(d / q as f32).round() as i16` -- round half away from
 * zero, then Rust's saturating float->int cast (NaN -> 0). */
int16_t ref_quantize_value(float d, uint8_t q) {
    float x = roundf(d / (float)q);
    if (x != x) return 0;
    if (x >= 32767.0f) return 32767;
    if (x <= -32768.0f) return -32768;
    return (int16_t)x;
}

/* frequency_block.rs:1-5 */
static const int ZIGZAG[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                               12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                               35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                               58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* ------------------------------------------------------------- categorize */

/* categorize.rs:22-32: category = 16 - leading_zeros(|v| as u16); > 15 panics */
int ref_category(int value) {
    unsigned a = (unsigned)(value < 0 ? -value : value) & 0xFFFFu;
    if (value == -32768) a = 32768u;
    int c = 0;
    while (a) {
        ++c;
        a >>= 1;
    }
    return c > 15 ? -1 : c;
}

/* categorize.rs:34-46: positive -> value, otherwise (1<<cat) - 1 - |value|,
 * left aligned in a u16 */
uint16_t ref_category_pattern(int value, int category) {
    if (category == 0) return 0; /* CategoryEncodedInteger::zero(), 48-53 */
    unsigned pat = value > 0 ? (unsigned)value : ((1u << category) - 1u - (unsigned)(-value));
    return (uint16_t)((pat << (16 - category)) & 0xFFFFu);
}

/* ---------------------------------------------------------- package-merge */

typedef struct {
    uint64_t freq;
    int kind; /* 0 = Leaf < 1 = Package (length_limited.rs:7-26, derived Ord) */
} pm_node;

static int pm_less(pm_node a, pm_node b) {
    return a.freq < b.freq || (a.freq == b.freq && a.kind < b.kind);
}

/* length_limited.rs:37-134.  Level 0 holds the leaves; level k is the sorted
 * union of pairwise packages of level k-1 (chunks_exact(2), odd tail dropped)
 * and the leaves (calculate_next_package, 82-86: BinaryHeap::into_sorted_vec,
 * equal keys are indistinguishable so a stable merge is identical).  The
 * solution walks the levels from the deepest with n-1 packages, takes the first
 * 2*packages nodes and counts leaves/packages (88-101, 108-134); symbol i gets
 * one bit per level whose leaf count exceeds i (62-72). */
int ref_package_merge(const uint64_t* sorted_freq, int n, int limit, int* lengths) {
    if (n <= 0) return -1; /* `code_length - 1` underflows: reference panics */
    if (limit < 31 && (uint64_t)n > (1ull << limit)) return -1; /* length_limited.rs:43-48 */
    pm_node** levels = (pm_node**)calloc((size_t)limit, sizeof(pm_node*));
    int* sizes = (int*)calloc((size_t)limit, sizeof(int));
    if (!levels || !sizes) return -1;
    levels[0] = (pm_node*)malloc(sizeof(pm_node) * (size_t)n);
    for (int i = 0; i < n; ++i) {
        levels[0][i].freq = sorted_freq[i];
        levels[0][i].kind = 0;
    }
    sizes[0] = n;
    for (int k = 1; k < limit; ++k) {
        int np = sizes[k - 1] / 2;
        int total = np + n;
        pm_node* out = (pm_node*)malloc(sizeof(pm_node) * (size_t)total);
        int i = 0, j = 0, o = 0;
        while (i < n || j < np) {
            pm_node pk;
            if (j < np) {
                pk.freq = levels[k - 1][2 * j].freq + levels[k - 1][2 * j + 1].freq;
                pk.kind = 1;
            }
            if (j >= np || (i < n && !pm_less(pk, levels[0][i]))) {
                out[o++] = levels[0][i++];
            } else {
                out[o++] = pk;
                ++j;
            }
        }
        levels[k] = out;
        sizes[k] = total;
    }
    for (int i = 0; i < n; ++i) lengths[i] = 0;
    size_t packages = (size_t)(n - 1);
    int rc = 0;
    for (int k = limit - 1; k >= 0; --k) {
        size_t count = packages * 2;
        if (count > (size_t)sizes[k]) { /* slice out of range: reference panics */
            rc = -1;
            break;
        }
        size_t leafs = 0, pk = 0;
        for (size_t t = 0; t < count; ++t) {
            if (levels[k][t].kind == 0)
                ++leafs;
            else
                ++pk;
        }
        for (size_t t = 0; t < leafs; ++t) lengths[t] += 1;
        packages = pk;
    }
    for (int k = 0; k < limit; ++k) free(levels[k]);
    free(levels);
    free(sizes);
    return rc;
}

/* symbol_counting.rs:25-32 (filter f > 0 in symbol order), 92-94 (stable sort
 * by frequency), 85-90 (package-merge with limit 15, then lengths[0] += 1). */
int ref_code_lengths(const uint64_t* hist, int nsym_max, uint8_t* symbols, int* lengths) {
    int n = 0;
    for (int s = 0; s < nsym_max; ++s)
        if (hist[s] > 0) symbols[n++] = (uint8_t)s;
    /* stable insertion sort by frequency */
    for (int i = 1; i < n; ++i) {
        uint8_t s = symbols[i];
        int j = i - 1;
        while (j >= 0 && hist[symbols[j]] > hist[s]) {
            symbols[j + 1] = symbols[j];
            --j;
        }
        symbols[j + 1] = s;
    }
    if (n == 0) return 0;
    uint64_t freq[256];
    for (int i = 0; i < n; ++i) freq[i] = hist[symbols[i]];
    if (ref_package_merge(freq, n, 15, lengths) != 0) return -1;
    lengths[0] += 1;
    return n;
}

/* huffman/encoder.rs:45-67,109-119: the last (most frequent) symbol gets code 0;
 * walking backwards each next code is previous + (1 << (16 - previous length))
 * in a left-aligned u16.  Returned right aligned. */
void ref_assign_codes(const uint8_t* symbols, const int* lengths, int n, uint16_t* code, uint8_t* len) {
    uint16_t prev_pat = 0;
    int prev_len = 0;
    for (int idx = n - 1; idx >= 0; --idx) {
        uint16_t pat;
        if (idx == n - 1)
            pat = 0;
        else
            pat = (uint16_t)(prev_pat + (uint16_t)(1u << (16 - prev_len)));
        int l = lengths[idx];
        code[symbols[idx]] = (uint16_t)(l ? (pat >> (16 - l)) : 0);
        len[symbols[idx]] = (uint8_t)l;
        prev_pat = pat;
        prev_len = l;
    }
}

/* ------------------------------------------------------------------ output */

typedef struct {
    uint8_t* data;
    size_t len, cap;
    int oom;
} bytebuf;

static void bb_put(bytebuf* b, uint8_t v) {
    if (b->len == b->cap) {
        size_t nc = b->cap ? b->cap * 2 : 4096;
        uint8_t* nd = (uint8_t*)realloc(b->data, nc);
        if (!nd) {
            b->oom = 1;
            return;
        }
        b->data = nd;
        b->cap = nc;
    }
    b->data[b->len++] = v;
}

/* segment_marker_injector.rs:13-30: every 0xFF is followed by 0x00 */
static void stuffed_put(bytebuf* b, uint8_t v) {
    bb_put(b, v);
    if (v == 0xFF) bb_put(b, 0x00);
}

/* binary_stream.rs:38-66 MSB-first, 89-96 flush; init 0xFF = pad with ones */
typedef struct {
    bytebuf* out;
    uint8_t buffer;
    int used;
} bitwriter;

static void bw_bits(bitwriter* w, unsigned value, int count) {
    for (int i = count - 1; i >= 0; --i) {
        int bit = (value >> i) & 1;
        if (bit)
            w->buffer |= (uint8_t)(0x80u >> w->used);
        else
            w->buffer &= (uint8_t)~(0x80u >> w->used);
        if (++w->used == 8) {
            stuffed_put(w->out, w->buffer);
            w->used = 0;
            w->buffer = 0xFF;
        }
    }
}

static void bw_flush(bitwriter* w) {
    if (w->used) {
        stuffed_put(w->out, w->buffer);
        w->used = 0;
        w->buffer = 0xFF;
    }
}

static void put_segment(bytebuf* b, uint8_t m1, uint8_t m2, const uint8_t* content, size_t n) {
    /* encoder.rs:137-153: length = marker bytes (2) + content */
    size_t seglen = 2 + n;
    bb_put(b, m1);
    bb_put(b, m2);
    bb_put(b, (uint8_t)(seglen >> 8));
    bb_put(b, (uint8_t)(seglen & 0xFF));
    for (size_t i = 0; i < n; ++i) bb_put(b, content[i]);
}

static void put_dht(bytebuf* b, uint8_t kind, const uint8_t* symbols, const int* lengths, int n) {
    /* encoder.rs:92-98,169-181: class/id byte, BITS[16], symbols reversed */
    uint8_t content[1 + 16 + 256];
    memset(content, 0, sizeof content);
    content[0] = kind;
    for (int i = 0; i < n; ++i) content[1 + lengths[i] - 1] += 1;
    for (int i = 0; i < n; ++i) content[17 + i] = symbols[n - 1 - i];
    put_segment(b, 0xFF, 0xC4, content, (size_t)(17 + n));
}

static void block_layout(int preset, int* n_luma) {
    *n_luma = preset == REF_P444 ? 1 : (preset == REF_P422 ? 2 : 4);
}

/* Back half.  Blocks arrive in MCU emission order (block_fold_iterator.rs:53-148):
 * per MCU n_luma Y blocks, then Cb, then Cr. */
int ref_encode_coefficients(const int16_t* coef_zz, size_t nblocks, int width, int height,
                            const ref_options* opt, uint8_t** out, size_t* out_len) {
    int n_luma;
    block_layout(opt->preset, &n_luma);
    int bpm = n_luma + 2;
    if (nblocks == 0 || nblocks % (size_t)bpm) return REF_E_INVALID_ARGUMENT;

    /* categorize_channel (categorize.rs:153-169) per component, DC predictor
     * per component; symbol histograms (symbol_counting.rs:55-74):
     * luma = Y blocks, chroma = Cb blocks then Cr blocks (transformer.rs:201-207). */
    uint64_t hist[4][256]; /* 0 luma DC, 1 luma AC, 2 chroma DC, 3 chroma AC */
    memset(hist, 0, sizeof hist);
    int16_t* dcdiff = (int16_t*)malloc(sizeof(int16_t) * nblocks);
    if (!dcdiff) return REF_E_OOM;
    const int ri = opt->restart_interval > 0 ? opt->restart_interval : 0;
    int last_dc[3] = {0, 0, 0};
    for (size_t e = 0; e < nblocks; ++e) {
        int k = (int)(e % (size_t)bpm);
        if (ri && k == 0 && (e / (size_t)bpm) % (size_t)ri == 0) /* extension: predictors reset per interval */
            last_dc[0] = last_dc[1] = last_dc[2] = 0;
        int comp = k < n_luma ? 0 : (k == n_luma ? 1 : 2);
        const int16_t* blk = coef_zz + e * 64;
        int16_t diff = (int16_t)(blk[0] - last_dc[comp]); /* i16 subtraction */
        last_dc[comp] = blk[0];
        dcdiff[e] = diff;
        int cat = ref_category(diff);
        if (cat < 0) {
            free(dcdiff);
            return REF_E_CATEGORY_RANGE;
        }
        int t = comp == 0 ? 0 : 2;
        hist[t][cat] += 1;
        /* sum_zeros_before_values, categorize.rs:132-151 */
        int zeros = 0;
        for (int i = 1; i < 64; ++i) {
            int v = blk[i];
            if (v == 0) {
                ++zeros;
            } else {
                while (zeros > 15) {
                    hist[t + 1][0xF0] += 1;
                    zeros -= 16;
                }
                int c = ref_category(v);
                if (c < 0) {
                    free(dcdiff);
                    return REF_E_CATEGORY_RANGE;
                }
                hist[t + 1][(zeros << 4) | c] += 1;
                zeros = 0;
            }
        }
        if (zeros) hist[t + 1][0x00] += 1;
    }

    uint8_t sym[4][256];
    int lens[4][256];
    int nsym[4];
    uint16_t code[4][256];
    uint8_t clen[4][256];
    memset(clen, 0, sizeof clen);
    for (int t = 0; t < 4; ++t) {
        nsym[t] = ref_code_lengths(hist[t], 256, sym[t], lens[t]);
        if (nsym[t] <= 0) {
            free(dcdiff);
            return REF_E_INVALID_ARGUMENT;
        }
        ref_assign_codes(sym[t], lens[t], nsym[t], code[t], clen[t]);
    }

    bytebuf b = {0};
    /* encoder.rs:125-135 */
    bb_put(&b, 0xFF);
    bb_put(&b, 0xD8);
    static const uint8_t app0[14] = {'J', 'F', 'I', 'F', 0, 0x01, 0x02, 0x00, 0x00, 0x48, 0x00, 0x48, 0, 0};
    put_segment(&b, 0xFF, 0xE0, app0, 14);
    for (int t = 0; t < 2; ++t) { /* encoder.rs:193-212: id, table in zigzag order */
        uint8_t dqt[65];
        const uint8_t* q = t == 0 ? opt->luma_q : opt->chroma_q;
        dqt[0] = (uint8_t)t;
        for (int i = 0; i < 64; ++i) dqt[1 + i] = q[ZIGZAG[i]];
        put_segment(&b, 0xFF, 0xDB, dqt, 65);
    }
    { /* encoder.rs:227-245 */
        int hr = opt->preset == REF_P444 ? 1 : 2, vr = opt->preset == REF_P420 ? 2 : 1;
        uint8_t sof[15] = {(uint8_t)opt->bits_per_channel,
                           (uint8_t)(height >> 8),
                           (uint8_t)height,
                           (uint8_t)(width >> 8),
                           (uint8_t)width,
                           0x03,
                           0x01,
                           (uint8_t)((hr << 4) | vr),
                           0x00,
                           0x02,
                           0x11,
                           0x01,
                           0x03,
                           0x11,
                           0x01};
        put_segment(&b, 0xFF, 0xC0, sof, 15);
    }
    /* encoder.rs:183-188: LumaAC 0x11, LumaDC 0x00, ChromaAC 0x13, ChromaDC 0x02 */
    put_dht(&b, 0x11, sym[1], lens[1], nsym[1]);
    put_dht(&b, 0x00, sym[0], lens[0], nsym[0]);
    put_dht(&b, 0x13, sym[3], lens[3], nsym[3]);
    put_dht(&b, 0x02, sym[2], lens[2], nsym[2]);
    if (ri) { /* extension: DRI (ITU T.81 B.2.4.4) */
        uint8_t dri[2] = {(uint8_t)(ri >> 8), (uint8_t)ri};
        put_segment(&b, 0xFF, 0xDD, dri, 2);
    }
    { /* encoder.rs:247-262 */
        static const uint8_t sos[10] = {0x03, 0x01, 0x01, 0x02, 0x23, 0x03, 0x23, 0x00, 0x3F, 0x00};
        put_segment(&b, 0xFF, 0xDA, sos, 10);
    }

    /* write_image_data, encoder.rs:264-282,356-404 */
    bitwriter w = {&b, 0xFF, 0};
    int rc = REF_OK;
    for (size_t e = 0; e < nblocks && rc == REF_OK; ++e) {
        int k = (int)(e % (size_t)bpm);
        int t = k < n_luma ? 0 : 2;
        const int16_t* blk = coef_zz + e * 64;
        if (ri && k == 0 && e > 0 && (e / (size_t)bpm) % (size_t)ri == 0) {
            /* extension: end of a restart interval -- 1-padding to a byte boundary
             * (the pad byte stuffed like any other), then RSTm, m = interval index mod 8,
             * which is not stuffed (ITU T.81 F.1.2.3) */
            bw_flush(&w);
            bb_put(&b, 0xFF);
            bb_put(&b, (uint8_t)(0xD0 + ((e / (size_t)bpm / (size_t)ri - 1) & 7)));
        }
        int diff = dcdiff[e];
        int cat = ref_category(diff);
        if (clen[t][cat] == 0) {
            rc = REF_E_SYMBOL_MISSING;
            break;
        }
        bw_bits(&w, code[t][cat], clen[t][cat]);
        bw_bits(&w, (unsigned)ref_category_pattern(diff, cat) >> (16 - cat), cat);
        int zeros = 0;
        for (int i = 1; i < 64; ++i) {
            int v = blk[i];
            if (v == 0) {
                ++zeros;
                continue;
            }
            while (zeros > 15) {
                bw_bits(&w, code[t + 1][0xF0], clen[t + 1][0xF0]);
                zeros -= 16;
            }
            int c = ref_category(v);
            int s = (zeros << 4) | c;
            if (s == 0xFF) { /* lookup table has Symbol::MAX (255) slots */
                rc = REF_E_SYMBOL_MISSING;
                break;
            }
            bw_bits(&w, code[t + 1][s], clen[t + 1][s]);
            bw_bits(&w, (unsigned)ref_category_pattern(v, c) >> (16 - c), c);
            zeros = 0;
        }
        if (zeros) bw_bits(&w, code[t + 1][0x00], clen[t + 1][0x00]);
    }
    free(dcdiff);
    if (rc != REF_OK) {
        free(b.data);
        return rc;
    }
    bw_flush(&w);
    bb_put(&b, 0xFF);
    bb_put(&b, 0xD9);
    if (b.oom) {
        free(b.data);
        return REF_E_OOM;
    }
    *out = b.data;
    *out_len = b.len;
    return REF_OK;
}

/* ------------------------------------------------------------ front half */

typedef struct {
    float* blocks;
    size_t first, count;
} dct_job;

static void* dct_worker(void* arg) {
    dct_job* j = (dct_job*)arg;
    for (size_t i = 0; i < j->count; ++i) ref_dct_block(j->blocks + (j->first + i) * 64);
    return NULL;
}

/* Transformer::transform (transformer.rs:188-221) up to the quantised,
 * entangled blocks, then MCU interleave (block_fold_iterator.rs). */
static int ref_forward_impl(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt,
                            int n_threads, int16_t** coef_zz, size_t* nblocks) {
    int hr = opt->preset == REF_P444 ? 1 : 2, vr = opt->preset == REF_P420 ? 2 : 1;
    if (width <= 0 || height <= 0) return REF_E_INVALID_ARGUMENT;
    /* padder.rs:12-17 with multiples (8*hr, 8*vr) (transformer.rs:48-51), u16 */
    int wp = (width + 8 * hr - 1) / (8 * hr) * (8 * hr);
    int hp = (height + 8 * vr - 1) / (8 * vr) * (8 * vr);
    if (wp > 65535 || hp > 65535) return REF_E_INVALID_ARGUMENT;
    size_t npx = (size_t)wp * hp;

    float* planes = (float*)malloc(sizeof(float) * npx * 3);
    if (!planes) return REF_E_OOM;
    float* py = planes;
    float* pcb = planes + npx;
    float* pcr = planes + 2 * npx;
    /* ppm.rs:153-157 (RangeColorFormat::new panics above max, color.rs:63-65),
     * padder.rs:19-34 (black pad), color.rs:75-100, transformer.rs:65-85 */
    for (int y = 0; y < hp; ++y) {
        for (int x = 0; x < wp; ++x) {
            float r = 0.0f, g = 0.0f, b = 0.0f;
            if (x < width && y < height) {
                const uint16_t* px = rgb + ((size_t)y * width + x) * 3;
                if (px[0] > maxval || px[1] > maxval || px[2] > maxval) {
                    free(planes);
                    return REF_E_VALUE_EXCEEDS_MAX;
                }
                r = ref_normalize(px[0], (uint16_t)maxval);
                g = ref_normalize(px[1], (uint16_t)maxval);
                b = ref_normalize(px[2], (uint16_t)maxval);
            }
            float ycc[3];
            ref_rgb_to_ycbcr(r, g, b, ycc);
            size_t i = (size_t)y * wp + x;
            py[i] = ycc[0];
            pcb[i] = ycc[1];
            pcr[i] = ycc[2];
        }
    }
    /* transformer.rs:87-124 */
    size_t ny = npx, nc = npx / (size_t)(hr * vr);
    float* by = (float*)malloc(sizeof(float) * (ny + 2 * nc));
    if (!by) {
        free(planes);
        return REF_E_OOM;
    }
    float* bcb = by + ny;
    float* bcr = bcb + nc;
    ref_subsample_resort(py, wp, hp, 1, 1, 0, 8, by);
    ref_subsample_resort(pcb, wp, hp, hr, vr, opt->preset != REF_P444, 8, bcb);
    ref_subsample_resort(pcr, wp, hp, hr, vr, opt->preset != REF_P444, 8, bcr);
    free(planes);

    /* transformer.rs:126-148: Arai DCT over all blocks (thread pool, 700-block jobs) */
    size_t total_blocks = (ny + 2 * nc) / 64;
    if (n_threads <= 1) {
        for (size_t i = 0; i < total_blocks; ++i) ref_dct_block(by + i * 64);
    } else {
        size_t njobs = (total_blocks + 699) / 700;
        dct_job* jobs = (dct_job*)malloc(sizeof(dct_job) * njobs);
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
        /* static round-robin of the 700-block jobs over n_threads workers */
        for (size_t j = 0; j < njobs; ++j) {
            jobs[j].blocks = by;
            jobs[j].first = j * 700;
            jobs[j].count = (j + 1) * 700 <= total_blocks ? 700 : total_blocks - j * 700;
        }
        for (size_t base = 0; base < njobs; base += (size_t)n_threads) {
            int launched = 0;
            for (int t = 0; t < n_threads && base + (size_t)t < njobs; ++t, ++launched)
                pthread_create(&th[t], NULL, dct_worker, &jobs[base + (size_t)t]);
            for (int t = 0; t < launched; ++t) pthread_join(th[t], NULL);
        }
        free(jobs);
        free(th);
    }

    /* quantizer.rs:53-62 (natural order table), block_entangler.rs:5-22,69-77,
     * block_fold_iterator.rs:53-148, zigzag frequency_block.rs:26-61 */
    int n_luma;
    block_layout(opt->preset, &n_luma);
    size_t nmcu = nc / 64;
    size_t nb = nmcu * (size_t)(n_luma + 2);
    int16_t* out = (int16_t*)malloc(sizeof(int16_t) * nb * 64);
    if (!out) {
        free(by);
        return REF_E_OOM;
    }
    size_t line = (size_t)wp / 8; /* luma blocks per block row */
    size_t cbx = (size_t)(wp / hr) / 8;
    size_t e = 0;
    for (size_t m = 0; m < nmcu; ++m) {
        size_t mx = m % cbx, my = m / cbx;
        size_t src[6];
        int ns = 0;
        if (opt->preset == REF_P444) {
            src[ns++] = m;
        } else if (opt->preset == REF_P422) {
            src[ns++] = my * line + 2 * mx;
            src[ns++] = my * line + 2 * mx + 1;
        } else {
            /* QuadFoldingIterator: TL, TR, BL, BR of a two-block-row strip */
            size_t r0 = 2 * my * line;
            src[ns++] = r0 + 2 * mx;
            src[ns++] = r0 + 2 * mx + 1;
            src[ns++] = r0 + line + 2 * mx;
            src[ns++] = r0 + line + 2 * mx + 1;
        }
        for (int s = 0; s < ns + 2; ++s) {
            const float* blk;
            const uint8_t* q;
            if (s < ns) {
                blk = by + src[s] * 64;
                q = opt->luma_q;
            } else {
                blk = (s == ns ? bcb : bcr) + m * 64;
                q = opt->chroma_q;
            }
            int16_t* o = out + e * 64;
            for (int i = 0; i < 64; ++i) o[i] = ref_quantize_value(blk[ZIGZAG[i]], q[ZIGZAG[i]]);
            ++e;
        }
    }
    free(by);
    *coef_zz = out;
    *nblocks = nb;
    return REF_OK;
}

/* ------------------------------------------------------------ parallel front half
 * The same stages as ref_forward_impl with every one of them split over threads
 * (rows of the colour conversion and of the subsampling, blocks of the DCT, MCUs of
 * quantisation).  Each output element is computed by exactly the function above,
 * so the result is identical to ref_forward; only the wall time differs.  It keeps
 * the parity tests of the BASELINE configs at their full size (32768^2, 1.07 Gpx)
 * within a few seconds of oracle time.  Not the CPU baseline (ref_encode_mt keeps
 * the reference's structure: only the DCT on the pool, transformer.rs:126-148). */
typedef struct {
    void (*fn)(void* ctx, size_t lo, size_t hi);
    void* ctx;
    size_t lo, hi;
} par_job;

static void* par_run(void* a) {
    par_job* j = (par_job*)a;
    j->fn(j->ctx, j->lo, j->hi);
    return NULL;
}

static void parallel_for(size_t n, int threads, void (*fn)(void*, size_t, size_t), void* ctx) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > n) threads = n ? (int)n : 1;
    par_job jobs[256];
    pthread_t th[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; ++t) {
        jobs[t].fn = fn;
        jobs[t].ctx = ctx;
        jobs[t].lo = n * (size_t)t / (size_t)threads;
        jobs[t].hi = n * (size_t)(t + 1) / (size_t)threads;
    }
    for (int t = 1; t < threads; ++t) pthread_create(&th[t], NULL, par_run, &jobs[t]);
    par_run(&jobs[0]);
    for (int t = 1; t < threads; ++t) pthread_join(th[t], NULL);
}

typedef struct {
    const uint16_t* rgb;
    int width, height, wp, maxval;
    float *py, *pcb, *pcr;
    volatile int bad;
} par_color;

static void par_color_rows(void* c_, size_t lo, size_t hi) {
    par_color* c = (par_color*)c_;
    for (size_t y = lo; y < hi; ++y) {
        for (int x = 0; x < c->wp; ++x) {
            float r = 0.0f, g = 0.0f, b = 0.0f;
            if (x < c->width && (int)y < c->height) {
                const uint16_t* px = c->rgb + (y * (size_t)c->width + (size_t)x) * 3;
                if (px[0] > c->maxval || px[1] > c->maxval || px[2] > c->maxval) {
                    c->bad = 1;
                    return;
                }
                r = ref_normalize(px[0], (uint16_t)c->maxval);
                g = ref_normalize(px[1], (uint16_t)c->maxval);
                b = ref_normalize(px[2], (uint16_t)c->maxval);
            }
            float ycc[3];
            ref_rgb_to_ycbcr(r, g, b, ycc);
            size_t i = y * (size_t)c->wp + (size_t)x;
            c->py[i] = ycc[0];
            c->pcb[i] = ycc[1];
            c->pcr[i] = ycc[2];
        }
    }
}

/* the subsampling of plane rows in whole 8-row block rows: ref_subsample_resort of
 * a horizontal slab writes exactly the slab's part of the block-contiguous output */
typedef struct {
    const float* plane[3];
    float* out[3];
    int wp, hp, hr, vr, average;
} par_sub;

static void par_sub_rows(void* c_, size_t lo, size_t hi) {
    par_sub* c = (par_sub*)c_;
    for (size_t u = lo; u < hi; ++u) {  /* unit = (plane, block row of its output) */
        int p = (int)(u % 3);
        size_t br = u / 3;
        int hr = p ? c->hr : 1, vr = p ? c->vr : 1;
        int sw = c->wp / hr, sh = c->hp / vr;
        if ((int)br * 8 >= sh) continue;
        /* output rows [8 br, 8 br + 8) read plane rows [8 br vr, 8 (br + 1) vr) */
        const float* slab = c->plane[p] + (size_t)br * 8 * (size_t)vr * (size_t)c->wp;
        ref_subsample_resort(slab, c->wp, 8 * vr, hr, vr, p ? c->average : 0, 8,
                             c->out[p] + (size_t)br * 8 * (size_t)sw);
    }
}

typedef struct {
    float* blocks;
} par_dct;

static void par_dct_blocks(void* c_, size_t lo, size_t hi) {
    par_dct* c = (par_dct*)c_;
    for (size_t i = lo; i < hi; ++i) ref_dct_block(c->blocks + i * 64);
}

typedef struct {
    const float *by, *bcb, *bcr;
    const ref_options* opt;
    size_t line, cbx;
    int n_luma;
    int16_t* out;
} par_quant;

static void par_quant_mcus(void* c_, size_t lo, size_t hi) {
    par_quant* c = (par_quant*)c_;
    const int bpm = c->n_luma + 2;
    for (size_t m = lo; m < hi; ++m) {
        size_t mx = m % c->cbx, my = m / c->cbx;
        size_t src[4];
        int ns = 0;
        if (c->opt->preset == REF_P444) {
            src[ns++] = m;
        } else if (c->opt->preset == REF_P422) {
            src[ns++] = my * c->line + 2 * mx;
            src[ns++] = my * c->line + 2 * mx + 1;
        } else {
            size_t r0 = 2 * my * c->line;
            src[ns++] = r0 + 2 * mx;
            src[ns++] = r0 + 2 * mx + 1;
            src[ns++] = r0 + c->line + 2 * mx;
            src[ns++] = r0 + c->line + 2 * mx + 1;
        }
        for (int s = 0; s < ns + 2; ++s) {
            const float* blk = s < ns ? c->by + src[s] * 64 : (s == ns ? c->bcb : c->bcr) + m * 64;
            const uint8_t* q = s < ns ? c->opt->luma_q : c->opt->chroma_q;
            int16_t* o = c->out + (m * (size_t)bpm + (size_t)s) * 64;
            for (int i = 0; i < 64; ++i) o[i] = ref_quantize_value(blk[ZIGZAG[i]], q[ZIGZAG[i]]);
        }
    }
}

int ref_forward_par(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt, int n_threads,
                    int16_t** coef_zz, size_t* nblocks) {
    int hr = opt->preset == REF_P444 ? 1 : 2, vr = opt->preset == REF_P420 ? 2 : 1;
    if (width <= 0 || height <= 0) return REF_E_INVALID_ARGUMENT;
    int wp = (width + 8 * hr - 1) / (8 * hr) * (8 * hr);
    int hp = (height + 8 * vr - 1) / (8 * vr) * (8 * vr);
    if (wp > 65535 || hp > 65535) return REF_E_INVALID_ARGUMENT;
    size_t npx = (size_t)wp * hp;
    float* planes = (float*)malloc(sizeof(float) * npx * 3);
    if (!planes) return REF_E_OOM;
    par_color pc = {rgb, width, height, wp, maxval, planes, planes + npx, planes + 2 * npx, 0};
    parallel_for((size_t)hp, n_threads, par_color_rows, &pc);
    if (pc.bad) {
        free(planes);
        return REF_E_VALUE_EXCEEDS_MAX;
    }
    size_t ny = npx, nc = npx / (size_t)(hr * vr);
    float* by = (float*)malloc(sizeof(float) * (ny + 2 * nc));
    if (!by) {
        free(planes);
        return REF_E_OOM;
    }
    par_sub ps = {{planes, planes + npx, planes + 2 * npx}, {by, by + ny, by + ny + nc}, wp, hp, hr, vr,
                  opt->preset != REF_P444};
    parallel_for((size_t)(hp / 8) * 3, n_threads, par_sub_rows, &ps);
    free(planes);
    par_dct pd = {by};
    parallel_for((ny + 2 * nc) / 64, n_threads, par_dct_blocks, &pd);
    int n_luma;
    block_layout(opt->preset, &n_luma);
    size_t nmcu = nc / 64;
    size_t nb = nmcu * (size_t)(n_luma + 2);
    int16_t* out = (int16_t*)malloc(sizeof(int16_t) * nb * 64);
    if (!out) {
        free(by);
        return REF_E_OOM;
    }
    par_quant pq = {by, by + ny, by + ny + nc, opt, (size_t)wp / 8, (size_t)(wp / hr) / 8, n_luma, out};
    parallel_for(nmcu, n_threads, par_quant_mcus, &pq);
    free(by);
    *coef_zz = out;
    *nblocks = nb;
    return REF_OK;
}

int ref_encode_par(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt, int n_threads,
                   uint8_t** out, size_t* out_len) {
    int16_t* coef = NULL;
    size_t nb = 0;
    int rc = ref_forward_par(rgb, width, height, maxval, opt, n_threads, &coef, &nb);
    if (rc != REF_OK) return rc;
    rc = ref_encode_coefficients(coef, nb, width, height, opt, out, out_len);
    free(coef);
    return rc;
}

int ref_forward(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt,
                int16_t** coef_zz, size_t* nblocks) {
    return ref_forward_impl(rgb, width, height, maxval, opt, 1, coef_zz, nblocks);
}

static int encode_common(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt,
                         int n_threads, uint8_t** out, size_t* out_len) {
    int16_t* coef = NULL;
    size_t nb = 0;
    int rc = ref_forward_impl(rgb, width, height, maxval, opt, n_threads, &coef, &nb);
    if (rc != REF_OK) return rc;
    rc = ref_encode_coefficients(coef, nb, width, height, opt, out, out_len);
    free(coef);
    return rc;
}

int ref_encode(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt,
               uint8_t** out, size_t* out_len) {
    return encode_common(rgb, width, height, maxval, opt, 1, out, out_len);
}

int ref_encode_mt(const uint16_t* rgb, int width, int height, int maxval, const ref_options* opt,
                  int n_threads, uint8_t** out, size_t* out_len) {
    return encode_common(rgb, width, height, maxval, opt, n_threads, out, out_len);
}

void ref_free(void* p) { free(p); }
