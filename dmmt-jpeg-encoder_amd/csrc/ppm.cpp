// ppm.cpp -- PPMImageReader (ppm.rs:19-252): ASCII P3 exactly as the reference
// tokenises it, plus binary P6 (extension).  Host I/O, not part of the GPU path.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <string>
#include <vector>

#include "../../include/dmmt_jpeg.h"

namespace {

// Rust's char::is_ascii_whitespace: space, \t, \n, \x0C, \r (not \x0B)
inline bool is_ws(uint8_t b) { return b == ' ' || b == '\t' || b == '\n' || b == 0x0C || b == '\r'; }

// PPMTokenizer::next (ppm.rs:41-77).  A '#' comment runs to the next '\n',
// which is consumed without ending the current token (ppm.rs:50-55).
struct Tokenizer {
    const uint8_t* p;
    size_t n, i = 0;
    bool next(std::string& tok) {
        tok.clear();
        bool in_comment = false;
        while (i < n) {
            const uint8_t b = p[i++];
            if (in_comment) {
                if (b == '\n') in_comment = false;
                continue;
            }
            if (b == '#') {
                in_comment = true;
                continue;
            }
            if (is_ws(b)) {
                if (!tok.empty()) break;
            } else {
                tok.push_back((char)b);
            }
        }
        return !tok.empty();
    }
};

// `str::parse::<u16>()`: optional '+', decimal digits, no overflow
bool parse_u16(const std::string& t, uint16_t* out) {
    size_t k = 0;
    if (!t.empty() && t[0] == '+') k = 1;
    if (k >= t.size()) return false;
    uint32_t v = 0;
    for (; k < t.size(); ++k) {
        const char c = t[k];
        if (c < '0' || c > '9') return false;
        v = v * 10 + (uint32_t)(c - '0');
        if (v > 65535) return false;
    }
    *out = (uint16_t)v;
    return true;
}

}  // namespace

// The payload the reference's error::Error variants carry (error.rs:3-22), for the
// last error a PPM entry point returned on this thread: IncompletePixelParsed(n)
// carries n, the components of the unfinished pixel (ppm.rs:239-245);
// PPMFileDoesNotContainRequiredToken and ParsingOfTokenFailed the token's name
// (ppm.rs:80-84) -- here its index.
static thread_local int t_err_code = 0, t_err_detail = 0;
static const char* const kTokenNames[5] = {"P3 Header", "Width Header", "Height Header", "Max Value Header",
                                           "Color Component Value"};
enum { TOK_P3 = 0, TOK_WIDTH, TOK_HEIGHT, TOK_MAXVAL, TOK_COMPONENT };

namespace dmmt {
int error_detail(int code, int detail) {
    t_err_code = code;
    t_err_detail = detail;
    return code;
}
}  // namespace dmmt
using dmmt::error_detail;

extern "C" int dmmt_last_error_detail(void) { return t_err_detail; }

extern "C" const char* dmmt_last_error_message(void) {
    // error.rs:25-60 Display of the variant, with its payload
    static thread_local char msg[160];
    switch (t_err_code) {
    case DMMT_E_PPM_MISSING_TOKEN:
        snprintf(msg, sizeof msg, "Expected token '%s' not found in PPM file", kTokenNames[t_err_detail % 5]);
        break;
    case DMMT_E_PPM_PARSE_TOKEN:
        snprintf(msg, sizeof msg, "Parsing of token '%s' failed", kTokenNames[t_err_detail % 5]);
        break;
    case DMMT_E_PPM_INCOMPLETE_PIXEL:
        snprintf(msg, sizeof msg, "Incomplete pixel parsed. Expected 3 components, but got %d.", t_err_detail);
        break;
    case DMMT_E_PPM_SIZE_MISMATCH:  // (sic, error.rs:39-42)
        snprintf(msg, sizeof msg, "Nubmer of pixels do not match the size, provided in header");
        break;
    default:
        msg[0] = 0;  // no PPM error on this thread: see dmmt_strerror
    }
    return msg;
}

// parse_header .. parse_max_value (ppm.rs:145-222): the four header tokens; the
// body starts after the whitespace byte that ended the max value
static int parse_header(Tokenizer& tz, dmmt_ppm_header* hdr) {
    std::string tok;
    memset(hdr, 0, sizeof *hdr);
    // parse_header + check_header_version (ppm.rs:177-192)
    error_detail(DMMT_OK, 0);
    if (!tz.next(tok)) return error_detail(DMMT_E_PPM_MISSING_TOKEN, TOK_P3);
    const bool binary = tok == "P6";
    if (tok != "P3" && !binary) return error_detail(DMMT_E_PPM_MISSING_TOKEN, TOK_P3);
    uint16_t w, h, mx;
    if (!tz.next(tok)) return error_detail(DMMT_E_PPM_MISSING_TOKEN, TOK_WIDTH);
    if (!parse_u16(tok, &w)) return error_detail(DMMT_E_PPM_PARSE_TOKEN, TOK_WIDTH);
    if (!tz.next(tok)) return error_detail(DMMT_E_PPM_MISSING_TOKEN, TOK_HEIGHT);
    if (!parse_u16(tok, &h)) return error_detail(DMMT_E_PPM_PARSE_TOKEN, TOK_HEIGHT);
    if (!tz.next(tok)) return error_detail(DMMT_E_PPM_MISSING_TOKEN, TOK_MAXVAL);
    if (!parse_u16(tok, &mx)) return error_detail(DMMT_E_PPM_PARSE_TOKEN, TOK_MAXVAL);
    hdr->width = w;
    hdr->height = h;
    hdr->maxval = mx;
    hdr->binary = binary ? 1 : 0;
    hdr->body_offset = tz.i;
    return DMMT_OK;
}

extern "C" int dmmt_parse_ppm_header(const uint8_t* data, size_t len, dmmt_ppm_header* hdr) {
    if (!hdr || (!data && len)) return DMMT_E_INVALID_ARGUMENT;
    Tokenizer tz{data, len};
    return parse_header(tz, hdr);
}

extern "C" int dmmt_parse_ppm(const uint8_t* data, size_t len, dmmt_image* img) {
    if (!img || (!data && len)) return DMMT_E_INVALID_ARGUMENT;
    memset(img, 0, sizeof *img);
    Tokenizer tz{data, len};
    std::string tok;
    dmmt_ppm_header hdr;
    int rc = parse_header(tz, &hdr);
    if (rc) return rc;
    const bool binary = hdr.binary != 0;
    const uint16_t w = hdr.width, h = hdr.height, mx = hdr.maxval;
    const size_t npx = (size_t)w * h;
    const int sb = mx > 255 ? 2 : 1;
    // The samples a body of this length can hold, at most: a P3 sample takes a
    // digit and a separator (a success needs all npx * 3 of them), a P6 sample
    // sb bytes.  A short file claiming a large image allocates no more than that.
    const size_t body = len - tz.i;
    const size_t fit = binary ? body / (size_t)sb : body / 2 + 1;
    if (binary && fit < npx * 3) return error_detail(DMMT_E_PPM_SIZE_MISMATCH, 0);
    const size_t cap = npx * 3 < fit ? npx * 3 : fit;
    uint8_t* buf = (uint8_t*)malloc(cap * (size_t)sb + 1);
    if (!buf) return DMMT_E_OUT_OF_MEMORY;
    if (binary) {
        // P6: exactly one whitespace byte after maxval (already consumed by the
        // tokenizer), then raw big-endian samples.
        const size_t need = npx * 3 * (size_t)sb;
        const uint8_t* s = data + tz.i;
        if (sb == 1) {
            memcpy(buf, s, need);
        } else {
            uint16_t* d = (uint16_t*)buf;
            for (size_t k = 0; k < npx * 3; ++k) d[k] = (uint16_t)((s[2 * k] << 8) | s[2 * k + 1]);
        }
    } else {
        // parse_all_dots (ppm.rs:224-252)
        size_t count = 0;
        bool over = false;
        while (tz.next(tok)) {
            uint16_t v;
            if (!parse_u16(tok, &v)) {
                free(buf);
                return error_detail(DMMT_E_PPM_PARSE_TOKEN, TOK_COMPONENT);
            }
            if (count < cap) {
                if (sb == 1)
                    buf[count] = (uint8_t)(v > 255 ? 255 : v);
                else
                    ((uint16_t*)buf)[count] = v;
            }
            if (v > mx) over = true;
            ++count;
        }
        if (count % 3) {  // check_pixel_was_complete (ppm.rs:239-245)
            free(buf);
            return error_detail(DMMT_E_PPM_INCOMPLETE_PIXEL, (int)(count % 3));
        }
        if (count != npx * 3) {  // ppm.rs:165-175
            free(buf);
            return error_detail(DMMT_E_PPM_SIZE_MISMATCH, 0);
        }
        if (over) {  // RangeColorFormat::new panics (ppm.rs:155, color.rs:63-65)
            free(buf);
            return DMMT_E_VALUE_EXCEEDS_MAX;
        }
    }
    img->width = w;
    img->height = h;
    img->maxval = mx;
    img->sample_bytes = (uint16_t)sb;
    img->rgb = buf;
    return DMMT_OK;
}

extern "C" int dmmt_read_ppm(const char* path, dmmt_image* img) {
    if (!path || !img) return DMMT_E_INVALID_ARGUMENT;
    struct stat st;
    if (stat(path, &st) != 0) return errno == EACCES ? DMMT_E_NO_READ_PERMISSION : DMMT_E_INPUT_NOT_FOUND;
    FILE* f = fopen(path, "rb");
    if (!f) return errno == EACCES ? DMMT_E_NO_READ_PERMISSION : DMMT_E_OPEN_INPUT;
    std::vector<uint8_t> data;
    data.resize((size_t)st.st_size);
    const size_t got = st.st_size ? fread(data.data(), 1, data.size(), f) : 0;
    fclose(f);
    if (got != data.size()) return DMMT_E_OPEN_INPUT;
    return dmmt_parse_ppm(data.data(), data.size(), img);
}
