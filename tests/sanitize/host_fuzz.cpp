// host_fuzz.cpp -- seeded fuzz of the product's host-only code (PPM parser,
// quantisation tables) for the ASan/UBSan build of tests/test_sanitizers.py.
// Inputs: well-formed P3/P6 files of random size, separators and comments, and
// mutations of them (byte flips, truncation, inserted garbage).  Every call must
// return one of the documented codes; a successful parse must agree with the
// header and hold exactly width*height*3 samples.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>

#include "../../include/dmmt_jpeg.h"

extern "C" void dmmt_free(void* p) { free(p); }  // (the library's own is in encoder.cpp, a HIP unit)

static std::mt19937_64 rng;
static int rnd(int n) { return (int)(rng() % (uint64_t)n); }

static std::string sep() {
    static const char* ws[] = {" ", "\n", "\t", "\r", "\f", "  ", "\n\n"};
    std::string s = ws[rnd(7)];
    if (rnd(10) == 0) s += "# a comment 12 34\n";
    return s;
}

static std::string make_ppm(bool binary, int w, int h, int mx) {
    std::string s = binary ? "P6" : "P3";
    s += sep() + std::to_string(w) + sep() + std::to_string(h) + sep() + std::to_string(mx);
    s += binary ? "\n" : sep();
    for (long k = 0; k < (long)w * h * 3; ++k) {
        const int v = rnd(mx + 1);
        if (binary) {
            if (mx > 255) s += (char)(v >> 8);
            s += (char)(v & 0xFF);
        } else {
            s += std::to_string(v) + sep();
        }
    }
    return s;
}

int main(int argc, char** argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 20000;
    rng.seed(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
    long ok = 0, err = 0;
    for (long it = 0; it < iters; ++it) {
        const bool binary = rnd(3) == 0;
        const int w = rnd(9), h = rnd(9);
        const int mx = rnd(4) == 0 ? 1 + rnd(65535) : (rnd(2) ? 255 : 1 + rnd(255));
        std::string s = make_ppm(binary, w, h, mx);
        switch (rnd(6)) {  // mutations
            case 0: break;
            case 1: if (!s.empty()) s[rnd((int)s.size())] = (char)rnd(256); break;
            case 2: s.resize(rnd((int)s.size() + 1)); break;
            case 3: s.insert(rnd((int)s.size() + 1), std::string(1 + rnd(4), (char)rnd(256))); break;
            case 4: s.insert(rnd((int)s.size() + 1), "#"); break;
            case 5: {  // a header that claims a huge image over a short body
                s = std::string(binary ? "P6 " : "P3 ") + "65535 65535 " + std::to_string(mx) + " 1 2 3";
                break;
            }
        }
        dmmt_ppm_header hdr;
        const int rh = dmmt_parse_ppm_header((const uint8_t*)s.data(), s.size(), &hdr);
        dmmt_image img;
        const int rc = dmmt_parse_ppm((const uint8_t*)s.data(), s.size(), &img);
        const bool known = rc == DMMT_OK || rc == DMMT_E_PPM_MISSING_TOKEN || rc == DMMT_E_PPM_PARSE_TOKEN ||
                           rc == DMMT_E_PPM_INCOMPLETE_PIXEL || rc == DMMT_E_PPM_SIZE_MISMATCH ||
                           rc == DMMT_E_VALUE_EXCEEDS_MAX;
        if (!known) {
            fprintf(stderr, "iteration %ld: unexpected code %d\n", it, rc);
            return 1;
        }
        if (rh != DMMT_OK && rc == DMMT_OK) {
            fprintf(stderr, "iteration %ld: body parsed without a header\n", it);
            return 1;
        }
        if (rc == DMMT_OK) {
            const size_t n = (size_t)img.width * img.height * 3;
            if (img.width != hdr.width || img.height != hdr.height || img.maxval != hdr.maxval ||
                img.sample_bytes != (img.maxval > 255 ? 2 : 1)) {
                fprintf(stderr, "iteration %ld: image disagrees with its header\n", it);
                return 1;
            }
            unsigned long sum = 0;  // touch every sample (ASan: all inside the buffer)
            for (size_t k = 0; k < n; ++k)
                sum += img.sample_bytes == 1 ? ((const uint8_t*)img.rgb)[k] : ((const uint16_t*)img.rgb)[k];
            (void)sum;
            dmmt_free((void*)img.rgb);
            ++ok;
        } else {
            ++err;
        }
    }
    uint8_t l[64], c[64];
    for (int q = -5; q <= 105; ++q) {
        const int r = dmmt_quality_tables(q, l, c);
        if ((r == DMMT_OK) != (q >= 1 && q <= 100)) return 1;
        if (r == DMMT_OK)
            for (int i = 0; i < 64; ++i)
                if (!l[i] || !c[i]) return 1;
    }
    for (int p = -2; p <= 9; ++p)
        if ((dmmt_quantization_preset(p, l, c) == DMMT_OK) != (p >= 0 && p < 7)) return 1;
    dmmt_options o;
    dmmt_default_options(&o);
    printf("host_fuzz: %ld parsed, %ld rejected, tables checked\n", ok, err);
    return 0;
}
