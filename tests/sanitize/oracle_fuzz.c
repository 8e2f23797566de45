/* oracle_fuzz.c -- seeded run of the CPU oracle (oracle/cpu_ref.c) for the
 * sanitizer builds of tests/test_sanitizers.py: ASan/UBSan over random images,
 * options and restart intervals, and ThreadSanitizer over the pthread DCT
 * (ref_encode_mt, the reference's threadpool stage), whose output must equal
 * the single-threaded encode byte for byte.  Test infrastructure only. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/cpu_ref.h"

static uint64_t s_state = 88172645463325252ull;
static uint32_t rnd(uint32_t n) {
    s_state ^= s_state << 13;
    s_state ^= s_state >> 7;
    s_state ^= s_state << 17;
    return (uint32_t)(s_state % n);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 60;
    const int threads = argc > 2 ? atoi(argv[2]) : 4;
    if (argc > 3) s_state ^= strtoull(argv[3], NULL, 10);
    int done = 0;
    for (int it = 0; it < iters; ++it) {
        /* every fourth image large enough for several 700-block DCT jobs per channel */
        const int big = it % 4 == 0;
        const int w = 1 + (int)rnd(big ? 600 : 120), h = (big ? 240 : 1) + (int)rnd(big ? 300 : 120);
        const int maxval = rnd(3) == 0 ? 1 + (int)rnd(65535) : 255;
        uint16_t* rgb = (uint16_t*)malloc(sizeof(uint16_t) * 3 * (size_t)w * h);
        const int kind = (int)rnd(3);
        for (int k = 0; k < 3 * w * h; ++k)
            rgb[k] = (uint16_t)(kind == 0 ? rnd(maxval + 1) : kind == 1 ? (k * 7 / 3) % (maxval + 1) : maxval / 2);
        ref_options o;
        memset(&o, 0, sizeof o);
        o.preset = (int)rnd(3);
        o.bits_per_channel = 8;
        for (int i = 0; i < 64; ++i) {
            o.luma_q[i] = (uint8_t)(1 + rnd(255));
            o.chroma_q[i] = (uint8_t)(1 + rnd(255));
        }
        o.restart_interval = rnd(2) ? 0 : 1 + (int)rnd(20);
        uint8_t *a = NULL, *b = NULL;
        size_t na = 0, nb = 0;
        const int ra = ref_encode(rgb, w, h, maxval, &o, &a, &na);
        const int rb = ref_encode_mt(rgb, w, h, maxval, &o, threads, &b, &nb);
        if (ra != rb || (ra == REF_OK && (na != nb || memcmp(a, b, na) != 0))) {
            fprintf(stderr, "iteration %d: threaded encode differs (%d/%d, %zu/%zu bytes)\n", it, ra, rb, na, nb);
            return 1;
        }
        int16_t* coef = NULL;
        size_t nblk = 0;
        if (ref_forward(rgb, w, h, maxval, &o, &coef, &nblk) == REF_OK) {
            uint8_t* c = NULL;
            size_t nc = 0;
            const int rc = ref_encode_coefficients(coef, nblk, w, h, &o, &c, &nc);
            if (ra == REF_OK && (rc != REF_OK || nc != na || memcmp(c, a, na) != 0)) {
                fprintf(stderr, "iteration %d: forward + back half differs from the whole encode\n", it);
                return 1;
            }
            ref_free(c);
            ref_free(coef);
        }
        ref_free(a);
        ref_free(b);
        free(rgb);
        ++done;
    }
    printf("oracle_fuzz: %d encodes, %d threads, identical\n", done, threads);
    return 0;
}
