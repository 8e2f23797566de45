// PCIe-inclusive encode rate at the C ABI (no Python between the caller and the
// library): host RGB frames -> dmmt_jpeg_encode_batch -> host JPEG buffers, the
// way a Rust caller of the reference's JpegImageWriter would use it.
//   e2e_c [width height subsampling quality frames_per_call distinct seconds]
// build: g++ -O2 -std=c++17 -Iinclude tools/e2e_c.cpp -Ldmmt-jpeg-encoder_amd/lib -ldmmt_jpeg \
//        -Wl,-rpath,$PWD/dmmt-jpeg-encoder_amd/lib -o tools/e2e_c
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "dmmt_jpeg.h"

int main(int argc, char** argv) {
    const int w = argc > 1 ? atoi(argv[1]) : 3840, h = argc > 2 ? atoi(argv[2]) : 2160;
    const int sub = argc > 3 ? atoi(argv[3]) : 0, q = argc > 4 ? atoi(argv[4]) : 90;
    const int fpc = argc > 5 ? atoi(argv[5]) : 8, distinct = argc > 6 ? atoi(argv[6]) : 8;
    const double seconds = argc > 7 ? atof(argv[7]) : 4.0;
    // the synthetic pattern of SURVEY 8(d) (noise-free variant is enough for rates)
    std::vector<std::vector<uint8_t>> frames(distinct, std::vector<uint8_t>((size_t)w * h * 3));
    for (int f = 0; f < distinct; ++f)
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x) {
                const int base = (x + 8 * y) % 256;
                uint8_t* p = &frames[f][((size_t)y * w + x) * 3];
                p[0] = (uint8_t)base;
                p[1] = (uint8_t)((base + 85 * f + (y >> 3)) % 256);
                p[2] = (uint8_t)((255 - base + (x >> 4)) % 256);
            }
    dmmt_ctx* ctx = nullptr;
    if (dmmt_ctx_create(0, &ctx) != DMMT_OK) return fprintf(stderr, "no device\n"), 1;
    dmmt_options opt;
    dmmt_default_options(&opt);
    opt.subsampling = sub;
    dmmt_quality_tables(q, opt.luma_q, opt.chroma_q);
    std::vector<dmmt_image> imgs(fpc);
    for (int i = 0; i < fpc; ++i) imgs[i] = dmmt_image{(uint16_t)w, (uint16_t)h, 255, 1, frames[i % distinct].data()};
    std::vector<uint8_t*> outs(fpc);
    std::vector<size_t> lens(fpc);
    auto call = [&]() {
        const int rc = dmmt_jpeg_encode_batch(ctx, imgs.data(), fpc, &opt, outs.data(), lens.data());
        if (rc != DMMT_OK) {
            fprintf(stderr, "encode failed: %d\n", rc);
            exit(1);
        }
        for (int i = 0; i < fpc; ++i) dmmt_free(outs[i]);
    };
    call();  // workspace, tables
    int calls = 0;
    const auto t0 = std::chrono::steady_clock::now();
    double dt = 0;
    do {
        call();
        ++calls;
        dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } while (dt < seconds);
    printf("{\"tool\": \"e2e_c\", \"width\": %d, \"height\": %d, \"subsampling\": %d, \"quality\": %d, "
           "\"frames_per_call\": %d, \"distinct_frames\": %d, \"calls\": %d, \"ms_per_call\": %.3f, "
           "\"mpixel_per_s\": %.1f, \"jpeg_bytes_first\": %zu}\n",
           w, h, sub, q, fpc, distinct, calls, 1e3 * dt / calls, (double)calls * fpc * w * h / dt / 1e6, lens[0]);
    dmmt_ctx_destroy(ctx);
    return 0;
}
