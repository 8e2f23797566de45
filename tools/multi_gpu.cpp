// Multi-GPU C-ABI driver (no Python): one multi-GPU context (dmmt_ctx_create_multi)
// against a single-device context on the same synthetic image and frames.
//   multi_gpu [width height subsampling quality members devices frames]
//     devices: comma list of GPU ids for the members ("all": 0..members-1 when the
//     machine has that many GPUs, else every member on GPU 0)
// Checks, byte for byte:
//   * dmmt_jpeg_encode on the group (MCU-row stripes, joined mid-byte: the
//     reference's own stream) == dmmt_jpeg_encode on one context
//   * the same with a restart interval of one MCU row (stripes of whole intervals)
//   * dmmt_jpeg_encode_batch on the group (frames round-robin) == on one context
// and prints one JSON line with the wall times; exit 1 on any difference.
// build: make -C dmmt-jpeg-encoder_amd (bin/multi_gpu)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dmmt_jpeg.h"

// SURVEY.md 8(d) generator, as the library's k_synthetic: base = (x + 8y) % 256
// (dct_timing.rs:150-160), 4-bit xorshift32 noise per channel, clamped
static void synthetic(std::vector<uint8_t>& rgb, int w, int h, uint32_t f, uint32_t seed = 0x9E3779B9u) {
    rgb.resize((size_t)w * h * 3);
    const uint32_t npx = (uint32_t)((uint64_t)w * h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const uint32_t pi = (uint32_t)y * (uint32_t)w + (uint32_t)x;
            uint32_t n = seed ^ (f * npx + pi);
            n ^= n << 13;
            n ^= n >> 17;
            n ^= n << 5;
            const uint32_t base = (uint32_t)(x + 8 * y) & 255u;
            const uint32_t r = base + (n & 15u);
            const uint32_t g = ((base + 85u * f + ((uint32_t)y >> 3)) & 255u) + ((n >> 4) & 15u);
            const uint32_t b = ((255u - base + ((uint32_t)x >> 4)) & 255u) + ((n >> 8) & 15u);
            uint8_t* p = &rgb[(size_t)pi * 3];
            p[0] = (uint8_t)(r < 255 ? r : 255);
            p[1] = (uint8_t)(g < 255 ? g : 255);
            p[2] = (uint8_t)(b < 255 ? b : 255);
        }
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int fail(const char* what, int rc) {
    fprintf(stderr, "%s failed: %d (%s)\n", what, rc, dmmt_error_name(rc));
    return 1;
}

int main(int argc, char** argv) {
    const int w = argc > 1 ? atoi(argv[1]) : 3840, h = argc > 2 ? atoi(argv[2]) : 2160;
    const int sub = argc > 3 ? atoi(argv[3]) : 0, q = argc > 4 ? atoi(argv[4]) : 90;
    const int members = argc > 5 ? atoi(argv[5]) : 8;
    const std::string devs = argc > 6 ? argv[6] : "all";
    const int frames = argc > 7 ? atoi(argv[7]) : 16;
    int ngpu = 0;
    dmmt_device_count(&ngpu);
    std::vector<int> ids;
    if (devs == "all") {
        for (int i = 0; i < members; ++i) ids.push_back(ngpu >= members ? i : 0);
    } else {
        for (size_t p = 0; p <= devs.size();) {
            size_t e = devs.find(',', p);
            if (e == std::string::npos) e = devs.size();
            ids.push_back(atoi(devs.substr(p, e - p).c_str()));
            p = e + 1;
        }
    }
    dmmt_options opt;
    dmmt_default_options(&opt);
    opt.subsampling = sub;
    dmmt_quality_tables(q, opt.luma_q, opt.chroma_q);
    const int mcu_w = sub == DMMT_P444 ? 8 : 16;
    const int mcux = (w + mcu_w - 1) / mcu_w;

    dmmt_ctx *one = nullptr, *grp = nullptr;
    int rc;
    if ((rc = dmmt_ctx_create(ids[0], &one))) return fail("dmmt_ctx_create", rc);
    if ((rc = dmmt_ctx_create_multi(ids.data(), (int)ids.size(), &grp))) return fail("dmmt_ctx_create_multi", rc);

    std::vector<uint8_t> img;
    synthetic(img, w, h, 0);
    const dmmt_image im{(uint16_t)w, (uint16_t)h, 255, 1, img.data()};
    bool ok = true;
    double t_one[2] = {0, 0}, t_grp[2] = {0, 0};
    size_t bytes[2] = {0, 0};
    for (int mode = 0; mode < 2; ++mode) {  // 0: joined (restart_interval 0), 1: restart every MCU row
        opt.restart_interval = mode ? mcux : 0;
        uint8_t *a = nullptr, *b = nullptr;
        size_t na = 0, nb = 0;
        for (int rep = 0; rep < 2; ++rep) {  // the second call is timed (workspaces allocated)
            dmmt_free(a);
            dmmt_free(b);
            double t0 = now();
            if ((rc = dmmt_jpeg_encode(one, &im, &opt, &a, &na))) return fail("dmmt_jpeg_encode (one)", rc);
            t_one[mode] = now() - t0;
            t0 = now();
            if ((rc = dmmt_jpeg_encode(grp, &im, &opt, &b, &nb))) return fail("dmmt_jpeg_encode (group)", rc);
            t_grp[mode] = now() - t0;
        }
        if (na != nb || memcmp(a, b, na) != 0) {
            fprintf(stderr, "mode %d: striped %zu bytes differ from single %zu bytes\n", mode, nb, na);
            ok = false;
        }
        bytes[mode] = na;
        dmmt_free(a);
        dmmt_free(b);
    }
    opt.restart_interval = 0;
    // frames round-robin over the members
    std::vector<std::vector<uint8_t>> fr(frames);
    std::vector<dmmt_image> ims(frames);
    for (int f = 0; f < frames; ++f) {
        synthetic(fr[f], w, h, (uint32_t)(f + 1));
        ims[f] = dmmt_image{(uint16_t)w, (uint16_t)h, 255, 1, fr[f].data()};
    }
    std::vector<uint8_t*> oa(frames), ob(frames);
    std::vector<size_t> la(frames), lb(frames);
    double t_batch_one = 0, t_batch_grp = 0;
    for (int rep = 0; rep < 2; ++rep) {
        if (rep)
            for (int f = 0; f < frames; ++f) dmmt_free(oa[f]), dmmt_free(ob[f]);
        double t0 = now();
        if ((rc = dmmt_jpeg_encode_batch(one, ims.data(), frames, &opt, oa.data(), la.data())))
            return fail("batch (one)", rc);
        t_batch_one = now() - t0;
        t0 = now();
        if ((rc = dmmt_jpeg_encode_batch(grp, ims.data(), frames, &opt, ob.data(), lb.data())))
            return fail("batch (group)", rc);
        t_batch_grp = now() - t0;
    }
    int batch_diff = 0;
    for (int f = 0; f < frames; ++f) {
        if (la[f] != lb[f] || memcmp(oa[f], ob[f], la[f]) != 0) ++batch_diff;
        dmmt_free(oa[f]);
        dmmt_free(ob[f]);
    }
    ok = ok && batch_diff == 0;
    std::string dl;
    for (size_t i = 0; i < ids.size(); ++i) dl += (i ? "," : "") + std::to_string(ids[i]);
    printf("{\"tool\": \"multi_gpu\", \"width\": %d, \"height\": %d, \"subsampling\": %d, \"quality\": %d, "
           "\"members\": %d, \"devices\": [%s], \"gpus_visible\": %d, \"match\": %s, "
           "\"joined\": {\"bytes\": %zu, \"ms_one_context\": %.3f, \"ms_group\": %.3f}, "
           "\"restart_every_row\": {\"bytes\": %zu, \"ms_one_context\": %.3f, \"ms_group\": %.3f}, "
           "\"batch\": {\"frames\": %d, \"mismatched\": %d, \"ms_one_context\": %.3f, \"ms_group\": %.3f}}\n",
           w, h, sub, q, dmmt_ctx_num_devices(grp), dl.c_str(), ngpu, ok ? "true" : "false", bytes[0],
           1e3 * t_one[0], 1e3 * t_grp[0], bytes[1], 1e3 * t_one[1], 1e3 * t_grp[1], frames, batch_diff,
           1e3 * t_batch_one, 1e3 * t_batch_grp);
    dmmt_ctx_destroy(grp);
    dmmt_ctx_destroy(one);
    return ok ? 0 : 1;
}
