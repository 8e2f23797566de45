// cli.cpp -- command line mirroring the reference's clap CLI (cli.rs:23-126,
// main.rs:5-12): dmmt-jpeg-encoder <input_file> <output_file> [-b 8|16|32]
// [-p P444|P422|P420] [-t N] [-q PRESET]; extensions: --quality Q, --device D,
// --gpus N / --devices A,B,.. (the image as MCU-row stripes over several GPUs),
// --restart-interval N (DRI/RSTn every N MCUs).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/dmmt_jpeg.h"

static int preset_from_name(const std::string& s) {
    // quantization_tables.rs:245-284 names and aliases
    if (s == "Specification" || s == "Spec" || s == "Default" || s == "0") return DMMT_Q_SPECIFICATION;
    if (s == "Flat" || s == "1") return DMMT_Q_FLAT;
    if (s == "MSSIM-Kodak-Tuned" || s == "2") return DMMT_Q_MSSIM_KODAK_TUNED;
    if (s == "PSNR-HVS-N-Kodak-Tuned" || s == "4") return DMMT_Q_PSNR_HVS_N_KODAK_TUNED;
    if (s == "DCTune-Perceptual-Optimization" || s == "6") return DMMT_Q_DCTUNE_PERCEPTUAL_OPTIMIZATION;
    if (s == "A-visual-detection-model" || s == "7") return DMMT_Q_A_VISUAL_DETECTION_MODEL;
    if (s == "An-improved-detection-model" || s == "8") return DMMT_Q_AN_IMPROVED_DETECTION_MODEL;
    return -1;
}

static void usage() {
    fprintf(stderr,
            "Usage: dmmt-jpeg-encoder [OPTIONS] <input_file> <output_file>\n"
            "  -b, --bits_per_channel <BITS>            8|16|32 [default: 8]\n"
            "  -p, --chroma_subsampling_preset <PRESET> P444|P422|P420 [default: P420]\n"
            "  -t, --threads <THREADS>                  accepted for compatibility (GPU encoder)\n"
            "  -q, --quantization_table <TABLE>         preset name or alias [default: Specification]\n"
            "      --quality <Q>                        IJG-scaled Annex K tables (extension)\n"
            "      --device <D>                         GPU ordinal [default: 0]\n"
            "      --gpus <N>                           encode as MCU-row stripes on GPUs 0..N-1 (extension)\n"
            "      --devices <A,B,..>                   encode as MCU-row stripes on these GPUs (repeats allowed)\n"
            "      --restart-interval <N>               DRI/RSTn every N MCUs [default: 0 = none] (extension)\n");
}

int main(int argc, char** argv) {
    dmmt_options opt;
    dmmt_default_options(&opt);
    const char* in = nullptr;
    const char* out = nullptr;
    int device = 0;
    std::vector<int> devices;  // several GPUs: a multi-GPU context
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto value = [&](const char* name) -> std::string {
            if (i + 1 >= argc) {
                fprintf(stderr, "error: a value is required for '%s'\n", name);
                exit(2);
            }
            return argv[++i];
        };
        if (a == "-b" || a == "--bits_per_channel") {
            std::string v = value("--bits_per_channel");
            if (v != "8" && v != "16" && v != "32") {
                fprintf(stderr, "error: invalid value '%s' for '--bits_per_channel'\n", v.c_str());
                return 2;
            }
            opt.bits_per_channel = atoi(v.c_str());
        } else if (a == "-p" || a == "--chroma_subsampling_preset") {
            std::string v = value("--chroma_subsampling_preset");
            if (v == "P444")
                opt.subsampling = DMMT_P444;
            else if (v == "P422")
                opt.subsampling = DMMT_P422;
            else if (v == "P420")
                opt.subsampling = DMMT_P420;
            else {
                fprintf(stderr, "error: invalid value '%s' for '--chroma_subsampling_preset'\n", v.c_str());
                return 2;
            }
        } else if (a == "-t" || a == "--threads") {
            opt.n_threads = atoi(value("--threads").c_str());
        } else if (a == "-q" || a == "--quantization_table") {
            std::string v = value("--quantization_table");
            int p = preset_from_name(v);
            if (p < 0) {
                fprintf(stderr, "error: invalid value '%s' for '--quantization_table'\n", v.c_str());
                return 2;
            }
            dmmt_quantization_preset(p, opt.luma_q, opt.chroma_q);
        } else if (a == "--quality") {
            if (dmmt_quality_tables(atoi(value("--quality").c_str()), opt.luma_q, opt.chroma_q)) {
                fprintf(stderr, "error: quality must be 1..100\n");
                return 2;
            }
        } else if (a == "--device") {
            device = atoi(value("--device").c_str());
        } else if (a == "--gpus") {
            const int n = atoi(value("--gpus").c_str());
            if (n < 1 || n > DMMT_MAX_GROUP) {
                fprintf(stderr, "error: --gpus must be 1..%d\n", DMMT_MAX_GROUP);
                return 2;
            }
            devices.clear();
            for (int d = 0; d < n; ++d) devices.push_back(d);
        } else if (a == "--devices") {
            std::string v = value("--devices");
            devices.clear();
            for (size_t p = 0; p <= v.size();) {
                size_t q = v.find(',', p);
                if (q == std::string::npos) q = v.size();
                const std::string t = v.substr(p, q - p);
                if (t.empty() || t.find_first_not_of("0123456789") != std::string::npos) {
                    fprintf(stderr, "error: invalid value '%s' for '--devices'\n", v.c_str());
                    return 2;
                }
                devices.push_back(atoi(t.c_str()));
                p = q + 1;
            }
        } else if (a == "--restart-interval") {
            opt.restart_interval = atoi(value("--restart-interval").c_str());
        } else if (a == "-h" || a == "--help") {
            usage();
            return 0;
        } else if (!in) {
            in = argv[i];
        } else if (!out) {
            out = argv[i];
        } else {
            usage();
            return 2;
        }
    }
    if (!in || !out) {
        usage();
        return 2;
    }
    dmmt_ctx* ctx = nullptr;
    int rc = devices.size() > 1 ? dmmt_ctx_create_multi(devices.data(), (int)devices.size(), &ctx)
                                : dmmt_ctx_create(devices.empty() ? device : devices[0], &ctx);
    if (rc == DMMT_OK) rc = dmmt_convert_ppm_to_jpeg(ctx, in, out, &opt);
    dmmt_ctx_destroy(ctx);
    if (rc != DMMT_OK) {  // main.rs:8-11
        fprintf(stderr, "Conversion failed because of: %s (%s)\n", dmmt_strerror(rc), dmmt_error_name(rc));
        return 1;
    }
    return 0;
}
