// cli.cpp -- command line mirroring the reference's clap CLI (cli.rs:23-126,
// main.rs:5-12): dmmt-jpeg-encoder <input_file> <output_file> [-b 8|16|32]
// [-p P444|P422|P420] [-t N] [-q PRESET]; extensions: --quality Q, --device D.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

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
            "      --device <D>                         GPU ordinal [default: 0]\n");
}

int main(int argc, char** argv) {
    dmmt_options opt;
    dmmt_default_options(&opt);
    const char* in = nullptr;
    const char* out = nullptr;
    int device = 0;
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
    int rc = dmmt_ctx_create(device, &ctx);
    if (rc == DMMT_OK) rc = dmmt_convert_ppm_to_jpeg(ctx, in, out, &opt);
    dmmt_ctx_destroy(ctx);
    if (rc != DMMT_OK) {  // main.rs:8-11
        fprintf(stderr, "Conversion failed because of: %s (%s)\n", dmmt_strerror(rc), dmmt_error_name(rc));
        return 1;
    }
    return 0;
}
