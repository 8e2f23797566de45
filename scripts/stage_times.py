"""Per-stage device time of one bench config for one library build, from the
library's own HIP-event stage profiling (dmmt_ctx_set_profiling), one lane.
Errors the kernels report (e.g. an ablation build that skips the histogram) are
ignored: this measures time only.
  DMMT_LIB_PATH=.../lib_x/libdmmt_jpeg.so python scripts/stage_times.py [--config 4k444q90]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import dmmt_jpeg  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k444q90", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--tag", default=os.path.basename(os.path.dirname(os.environ.get("DMMT_LIB_PATH", "lib/x"))))
    args = ap.parse_args()
    w, h, sub, q, fps = bench.CONFIGS[args.config]
    luma, chroma = dmmt_jpeg.quality_tables(q)
    opt_c = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                                chroma_table=chroma).to_c()
    enc = dmmt_jpeg.Encoder(0)
    out_stride = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
    d_in = enc.malloc(w * h * 3 * fps)
    d_out = enc.malloc(out_stride * fps)
    d_len = enc.malloc(4 * fps)
    enc.fill_synthetic(d_in, w, h, fps)

    def run(n):
        for _ in range(n):
            enc.encode_device(d_in, fps, w, h, None, d_out, out_stride, d_len, frame_stride=w * h * 3, opt_c=opt_c)
        try:
            enc.synchronize()
        except dmmt_jpeg.Error:
            pass

    run(5)
    enc.set_profiling(True)
    run(args.steps)
    prof = enc.profile()
    enc.set_profiling(False)
    res = {"tag": args.tag, "config": args.config}
    for k, (ms, n) in prof.items():
        if n:
            res[k] = round(1000.0 * ms / n, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
