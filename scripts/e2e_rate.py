"""PCIe-inclusive encode rate (host RGB -> host JPEG bytes through dmmt_jpeg_encode),
for DESIGN.md; bench.py's `value` is the device-resident rate.
usage: python scripts/e2e_rate.py [--config 4k444q90] [--seconds 5]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process)
import dmmt_jpeg  # noqa: E402
import bench  # noqa: E402
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k444q90", choices=sorted(bench.CONFIGS))
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--batch", type=int, default=0, help="frames per call (default: the config's)")
    a = ap.parse_args()
    w, h, sub, q, fps = bench.CONFIGS[a.config]
    fps = a.batch or fps
    luma, chroma = dmmt_jpeg.quality_tables(q)
    opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                               chroma_table=chroma)
    enc = dmmt_jpeg.Encoder(0)

    def synthetic(frame):  # the SURVEY 8(d) frames from the library's own device generator
        d = enc.malloc(w * h * 3)
        enc.fill_synthetic(d, w, h, 1, first_frame=frame)
        rgb = np.frombuffer(enc.d2h(d, w * h * 3), np.uint8).reshape(h, w, 3).copy()
        enc.free(d)
        return rgb

    imgs = [dmmt_jpeg.Image.from_array(synthetic(f)) for f in range(min(fps, 8))]
    batch = [imgs[i % len(imgs)] for i in range(fps)]
    enc.encode_batch(batch, opts)  # warm-up: workspace, tables
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        outs = enc.encode_batch(batch, opts)
        n += 1
    dt = time.perf_counter() - t0
    print(json.dumps({"config": a.config, "mode": "host RGB -> host JPEG (PCIe both ways, dmmt_jpeg_encode_batch)",
                      "frames_per_call": fps, "distinct_frames": min(fps, 8),
                      "mpixel_per_s": round(n * fps * w * h / dt / 1e6, 1), "calls": n,
                      "ms_per_call": round(dt / n * 1e3, 3), "mean_jpeg_bytes": sum(map(len, outs)) / len(outs)}))
    enc.close()


if __name__ == "__main__":
    main()
