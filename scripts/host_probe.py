"""Is the pipelined 4K bench bound by the host?  Times N dmmt_encode_device calls
(4 lanes) as enqueue time (loop without sync) and total time (to the final sync),
for 1, 2 and 4 frames per call, with and without graph replay (DMMT_GRAPHS=1
must be set in the environment for the latter: pass --tag).
  python scripts/host_probe.py [--tag name]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
import torch  # noqa: E402,F401
import dmmt_jpeg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tag", default="direct")
ap.add_argument("--calls", type=int, default=400)
args = ap.parse_args()
w, h, sub, q = 3840, 2160, 0, 90
luma, chroma = dmmt_jpeg.quality_tables(q)
opt_c = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                            chroma_table=chroma).to_c()
out_stride = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
enc = dmmt_jpeg.Encoder(0)
enc.set_lanes(4)
for fps in (1, 2, 4):
    d_in = enc.malloc(w * h * 3 * fps)
    enc.fill_synthetic(d_in, w, h, fps)
    d_out = [enc.malloc(out_stride * fps) for _ in range(4)]
    d_len = [enc.malloc(4 * fps) for _ in range(4)]

    def run(n):
        for i in range(n):
            enc.encode_device(d_in, fps, w, h, None, d_out[i % 4], out_stride, d_len[i % 4], frame_stride=w * h * 3,
                              opt_c=opt_c)

    run(20)
    enc.synchronize()
    n = args.calls // fps
    t0 = time.perf_counter()
    run(n)
    t1 = time.perf_counter()
    enc.synchronize()
    t2 = time.perf_counter()
    print(f"{args.tag} frames/call={fps} enqueue_us/frame={(t1 - t0) / (n * fps) * 1e6:.1f} "
          f"total_us/frame={(t2 - t0) / (n * fps) * 1e6:.1f} Gpx/s={n * fps * w * h / (t2 - t0) / 1e9:.1f}", flush=True)
    for b in d_out + d_len + [d_in]:
        enc.free(b)
enc.close()
