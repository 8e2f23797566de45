"""Where does a short timed region (the driver's 20 bench steps) lose time?  Per
run: enqueue time of the steps, time to the device being idle, then the context's
status collection (dmmt_ctx_synchronize).
  python scripts/short_probe.py [--steps 20] [--runs 8]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
import torch  # noqa: E402
import dmmt_jpeg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--runs", type=int, default=8)
ap.add_argument("--lanes", type=int, default=4)
args = ap.parse_args()
w, h, sub, q = 3840, 2160, 0, 90
luma, chroma = dmmt_jpeg.quality_tables(q)
opt_c = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                            chroma_table=chroma).to_c()
out_stride = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
enc = dmmt_jpeg.Encoder(0)
enc.set_lanes(args.lanes)
d_in = [enc.malloc(w * h * 3) for _ in range(4)]
for s in range(4):
    enc.fill_synthetic(d_in[s], w, h, 1, first_frame=s)
d_out = [enc.malloc(out_stride) for _ in range(args.lanes)]
d_len = [enc.malloc(4) for _ in range(args.lanes)]


def run(n):
    for i in range(n):
        enc.encode_device(d_in[i % 4], 1, w, h, None, d_out[i % args.lanes], out_stride, d_len[i % args.lanes],
                          frame_stride=w * h * 3, opt_c=opt_c)


run(8)
enc.synchronize()
for r in range(args.runs):
    torch.cuda.synchronize()
    enc.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    enc.synchronize()
    t3 = time.perf_counter()
    us = lambda a, b: (b - a) * 1e6  # noqa: E731
    print(f"steps={args.steps} lanes={args.lanes} enqueue={us(t0, t1):.0f}us idle_at={us(t0, t2):.0f}us "
          f"status={us(t2, t3):.0f}us per_step={us(t0, t3) / args.steps:.1f}us", flush=True)
enc.close()
