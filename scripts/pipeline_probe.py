"""Throughput of 4K q90 encodes with 1, 2 or 3 contexts (own workspace and HIP
stream each) fed round-robin: do the latency-bound kernels of one frame overlap
the other frames' kernels?  python scripts/pipeline_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
import torch  # noqa: E402,F401
import dmmt_jpeg  # noqa: E402

w, h, sub, q = 3840, 2160, 0, 90
luma, chroma = dmmt_jpeg.quality_tables(q)
opt_c = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                            chroma_table=chroma).to_c()
out_stride = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
for nctx in (1, 2, 3):
    encs = [dmmt_jpeg.Encoder(0) for _ in range(nctx)]
    bufs = []
    for i, e in enumerate(encs):
        d_in = e.malloc(w * h * 3)
        e.fill_synthetic(d_in, w, h, 1, first_frame=i)
        bufs.append((d_in, e.malloc(out_stride), e.malloc(4)))

    def run(n):
        for i in range(n):
            e = encs[i % nctx]
            d_in, d_out, d_len = bufs[i % nctx]
            e.encode_device(d_in, 1, w, h, None, d_out, out_stride, d_len, frame_stride=w * h * 3, opt_c=opt_c)
        for e in encs:
            e.synchronize()

    run(30)
    n = 300
    t0 = time.perf_counter()
    run(n)
    dt = time.perf_counter() - t0
    print(f"contexts={nctx} us/frame={dt / n * 1e6:8.2f} Gpx/s={w * h * n / dt / 1e9:7.2f}", flush=True)
    for e, (a, b, c) in zip(encs, bufs):
        e.free(a)
        e.free(b)
        e.free(c)
        e.close()
