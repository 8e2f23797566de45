"""Per-phase cycle counts of the kernels from the `make TRACE=1` build.

Runs the bench workload through lib_trace/libdmmt_jpeg.so and prints, for
every traced phase, the time per mark (s_memrealtime, 100 MHz) (thread 0 of every
workgroup marks once per phase pass) and the summed cycles.
  python scripts/phase_trace.py [--config 4k444q90] [--steps 20]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DMMT_LIB_PATH"] = os.path.join(ROOT, "dmmt-jpeg-encoder_amd", os.environ.get("DMMT_TRACE_LIB", "lib_trace"), "libdmmt_jpeg.so")
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import dmmt_jpeg  # noqa: E402
import bench  # noqa: E402

NAMES = {
    "kernels": {0: "front A colour", 1: "front B rows", 2: "front C cols+quant", 3: "front D store",
                4: "front E symbols", 5: "front hist flush", 10: "tables 1 hist", 6: "tables merge leafsearch", 7: "tables merge pkgsearch", 8: "tables merge barrier", 11: "tables 2 rank",
                12: "tables 3 merge", 13: "tables 4 leaves", 14: "tables 5 codes", 15: "tables 6 header"},
    "entropy": {0: "emit tables+sort", 4: "emit block load+zigzag", 5: "emit walk", 1: "emit scan",
                2: "emit windows+store", 3: "emit ff/edges", 6: "emit summary+arrival",
                7: "emit tail bits/edges+scan", 8: "emit tail ff loads+bytes", 9: "emit tail byte scan",
                10: "emit tail stores"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k444q90", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    w, h, sub, q, fps = bench.CONFIGS[args.config]
    luma, chroma = dmmt_jpeg.quality_tables(q)
    opt_c = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                                chroma_table=chroma).to_c()
    enc = dmmt_jpeg.Encoder(0)
    L = dmmt_jpeg.lib()
    buf = (ctypes.c_ulonglong * 64)()
    out_stride = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
    d_in = enc.malloc(w * h * 3 * fps)
    d_out = enc.malloc(out_stride * fps)
    d_len = enc.malloc(4 * fps)
    enc.fill_synthetic(d_in, w, h, fps)
    for _ in range(3):
        enc.encode_device(d_in, fps, w, h, None, d_out, out_stride, d_len, frame_stride=w * h * 3, opt_c=opt_c)
    enc.synchronize()
    for tu in ("kernels", "entropy"):
        getattr(L, f"dmmt_debug_trace_{tu}")(buf)
    acc = {tu: [0] * 48 for tu in ("kernels", "entropy")}
    spans = {tu: [[0.0, 0.0, 0] for _ in range(4)] for tu in ("kernels", "entropy")}
    for _ in range(args.steps):  # one readout per step: the span slots hold per-launch extrema
        enc.encode_device(d_in, fps, w, h, None, d_out, out_stride, d_len, frame_stride=w * h * 3, opt_c=opt_c)
        enc.synchronize()
        for tu in ("kernels", "entropy"):
            getattr(L, f"dmmt_debug_trace_{tu}")(buf)
            v = list(buf)
            for i in range(48):
                acc[tu][i] += v[i]
            for s in range(4):
                t0, t1, life, n = (~v[48 + 4 * s]) & (2**64 - 1), v[49 + 4 * s], v[50 + 4 * s], v[51 + 4 * s]
                if n:
                    spans[tu][s][0] += (t1 - t0) / 100
                    spans[tu][s][1] += life / n / 100
                    spans[tu][s][2] = n
    for tu in ("kernels", "entropy"):
        v = acc[tu]
        for i in range(16):
            if v[32 + i]:
                print(f"{tu:8s} {i:2d} {NAMES[tu].get(i, '?'):22s} marks/step={v[32 + i] / args.steps:9.1f} "
                      f"us/mark={v[i] / v[32 + i] / 100:9.3f} us/step(sum over marks)={v[i] / args.steps / 100:12.1f} "
                      f"clock={v[16 + i] / max(v[i], 1) * 100:6.0f} MHz")
        for s in range(4):
            if spans[tu][s][2]:
                print(f"{tu:8s} span {s}: workgroups={spans[tu][s][2]} first start->last end="
                      f"{spans[tu][s][0] / args.steps:8.2f} us  mean workgroup lifetime={spans[tu][s][1] / args.steps:8.2f} us")
    enc.close()


if __name__ == "__main__":
    main()
