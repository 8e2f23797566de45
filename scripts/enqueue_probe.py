"""Host enqueue rate against the GPU's frame period (4K q90, the bench's pipelined
steps): how long the host takes to enqueue N frames (dmmt_encode_device through the
Python mirror, no synchronisation) against the time until they have all finished.
If the enqueue time per frame approaches the period, the host bounds the bench.
  python scripts/enqueue_probe.py [--steps 200] [--lanes 4] [--graphs]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process, as bench.py)
import dmmt_jpeg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--lanes", type=int, default=4)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--pre", choices=("onelane", "synthetic"), default="onelane")
    ap.add_argument("--pre-frames", type=int, default=0)
    ap.add_argument("--clocks", action="store_true", help="sample the current sclk level (sysfs pp_dpm_sclk) per rep")
    args = ap.parse_args()
    w, h = args.width, args.height
    luma, chroma = dmmt_jpeg.quality_tables(90)
    opt_c = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(0), 8, luma_table=luma,
                                                chroma_table=chroma).to_c()
    enc = dmmt_jpeg.Encoder(0)
    nslots = 12
    d_in = [enc.malloc(w * h * 3) for _ in range(nslots)]
    cap = (dmmt_jpeg.max_jpeg_bytes(w, h, 0) + 255) // 256 * 256
    d_out = [enc.malloc(cap) for _ in range(args.lanes)]
    d_len = [enc.malloc(4) for _ in range(args.lanes)]
    for s in range(nslots):
        enc.fill_synthetic(d_in[s], w, h, 1, first_frame=s)
    if args.pre_frames:  # a pre-load of another kind before the reps (what warms the path up?)
        if args.pre == "onelane":
            enc.set_lanes(1)
            for i in range(args.pre_frames):
                enc.encode_device(d_in[i % nslots], 1, w, h, None, d_out[0], cap, d_len[0], frame_stride=w * h * 3,
                                  opt_c=opt_c)
        elif args.pre == "synthetic":
            for i in range(args.pre_frames):
                enc.fill_synthetic(d_in[i % nslots], w, h, 1, first_frame=i % nslots)
        enc.synchronize()
    enc.set_lanes(args.lanes)
    res = {}
    import glob
    import threading
    sclk = []
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):  # the GPUs this process sees
        try:
            kv = dict(l.split()[:2] for l in open(props).read().splitlines() if len(l.split()) >= 2)
        except OSError:  # (nodes of GPUs this container does not see)
            continue
        if int(kv.get("simd_count", 0)) > 0 and "drm_render_minor" in kv:
            for clk in ("sclk", "fclk", "mclk", "socclk"):
                f = f"/sys/class/drm/renderD{kv['drm_render_minor']}/device/pp_dpm_{clk}"
                if os.path.exists(f):
                    sclk.append(f)
    samples = []
    stop = threading.Event()

    def sampler():  # the active DPM level line ("N: xxxMhz *") every ~1 ms
        while not stop.is_set():
            lv = []
            for p in sclk:
                try:
                    cur = [l for l in open(p).read().splitlines() if l.endswith("*")]
                    lv.append(p.split("_")[-1] + " " + (cur[0].split(":")[1].strip(" *") if cur else "?"))
                except OSError:
                    pass
            samples.append((time.perf_counter(), ", ".join(lv)))
            time.sleep(0.0005)
    th = threading.Thread(target=sampler, daemon=True)
    if args.clocks and sclk:
        th.start()
    for rep in range(args.reps):
        for i in range(args.warmup):
            enc.encode_device(d_in[i % nslots], 1, w, h, None, d_out[i % args.lanes], cap, d_len[i % args.lanes],
                              frame_stride=w * h * 3, opt_c=opt_c)
        enc.synchronize()
        t0 = time.perf_counter()
        marks = []
        for i in range(args.steps):
            enc.encode_device(d_in[i % nslots], 1, w, h, None, d_out[i % args.lanes], cap, d_len[i % args.lanes],
                              frame_stride=w * h * 3, opt_c=opt_c)
            if i in (0, args.steps // 2 - 1, args.steps - 1):
                marks.append(time.perf_counter() - t0)
        t_enq = time.perf_counter() - t0
        enc.synchronize()
        t_all = time.perf_counter() - t0
        if args.clocks:
            seen = {}
            for t, lv in samples:
                if t0 <= t <= t0 + t_all:
                    seen[lv] = seen.get(lv, 0) + 1
            res[f"rep{rep}_sclk"] = seen
        res[f"rep{rep}"] = {"enqueue_us_per_frame": round(t_enq / args.steps * 1e6, 2),
                            "done_us_per_frame": round(t_all / args.steps * 1e6, 2),
                            "first_call_us": round(marks[0] * 1e6, 1), "gpx_s": round(w * h * args.steps / t_all / 1e9, 2)}
    stop.set()
    print(json.dumps({"clock_files": sclk, "steps": args.steps, "lanes": args.lanes, "graphs": os.environ.get("DMMT_GRAPHS", "0"),
                      **res}))


if __name__ == "__main__":
    main()
