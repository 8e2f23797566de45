"""Benchmark of the gfx950 baseline-JPEG encode path (BASELINE.json metric).

One step = one pass of the whole encode path (pixels in HBM -> complete JPEG
file in HBM: colour, subsampling, Arai DCT, quantisation, symbols, Huffman
tables, bit packing, byte stuffing, headers) over one batch of synthetic frames.
At N=1 the workload is BASELINE config 2: one 3840x2160 frame, 4:4:4, IJG
quality 90.  With N GPUs every rank encodes its own frames (independent
images: weak scaling, no data-path collective); the driver launches one process
per GPU via torch.distributed.run, and `--gpus N` without a launcher spawns the
N rank processes itself (before anything touches a GPU).

Prints ONE JSON line on rank 0.  `value` comes from the timed region: the
production path, every call launched directly (four kernels per frame: k_front,
k_hist with the fused tables, k_emit with the fused offsets, k_stuffwrite),
consecutive frames pipelined over the context's lanes, after an untimed settle
phase of the same steps (--settle-ms, profiles/r06_settle_study.txt), the input frames rotating
over enough distinct slots (> 256 MiB together) that their pixels stream from
HBM rather than the 256 MiB Infinity Cache.  `roofline` comes from a second
pass over the same steps, one frame at a time, with HIP events around every
kernel launch, recorded on the stream the kernel runs on: per kernel the average
launch duration, the SURVEY.md 8(d) algorithmic bytes over it, and the PMC
traffic from profiles/; the dominant (longest) kernel is the headline.
`rocprofv3 --kernel-trace` of this command times the same dispatches:
scripts/kstats_passes.py splits its trace into the settle phase and the two
passes (profiles/r06_v01_kernel_passes.csv).
`cpu_baseline` times the CPU restatement of the reference encoder (oracle/, C,
the reference's DCT thread-pool structure) on a bounded sample of the same
workload on this host.
`extra_configs` (on by default; `--no-extras` skips it) measures, after the
headline and on every rank, the BASELINE configs that shard over the GPUs: config
4 (one 32768x32768 image as MCU-row stripes, with and without restart intervals,
strong scaling) and config 5 (a stream of 8K 4:2:0 frames at q50/75/95, weak
scaling), each with its own per-rank block -- so the one `--gpus N` run the
driver makes per N covers configs 2, 4 and 5.
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before the library: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import dmmt_jpeg  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
MALL_BYTES = 256 << 20  # Infinity Cache (MI355X_MICROARCH.md): inputs beyond it stream from HBM
# f32 VALU issue rate measured on MI355X by tools/pk_rate.hip: 64.2 T lane-ops/s of
# independent v_add_f32 = 1.003 T wave64 instructions/s over the chip
VALU_PEAK_PER_S = 1.003e12
KERNELS = {"front": "k_front", "hist": "k_hist", "tables": "k_tables", "emit": "k_emit", "offsets": "k_offsets",
           "stuffwrite": "k_stuffwrite"}

CONFIGS = {
    # name: (width, height, subsampling, quality, frames per step)
    "4k444q90": (3840, 2160, 0, 90, 1),
    "1080p420q75x256": (1920, 1080, 2, 75, 256),
    "8k420q50": (7680, 4320, 2, 50, 1),   # BASELINE config 5 quality sweep (q50 = the Specification tables)
    "8k420q75": (7680, 4320, 2, 75, 1),
    "8k420q95": (7680, 4320, 2, 95, 1),
}


# one image over all ranks as MCU-row stripes (BASELINE config 4):
# name: (width, height, subsampling, quality, MCU rows per restart interval; 0 = none, joined stripes)
STRIPED = {
    "32k420r": (32768, 32768, 2, 75, 1),
    "32k420": (32768, 32768, 2, 75, 0),
}


def run_striped(args, world, rank, local_rank, make_encoder, barrier_sync, xgroup=None):
    """BASELINE config 4: one 32768x32768 image, MCU-row stripes (one per rank).
    "32k420r": a restart interval of one MCU row; per step every rank runs
    dmmt_stripe_analyze, the 544-counter histogram all-reduce, dmmt_stripe_encode
    and the all-gather of the stripe sizes (dmmt_jpeg.encode_striped).  "32k420":
    no restart intervals (the reference's own stream, joined stripes): analyze,
    edge-DC all-gather, histogram all-reduce, measure, (bits, head) all-gather,
    write.  Total work is fixed: scaling "strong"; value = image pixels / MAX
    elapsed.  The small exchanges run over `xgroup` (bench: a gloo group of CPU
    tensors, the host reduction of SURVEY.md 8(e); None = the default group).
    Returns rank 0's line (None on the other ranks)."""
    w, h, sub, quality, rpi = STRIPED[args.config]
    mcu_w, mcu_h = (8, 8) if sub == 0 else ((16, 8) if sub == 1 else (16, 16))
    mcux, mcuy = -(-w // mcu_w), -(-h // mcu_h)
    luma, chroma = dmmt_jpeg.quality_tables(quality)
    opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                               chroma_table=chroma, restart_interval=mcux * rpi)
    enc = make_encoder(local_rank)
    row0, rows = dmmt_jpeg.stripe_rows(mcuy, world, rank, max(rpi, 1))
    y0, y1 = row0 * mcu_h, min((row0 + rows) * mcu_h, h)
    d_in = enc.malloc(w * (y1 - y0) * 3)
    enc.fill_synthetic_rows(d_in, w, h, y0, y1 - y0, frame=0)
    st = enc.stripe(d_in, w, h, row0, rows)
    cap = enc.stripe_max_bytes(st, opts)
    gather = world > 1 and args.gather
    if gather:  # a torch buffer: its bytes go to rank 0's file over RCCL (gather_striped)
        out_t = torch.empty(cap, dtype=torch.uint8, device=torch.device("cuda", local_rank))
        d_out = out_t.data_ptr()
    else:
        d_out = enc.malloc(cap)
    if world == 1 and rpi == 0:
        def step():
            hist = enc.stripe_analyze(st, opts)
            enc.stripe_measure(hist, [0, 0, 0], d_out, cap)
            return enc.stripe_write(0, 0, 0), 0, None
    elif world == 1:
        def step():
            hist = enc.stripe_analyze(st, opts)
            return enc.stripe_encode(hist, d_out, cap), 0, None
    elif gather:
        def step():
            n, off, total = dmmt_jpeg.encode_striped(enc, st, opts, d_out, cap, group=xgroup)
            dmmt_jpeg.gather_striped(out_t, n, off, total, root=0)
            return n, off, total
    else:
        def step():
            return dmmt_jpeg.encode_striped(enc, st, opts, d_out, cap, group=xgroup)
    for _ in range(args.warmup):
        step()
    barrier_sync(enc)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n, off, total = step()
    barrier_sync(enc)
    elapsed = time.perf_counter() - t0
    # (strong scaling: each rank's rate is its stripe's pixels over its own time)
    elapsed, ranks = gather_ranks(elapsed, world, enc, w * (y1 - y0) * args.steps)
    line = None
    if rank == 0:
        cpu = None
        if args.cpu_seconds > 0:  # the oracle on a bounded stripe of the same image (256 pixel rows)
            from oracle.synth import synthetic
            sample = synthetic(w, 256, frame=0)
            cpu = cpu_baseline(sample, sub, luma, chroma, args.cpu_seconds)
            cpu["sample"] = cpu["sample"].replace("frame(s) of the same synthetic workload",
                                                  "pixel rows (the top stripe pattern) of the same synthetic image")
        line = {
            "metric": f"Mpixel/s encoded ({args.config}: one {w}x{h} image over {world} GPU(s))",
            "value": round(w * h * args.steps / elapsed / 1e6, 2),
            "unit": "Mpixel/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{w}x{h} synthetic RGB u8, {['4:4:4', '4:2:2', '4:2:0'][sub]}, IJG quality {quality}, "
                            + (f"restart interval {mcux * rpi} MCUs, one MCU-row stripe per GPU, pixels in HBM -> "
                               f"stripe bytes in HBM (histogram all-reduce + size all-gather per step)" if rpi else
                               "no restart intervals (the reference's stream), one MCU-row stripe per GPU joined "
                               "mid-byte, pixels in HBM -> stripe bytes in HBM (edge-DC all-gather, histogram "
                               "all-reduce, bit-count all-gather, size all-gather per step)")
                            + (f"; exchanges over {dist.get_backend(xgroup)}" if world > 1 else "")
                            + ("; the stripes then sent to one file in rank 0's HBM (gather_striped)" if gather else ""),
                "width": w, "height": h, "subsampling": ["P444", "P422", "P420"][sub], "quality": quality,
                "restart_interval": mcux * rpi, "parallelism": f"MCU-row stripes x{world}",
                "jpeg_bytes": int(total) if total is not None else int(n),
                "ranks": ranks,
            },
            "roofline": None,
            "cpu_baseline": cpu,
        }
    enc.free(d_in)
    if not gather:
        enc.free(d_out)
    enc.close()
    return line


def run_frame_stream(args, config, world, rank, enc, barrier_sync, steps, warmup):
    """A stream of independent frames of `config` per rank (BASELINE config 5: 8K
    4:2:0 at one quality), pipelined over the lanes, every rank its own distinct
    frames: weak scaling, value = all ranks' pixels / MAX elapsed.  The lean form of
    the headline measurement (no roofline pass) for extra_configs."""
    w, h, sub, quality, fps = CONFIGS[config]
    luma, chroma = dmmt_jpeg.quality_tables(quality)
    opt_c = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                                chroma_table=chroma).to_c()
    frame_bytes = w * h * 3 * fps
    nslots = max(4, MALL_BYTES // frame_bytes + 2)
    out_stride = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
    lanes = max(1, args.lanes)
    d_in = [enc.malloc(frame_bytes) for _ in range(nslots)]
    d_out = [enc.malloc(out_stride * fps) for _ in range(lanes)]
    d_len = [enc.malloc(4 * fps) for _ in range(lanes)]
    try:
        for s in range(nslots):
            enc.fill_synthetic(d_in[s], w, h, fps, first_frame=1000 + (rank * nslots + s) * fps)
        enc.set_lanes(lanes)
        for i in range(warmup):
            enc.encode_device(d_in[i % nslots], fps, w, h, None, d_out[i % lanes], out_stride, d_len[i % lanes],
                              frame_stride=w * h * 3, opt_c=opt_c)
        barrier_sync(enc)
        t0 = time.perf_counter()
        for i in range(steps):
            enc.encode_device(d_in[i % nslots], fps, w, h, None, d_out[i % lanes], out_stride, d_len[i % lanes],
                              frame_stride=w * h * 3, opt_c=opt_c)
        barrier_sync(enc)
        elapsed = time.perf_counter() - t0
        elapsed, ranks = gather_ranks(elapsed, world, enc, w * h * fps * steps)
        lens = np.frombuffer(enc.d2h(d_len[0], 4 * fps), np.uint32)
    finally:
        for p in d_in + d_out + d_len:
            enc.free(p)
    if rank != 0:
        return None
    return {
        "metric": f"Mpixel/s encoded ({config})", "value": round(w * h * fps * steps * world / elapsed / 1e6, 2),
        "unit": "Mpixel/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4), "scaling": "weak",
        "config": {"workload": f"{w}x{h} synthetic RGB u8, {['4:4:4', '4:2:2', '4:2:0'][sub]}, IJG quality {quality}, "
                               f"{fps} frame(s) per step per GPU, pixels in HBM -> JPEG files in HBM, {lanes} lanes, "
                               f"{nslots} input slots",
                   "quality": quality, "mean_jpeg_bytes": float(lens.mean()), "lanes": lanes, "ranks": ranks},
    }


# the BASELINE configs that shard, measured after the headline (extra_configs):
# config 4 in both stripe modes (strong scaling), config 5's quality sweep (weak)
EXTRA_STRIPED = ("32k420r", "32k420")
EXTRA_STREAM = ("8k420q50", "8k420q75", "8k420q95")


def run_extras(args, world, rank, local_rank, make_encoder, enc, barrier_sync, xgroup):
    """extra_configs: every rank runs each config in turn (the same order on every
    rank); a config that raises is recorded with its error and the rest still run"""
    out = {}
    sargs = argparse.Namespace(**vars(args))
    sargs.steps, sargs.warmup, sargs.cpu_seconds, sargs.gather = args.extra_steps, 2, 0, False
    for name in EXTRA_STRIPED:
        sargs.config = name
        try:
            line = run_striped(sargs, world, rank, local_rank, make_encoder, barrier_sync, xgroup)
        except Exception as e:  # noqa: BLE001 -- reported in the line; the next config still runs
            line = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            out[name] = line
    for name in EXTRA_STREAM:
        try:
            line = run_frame_stream(args, name, world, rank, enc, barrier_sync, 4 * args.extra_steps, 5)
        except Exception as e:  # noqa: BLE001
            line = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            out[name] = line
    return out


def gather_ranks(elapsed, world, enc, pixels_per_rank):
    """every rank's own timed region and GPU, gathered on every rank, so that the
    line validates itself: the reported elapsed is their MAX, each rank's own rate
    is listed, and each rank names the device its context runs on (checked by
    dmmt_ctx_check_device: the thread's device and every pooled buffer on it)"""
    device = int(enc.check_device())
    secs, devs, backend = [elapsed], [device], None
    if world > 1:
        backend = dist.get_backend()
        t = torch.tensor([elapsed, float(device)], dtype=torch.float64,
                         device=torch.device("cuda", device) if backend == "nccl" else "cpu")
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        secs = [float(x[0].item()) for x in out]
        devs = [int(x[1].item()) for x in out]
    info = {"world_size": world, "backend": backend, "seconds": [round(x, 6) for x in secs],
            "mpixel_s": [round(pixels_per_rank / x / 1e6, 2) for x in secs], "devices": devs,
            "one_device_per_rank": len(set(devs)) == world}
    return max(secs), info


def run_inproc(args, emit, make_group):
    """`--inproc`: the multi-GPU path a caller of the C ABI uses (one process, no
    torch.distributed): dmmt_ctx_create_multi over the device ids, every member
    with its own input frames in its own HBM, each step one dmmt_encode_device_multi
    call that enqueues one batch of frames per member (frames round-robin over the
    GPUs, the reference's thread-pool fan-out of lib.rs:62 / cosine_transform.rs:
    55-73 turned into one host thread per GPU).  Independent frames: weak scaling,
    value = all members' pixels / elapsed."""
    ids = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
    w, h, sub, quality, fps = CONFIGS[args.config]
    luma, chroma = dmmt_jpeg.quality_tables(quality)
    opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                               chroma_table=chroma)
    grp = make_group(ids)
    n = grp.num_devices()
    mem = [grp.member_encoder(i) for i in range(n)]
    frame_bytes = w * h * 3
    slot_bytes = frame_bytes * fps
    # per member enough distinct input slots to stream past its device's Infinity
    # Cache (members sharing one GPU share it: the same count per GPU in total)
    per_dev = {d: ids.count(d) for d in ids}
    nslots = args.distinct_frames if args.distinct_frames > 0 else max(
        2, -(-(MALL_BYTES // slot_bytes + 2) // max(per_dev.values())))
    out_stride = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
    lanes = max(1, args.lanes)
    bufs = []
    for i, m in enumerate(mem):
        d_in = [m.malloc(slot_bytes) for _ in range(nslots)]
        d_out = [m.malloc(out_stride * fps) for _ in range(lanes)]
        d_len = [m.malloc(4 * fps) for _ in range(lanes)]
        for k in range(nslots):
            m.fill_synthetic(d_in[k], w, h, fps, first_frame=(i * nslots + k) * fps)
        bufs.append((d_in, d_out, d_len))

    def frames(step):
        fs = []
        for d_in, d_out, d_len in bufs:
            f = dmmt_jpeg.DmmtDeviceFrames()
            f.d_rgb, f.frame_stride, f.n_frames = d_in[step % nslots], frame_bytes, fps
            f.width, f.height, f.maxval, f.sample_bytes = w, h, 255, 1
            f.d_out, f.out_stride, f.d_out_len = d_out[step % lanes], out_stride, d_len[step % lanes]
            fs.append(f)
        return fs

    grp.set_lanes(lanes)
    for i in range(args.warmup):
        grp.encode_device_multi(frames(i), opts)
    grp.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        grp.encode_device_multi(frames(i), opts)
    grp.synchronize()
    elapsed = time.perf_counter() - t0
    lens = np.frombuffer(mem[0].d2h(bufs[0][2][0], 4 * fps), np.uint32)
    ngpu = len(set(ids))
    value = n * w * h * fps * args.steps / elapsed / 1e6
    line = {
        "metric": "Mpixel/s encoded (4K PPM, q=90)" if args.config == "4k444q90" else f"Mpixel/s encoded ({args.config})",
        "value": round(value, 2), "unit": "Mpixel/s", "n_gpus": ngpu, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {
            "workload": f"{w}x{h} synthetic RGB u8, {['4:4:4', '4:2:2', '4:2:0'][sub]}, IJG quality {quality}, "
                        f"{fps} frame(s) per step per member, pixels in HBM -> JPEG files in HBM, one process: "
                        f"dmmt_ctx_create_multi({ids}), one dmmt_encode_device_multi call per step",
            "width": w, "height": h, "subsampling": ["P444", "P422", "P420"][sub], "quality": quality,
            "frames_per_step": fps * n, "members": n, "device_ids": ids, "mean_jpeg_bytes": float(lens.mean()),
            "parallelism": f"independent frames x{n} members on {ngpu} GPU(s), in-process C-ABI group",
            "lanes": lanes, "input_slots_per_member": nslots,
        },
        "roofline": None, "cpu_baseline": None,
    }
    emit(json.dumps(line))
    for m, (d_in, d_out, d_len) in zip(mem, bufs):
        for p in d_in + d_out + d_len:
            m.free(p)
    grp.close()


def p3_bytes(rgb, maxval=255, sep=b" "):
    """a P3 file of an (h, w, 3) uint8 image, built vectorised: every sample in decimal
    followed by one separator byte (the ingest workload of --ppm and its tests)"""
    h, w, _ = rgb.shape
    v = np.asarray(rgb, np.int64).reshape(-1)
    nd = 1 + (v >= 10) + (v >= 100)
    end = np.cumsum(nd + 1)  # one past each token's separator
    body = np.full(int(end[-1]) if v.size else 0, sep[0], np.uint8)
    last = end - 2           # each token's last digit
    body[last] = 48 + v % 10
    m = nd >= 2
    body[last[m] - 1] = 48 + (v[m] // 10) % 10
    m = nd >= 3
    body[last[m] - 2] = 48 + v[m] // 100
    return b"P3\n%d %d\n%d\n" % (w, h, maxval) + body.tobytes()


def _p3_in_hbm(enc, w, h):
    """one w x h frame of the synthetic workload as a P3 file in HBM: (rgb, text,
    header, d_text, d_rgb)"""
    d_rgb = enc.malloc(w * h * 3)
    enc.fill_synthetic(d_rgb, w, h, 1)
    enc.synchronize()
    rgb = np.frombuffer(enc.d2h(d_rgb, w * h * 3), np.uint8).reshape(h, w, 3)
    text = p3_bytes(rgb)
    hdr = dmmt_jpeg.parse_ppm_header(text)
    d_text = enc.malloc(len(text))
    enc.h2d(d_text, np.frombuffer(text, np.uint8))
    return rgb, text, hdr, d_text, d_rgb


def ppm_ingest(enc, w, h, steps):
    """SURVEY.md 8(f) row 1, timed apart from the encode (8(d)): one w x h frame of
    the synthetic workload as a P3 file (one space after every sample) in HBM ->
    its u8 samples in HBM, dmmt_decode_ppm_device per step (which synchronises).
    Algorithmic bytes: the file read once + the samples written once."""
    rgb, text, hdr, d_text, d_rgb = _p3_in_hbm(enc, w, h)
    for _ in range(3):
        enc.decode_ppm_device(d_text, len(text), hdr, d_rgb)
    t0 = time.perf_counter()
    for _ in range(steps):
        enc.decode_ppm_device(d_text, len(text), hdr, d_rgb)
    dt = (time.perf_counter() - t0) / steps
    ok = bytes(enc.d2h(d_rgb, w * h * 3)) == rgb.tobytes()
    enc.free(d_text)
    enc.free(d_rgb)
    algo = len(text) + w * h * 3
    return {"workload": f"{w}x{h} P3 text ({len(text)} B) in HBM -> u8 samples in HBM, per call incl. its sync",
            "ms": round(dt * 1e3, 4), "mpixel_per_s": round(w * h / dt / 1e6, 1),
            "achieved_gbs": round(algo / dt / 1e9, 1), "frac": round(algo / dt / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes": algo, "samples_match": ok}


def ppm_to_jpeg(enc, w, h, opts, opt_c, steps):
    """The reference's product path (convert_ppm_to_jpeg, lib.rs:59-77) minus the
    file I/O: one w x h synthetic frame as P3 text in HBM -> its JPEG file in HBM,
    one file at a time -- dmmt_decode_ppm_device (which synchronises to read its
    report), then dmmt_encode_device and a synchronisation.  Algorithmic bytes: the
    text read once + the JPEG written once."""
    rgb, text, hdr, d_text, d_rgb = _p3_in_hbm(enc, w, h)
    cap = (dmmt_jpeg.max_jpeg_bytes(w, h, int(opts.chroma_subsampling_preset)) + 255) // 256 * 256
    d_out, d_len = enc.malloc(cap), enc.malloc(4)
    enc.set_lanes(1)

    def one():
        enc.decode_ppm_device(d_text, len(text), hdr, d_rgb)
        enc.encode_device(d_rgb, 1, w, h, None, d_out, cap, d_len, frame_stride=w * h * 3, opt_c=opt_c)
        enc.synchronize()
    for _ in range(3):
        one()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    dt = (time.perf_counter() - t0) / steps
    n = int(np.frombuffer(enc.d2h(d_len, 4), np.uint32)[0])
    for p in (d_text, d_rgb, d_out, d_len):
        enc.free(p)
    algo = len(text) + n
    return {"workload": f"{w}x{h} P3 text ({len(text)} B) in HBM -> JPEG file ({n} B) in HBM, one file at a time "
                        f"(decode_ppm_device + encode_device + synchronize per file)",
            "ms": round(dt * 1e3, 4), "mpixel_per_s": round(w * h / dt / 1e6, 1),
            "achieved_gbs": round(algo / dt / 1e9, 1), "frac": round(algo / dt / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes": algo}


def ppm_to_jpeg_stream(enc, w, h, opt_c, steps, lanes, distinct=3, per_call=12):
    """The same path for a stream of files (dmmt_convert_ppm_device_batch, the
    extension for serving): per call `per_call` files of w x h P3 text already in
    HBM -> their JPEG files in HBM, decoded and encoded back to back over `lanes`
    lanes with no synchronisation between files (the comment-free decode is checked
    after the call).  The files rotate over `distinct` different frames' texts (3 x
    90 MB at 4K: more than the 256 MB Infinity Cache).  Algorithmic bytes per file:
    the text read once + the JPEG written once."""
    texts = []
    for k in range(distinct):
        d_rgb = enc.malloc(w * h * 3)
        enc.fill_synthetic(d_rgb, w, h, 1, first_frame=100 + k)
        enc.synchronize()
        rgb = np.frombuffer(enc.d2h(d_rgb, w * h * 3), np.uint8).reshape(h, w, 3)
        enc.free(d_rgb)
        text = p3_bytes(rgb)
        d_text = enc.malloc(len(text))
        enc.h2d(d_text, np.frombuffer(text, np.uint8))
        texts.append((d_text, len(text), dmmt_jpeg.parse_ppm_header(text)))
    cap = (dmmt_jpeg.max_jpeg_bytes(w, h, opt_c.subsampling) + 255) // 256 * 256
    outs = [(enc.malloc(cap), enc.malloc(4)) for _ in range(per_call)]
    files = [(texts[i % distinct][0], texts[i % distinct][1], texts[i % distinct][2], outs[i][0], cap, outs[i][1])
             for i in range(per_call)]
    enc.set_lanes(lanes)
    try:
        for _ in range(2):
            enc.convert_ppm_device_batch(files, opt_c=opt_c)
        t0 = time.perf_counter()
        for _ in range(steps):
            enc.convert_ppm_device_batch(files, opt_c=opt_c)
        dt = (time.perf_counter() - t0) / (steps * per_call)
        sizes = [int(np.frombuffer(enc.d2h(d_len, 4), np.uint32)[0]) for _, d_len in outs]
    finally:
        enc.set_lanes(1)
        for d_out, d_len in outs:
            enc.free(d_out)
            enc.free(d_len)
        for d_text, _, _ in texts:
            enc.free(d_text)
    algo = sum(t[1] for t in texts) / distinct + sum(sizes) / len(sizes)
    return {"workload": f"{w}x{h} P3 texts ({distinct} distinct, {texts[0][1]} B) in HBM -> JPEG files in HBM, "
                        f"{per_call} files per dmmt_convert_ppm_device_batch call over {lanes} lanes",
            "ms_per_file": round(dt * 1e3, 4), "mpixel_per_s": round(w * h / dt / 1e6, 1),
            "achieved_gbs": round(algo / dt / 1e9, 1), "frac": round(algo / dt / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_file": round(algo)}


def available_parallelism():
    """std::thread::available_parallelism() as the reference's CLI default uses it
    (cli.rs:104-109): the CPUs this process may run on, capped by a cgroup CPU
    quota.  Returns (that count, nproc, cgroup quota or None)."""
    nproc = os.cpu_count() or 1
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - not Linux
        n = nproc
    quota = None
    try:  # cgroup v2
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(p))
    except (OSError, ValueError):
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // p)
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, quota)
    return max(1, n), nproc, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# the GPU box's CPU share per GPU: worker pools are sized to it (its nproc shows the
# whole machine)
BOX_CPU_SHARE = 16


def cpu_baseline(rgb, sub, luma, chroma, budget_s):
    """Oracle (C restatement, DCT on a thread pool like transformer.rs:126-148) on this
    host, with the reference's default thread count (available_parallelism,
    cli.rs:104-109), at most the GPU box's CPU share."""
    import oracle
    avail, nproc, quota = available_parallelism()
    threads = min(avail, BOX_CPU_SHARE)
    oracle.encode(rgb[:64, :64], 255, sub, luma, chroma)  # load/build
    n = 0
    t0 = time.perf_counter()
    while True:
        oracle.encode(rgb, 255, sub, luma, chroma, threads=threads)
        n += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    h, w = rgb.shape[:2]
    return {"value": round(n * w * h / dt / 1e6, 3), "unit": "Mpixel/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "nproc": nproc, "available_parallelism": avail, "cgroup_cpu_quota": quota,
            "sample": f"{n} x {w}x{h} frame(s) of the same synthetic workload, {dt:.1f} s, oracle/cpu_ref.c "
                      f"(C restatement of the reference encoder; DCT on {threads} threads in 700-block jobs, "
                      f"other stages serial, as transformer.rs:126-148; threads = available_parallelism "
                      f"(the reference's -t default) capped at the box's {BOX_CPU_SHARE}-CPU share)"}


def _spawned_rank(rank, argv, world, port, make_encoder, out_dir):
    """one rank of `bench.py --gpus N` started without a launcher (spawned, so
    nothing of the parent's process state -- and no GPU -- is inherited)"""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    lines = []
    main(argv, make_encoder=make_encoder, emit=lines.append)
    if lines:
        with open(os.path.join(out_dir, f"rank{rank}.jsonl"), "w") as f:
            f.write("\n".join(lines) + "\n")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(argv, n, make_encoder, emit):
    """`--gpus N` with no WORLD_SIZE: start N rank processes (spawn, one per GPU,
    rendezvous on 127.0.0.1) and emit rank 0's line.  Called before anything here
    has touched a GPU."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_spawned_rank, args=(argv, n, _free_port(), make_encoder, d), nprocs=n,
                           start_method="spawn")
        p = os.path.join(d, "rank0.jsonl")
        if not os.path.exists(p):
            raise SystemExit("bench: rank 0 printed no line")
        for line in open(p).read().splitlines():
            emit(line)


def kernel_roofline(prof, algo_bytes, frames_per_launch, pmc):
    """per kernel: average launch duration (HIP events on its stream), the SURVEY
    8(d) algorithmic bytes of the frames one launch processes over it, and the PMC
    traffic / instruction counts of profiles/pmc_<config>.json"""
    out = {}
    for stage, name in KERNELS.items():
        ms, n = prof.get(stage, (0.0, 0))
        if not n:
            continue
        avg_s = ms / 1e3 / n
        achieved = algo_bytes / avg_s / 1e9
        k = {"avg_launch_us": round(avg_s * 1e6, 2), "launches": n, "achieved": round(achieved, 1),
             "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None}
        pk = (pmc or {}).get("kernels", {}).get(name)
        if pk:
            if pk.get("hbm_bytes") is not None:
                k["traffic"] = round(pk["hbm_bytes"])
            if pk.get("SQ_INSTS_VALU") is not None:
                k["valu_wave_insts"] = round(pk["SQ_INSTS_VALU"])
                k["valu_frac"] = round(pk["SQ_INSTS_VALU"] / avg_s / VALU_PEAK_PER_S, 4)
            if pk.get("SQ_INSTS_SALU") is not None:
                k["salu_wave_insts"] = round(pk["SQ_INSTS_SALU"])
            if pk.get("SQ_WAIT_ANY") and pk.get("SQ_WAVE_CYCLES"):
                k["parked_frac"] = round(pk["SQ_WAIT_ANY"] / pk["SQ_WAVE_CYCLES"], 3)
        out[name] = k
    return out


def path_roofline(algo_bytes, achieved, step_s, pmc, launched):
    """the whole step against both ceilings: the HBM fraction of the
    step's algorithmic bytes, and the issue ceiling -- the VALU wave-instructions all
    kernels of a step issue (PMC, profiles/pmc_<config>.json) over the step time
    against the measured 1.003 T wave-instructions/s (tools/pk_rate.hip).  `launched`:
    the kernels the step ran (k_offsets only when k_emit did not fuse the offsets)"""
    out = {"algorithmic_bytes_per_step": round(algo_bytes), "achieved": round(achieved, 1),
           "frac": round(achieved / HBM_PEAK_GBS, 4), "valu_wave_insts": None, "salu_wave_insts": None,
           "valu_frac": None}
    ks = {n: k for n, k in (pmc or {}).get("kernels", {}).items() if n in launched}  # the step's kernels
    if launched and len(ks) == len(launched) and all(k.get("SQ_INSTS_VALU") is not None for k in ks.values()):
        valu = sum(k["SQ_INSTS_VALU"] for k in ks.values())
        out["valu_wave_insts"] = round(valu)
        out["valu_frac"] = round(valu / step_s / VALU_PEAK_PER_S, 4)
        if all(k.get("SQ_INSTS_SALU") is not None for k in ks.values()):
            out["salu_wave_insts"] = round(sum(k["SQ_INSTS_SALU"] for k in ks.values()))
        out["valu_frac_def"] = ("sum over the step's kernels of PMC SQ_INSTS_VALU / step time / "
                                f"{VALU_PEAK_PER_S:.4g} wave-instructions/s")
    return out


def main(argv=None, make_encoder=None, emit=None, make_group=None):
    """The bench; `make_encoder(local_rank)`, `make_group(device_ids)` and
    `emit(line)` are test seams (tests/test_bench_dist.py drives the N>1 path with
    gloo on CPU, and the --inproc path with a stand-in group)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="4k444q90", choices=sorted(CONFIGS) + sorted(STRIPED))
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--distinct-frames", type=int, default=0,
                    help="input slots the steps rotate over (0 = enough to exceed the 256 MiB Infinity Cache)")
    ap.add_argument("--mall-compare", action="store_true",
                    help="also time the steps over 4 input slots (inputs resident in the Infinity Cache)")
    ap.add_argument("--ppm-steps", type=int, default=20,
                    help="PPM ingest line: P3 decodes of one synthetic frame timed on rank 0 (0 = skip)")
    ap.add_argument("--gather", action="store_true",
                    help="striped configs, N>1: every step also sends the stripes to one file on rank 0 (RCCL p2p)")
    ap.add_argument("--lanes", type=int, default=4,
                    help="pipeline lanes: consecutive steps overlap on this many workspaces/streams (1 = serial)")
    ap.add_argument("--inproc", action="store_true",
                    help="one process drives all GPUs through the C ABI's multi-GPU context (dmmt_ctx_create_multi)")
    ap.add_argument("--devices", default="",
                    help="--inproc: comma-separated device ids of the members (default 0..gpus-1; repeats allowed)")
    ap.add_argument("--settle-ms", type=float, default=60.0,
                    help="untimed pipelined steps for this long before the warmup steps (0 = from cold)")
    ap.add_argument("--roofline-order", choices=("first", "last"), default="last",
                    help="run the one-lane roofline pass before or after the timed region")
    ap.add_argument("--no-extras", dest="extras", action="store_false",
                    help="skip extra_configs (BASELINE configs 4 and 5 after the headline)")
    ap.add_argument("--extra-steps", type=int, default=5,
                    help="extra_configs: timed steps per striped config (x4 per 8K stream config)")
    ap.add_argument("--exchange", choices=("host", "device"), default="host",
                    help="striped configs, N>1: the small exchanges as CPU tensors over gloo (host) or GPU "
                         "tensors over the main backend (device)")
    ap.add_argument("--same-device", action="store_true",
                    help="N>1 rehearsal on a one-GPU box: every rank on device 0, gloo for the barrier and the "
                         "gather (RCCL refuses two ranks on one GPU); the line says so (ranks.devices)")
    args = ap.parse_args(argv)
    emit = emit or (lambda line: print(line, flush=True))
    if args.inproc:
        if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
            raise SystemExit("bench: --inproc drives every GPU from one process; do not launch it per rank")
        if args.config not in CONFIGS:
            raise SystemExit("bench: --inproc runs the independent-frame configs")
        return run_inproc(args, emit, make_group or (lambda ids: dmmt_jpeg.Encoder(devices=ids)))

    if args.same_device and args.config in STRIPED and args.exchange == "device":
        raise SystemExit("bench: --same-device runs the stripes' exchanges on the host (gloo), not --exchange device")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:  # no launcher: start the ranks here
        return spawn_ranks(list(argv if argv is not None else sys.argv[1:]), args.gpus, make_encoder, emit)
    make_encoder = make_encoder or dmmt_jpeg.Encoder
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # the GPU of this rank (--same-device: all on GPU 0, a rehearsal of the N>1 path)
    local_rank = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a wrong n_gpus")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if torch.cuda.is_available() and not args.same_device else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)
    dev = torch.device("cuda", local_rank) if torch.cuda.is_available() else None

    def barrier_sync(enc):
        if world > 1:
            dist.barrier()
        if dev is not None:
            torch.cuda.synchronize(dev)
        enc.synchronize()

    # the stripes' small exchanges (histograms, edge DCs, bit counts, sizes): CPU
    # tensors over gloo, i.e. a host reduction; --exchange device
    # keeps them on GPU tensors over the main backend (RCCL)
    xgroup = None
    if world > 1 and args.exchange == "host" and dist.get_backend() != "gloo":
        xgroup = dist.new_group(backend="gloo")

    if args.config in STRIPED:
        line = run_striped(args, world, rank, local_rank, make_encoder, barrier_sync, xgroup)
        if rank == 0:
            emit(json.dumps(line))
        if world > 1:
            dist.destroy_process_group()
        return

    w, h, sub, quality, fps = CONFIGS[args.config]
    luma, chroma = dmmt_jpeg.quality_tables(quality)
    opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                               chroma_table=chroma)
    opt_c = opts.to_c()
    enc = make_encoder(local_rank)

    frame_bytes = w * h * 3
    slot_bytes = frame_bytes * fps
    # distinct input slots: enough that between two reads of a slot more than the
    # Infinity Cache's capacity of other frames has streamed past (4K: 13 x 24.9 MB)
    nslots = args.distinct_frames if args.distinct_frames > 0 else max(4, MALL_BYTES // slot_bytes + 2)
    out_stride = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
    lanes = max(1, args.lanes)
    d_in = [enc.malloc(slot_bytes) for _ in range(nslots)]
    d_out = [enc.malloc(out_stride * fps) for _ in range(lanes)]  # one per lane: never shared by concurrent steps
    d_len = [enc.malloc(4 * fps) for _ in range(lanes)]
    for s in range(nslots):  # distinct synthetic frames per slot and per rank
        enc.fill_synthetic(d_in[s], w, h, fps, first_frame=(rank * nslots + s) * fps)

    def step(i, nl, ns):
        enc.encode_device(d_in[i % ns], fps, w, h, None, d_out[i % nl], out_stride, d_len[i % nl],
                          frame_stride=frame_bytes, opt_c=opt_c)

    def timed(nl, ns=nslots):
        enc.set_lanes(nl)
        for i in range(args.warmup):
            step(i, nl, ns)
        barrier_sync(enc)
        barrier_sync(enc)
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i, nl, ns)
        barrier_sync(enc)
        return time.perf_counter() - t0

    # roofline pass: the same steps one at a time (one lane) with HIP events around
    # every kernel launch, on the stream it is launched on: each kernel's own launch
    # duration (pipelined, the kernels of consecutive frames share the CUs and each
    # one's duration is stretched by the others).  --roofline-order first runs it
    # before the timed region (the GPU then enters the timed steps busy, as a
    # serving GPU is, rather than from idle)
    def roofline_pass():
        enc.set_profiling(1)
        t = timed(1)
        p = enc.profile()
        enc.set_profiling(0)
        return t, p
    if args.roofline_order == "first":
        single, prof = roofline_pass()
    # settle: the same pipelined steps, untimed, for --settle-ms of wall time before
    # the W warmup steps.  A fresh process runs its first few hundred 4K frames up to
    # 10 % slower than later ones at unchanged clocks (profiles/r06_settle_study.txt:
    # 162 -> 175 -> 178 Gpx/s over consecutive 200-frame reps); a serving GPU is
    # past that, so the timed steps are measured there.  0: from cold.
    settle_frames, settle_s = 0, 0.0
    if args.settle_ms > 0:
        enc.set_lanes(lanes)
        t_s = time.perf_counter()
        while time.perf_counter() - t_s < args.settle_ms / 1e3:
            for _ in range(32):
                step(settle_frames, lanes, nslots)
                settle_frames += 1
            enc.synchronize()
        settle_s = time.perf_counter() - t_s
    # timed region: the production path (no event timing inside); with lanes > 1
    # consecutive frames are pipelined over the context's lanes (dmmt_ctx_set_lanes)
    elapsed = timed(lanes)
    if args.roofline_order == "last":
        single, prof = roofline_pass()
    # the same one-lane steps without the event records: a frame's latency on the
    # production path (the roofline pass's 8 event records per frame stretch it)
    single_plain = timed(1)
    extra = {}
    if args.mall_compare:  # inputs resident in the Infinity Cache: 4 slots
        extra["mall_resident_4_slots"] = timed(lanes, min(4, nslots))

    elapsed, ranks = gather_ranks(elapsed, world, enc, w * h * fps * args.steps)

    lens = np.frombuffer(enc.d2h(d_len[0], 4 * fps), np.uint32)
    jpeg_bytes = float(lens.mean())

    if rank == 0:
        pixels = w * h * fps * args.steps * world
        value = pixels / elapsed / 1e6
        # the path's algorithmic bytes per frame are 3 B/px of RGB in
        # + the JPEG bytes out; a launch processes `fps` frames
        algo_bytes = fps * (w * h * 3 + jpeg_bytes)
        path_achieved = algo_bytes / (elapsed / args.steps) / 1e9
        pmc = None
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")
        if os.path.exists(pmc_path):
            try:
                pmc = json.load(open(pmc_path))
            except ValueError:
                pmc = None
        kern = kernel_roofline(prof, algo_bytes, fps, pmc)
        if "k_emit" in kern and "k_offsets" not in kern:  # frames of <= 6144 chunks
            kern["k_emit"]["includes"] = "the frame's chunk-offset scans (k_offsets fused into its last workgroup)"
        dom = max(kern, key=lambda k: kern[k]["avg_launch_us"]) if kern else None
        d = kern.get(dom, {})
        ingest = ppm_ingest(enc, w, h, args.ppm_steps) if args.ppm_steps > 0 else None
        ppm_jpeg = ppm_to_jpeg(enc, w, h, opts, opt_c, args.ppm_steps) if args.ppm_steps > 0 and fps == 1 else None
        ppm_stream = (ppm_to_jpeg_stream(enc, w, h, opt_c, max(2, args.ppm_steps // 4), lanes)
                      if args.ppm_steps > 0 and fps == 1 else None)
        # one file per call through the same API: decode and encode back to back,
        # one synchronisation (the report checked after it), one lane
        ppm_one = (ppm_to_jpeg_stream(enc, w, h, opt_c, args.ppm_steps, 1, distinct=1, per_call=1)
                   if args.ppm_steps > 0 and fps == 1 else None)
        cpu = None
        if args.cpu_seconds > 0 and world == 1:  # the CPU baseline is an N=1 figure
            from oracle.synth import synthetic  # numpy twin of the device generator
            rgb = synthetic(w, h, frame=0)
            cpu = cpu_baseline(rgb, sub, luma, chroma, args.cpu_seconds)
        cfg = {
            "workload": f"{w}x{h} synthetic RGB u8, {['4:4:4', '4:2:2', '4:2:0'][sub]}, IJG quality {quality}, "
                        f"{fps} frame(s) per step per GPU, pixels in HBM -> JPEG files in HBM, inputs rotating "
                        f"over {nslots} distinct slots ({nslots * slot_bytes / 2**20:.0f} MiB: streamed from HBM)",
            "width": w, "height": h, "subsampling": ["P444", "P422", "P420"][sub], "quality": quality,
            "frames_per_step": fps, "mean_jpeg_bytes": jpeg_bytes, "parallelism": f"independent frames x{world}",
            "lanes": lanes, "input_slots": nslots, "ranks": ranks,
            "settle": {"ms": round(settle_s * 1e3, 1), "frames": settle_frames * fps,
                       "what": "untimed pipelined steps of the same workload before the warmup steps (--settle-ms)"},
        }
        if "mall_resident_4_slots" in extra:
            t4 = extra["mall_resident_4_slots"]
            cfg["mall_resident_4_slots_value"] = round(pixels / world / t4 / 1e6, 2)
        # the roofline pass's wall time: one frame at a time, events on (the latency of
        # a frame plus the event records)
        cfg["single_lane_ms_per_step"] = round(single / args.steps * 1e3, 4)
        cfg["single_lane_plain_ms_per_step"] = round(single_plain / args.steps * 1e3, 4)
        line = {
            "metric": "Mpixel/s encoded (4K PPM, q=90)" if args.config == "4k444q90" else f"Mpixel/s encoded ({args.config})",
            "value": round(value, 2),
            "unit": "Mpixel/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": cfg,
            "roofline": {
                # bound: the roofline the fraction is priced against (no MFMA work:
                # HBM); what limits the kernels is `limiter`
                "bound": "hbm",
                "limiter": "issue/latency: wave-cycles parked at s_waitcnt/barrier and VALU+SALU issue "
                           "(PMC parked_frac, valu_frac per kernel), not HBM bandwidth",
                "kernel": dom,
                "achieved": d.get("achieved"),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": d.get("frac"),
                "traffic": d.get("traffic"),
                "avg_launch_us": d.get("avg_launch_us"),
                "algorithmic_bytes_per_launch": round(algo_bytes),
                "algorithmic_bytes_def": "SURVEY 8(d): 3 B/px RGB in + JPEG bytes out, per frame, x frames per launch",
                "kernels": kern,
                "path": path_roofline(algo_bytes, path_achieved, elapsed / args.steps, pmc, set(kern)),
                "pmc_source": f"profiles/pmc_{args.config}.json" if pmc else None,
            },
            "cpu_baseline": cpu,
            "ppm_ingest": ingest,
            "ppm_to_jpeg": ppm_jpeg,
            "ppm_to_jpeg_one_call": ppm_one,
            "ppm_to_jpeg_stream": ppm_stream,
        }
    for p in d_in + d_out + d_len:
        enc.free(p)
    if args.extras:  # (every rank: the configs' collectives)
        extras = run_extras(args, world, rank, local_rank, make_encoder, enc, barrier_sync, xgroup)
        if rank == 0:
            line["extra_configs"] = extras
    if rank == 0:
        emit(json.dumps(line))
    enc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
