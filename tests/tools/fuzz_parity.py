"""Long seeded parity sweep (GPU; not part of the pytest suite): random images
across the option space, each JPEG byte-compared with the oracle.  Extends
tests/test_gpu_parity.py::test_seeded_random_sweep with larger sizes, Image<f32>
dots, batches of mixed geometry and pipelined device encodes.
  python tests/tools/fuzz_parity.py --cases 5000 --seed 1 [--minutes 5]
Prints one JSON line per 250 cases and a summary line; exits 1 on the first
mismatch (the failing case's parameters in the line)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmmt-jpeg-encoder_amd")]
import dmmt_jpeg  # noqa: E402
import oracle  # noqa: E402  (checker)


def image(rng, h, w, maxval):
    kind = int(rng.integers(0, 5))
    if kind == 0:
        px = rng.integers(0, maxval + 1, (h, w, 3))
    elif kind == 1:
        yy, xx = np.mgrid[0:h, 0:w]
        px = ((np.stack([xx, yy, xx + yy], -1) * maxval) // max(w + h, 1)) % (maxval + 1)
    elif kind == 2:
        px = np.full((h, w, 3), int(rng.integers(0, maxval + 1)))
    elif kind == 3:
        px = np.where(rng.random((h, w, 3)) < 0.02, rng.integers(0, maxval + 1, (h, w, 3)), 0)
    else:  # smooth base + small noise (natural-image-like statistics)
        yy, xx = np.mgrid[0:h, 0:w]
        base = (np.sin(xx / 17.0)[..., None] * np.cos(yy / 23.0)[..., None] * np.array([1.0, 0.7, 0.4]) + 1) / 2
        px = np.clip(base * maxval + rng.integers(-3, 4, (h, w, 3)), 0, maxval).astype(np.int64)
    return px.astype(np.uint8 if maxval < 256 else np.uint16), kind


def opts(sub, luma, chroma, ri):
    o = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(sub), 8, luma_table=luma,
                                            chroma_table=chroma)
    o.restart_interval = ri
    return o


def run(cases: int, seed: int, max_side: int = 1200, minutes: float = 0, log=print):
    """The sweep; returns its summary dict, or the failing case's parameters under
    "mismatch" (tests/test_gpu_fuzz.py runs a short one in the GPU suite)."""
    args = argparse.Namespace(cases=cases, seed=seed, max_side=max_side, minutes=minutes)
    rng = np.random.default_rng(args.seed)
    enc = dmmt_jpeg.Encoder(0)
    t0 = time.time()
    stats = {"single": 0, "f32": 0, "batch_images": 0, "device": 0, "pixels": 0}
    done = 0
    for case in range(args.cases):
        if args.minutes and time.time() - t0 > 60 * args.minutes:
            break
        h = int(rng.integers(1, args.max_side + 1)) if rng.random() < 0.3 else int(rng.integers(1, 129))
        w = int(rng.integers(1, args.max_side + 1)) if rng.random() < 0.3 else int(rng.integers(1, 129))
        sub = int(rng.integers(0, 3))
        q = int(rng.integers(1, 101))
        maxval = int(rng.choice([255, 255, int(rng.integers(1, 256)), int(rng.integers(256, 65536))]))
        ri = 0 if rng.random() < 0.6 else int(rng.integers(1, 65))
        luma, chroma = dmmt_jpeg.quality_tables(q)
        o = opts(sub, luma, chroma, ri)
        mode = int(rng.integers(0, 4))
        params = dict(case=case, h=h, w=w, sub=sub, q=q, maxval=maxval, ri=ri, mode=mode)
        if mode == 0:  # one image through dmmt_jpeg_encode
            rgb, params["kind"] = image(rng, h, w, maxval)
            ok = enc.encode(dmmt_jpeg.Image.from_array(rgb, maxval), o) == \
                oracle.encode(rgb, maxval, sub, luma, chroma, restart_interval=ri)
            stats["single"] += 1
            stats["pixels"] += h * w
        elif mode == 1:  # Image<f32> dots (sample_bytes 4), as JpegImageWriter receives them
            rgb, params["kind"] = image(rng, h, w, maxval)
            f32 = rgb.astype(np.float32) / np.float32(maxval)
            ok = enc.encode(dmmt_jpeg.Image.from_array(f32, maxval), o) == \
                oracle.encode(rgb, maxval, sub, luma, chroma, restart_interval=ri)
            stats["f32"] += 1
            stats["pixels"] += h * w
        elif mode == 2:  # a batch of mixed geometry (equal sizes share launches)
            n = int(rng.integers(2, 7))
            imgs = []
            for i in range(n):
                hh, ww = (h, w) if rng.random() < 0.5 else (int(rng.integers(1, 129)), int(rng.integers(1, 129)))
                imgs.append(image(rng, hh, ww, maxval)[0])
            outs = enc.encode_batch([dmmt_jpeg.Image.from_array(a, maxval) for a in imgs], o)
            ok = all(out == oracle.encode(a, maxval, sub, luma, chroma, restart_interval=ri)
                     for a, out in zip(imgs, outs))
            stats["batch_images"] += n
            stats["pixels"] += sum(a.shape[0] * a.shape[1] for a in imgs)
        else:  # frames in HBM, pipelined over lanes
            rgb, params["kind"] = image(rng, h, w, maxval)
            lanes = int(rng.integers(1, 5))
            nf = int(rng.integers(1, 4))
            frames = np.stack([rgb] * nf)
            sb = rgb.dtype.itemsize
            cap = (dmmt_jpeg.max_jpeg_bytes(w, h, sub) + 255) // 256 * 256
            d_in = enc.malloc(frames.nbytes)
            enc.h2d(d_in, frames)
            enc.set_lanes(lanes)
            outs = []
            for rep in range(lanes):  # the same frames on every lane, concurrently
                d_out, d_len = enc.malloc(cap * nf), enc.malloc(4 * nf)
                enc.encode_device(d_in, nf, w, h, o, d_out, cap, d_len, maxval=maxval, sample_bytes=sb)
                outs.append((d_out, d_len))
            enc.synchronize()
            ref = oracle.encode(rgb, maxval, sub, luma, chroma, restart_interval=ri)
            ok = True
            for d_out, d_len in outs:
                lens = np.frombuffer(enc.d2h(d_len, 4 * nf), np.uint32)
                for f in range(nf):
                    ok &= enc.d2h(d_out + f * cap, int(lens[f])) == ref
                enc.free(d_out)
                enc.free(d_len)
            enc.free(d_in)
            enc.set_lanes(1)
            stats["device"] += lanes * nf
            stats["pixels"] += lanes * nf * h * w
        if not ok:
            enc.close()
            return {"mismatch": params}
        done += 1
        if done % 250 == 0:
            log(json.dumps({"cases": done, "seconds": round(time.time() - t0, 1), **stats}))
    enc.close()
    return {"summary": "every JPEG byte-identical to the oracle", "cases": done, "seed": args.seed,
            "seconds": round(time.time() - t0, 1), **stats}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=5000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--minutes", type=float, default=0, help="stop early after this long (0 = no limit)")
    ap.add_argument("--max-side", type=int, default=1200)
    a = ap.parse_args()
    res = run(a.cases, a.seed, a.max_side, a.minutes, log=lambda line: print(line, flush=True))
    print(json.dumps(res), flush=True)
    sys.exit(1 if "mismatch" in res else 0)


if __name__ == "__main__":
    main()
