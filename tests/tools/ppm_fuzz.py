"""Long seeded sweep of the PPM ingest on the GPU (not part of the pytest suite):
random P3 files -- 8- and 16-bit, one to three separators of every whitespace
kind, sometimes comments, '+' signs or leading zeros, sometimes a broken token,
a missing or extra sample or a sample above maxval -- decoded by
dmmt_decode_ppm_device with the text and the sample buffer at random
misalignments.  A file the host reader (the reference's tokenizer and parser,
restated in csrc/ppm.cpp) accepts must give exactly the generated samples; any
other file must give the host reader's error code.
  python tests/tools/ppm_fuzz.py --cases 2000 --seed 1 [--minutes 5]
Prints one JSON line per 200 cases and a summary line; exits 1 on the first
mismatch (the failing case's parameters in the line)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"), os.path.join(ROOT, "tests")]
import dmmt_jpeg  # noqa: E402
from test_gpu_ppm import host_code, p3_text  # noqa: E402


def make_file(rng, max_side):
    big = rng.random() < 0.25
    w = int(rng.integers(1, max_side + 1 if big else 80))
    h = int(rng.integers(1, max_side + 1 if big else 60))
    mx = int(rng.choice([255, 255, 255, 9, 100, 1000, 65535]))
    rgb = rng.integers(0, mx + 1, (h, w, 3)).astype(np.uint16)
    if rng.random() < 0.15:  # only short tokens (values below 10 or 100)
        rgb = np.minimum(rgb, int(rng.choice([9, 99])))
    r = rng.random()
    kind = "clean"
    if r < 0.05:
        kind = "over"
        if mx < 65535:
            rgb.reshape(-1)[int(rng.integers(0, rgb.size))] = mx + 1
    data = p3_text(rgb, mx, rng, ws_max=int(rng.integers(1, 4)),
                   comments=0.01 if 0.05 <= r < 0.12 else 0.0, plus=0.01 if 0.12 <= r < 0.18 else 0.0,
                   zeros=0.05 if 0.18 <= r < 0.3 else 0.0)
    k = rng.random()
    if k < 0.04:
        kind, data = "broken", data[:-3] + b" 1x "
    elif k < 0.08:
        kind, data = "missing", data.rstrip()[:data.rstrip().rfind(b" ")] if b" " in data else data
    elif k < 0.12:
        kind, data = "extra", data + b" 7 "
    return data, rgb, mx, kind


def run(cases, seed, max_side=700, minutes=0.0, log=print):
    rng = np.random.default_rng(seed)
    enc = dmmt_jpeg.Encoder(0)
    t0, t_log = time.time(), time.time()
    stats = {"files": 0, "accepted": 0, "errors": 0, "bytes": 0, "samples": 0, "u16": 0}
    for case in range(cases):
        if minutes and time.time() - t0 > 60 * minutes:
            break
        data, rgb, mx, kind = make_file(rng, max_side)
        try:
            hdr = dmmt_jpeg.parse_ppm_header(data)
        except dmmt_jpeg.Error:  # (a truncation that reached into the header)
            continue
        sb = 1 if hdr.maxval <= 255 else 2
        n = hdr.width * hdr.height * 3
        ta, ra = int(rng.integers(0, 16)), int(rng.integers(0, 8))
        d_text = enc.malloc(len(data) + 64)
        d_rgb = enc.malloc(n * sb + 64)
        try:
            enc.h2d(d_text + ta, np.frombuffer(data, np.uint8))
            code = host_code(data)
            if code == 0 and int(rgb.max()) > mx:  # the host reader leaves the range check to the encoder
                code = -100  # DMMT_E_VALUE_EXCEEDS_MAX (color.rs:63-65)
            try:
                enc.decode_ppm_device(d_text + ta, len(data), hdr, d_rgb + ra)
                got = 0
            except dmmt_jpeg.Error as e:
                got = e.code
            ok = got == code
            if ok and code == 0:
                out = np.frombuffer(enc.d2h(d_rgb + ra, n * sb), np.uint8 if sb == 1 else np.uint16)
                ok = np.array_equal(out.astype(np.uint16), rgb.reshape(-1))
            if not ok:
                log(json.dumps({"mismatch": True, "case": case, "seed": seed, "kind": kind, "w": hdr.width,
                                "h": hdr.height, "maxval": mx, "text_align": ta, "rgb_align": ra,
                                "host_code": code, "gpu_code": got}))
                return {"mismatch": case}
        finally:
            enc.free(d_text)
            enc.free(d_rgb)
        stats["files"] += 1
        stats["accepted" if code == 0 else "errors"] += 1
        stats["bytes"] += len(data)
        stats["samples"] += n if code == 0 else 0
        stats["u16"] += sb == 2
        if stats["files"] % 200 == 0 or time.time() - t_log > 30:
            t_log = time.time()
            log(json.dumps({"progress": stats["files"], "s": round(time.time() - t0, 1), **stats}))
    summary = {"seed": seed, "seconds": round(time.time() - t0, 1), **stats, "mismatches": 0}
    log(json.dumps(summary))
    return summary


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-side", type=int, default=700)
    ap.add_argument("--minutes", type=float, default=0.0)
    a = ap.parse_args()
    res = run(a.cases, a.seed, a.max_side, a.minutes, log=lambda s: print(s, flush=True))
    sys.exit(1 if "mismatch" in res else 0)
