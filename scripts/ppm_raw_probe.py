"""Time dmmt_decode_ppm_device on bench.py's 4K P3 text, ignoring its return code
(timing-only ablation builds whose output is not a valid decode).
usage: python scripts/ppm_raw_probe.py [steps]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import dmmt_jpeg  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
enc = dmmt_jpeg.Encoder(0)
rgb, text, hdr, d_text, d_rgb = bench._p3_in_hbm(enc, 3840, 2160)
L = dmmt_jpeg.lib()
rc = L.dmmt_decode_ppm_device(enc._ctx, d_text, len(text), ctypes.byref(hdr), d_rgb, None)
for _ in range(3):
    L.dmmt_decode_ppm_device(enc._ctx, d_text, len(text), ctypes.byref(hdr), d_rgb, None)
t0 = time.perf_counter()
for _ in range(steps):
    L.dmmt_decode_ppm_device(enc._ctx, d_text, len(text), ctypes.byref(hdr), d_rgb, None)
dt = (time.perf_counter() - t0) / steps
print(json.dumps({"ms": round(dt * 1e3, 4), "rc": rc}))
