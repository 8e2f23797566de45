"""PPM ingest probe: decode one synthetic 4K frame's P3 text N times (for rocprof)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
import torch  # noqa: E402,F401
import bench  # noqa: E402
import dmmt_jpeg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
enc = dmmt_jpeg.Encoder(0)
print(bench.ppm_ingest(enc, 3840, 2160, n))
enc.close()
