"""Probe: one small flat frame through the fused tables (k_hist's tail) and the
k_tables launch; prints both files' first scan bytes next to the oracle's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmmt-jpeg-encoder_amd")]
import numpy as np  # noqa: E402

import dmmt_jpeg  # noqa: E402
import oracle  # noqa: E402

f = np.zeros((64, 96, 3), np.uint8)
f[5, 7] = 255
luma, chroma = dmmt_jpeg.quality_tables(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(0), 8, luma_table=luma,
                                          chroma_table=chroma)
ref = oracle.encode(f, 255, 0, luma, chroma)
for fuse in ("1", "0"):
    os.environ["DMMT_FUSE_TABLES"] = fuse
    enc = dmmt_jpeg.Encoder(0)
    got = enc.encode(dmmt_jpeg.Image.from_array(f), opts)
    enc.close()
    k = next((i for i in range(min(len(got), len(ref))) if got[i] != ref[i]), None)
    print("fuse", fuse, "len", len(got), len(ref), "first diff", k, got[270:300].hex(), ref[270:300].hex())
