"""Locate a GPU/oracle mismatch: front half (coefficients), back half (from the
oracle's coefficients) and the whole encode, for one synthetic image."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dmmt-jpeg-encoder_amd"))
sys.path.insert(0, ROOT)
import dmmt_jpeg  # noqa: E402
import oracle  # noqa: E402
from oracle.synth import synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--w", type=int, default=7680)
ap.add_argument("--h", type=int, default=4320)
ap.add_argument("--sub", type=int, default=2)
ap.add_argument("--q", type=int, default=95)
ap.add_argument("--frame", type=int, default=95)
a = ap.parse_args()
luma, chroma = dmmt_jpeg.quality_tables(a.q)
opts = dmmt_jpeg.JpegTransformationOptions(dmmt_jpeg.ChromaSubsamplingPreset(a.sub), 8, luma_table=luma,
                                           chroma_table=chroma)
rgb = synthetic(a.w, a.h, frame=a.frame)
enc = dmmt_jpeg.Encoder(0)
gc = enc.forward_blocks(dmmt_jpeg.Image.from_array(rgb), opts)
oc = oracle.forward(rgb, 255, a.sub, luma, chroma)
print("blocks", gc.shape, oc.shape)
n = min(len(gc), len(oc))
bad = np.nonzero((gc[:n] != oc[:n]).any(axis=1))[0]
print("front: differing blocks", len(bad), bad[:10])
for b in bad[:3]:
    print(b, "gpu", gc[b].tolist(), "\n   oracle", oc[b].tolist())
gb = enc.encode_coefficients(oc, a.w, a.h, opts)
ob = oracle.encode(rgb, 255, a.sub, luma, chroma, threads=8)
print("back half from oracle coefficients equal:", gb == ob, len(gb), len(ob))
if gb != ob:
    i = next(i for i in range(min(len(gb), len(ob))) if gb[i] != ob[i])
    print("  first diff at", i)
g = enc.encode(dmmt_jpeg.Image.from_array(rgb), opts)
print("whole encode equal:", g == ob, len(g))
if g != ob:
    i = next(i for i in range(min(len(g), len(ob))) if g[i] != ob[i])
    print("  first diff at", i)
